"""Static scratch-frame audit of a kernel's call tree in a gfx950 code object (no GPU).

  python tools/frame_check.py consensus-specs_amd/lib/libbls381.so k_final_exp_verdictEm

For the kernel and every function it reaches through s_swappc it prints:
  * the frame (the kernel's initial s32, or the callee's s_addk_i32 s32 adjustment);
  * the deepest call chain's frame sum, to compare with .private_segment_fixed_size;
  * the furthest frame-relative (s33) scratch access and whether it stays in the frame;
  * scratch accesses addressed by a VGPR (sret / by-reference operands) and flat
    accesses (by-reference operands passed as generic pointers);
  * whether every return path restores s32 / s33.
Used for DESIGN.md §10.7 (the round-2 max-ilp illegal-address fault), where the faulting
build is rebuilt from git and audited instead of being launched again.
"""
import bisect
import collections
import os
import re
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from extract_co import extract  # noqa: E402

OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"
READELF = "/opt/rocm/lib/llvm/bin/llvm-readelf"
WIDTH = {"dword": 4, "dwordx2": 8, "dwordx3": 12, "dwordx4": 16, "byte": 1, "short": 2, "ubyte": 1, "ushort": 2,
         "sbyte": 1, "sshort": 2}


def load(co):
    dis = subprocess.run([OBJDUMP, "-d", "--no-show-raw-insn", co], capture_output=True, text=True).stdout.splitlines()
    starts = []
    for i, ln in enumerate(dis):
        m = re.match(r"^([0-9a-f]+) <(.+)>:", ln)
        if m:
            starts.append((int(m.group(1), 16), m.group(2), i))
    starts.sort()
    bodies = {}
    for k, (a, n, i) in enumerate(starts):
        e = starts[k + 1][2] if k + 1 < len(starts) else len(dis)
        bodies[n] = dis[i + 1:e]
    return starts, bodies


def func_at(starts, addr):
    k = bisect.bisect_right([a for a, _, _ in starts], addr) - 1
    return starts[k][1] if k >= 0 else None


def callees(starts, body):
    regs, out = {}, set()
    for j, ln in enumerate(body):
        m = re.search(r"s_getpc_b64 s\[(\d+):\d+\]\s+//\s*([0-9A-F]+):", ln)
        if m:
            r0, pc = int(m.group(1)), int(m.group(2), 16) + 4
            for ln2 in body[j + 1:j + 4]:
                m2 = re.search(r"s_add_u32 s%d, s%d, (0x[0-9a-f]+|\d+)" % (r0, r0), ln2)
                if m2:
                    off = int(m2.group(1), 0)
                    regs[r0] = pc + (off - 2 ** 32 if off >= 2 ** 31 else off)
                    break
        m = re.search(r"s_swappc_b64 s\[\d+:\d+\], s\[(\d+):\d+\]", ln)
        if m and int(m.group(1)) in regs:
            out.add(func_at(starts, regs[int(m.group(1))]))
    return out


def frame(body):
    for ln in body:
        m = re.search(r"s_movk_i32 s32, (0x[0-9a-f]+|\d+)", ln)
        if m:
            return int(m.group(1), 0)
        m = re.search(r"s_(?:addk_i32|add_i32) s32, (?:s32, )?(0x[0-9a-f]+|\d+)", ln)
        if m:
            return int(m.group(1), 0)
    return 0


def audit(body):
    fr = frame(body)
    far, vaddr, flat = 0, 0, 0
    for ln in body:
        m = re.search(r"scratch_(?:load|store)_(\w+) .*s33(?: offset:(\d+))?", ln)
        if m:
            far = max(far, int(m.group(2) or 0) + WIDTH.get(m.group(1).split("_")[-1], 4))
        if re.search(r"scratch_store_\w+ v\d+,", ln) or re.search(r"scratch_load_\w+ v[\[\d][^,]*, v\d+,", ln):
            vaddr += 1
        if "flat_load" in ln or "flat_store" in ln:
            flat += 1
    rets = sum("s_setpc_b64" in ln for ln in body)
    restores = sum(bool(re.search(r"s_mov_b32 s32, s33|s_addk_i32 s32, 0x[89a-f]", ln)) for ln in body)
    return fr, far, vaddr, flat, rets, restores


def main():
    lib, kern = sys.argv[1], sys.argv[2]
    co = "/tmp/frame_check.co"
    extract(lib, co)
    starts, bodies = load(co)
    meta = subprocess.run([READELF, "--notes", co], capture_output=True, text=True).stdout
    names = [n for n in bodies if kern in n]
    if not names:
        raise SystemExit("no function matching %r" % kern)
    root = names[0]
    m = re.search(re.escape(root) + r".*?\.private_segment_fixed_size:\s+(\d+)", meta, re.S)
    pss = int(m.group(1)) if m else None
    seen, memo = [], {}

    def depth(n, path=()):
        if n in path:
            return 0, ["recursion " + n]
        if n not in memo:
            best, chain = 0, []
            for c in callees(starts, bodies[n]):
                if c is None or c not in bodies:
                    continue
                d, p = depth(c, path + (n,))
                if d > best:
                    best, chain = d, p
            memo[n] = (frame(bodies[n]) + best, [(n, frame(bodies[n]))] + chain)
        return memo[n]

    def walk(n):
        if n in seen or n not in bodies:
            return
        seen.append(n)
        for c in sorted(x for x in callees(starts, bodies[n]) if x):
            walk(c)
    walk(root)
    total, chain = depth(root)
    print("kernel %s: .private_segment_fixed_size %s, deepest chain %d B" % (root, pss, total))
    for n, f in chain:
        print("   %6d  %s" % (f, n[:90]))
    print("%-70s %6s %8s %6s %5s %5s" % ("function", "frame", "s33-end", "vaddr", "flat", "ret/restore"))
    ok = True
    for n in seen:
        fr, far, va, fl, rets, rest = audit(bodies[n])
        inside = far <= fr or n == root
        ok &= inside
        print("%-70s %6d %8d %6d %5d %3d/%d%s" % (n[:70], fr, far, va, fl, rets, rest, "" if inside else "  OUTSIDE FRAME"))
    print("frames consistent:", ok and (pss is None or total == pss))


if __name__ == "__main__":
    main()
