"""Extract the gfx950 code object from a HIP shared library's offload bundle and
summarise the instruction mix per function (static counts from llvm-objdump).

  python tools/extract_co.py consensus-specs_amd/lib/libbls381.so /tmp/bls.co [func ...]

Used to read the kernels' instruction classes (v_mad_u64_u32, DPP moves, scratch
accesses, plain moves) before spending GPU time on a build variant.
"""
import collections
import re
import subprocess
import sys

MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"


def extract(lib, out):
    data = open(lib, "rb").read()
    pos = data.find(MAGIC)
    while pos >= 0:
        p = pos + len(MAGIC)
        n = int.from_bytes(data[p:p + 8], "little"); p += 8
        for _ in range(n):
            off = int.from_bytes(data[p:p + 8], "little"); p += 8
            size = int.from_bytes(data[p:p + 8], "little"); p += 8
            tl = int.from_bytes(data[p:p + 8], "little"); p += 8
            triple = data[p:p + tl].decode(); p += tl
            if "gfx950" in triple and size:
                open(out, "wb").write(data[pos + off:pos + off + size])
                return triple
        pos = data.find(MAGIC, pos + 1)
    raise SystemExit("no gfx950 code object found")


def summarise(co, funcs):
    dis = subprocess.run([OBJDUMP, "-d", "--no-show-raw-insn", co], capture_output=True, text=True).stdout
    cur, stats = None, collections.defaultdict(collections.Counter)
    for line in dis.splitlines():
        m = re.match(r"^[0-9a-f]+ <(.+)>:", line)
        if m:
            cur = m.group(1)
            continue
        s = line.strip().split()
        if not cur or not s or s[0].startswith(";"):
            continue
        op = s[0]
        c = stats[cur]
        c["total"] += 1
        if op.startswith("v_mad_u64_u32") or op.startswith("v_mad_i64_i32"):
            c["mad64"] += 1
        elif "dpp" in line:
            c["dpp"] += 1
        elif op.startswith("scratch_store") or op.startswith("buffer_store"):
            c["scratch_st"] += 1
        elif op.startswith("scratch_load") or op.startswith("buffer_load"):
            c["scratch_ld"] += 1
        elif op.startswith("v_mov_b32") or op.startswith("v_mov_b64"):
            c["v_mov"] += 1
        elif op.startswith("v_accvgpr"):
            c["agpr_mov"] += 1
        elif op.startswith("s_"):
            c["salu"] += 1
        elif op.startswith("global_"):
            c["global"] += 1
        else:
            c["valu_other"] += 1
    names = [f for f in stats if any(x in f for x in funcs)] if funcs else sorted(stats, key=lambda f: -stats[f]["total"])[:40]
    for f in names:
        c = stats[f]
        print(f"{c['total']:7d} mad={c['mad64']:6d} dpp={c['dpp']:5d} mov={c['v_mov']:5d} agpr={c['agpr_mov']:5d} "
              f"scr_st={c['scratch_st']:4d} scr_ld={c['scratch_ld']:4d} other={c['valu_other']:6d} salu={c['salu']:5d}  {f[:110]}")


if __name__ == "__main__":
    lib, out = sys.argv[1], sys.argv[2]
    print(extract(lib, out))
    summarise(out, sys.argv[3:])
