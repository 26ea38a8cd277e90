"""Static call counts per function in a gfx950 code object (s_getpc + s_add_u32 -> s_swappc).

  python tools/call_graph.py /tmp/bls.co name_substring ...
Prints, for each matching function, its instruction count and the functions it calls
(how many call sites), so a kernel's dynamic work can be estimated from its loops."""
import collections
import re
import subprocess
import sys

dis = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-objdump", "-d", "--no-show-raw-insn", sys.argv[1]],
                     capture_output=True, text=True).stdout.splitlines()
funcs, cur = {}, None
addr_of = {}
for l in dis:
    m = re.match(r"^([0-9a-f]+) <(.+)>:", l)
    if m:
        cur = m.group(2); funcs[cur] = []; addr_of[int(m.group(1), 16)] = cur
        continue
    m = re.search(r"//\s*([0-9A-F]+):", l)
    if cur and m and not l.strip().startswith("//"):
        funcs[cur].append((int(m.group(1), 16), l.strip()))
for name, ins in funcs.items():
    if not any(s in name for s in sys.argv[2:]):
        continue
    calls = collections.Counter()
    pc = {}
    for a, t in ins:
        m = re.match(r"s_getpc_b64 s\[(\d+):", t)
        if m:
            pc[int(m.group(1))] = a + 4
            continue
        m = re.match(r"s_add_u32 s(\d+), s\1, (0x[0-9a-f]+|-?\d+)", t)
        if m and int(m.group(1)) in pc:
            off = int(m.group(2), 0) & 0xffffffff
            if off >= 1 << 31:
                off -= 1 << 32
            tgt = pc.pop(int(m.group(1))) + off
            calls[addr_of.get(tgt, hex(tgt))] += 1
    print(f"{len(ins):7d} {name[:90]}")
    for f, c in calls.most_common():
        print(f"        {c:4d} x {f[:90]} ({len(funcs.get(f, []))} instrs)")
