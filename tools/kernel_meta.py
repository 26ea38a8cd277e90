"""Per-kernel register and scratch metadata of a gfx950 code object (no GPU).

  python tools/kernel_meta.py consensus-specs_amd/lib/libbls381.so [name-substring ...]

Prints .vgpr_count, .agpr_count, .sgpr_count and .private_segment_fixed_size (the scratch
frame per lane) from the code object's AMDGPU metadata note, for comparing build variants.
"""
import os
import re
import subprocess
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from extract_co import extract  # noqa: E402

READELF = "/opt/rocm/lib/llvm/bin/llvm-readelf"


def meta(lib):
    with tempfile.TemporaryDirectory() as d:
        co = os.path.join(d, "k.co")
        extract(lib, co)
        txt = subprocess.run([READELF, "--notes", co], capture_output=True, text=True).stdout
    out, cur = {}, {}
    for line in txt.splitlines():
        s = line.strip()
        m = re.match(r"^-?\s*\.(\w+):\s*(.*)$", s.lstrip("- "))
        if s.startswith("- ") and cur:
            if "name" in cur:
                out[cur["name"]] = cur
            cur = {}
        if m:
            cur[m.group(1)] = m.group(2).strip()
    if "name" in cur:
        out[cur["name"]] = cur
    return out


if __name__ == "__main__":
    lib, pats = sys.argv[1], sys.argv[2:]
    for name, k in sorted(meta(lib).items()):
        if "private_segment_fixed_size" not in k:
            continue
        if pats and not any(p in name for p in pats):
            continue
        print(f"{k.get('vgpr_count', '?'):>4} v {k.get('agpr_count', '?'):>4} a {k.get('sgpr_count', '?'):>4} s "
              f"{k.get('private_segment_fixed_size', '?'):>6} B  {name}")
