"""Per-step prologue of the C2 pipeline from a rocprofv3 --kernel-trace database.

  python tools/prologue_spans.py <prof_dir_or_db>

For every C2 step: the one-lane launches (k_hash_cand_1, k_decode_g1, k_decode_g2_1 on three
streams, or the fused k_prologue_1) and the span from the first of them to the start of k_hash_bp,
which waits for all of them -- the prologue's length on the step's critical path.
"""
import glob
import os
import re
import sqlite3
import sys


def main():
    path = sys.argv[1]
    if os.path.isdir(path):
        path = glob.glob(os.path.join(path, "**", "*.db"), recursive=True)[0]
    rows = sqlite3.connect(path).execute("select name, start, end from kernels order by start").fetchall()
    name = lambda n: (re.search(r"(k_[A-Za-z0-9_]+)", n) or re.search(r"(.{1,30})", n)).group(1)
    rows = [(name(n), s, e) for n, s, e in rows]
    firsts = {"k_hash_cand_1", "k_decode_g1", "k_decode_g2_1", "k_prologue_1"}
    print("%-60s %s" % ("one-lane launches (ms)", "prologue span to k_hash_bp (ms), k_hash_bp (ms)"))
    i = 0
    while i < len(rows):
        if rows[i][0] not in firsts:
            i += 1
            continue
        grp, j = [], i
        while j < len(rows) and rows[j][0] in firsts:
            grp.append(rows[j])
            j += 1
        bp = next((r for r in rows[j:j + 3] if r[0] == "k_hash_bp"), None)
        t0 = min(s for _, s, _ in grp)
        desc = ", ".join("%s %.2f" % (n.replace("k_", ""), (e - s) / 1e6) for n, s, e in grp)
        if bp:
            print("%-60s %.2f, %.2f" % (desc, (bp[1] - t0) / 1e6, (bp[2] - bp[1]) / 1e6))
        i = j


if __name__ == "__main__":
    main()
