"""Kernel timeline of one traced call from a rocprofv3 --kernel-trace database.

Usage: python tools/timeline.py <prof_dir_or_db> [first_kernel_substring] [count]
Prints start offset, duration and queue of `count` consecutive dispatches starting at
the last dispatch whose name contains `first_kernel_substring` -- which kernels of a
pipeline overlap on the side stream and which sit on the critical path.
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
    first = sys.argv[2] if len(sys.argv) > 2 else ""
    count = int(sys.argv[3]) if len(sys.argv) > 3 else 40
    c = sqlite3.connect(path)
    rows = c.execute("select name, start, end, queue_id from kernels order by start").fetchall()
    idx = [i for i, r in enumerate(rows) if first in r[0]]
    i0 = idx[-1] if idx else 0
    t0 = rows[i0][1]
    for name, s, e, q in rows[i0:i0 + count]:
        m = re.search(r"(k_[A-Za-z0-9_]+(?:<[^>]*>)?)", name)
        print("%9.3f ms  +%8.3f ms  q%-3s %s" % ((s - t0) / 1e6, (e - s) / 1e6, q, m.group(1) if m else name[:50]))


if __name__ == "__main__":
    main()
