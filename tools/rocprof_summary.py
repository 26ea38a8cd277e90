"""Summarise a rocprofv3 kernel trace (SQLite .db or kernel_stats.csv) per kernel.

Usage: python tools/rocprof_summary.py <prof_dir_or_db> [out.md]
Writes a markdown table: kernel, calls, avg/min/max duration (ms), total share,
VGPRs, scratch bytes/lane -- the summary committed under profiles/.
"""
import glob
import os
import re
import sqlite3
import sys
from collections import defaultdict


def short(name):
    m = re.search(r"(k_[A-Za-z0-9_]+)", name)
    return m.group(1) if m else name[:60]


def from_db(path):
    c = sqlite3.connect(path)
    rows = c.execute("select name, duration, vgpr_count, accum_vgpr_count, scratch_size, grid_x, workgroup_x "
                     "from kernels").fetchall()
    agg = defaultdict(lambda: {"n": 0, "tot": 0.0, "mn": 1e30, "mx": 0.0, "vgpr": 0, "scratch": 0, "grid": 0})
    for name, dur, vg, ag, sc, gx, wx in rows:
        a = agg[short(name)]
        d = dur / 1e6
        a["n"] += 1; a["tot"] += d; a["mn"] = min(a["mn"], d); a["mx"] = max(a["mx"], d)
        a["vgpr"] = max(a["vgpr"], (vg or 0) + (ag or 0)); a["scratch"] = max(a["scratch"], sc or 0)
        a["grid"] = max(a["grid"], gx or 0)
    return agg


def from_csv(path):
    """the same aggregation from a --output-format csv kernel trace (*_kernel_trace.csv)"""
    import csv
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((r["Kernel_Name"], int(r["End_Timestamp"]) - int(r["Start_Timestamp"]), int(r["VGPR_Count"] or 0),
                         int(r["Accum_VGPR_Count"] or 0), int(r["Scratch_Size"] or 0), int(r["Grid_Size_X"] or 0),
                         int(r["Workgroup_Size_X"] or 0)))
    agg = defaultdict(lambda: {"n": 0, "tot": 0.0, "mn": 1e30, "mx": 0.0, "vgpr": 0, "scratch": 0, "grid": 0})
    for name, dur, vg, ag, sc, gx, wx in rows:
        a = agg[short(name)]
        d = dur / 1e6
        a["n"] += 1; a["tot"] += d; a["mn"] = min(a["mn"], d); a["mx"] = max(a["mx"], d)
        a["vgpr"] = max(a["vgpr"], vg + ag); a["scratch"] = max(a["scratch"], sc)
        a["grid"] = max(a["grid"], gx)
    return agg


def main():
    src = sys.argv[1]
    if os.path.isdir(src):
        dbs = glob.glob(os.path.join(src, "**", "*.db"), recursive=True)
        csvs = glob.glob(os.path.join(src, "**", "*kernel_trace.csv"), recursive=True)
        src = dbs[0] if dbs else csvs[0]
    agg = from_csv(src) if src.endswith(".csv") else from_db(src)
    total = sum(a["tot"] for a in agg.values())
    lines = ["| kernel | calls | avg ms | min ms | max ms | share | VGPR+AGPR | scratch B/lane | grid (lanes) |",
             "|---|---|---|---|---|---|---|---|---|"]
    for k, a in sorted(agg.items(), key=lambda kv: -kv[1]["tot"]):
        lines.append("| %s | %d | %.3f | %.3f | %.3f | %.1f%% | %d | %d | %d |" % (
            k, a["n"], a["tot"] / a["n"], a["mn"], a["mx"], 100 * a["tot"] / total, a["vgpr"], a["scratch"], a["grid"]))
    out = "\n".join(lines)
    print(out)
    if len(sys.argv) > 2:
        with open(sys.argv[2], "w") as f:
            f.write(out + "\n")


if __name__ == "__main__":
    main()
