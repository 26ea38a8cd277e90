"""Aggregate rocprofv3 --pmc CSV passes per kernel (last dispatch of each kernel).

Usage: python tools/pmc_summary.py gpurun_out/pmc_TAG [out.md]
"""
import csv
import json
import glob
import os
import re
import sys
from collections import defaultdict


def short(name):
    """k_name, or k_name<args> for a template instance (demangled names; namespaces dropped)"""
    m = re.search(r"(k_[A-Za-z0-9_]+)(<[^()]*>)?", name)
    if not m:
        return name[:50]
    return m.group(1) + (re.sub(r"\s+|[A-Za-z0-9_]+::", "", m.group(2)) if m.group(2) else "")


def kernel_ms(d):
    """average kernel duration (ms) per kernel from a --kernel-trace --stats pass under d/kt, if present"""
    tot = defaultdict(lambda: [0, 0.0])
    for f in glob.glob(os.path.join(d, "kt", "**", "*kernel_trace.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                t = tot[short(row["Kernel_Name"])]
                t[0] += 1
                t[1] += (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-6
    return {k: v[1] / v[0] for k, v in tot.items() if v[0]}


def main():
    d = sys.argv[1]
    data = defaultdict(dict)     # kernel -> counter -> value (last dispatch)
    last_disp = defaultdict(dict)
    for f in sorted(glob.glob(os.path.join(d, "p*", "*counter_collection.csv"))):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = short(row["Kernel_Name"])
                c = row["Counter_Name"]
                disp = int(row["Dispatch_Id"])
                v = float(row["Counter_Value"])
                key = (k, c)
                prev = last_disp[k].get(c)
                if prev is None or disp > prev[0]:
                    last_disp[k][c] = (disp, v)
                elif disp == prev[0]:
                    last_disp[k][c] = (disp, prev[1] + v)   # sum over dimensions
    for k, cs in last_disp.items():
        for c, (disp, v) in cs.items():
            data[k][c] = v
    cols = ["SQ_WAVES", "SQ_INSTS_VALU", "SQ_INSTS_VALU_INT32", "SQ_INSTS_VALU_INT64", "SQ_INSTS_SALU",
            "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR", "SQ_INSTS_FLAT", "SQ_INSTS_LDS", "SQ_WAVE_CYCLES",
            "SQ_BUSY_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_ANY",
            "GRBM_GUI_ACTIVE", "FETCH_SIZE", "WRITE_SIZE"]
    kernels = [k for k in data if k.startswith("k_")]
    lines = ["| counter | " + " | ".join(kernels) + " |", "|---|" + "---|" * len(kernels)]
    for c in cols:
        lines.append("| %s | " % c + " | ".join("%.4g" % data[k].get(c, float("nan")) for k in kernels) + " |")
    # derived
    lines.append("| VALU insts / wave | " + " | ".join(
        "%.4g" % (data[k].get("SQ_INSTS_VALU", 0) / max(data[k].get("SQ_WAVES", 1), 1)) for k in kernels) + " |")
    lines.append("| VMEM (rd+wr) / VALU | " + " | ".join(
        "%.3f" % ((data[k].get("SQ_INSTS_VMEM_RD", 0) + data[k].get("SQ_INSTS_VMEM_WR", 0)) /
                  max(data[k].get("SQ_INSTS_VALU", 1), 1)) for k in kernels) + " |")
    lines.append("| WAIT_ANY / WAVE_CYCLES | " + " | ".join(
        "%.3f" % (data[k].get("SQ_WAIT_ANY", 0) / max(data[k].get("SQ_WAVE_CYCLES", 1), 1)) for k in kernels) + " |")
    lines.append("| HBM bytes (2*FETCH_KB*1024 + WRITE_KB*1024) | " + " | ".join(
        "%.4g" % (2 * data[k].get("FETCH_SIZE", 0) * 1024 + data[k].get("WRITE_SIZE", 0) * 1024) for k in kernels) + " |")
    kms = kernel_ms(d)
    if kms:
        lines.append("| avg ms (kernel trace) | " + " | ".join("%.4g" % kms.get(k, float("nan")) for k in kernels) + " |")
        lines.append("| HBM GB/s | " + " | ".join(
            "%.4g" % ((2 * data[k].get("FETCH_SIZE", 0) * 1024 + data[k].get("WRITE_SIZE", 0) * 1024) /
                      (kms[k] * 1e-3) / 1e9 if kms.get(k) else float("nan")) for k in kernels) + " |")
    out = "\n".join(lines)
    print(out)
    if len(sys.argv) > 2:
        open(sys.argv[2], "w").write(out + "\n")
        # machine-readable companion read by bench.py (roofline.traffic): HBM bytes per launch of each
        # kernel, FETCH_SIZE doubled per MI355X_MICROARCH.md "HBM" (gfx950 tallies 128-B reads at 64 B)
        js = {k: {"hbm_bytes_per_launch": 2 * data[k].get("FETCH_SIZE", 0) * 1024 + data[k].get("WRITE_SIZE", 0) * 1024,
                  "fetch_kb": data[k].get("FETCH_SIZE"), "write_kb": data[k].get("WRITE_SIZE"),
                  "valu_insts": data[k].get("SQ_INSTS_VALU"), "valu_int64_insts": data[k].get("SQ_INSTS_VALU_INT64"),
                  "valu_int32_insts": data[k].get("SQ_INSTS_VALU_INT32"), "waves": data[k].get("SQ_WAVES"),
                  "wait_any_frac": data[k].get("SQ_WAIT_ANY", 0) / max(data[k].get("SQ_WAVE_CYCLES", 1), 1),
                  "avg_ms": kms.get(k)}
              for k in kernels}
        json.dump({"source": os.path.basename(os.path.normpath(d)), "workload": "tools/prof_workload.py",
                   "kernels": js}, open(os.path.splitext(sys.argv[2])[0] + ".json", "w"), indent=1)


if __name__ == "__main__":
    main()
