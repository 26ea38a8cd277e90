#!/bin/bash
# Single-call latency, padded (32 copies) against unpadded, alternating; then a kernel trace of each
# (rocprofv3 --kernel-trace --stats, no counters) for the per-kernel duration distributions.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
TAG=${1:-r05q}
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2; do
  for p in 1 32; do
    BLS381_LAT_PAD=$p timeout -k 10 120 python tools/lat_ab.py 40 > gpurun_out/lat_${TAG}_pad${p}_$r.txt 2>&1 || { cat gpurun_out/lat_${TAG}_pad${p}_$r.txt; exit 1; }
    echo "run $r: $(tail -1 gpurun_out/lat_${TAG}_pad${p}_$r.txt)"
  done
done
for p in 1 32; do
  BLS381_LAT_PAD=$p timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/lattrace_${TAG}_pad$p -o kt -- python3 tools/lat_ab.py 40 > gpurun_out/lattrace_${TAG}_pad$p.log 2>&1 || { tail -5 gpurun_out/lattrace_${TAG}_pad$p.log; exit 1; }
  echo "trace pad $p ok"
done
