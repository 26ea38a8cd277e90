#!/bin/bash
# Single-call latency against the pad count: 16 copies keep the quad kernels at one wave, 17 give them a
# second wave (the FE and the hash at 4 lanes per item, 64 lanes per wave).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
TAG=${1:-r05s}
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2; do
  for p in ${PADS:-1 9 16 17 32}; do
    BLS381_LAT_PAD=$p timeout -k 10 120 python tools/lat_ab.py 40 > gpurun_out/lat_${TAG}_pad${p}_$r.txt 2>&1 || { cat gpurun_out/lat_${TAG}_pad${p}_$r.txt; exit 1; }
    echo "run $r: $(tail -1 gpurun_out/lat_${TAG}_pad${p}_$r.txt)"
  done
done
