#!/bin/bash
# Roofline session: the integer-VALU rate table (tools/valu_peak, every launch shape), a quick
# C2 bench priced against it, then the PMC passes and kernel trace (tools/pmc_passes.sh).
# Usage: bash tools/gpu_roof.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
TAG=${1:-roof}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 180 ./tools/valu_peak > gpurun_out/valu_peak_$TAG.json \
 && cp gpurun_out/valu_peak_$TAG.json profiles/valu_peak_r04.json && echo "valu_peak ok" \
 && timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-secondary --no-cpu-baseline --no-aggregate > gpurun_out/qb_$TAG.json 2> gpurun_out/qb_$TAG.err \
 && echo "bench ok" \
 && bash tools/pmc_passes.sh $TAG
