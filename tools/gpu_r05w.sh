#!/bin/bash
# r05: full-wave latency kernels -- GPU suite, then single-call latency at 1 and 16 copies, alternating.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
TAG=${1:-r05w}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/ -x -v -m gpu -p no:cacheprovider --timeout 150 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1 \
 && echo "tests ok" && tail -1 gpurun_out/gpu_tests_$TAG.log || { tail -30 gpurun_out/gpu_tests_$TAG.log; exit 1; }
PADS="1 16" bash tools/gpu_lat_pads.sh $TAG
