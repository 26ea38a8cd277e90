#!/bin/bash
# Kernel trace of single unpadded calls (the default latency path): per-kernel durations and the
# timeline of one bls_verify call (tools/timeline.py reads the trace)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
TAG=${1:-r05ac}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/lattrace_${TAG} -o kt -- python3 tools/lat_ab.py 40 > gpurun_out/lattrace_${TAG}.log 2>&1 || { tail -5 gpurun_out/lattrace_${TAG}.log; exit 1; }
echo "trace ok: $(tail -1 gpurun_out/lattrace_${TAG}.log)"
