#!/bin/bash
# Kernel timeline of one clean randomized batch (tools/prof_rb.py) under rocprofv3.
# Usage: tools/gpu_rbprof.sh TAG B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
TAG=${1:-rbp}; B=${2:-64}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_$TAG -o run -- python3 tools/prof_rb.py 65536 $B > gpurun_out/prof_$TAG.log 2>&1 || { tail -5 gpurun_out/prof_$TAG.log; exit 1; }
python tools/timeline.py gpurun_out/prof_$TAG k_decode_g1 40 > gpurun_out/timeline_$TAG.txt && cat gpurun_out/timeline_$TAG.txt
