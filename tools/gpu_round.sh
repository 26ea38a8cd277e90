#!/bin/bash
# One GPU-box session: parity tests -> smoke -> bench -> rocprofv3 kernel trace.
# Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
TAG=${1:-r01}
STEPS=${BENCH_STEPS:-3}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/ -x -v -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1 \
 && echo "tests ok" \
 && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 \
 && echo "smoke ok" \
 && timeout -k 10 900 python bench.py --steps $STEPS --warmup 1 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err \
 && echo "bench ok" && cat gpurun_out/bench_$TAG.json \
 && timeout -k 10 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o prof -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-secondary > gpurun_out/rocprof_$TAG.log 2>&1 \
 && echo "rocprof ok"
rc=$?
tail -5 gpurun_out/gpu_tests_$TAG.log
exit $rc
