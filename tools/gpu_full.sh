#!/bin/bash
# GPU-box session: parity tests -> smoke -> full bench (all lines).  Usage: tools/gpu_full.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
TAG=${1:-full}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/ -x -v -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1 \
 && echo "tests ok" \
 && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 \
 && echo "smoke ok" \
 && timeout -k 10 600 python bench.py --steps 3 --warmup 1 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err \
 && echo "bench ok"
rc=$?
tail -3 gpurun_out/gpu_tests_$TAG.log
[ -s gpurun_out/bench_$TAG.err ] && tail -3 gpurun_out/bench_$TAG.err
exit $rc
