#!/bin/bash
# Round-end measurement session: GPU parity tests -> smoke -> full bench -> rocprofv3 kernel
# trace of the C2 bench -> PMC passes + kernel trace of the profiling workload.  Every GPU step
# has its own time limit and the chain stops at the first failure.  Usage: tools/gpu_final.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
TAG=${1:-final}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/ -x -v -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1 \
 && echo "tests ok" && tail -1 gpurun_out/gpu_tests_$TAG.log \
 && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 \
 && echo "smoke ok" \
 && timeout -k 10 900 python bench.py --steps 5 --warmup 1 --fail-on-secondary-error > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err \
 && echo "bench ok" \
 && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o prof -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-secondary --no-aggregate > gpurun_out/rocprof_$TAG.log 2>&1 \
 && echo "rocprof ok" \
 && bash tools/pmc_passes.sh $TAG
rc=$?
tail -2 gpurun_out/gpu_tests_$TAG.log
exit $rc
