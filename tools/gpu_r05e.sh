#!/bin/bash
# r05: GPU parity tests with the pair-split inversion, the Fp2-product leaf micro-bench, and
# fe_phases cycle counts before (fe_phases_v2) / after (fe_phases_pinv) the pair inversion.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
TAG=${1:-r05e}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/ -x -v -m gpu -p no:cacheprovider --timeout 150 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1 \
 && echo "tests ok" && tail -1 gpurun_out/gpu_tests_$TAG.log \
 && timeout -k 5 120 ./tools/leaf_bench 65536 2.1 > gpurun_out/leaf_$TAG.json && cat gpurun_out/leaf_$TAG.json \
 && timeout -k 5 120 ./tools/fe_phases_v2 > gpurun_out/fe_v2_$TAG.txt && cat gpurun_out/fe_v2_$TAG.txt \
 && timeout -k 5 120 ./tools/fe_phases_pinv > gpurun_out/fe_pinv_$TAG.txt && cat gpurun_out/fe_pinv_$TAG.txt
rc=$?
tail -3 gpurun_out/gpu_tests_$TAG.log
exit $rc
