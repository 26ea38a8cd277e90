#!/bin/bash
# r05: GPU parity tests on the flat-free library, then a same-box A/B of the pre-refactor
# library (variants/pre), the flat-free library (base) and flat-free + csqr diet (variants/csqr).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
TAG=${1:-r05c}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/ -x -v -m gpu -p no:cacheprovider --timeout 150 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1 \
 && echo "tests ok" && tail -1 gpurun_out/gpu_tests_$TAG.log \
 && bash tools/ab_variants.sh $TAG 2 pre csqr
rc=$?
tail -3 gpurun_out/gpu_tests_$TAG.log
exit $rc
