#!/bin/bash
# r05: octet pair tasks for verify_multiple -- GPU suite, then latency: default, and with the octet FE
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
TAG=${1:-r05z}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/ -x -v -m gpu -p no:cacheprovider --timeout 150 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1 \
 && echo "tests ok" && tail -1 gpurun_out/gpu_tests_$TAG.log || { tail -30 gpurun_out/gpu_tests_$TAG.log; exit 1; }
for r in 1 2; do
  for fo in 0 1; do
    BLS381_FE_OCT=$fo timeout -k 10 120 python tools/lat_ab.py 40 > gpurun_out/lat_${TAG}_feoct${fo}_$r.txt 2>&1 || { cat gpurun_out/lat_${TAG}_feoct${fo}_$r.txt; exit 1; }
    echo "fe_oct=$fo run $r: $(tail -1 gpurun_out/lat_${TAG}_feoct${fo}_$r.txt)"
  done
done
