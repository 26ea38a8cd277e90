#!/bin/bash
# r05: octet Miller loop for single calls -- GPU suite, then latency with BLS381_ML_OCTET=0 / 1 alternating.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
TAG=${1:-r05y}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/ -x -v -m gpu -p no:cacheprovider --timeout 150 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1 \
 && echo "tests ok" && tail -1 gpurun_out/gpu_tests_$TAG.log || { tail -30 gpurun_out/gpu_tests_$TAG.log; exit 1; }
for r in 1 2; do
  for o in 0 1; do
    BLS381_ML_OCTET=$o timeout -k 10 120 python tools/lat_ab.py 40 > gpurun_out/lat_${TAG}_oct${o}_$r.txt 2>&1 || { cat gpurun_out/lat_${TAG}_oct${o}_$r.txt; exit 1; }
    echo "octet=$o run $r: $(tail -1 gpurun_out/lat_${TAG}_oct${o}_$r.txt)"
  done
done
