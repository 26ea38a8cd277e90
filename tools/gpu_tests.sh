#!/bin/bash
# The GPU suite alone: bash tools/gpu_tests.sh TAG  (log gpurun_out/gpu_tests_TAG.log)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -x -v -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_${1:-r06}.log 2>&1; rc=$?; tail -3 gpurun_out/gpu_tests_${1:-r06}.log; exit $rc
