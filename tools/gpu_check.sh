#!/bin/bash
# GPU-box check: parity tests -> smoke -> short C2 bench.  Each GPU step has its
# own time limit; the chain stops at the first failure.  Usage: tools/gpu_check.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
TAG=${1:-chk}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/ -x -v -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1 \
 && echo "tests ok" \
 && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 \
 && echo "smoke ok" \
 && timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-secondary --no-cpu-baseline --no-aggregate > gpurun_out/qb_$TAG.json 2> gpurun_out/qb_$TAG.err \
 && echo "bench ok" && python -c "
import json; d=json.loads(open('gpurun_out/qb_$TAG.json').read().splitlines()[-1]); print(d['value'], {k: round(v, 2) for k, v in d['roofline']['kernel_avg_ms'].items()})"
rc=$?
tail -3 gpurun_out/gpu_tests_$TAG.log
exit $rc
