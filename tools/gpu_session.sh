#!/bin/bash
# One GPU-box session: microbenchmarks, parity tests, smoke, quick C2 bench, then optional
# build variants (variants/<name>/libbls381.so) last -- a variant that faults ends the call.
# Usage: tools/gpu_session.sh TAG [variant ...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
TAG=${1:-s}; shift
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -x tools/csqr_bench ]; then
  timeout -k 10 120 ./tools/csqr_bench > gpurun_out/csqr_bench_$TAG.json 2>&1 || { echo "csqr_bench failed"; exit 1; }
  cat gpurun_out/csqr_bench_$TAG.json
fi
timeout -k 10 600 python -u -m pytest tests/ -x -v -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1 \
 && echo "tests ok" \
 && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 \
 && echo "smoke ok" \
 && timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-secondary --no-cpu-baseline --no-aggregate > gpurun_out/qb_$TAG.json 2> gpurun_out/qb_$TAG.err \
 && python -c "
import json; d=json.loads(open('gpurun_out/qb_$TAG.json').read().splitlines()[-1]); print(d['value'], {k: round(v, 2) for k, v in d['roofline']['kernel_avg_ms'].items()})"
rc=$?
tail -3 gpurun_out/gpu_tests_$TAG.log
[ $rc -ne 0 ] && exit $rc
for v in "$@"; do
  BLS381_LIB=$PWD/variants/$v/libbls381.so timeout -k 10 240 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-aggregate --no-secondary > gpurun_out/variant_${v}_$TAG.json 2> gpurun_out/variant_${v}_$TAG.err || { echo "variant $v failed rc=$?"; tail -5 gpurun_out/variant_${v}_$TAG.err; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/variant_${v}_$TAG.json').read().splitlines()[-1]); print('$v', round(d['value']), {k: round(x,2) for k,x in d['roofline']['kernel_avg_ms'].items()})"
done
