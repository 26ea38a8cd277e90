#!/bin/bash
# r05: the native-communicator tests (host and device aggregation forms share one protocol now),
# then the full GPU suite, then the RCCL bench lines.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
TAG=${1:-r05o}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v -m gpu -p no:cacheprovider --timeout 150 --timeout-method thread -k "native_comm" > gpurun_out/gpu_comm_$TAG.log 2>&1 \
 && echo "comm tests ok" && tail -1 gpurun_out/gpu_comm_$TAG.log || { tail -40 gpurun_out/gpu_comm_$TAG.log; exit 1; }
timeout -k 10 900 python -u -m pytest tests/ -x -v -m gpu -p no:cacheprovider --timeout 150 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1 \
 && echo "tests ok" && tail -1 gpurun_out/gpu_tests_$TAG.log || { tail -30 gpurun_out/gpu_tests_$TAG.log; exit 1; }
timeout -k 10 600 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-aggregate --sections rccl,c4 > gpurun_out/bench_${TAG}_sec.json 2> gpurun_out/bench_${TAG}_sec.err || { tail -5 gpurun_out/bench_${TAG}_sec.err; exit 1; }
python -c "
import json; d=json.loads(open('gpurun_out/bench_${TAG}_sec.json').read().splitlines()[-1])
print('value', d['value'], 'no_events', d.get('no_profiling_events'))
r=d.get('native_rccl') or {}
print('rccl c4 host', (r.get('c4_aggregate') or {}).get('pubkeys_aggregated_per_s'), 'device', (r.get('c4_aggregate_device') or {}).get('pubkeys_aggregated_per_s'))
print('c4 plain', (d.get('c4_aggregate') or {}).get('pubkeys_aggregated_per_s'))
"
