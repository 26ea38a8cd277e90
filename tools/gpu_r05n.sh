#!/bin/bash
# r05: GPU parity tests (device-resident sharded aggregation, quad-form hash for latency batches),
# then the single-verify latency with the quad hash off / on, alternating, and the native RCCL lines.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
TAG=${1:-r05n}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/ -x -v -m gpu -p no:cacheprovider --timeout 150 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1 \
 && echo "tests ok" && tail -1 gpurun_out/gpu_tests_$TAG.log || { tail -30 gpurun_out/gpu_tests_$TAG.log; exit 1; }
for r in 1 2; do
  for q in 0 8192; do
    BLS381_HASH_QUAD_MAX_N=$q timeout -k 10 120 python tools/lat_ab.py 40 > gpurun_out/lat_${TAG}_q${q}_$r.txt 2>&1 || { cat gpurun_out/lat_${TAG}_q${q}_$r.txt; exit 1; }
    echo "quad_max=$q run $r: $(tail -1 gpurun_out/lat_${TAG}_q${q}_$r.txt)"
  done
done
timeout -k 10 600 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-aggregate --sections latency,rccl > gpurun_out/bench_${TAG}_sec.json 2> gpurun_out/bench_${TAG}_sec.err || { tail -5 gpurun_out/bench_${TAG}_sec.err; exit 1; }
python -c "
import json; d=json.loads(open('gpurun_out/bench_${TAG}_sec.json').read().splitlines()[-1])
print('value', d['value'], 'no_events', d.get('no_profiling_events'))
print('latency', d.get('latency'))
r=d.get('native_rccl') or {}
print('rccl c4 host', (r.get('c4_aggregate') or {}).get('pubkeys_aggregated_per_s'), 'device', (r.get('c4_aggregate_device') or {}).get('pubkeys_aggregated_per_s'))
"
