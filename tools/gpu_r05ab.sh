#!/bin/bash
# r05: octet FE with octet squarings too -- GPU suite, latency with BLS381_FE_OCT=2 / 3, then the secondary
# lines that use small-batch final exponentiations (C3 epoch, randomized) under each
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
TAG=${1:-r05ab}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/ -x -v -m gpu -p no:cacheprovider --timeout 150 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1 \
 && echo "tests ok" && tail -1 gpurun_out/gpu_tests_$TAG.log || { tail -30 gpurun_out/gpu_tests_$TAG.log; exit 1; }
for r in 1 2; do
  for fo in 2 3; do
    BLS381_FE_OCT=$fo timeout -k 10 120 python tools/lat_ab.py 40 > gpurun_out/lat_${TAG}_feoct${fo}_$r.txt 2>&1 || { cat gpurun_out/lat_${TAG}_feoct${fo}_$r.txt; exit 1; }
    echo "fe_oct=$fo run $r: $(tail -1 gpurun_out/lat_${TAG}_feoct${fo}_$r.txt)"
  done
done
for fo in 2 3; do
  BLS381_FE_OCT=$fo timeout -k 10 600 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-aggregate --sections c3,randomized > gpurun_out/bench_${TAG}_fe$fo.json 2> gpurun_out/bench_${TAG}_fe$fo.err || { tail -5 gpurun_out/bench_${TAG}_fe$fo.err; exit 1; }
  python -c "
import json; d=json.loads(open('gpurun_out/bench_${TAG}_fe$fo.json').read().splitlines()[-1])
c3=d.get('c3_epoch') or {}; rb=d.get('c2_randomized_batch') or {}
print('fe_oct=$fo', 'c2', round(d['value']), 'c3', {k: (round(v) if isinstance(v,(int,float)) else v) for k,v in c3.items() if 'per_s' in k or k.startswith('ms')}, 'rb clean', round((rb.get('clean') or {}).get('verifications_per_s', 0)))
"
done
