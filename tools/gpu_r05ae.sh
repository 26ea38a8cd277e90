#!/bin/bash
# r05: hash_to_G2's cofactor-map doublings on octets (k_hash_g2_o, lib/libbls381_hoct.so) --
# GPU suite on it, then latency and the C3 epoch with BLS381_HASH_OCT=0 / 1, alternating
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
TAG=${1:-r05ae}
mkdir -p gpurun_out
export TMPDIR=/tmp
export BLS381_LIB=$PWD/consensus-specs_amd/lib/libbls381_hoct.so
timeout -k 10 600 python -u -m pytest tests/ -x -v -m gpu -p no:cacheprovider --timeout 150 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1 \
 && echo "tests ok" && tail -1 gpurun_out/gpu_tests_$TAG.log || { tail -30 gpurun_out/gpu_tests_$TAG.log; exit 1; }
for r in 1 2; do
  for ho in 0 1; do
    BLS381_HASH_OCT=$ho timeout -k 10 120 python tools/lat_ab.py 40 > gpurun_out/lat_${TAG}_hoct${ho}_$r.txt 2>&1 || { cat gpurun_out/lat_${TAG}_hoct${ho}_$r.txt; exit 1; }
    echo "hash_oct=$ho run $r: $(tail -1 gpurun_out/lat_${TAG}_hoct${ho}_$r.txt)"
  done
done
for ho in 0 1; do
  BLS381_HASH_OCT=$ho timeout -k 10 600 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-aggregate --sections c3 > gpurun_out/bench_${TAG}_hoct$ho.json 2> gpurun_out/bench_${TAG}_hoct$ho.err || { tail -5 gpurun_out/bench_${TAG}_hoct$ho.err; exit 1; }
  python -c "
import json; d=json.loads(open('gpurun_out/bench_${TAG}_hoct$ho.json').read().splitlines()[-1])
c3=d.get('c3_epoch') or {}; lat=d.get('latency') or {}
print('hash_oct=$ho', 'c3', round(c3.get('attestations_per_s', 0)), 'grouped', round((c3.get('grouped') or {}).get('attestations_per_s', 0)), 'lat', {k: (round(v['ms'], 2) if isinstance(v, dict) and 'ms' in v else v) for k, v in lat.items()})
"
done
