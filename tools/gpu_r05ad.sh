#!/bin/bash
# r05: the pair-split exponentiation in the Fp2 square root (lib/libbls381_pow.so) against the
# current library -- GPU suite on the new one, then latency and C2 alternating
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
TAG=${1:-r05ad}
mkdir -p gpurun_out
export TMPDIR=/tmp
NEW=$PWD/consensus-specs_amd/lib/libbls381_pow.so
OLD=$PWD/consensus-specs_amd/lib/libbls381.so
BLS381_LIB=$NEW timeout -k 10 600 python -u -m pytest tests/ -x -v -m gpu -p no:cacheprovider --timeout 150 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1 \
 && echo "tests ok" && tail -1 gpurun_out/gpu_tests_$TAG.log || { tail -30 gpurun_out/gpu_tests_$TAG.log; exit 1; }
for r in 1 2; do
  for v in old new; do
    L=$OLD; [ $v = new ] && L=$NEW
    BLS381_LIB=$L timeout -k 10 120 python tools/lat_ab.py 40 > gpurun_out/lat_${TAG}_${v}_$r.txt 2>&1 || { cat gpurun_out/lat_${TAG}_${v}_$r.txt; exit 1; }
    echo "$v run $r: $(tail -1 gpurun_out/lat_${TAG}_${v}_$r.txt)"
    BLS381_LIB=$L timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-secondary --no-aggregate > gpurun_out/bench_${TAG}_${v}_$r.json 2> gpurun_out/bench_${TAG}_${v}_$r.err || { tail -5 gpurun_out/bench_${TAG}_${v}_$r.err; exit 1; }
    python -c "
import json; d=json.loads(open('gpurun_out/bench_${TAG}_${v}_$r.json').read().splitlines()[-1])
k=d['roofline']['kernel_avg_ms']; print('$v c2', round(d['value']), {n: round(k[n], 3) for n in ('decode_g2', 'hash_cand', 'hash_bp', 'final_exp')})
"
  done
done
