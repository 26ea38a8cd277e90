#!/bin/bash
# Time several builds of libbls381 (BLS381_LIB) on the same workload in one session.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for v in "$@"; do
  BLS381_LIB=$PWD/consensus-specs_amd/lib/libbls381_$v.so timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-aggregate > gpurun_out/variant_$v.json 2> gpurun_out/variant_$v.err || { echo "variant $v failed"; tail -3 gpurun_out/variant_$v.err; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/variant_$v.json')); print('$v', round(d['value']), {k: round(v,2) for k,v in d['roofline']['kernel_avg_ms'].items()})"
done
