#!/bin/bash
# Time several builds of libbls381 on the C2 workload in one session:
# variants/<name>/libbls381.so, selected through BLS381_LIB.  bench.py checks every
# verdict of the 2^16 batch against the expected ones, so a wrong build fails.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for v in "$@"; do
  BLS381_LIB=$PWD/variants/$v/libbls381.so timeout -k 10 240 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-aggregate --no-secondary > gpurun_out/variant_$v.json 2> gpurun_out/variant_$v.err || { echo "variant $v failed"; tail -3 gpurun_out/variant_$v.err; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/variant_$v.json').read().splitlines()[-1]); print('$v', round(d['value']), {k: round(v,2) for k,v in d['roofline']['kernel_avg_ms'].items()})"
done
