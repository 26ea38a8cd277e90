#!/bin/bash
# Same-box A/B of build variants (variants/<name>/libbls381.so, selected through BLS381_LIB) against
# the in-tree library on the C2 headline, alternating.  Usage: tools/ab_variants.sh TAG REPS name...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
TAG=$1; REPS=$2; shift 2
mkdir -p gpurun_out
for rep in $(seq 1 $REPS); do
  for v in base "$@"; do
    if [ "$v" = base ]; then unset BLS381_LIB; else export BLS381_LIB="variants/$v/libbls381.so"; fi
    timeout -k 10 240 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-aggregate --no-secondary \
      > gpurun_out/ab_${TAG}_${v}_$rep.json 2> gpurun_out/ab_${TAG}_${v}_$rep.err || { echo "$v failed"; tail -5 gpurun_out/ab_${TAG}_${v}_$rep.err; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/ab_${TAG}_${v}_$rep.json').read().splitlines()[-1]); print('$v', round(d['value']), d['ms_per_step'], {k: round(x,2) for k,x in d['roofline']['kernel_avg_ms'].items()})"
  done
done
