#!/bin/bash
# Same-box A/B of library variants on the C2 bench, alternating: base (lib/libbls381.so) and
# variants/<name>/libbls381.so, REPS rounds.  bench.py checks every verdict of the batch.
# Usage: bash tools/ab_variants.sh TAG REPS name...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
TAG=$1; REPS=$2; shift 2
mkdir -p gpurun_out
for r in $(seq 1 $REPS); do
  for v in base "$@"; do
    if [ "$v" = base ]; then LIBV=$PWD/consensus-specs_amd/lib/libbls381.so; else LIBV=$PWD/variants/$v/libbls381.so; fi
    BLS381_LIB=$LIBV timeout -k 10 240 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-aggregate --no-secondary > gpurun_out/ab_${TAG}_${v}_$r.json 2> gpurun_out/ab_${TAG}_${v}_$r.err || { echo "variant $v failed"; tail -3 gpurun_out/ab_${TAG}_${v}_$r.err; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/ab_${TAG}_${v}_$r.json').read().splitlines()[-1]); print('$v', $r, round(d['value']), {k: round(x,2) for k,x in d['roofline']['kernel_avg_ms'].items()})"
  done
done
