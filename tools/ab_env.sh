#!/bin/bash
# A/B of runtime knobs on the C2 bench: each argument is NAME=VALUE (or "base");
# runs alternate (a b a b) on one box.  Usage: tools/ab_env.sh TAG base BLS381_G2_ONE_LANE=1 ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
TAG=$1; shift
mkdir -p gpurun_out
for rep in $(seq 1 ${REPS:-2}); do
  for kv in "$@"; do
    name=${kv//[^A-Za-z0-9_]/_}
    if [ "$kv" = base ]; then envs=(); else envs=("$kv"); fi
    env "${envs[@]}" timeout -k 10 240 python bench.py --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline --no-aggregate --no-secondary ${EXTRA:-} > gpurun_out/ab_${TAG}_${name}_$rep.json 2> gpurun_out/ab_${TAG}_${name}_$rep.err || { echo "$kv failed"; tail -5 gpurun_out/ab_${TAG}_${name}_$rep.err; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/ab_${TAG}_${name}_$rep.json').read().splitlines()[-1]); print('$kv', round(d['value']), d['ms_per_step'], {k: round(x,2) for k,x in d['roofline']['kernel_avg_ms'].items()})"
  done
done
