#!/bin/bash
# Same-box A/B of this tree's C2 bench against another source tree's own bench + library
# (e.g. a previous round's final commit, exported with git archive and built in place).
# Usage: tools/ab_tree.sh TAG OTHER_TREE_DIR
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
TAG=$1; OTHER=$2
mkdir -p gpurun_out
HERE=$PWD
for rep in 1 2; do
  timeout -k 10 240 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-aggregate --no-secondary > gpurun_out/abt_${TAG}_head_$rep.json 2> gpurun_out/abt_${TAG}_head_$rep.err || { echo "head failed"; tail -5 gpurun_out/abt_${TAG}_head_$rep.err; exit 1; }
  (cd "$OTHER" && timeout -k 10 240 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-aggregate --no-secondary) > gpurun_out/abt_${TAG}_other_$rep.json 2> gpurun_out/abt_${TAG}_other_$rep.err || { echo "other failed"; tail -5 gpurun_out/abt_${TAG}_other_$rep.err; exit 1; }
  for w in head other; do
    python -c "import json; d=json.loads(open('gpurun_out/abt_${TAG}_${w}_$rep.json').read().splitlines()[-1]); print('$w', round(d['value']), {k: round(x,2) for k,x in d['roofline']['kernel_avg_ms'].items()})"
  done
done
