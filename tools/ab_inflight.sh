#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for rep in 1 2 3; do
  for k in 1 2; do
    timeout -k 10 240 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-aggregate --no-secondary --inflight $k > gpurun_out/ab_r06f_inflight${k}_$rep.json 2> gpurun_out/ab_r06f_inflight${k}_$rep.err || { echo "inflight $k failed"; tail -5 gpurun_out/ab_r06f_inflight${k}_$rep.err; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/ab_r06f_inflight${k}_$rep.json').read().splitlines()[-1]); print('inflight $k', round(d['value']), d['ms_per_step'], {kk: round(x,2) for kk,x in d['roofline']['kernel_avg_ms'].items()})"
  done
done
