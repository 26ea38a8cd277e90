#!/bin/bash
# The C2 headline three times in a row on one box (run-to-run spread): bash tools/bench_repeat.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
for r in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-aggregate --no-secondary > gpurun_out/rep_r06ze_$r.json 2> gpurun_out/rep_r06ze_$r.err || exit 1
  python -c "import json; d=json.loads(open('gpurun_out/rep_r06ze_$r.json').read().splitlines()[-1]); print($r, round(d['value']), d['ms_per_step'], {k: round(x,3) for k,x in d['roofline']['kernel_avg_ms'].items()})"
done
