#!/bin/bash
# Short C2-only bench on the GPU box (no tests / secondary configs): kernel times.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
TAG=${1:-q}
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-secondary --no-cpu-baseline --no-aggregate > gpurun_out/qb_$TAG.json 2> gpurun_out/qb_$TAG.err || { tail -5 gpurun_out/qb_$TAG.err; exit 1; }
python -c "
import json; d=json.loads(open('gpurun_out/qb_$TAG.json').read().splitlines()[-1]); print(d['value'], {k: round(v, 2) for k, v in d['roofline']['kernel_avg_ms'].items()})"
