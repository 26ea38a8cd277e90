#!/bin/bash
# r04e: same-box A/B of the build variants on C2, then the randomized batch line with the
# bucket MSM and with the per-item ladder (BLS381_RB_MSM=0).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/ab_variants.sh r04e 2 fesplit1 fe1w ml1w mlnt || exit 1
for msm in 1 0; do
  BLS381_RB_MSM=$msm timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-aggregate --sections randomized --rb-batch 64,256 > gpurun_out/rb_r04e_msm$msm.json 2> gpurun_out/rb_r04e_msm$msm.err || { echo "rb $msm failed"; tail -5 gpurun_out/rb_r04e_msm$msm.err; exit 1; }
  python -c "
import json; d=json.loads(open('gpurun_out/rb_r04e_msm$msm.json').read().splitlines()[-1]); r=d['c2_randomized_batch']
print('msm=$msm default', round(d['value']))
for B, v in r.get('by_sub_batch', {r['sub_batch']: r}).items():
    print('  B', B, {k: (round(x['verifications_per_s']), x.get('failed_sub_batches')) for k, x in v.items() if isinstance(x, dict) and 'verifications_per_s' in x})"
done
