#!/bin/bash
# r04d: GPU parity tests on the split-FE + MSM library, then same-box A/B against the
# unsplit FE (variants/fesplit0) and the one-wave FE / Miller builds, then the randomized
# batch line with the MSM and with the per-item ladder (BLS381_RB_MSM=0).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/ -x -v -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_r04d.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/gpu_tests_r04d.log; exit 1; }
tail -2 gpurun_out/gpu_tests_r04d.log
bash tools/ab_variants.sh r04d 2 fesplit0 fe1w ml1w || exit 1
for msm in 1 0; do
  BLS381_RB_MSM=$msm timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-aggregate --sections randomized --rb-batch 64,256 > gpurun_out/rb_r04d_msm$msm.json 2> gpurun_out/rb_r04d_msm$msm.err || { echo "rb $msm failed"; tail -5 gpurun_out/rb_r04d_msm$msm.err; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/rb_r04d_msm$msm.json').read().splitlines()[-1]); print('msm=$msm default', round(d['value']), {k: (round(v['verifications_per_s']), v.get('failed_sub_batches')) for k, v in d['c2_randomized_batch'].items() if isinstance(v, dict) and 'verifications_per_s' in v})"
done
