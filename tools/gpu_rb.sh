#!/bin/bash
# Randomized-batch GPU check: the per-item-verdict tests, then the bench's randomized line
# at several sub-batch sizes.  Usage: tools/gpu_rb.sh TAG [sizes]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
TAG=${1:-rb}; SIZES=${2:-8,16,64}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "randomized" -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/rb_tests_$TAG.log 2>&1 || { tail -30 gpurun_out/rb_tests_$TAG.log; exit 1; }
tail -2 gpurun_out/rb_tests_$TAG.log
timeout -k 10 400 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-aggregate --no-secondary --sections randomized --rb-batch $SIZES > gpurun_out/rb_$TAG.json 2> gpurun_out/rb_$TAG.err || { tail -5 gpurun_out/rb_$TAG.err; exit 1; }
python - <<PY
import json
d = json.loads(open("gpurun_out/rb_$TAG.json").read().splitlines()[-1])
print("default", round(d["value"]), {k: round(v, 2) for k, v in d["roofline"]["kernel_avg_ms"].items()})
r = d["c2_randomized_batch"]
for k, v in (r.get("by_sub_batch") or {r["sub_batch"]: r}).items():
    print("B=%s" % k, {n: (round(v[n]["verifications_per_s"]), v[n]["failed_sub_batches"], v[n]["verified_singly"])
                       for n in ("clean", "tampered_1_in_16")})
PY
