#!/bin/bash
# Randomized-batch A/B over an env knob: tests once, then the randomized line per setting.
# Usage: tools/gpu_rb_ab.sh TAG SIZES KNOB=V1 KNOB=V2 ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
TAG=$1; SIZES=$2; shift 2
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "randomized" -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/rb_tests_$TAG.log 2>&1 || { tail -30 gpurun_out/rb_tests_$TAG.log; exit 1; }
tail -1 gpurun_out/rb_tests_$TAG.log
for kv in "$@"; do
  name=${kv//[^A-Za-z0-9_]/_}
  env "$kv" timeout -k 10 400 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-aggregate --no-secondary --sections randomized --rb-batch $SIZES > gpurun_out/rb_${TAG}_$name.json 2> gpurun_out/rb_${TAG}_$name.err || { tail -5 gpurun_out/rb_${TAG}_$name.err; exit 1; }
  python - <<PY
import json
d = json.loads(open("gpurun_out/rb_${TAG}_$name.json").read().splitlines()[-1])
r = d["c2_randomized_batch"]
for k, v in (r.get("by_sub_batch") or {r["sub_batch"]: r}).items():
    print("$kv default %d B=%s" % (d["value"], k), {n: (round(v[n]["verifications_per_s"]), round(v[n]["ms_per_step"], 2), v[n]["failed_sub_batches"]) for n in ("clean", "tampered_1_in_16")})
PY
done
