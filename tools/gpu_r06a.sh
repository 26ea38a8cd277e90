#!/bin/bash
# Round-6 baseline: the randomized line at large sub-batches (never measured above B = 256 with
# the ladder + tree-sum path), then a kernel trace of one clean 2^16 call at B = 4096.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r06a}
timeout -k 10 500 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-aggregate --no-secondary \
  --sections randomized --rb-batch 32,512,4096,32768 > gpurun_out/rb_$TAG.json 2> gpurun_out/rb_$TAG.err \
  || { tail -5 gpurun_out/rb_$TAG.err; exit 1; }
python - <<PY
import json
d = json.loads(open("gpurun_out/rb_$TAG.json").read().splitlines()[-1])
print("default", round(d["value"]), {k: round(v, 2) for k, v in d["roofline"]["kernel_avg_ms"].items()})
r = d["c2_randomized_batch"]
for k, v in (r.get("by_sub_batch") or {r["sub_batch"]: r}).items():
    print("B=%s" % k, {n: (round(v[n]["verifications_per_s"]), round(v[n]["ms_per_step"], 2), v[n]["failed_sub_batches"],
                           v[n]["verified_singly"]) for n in ("clean", "tampered_1_in_16")})
PY
cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --output-format sqlite -d $GRAFT_REPO_ROOT/gpurun_out/tr_$TAG -- \
  python3 $GRAFT_REPO_ROOT/tools/prof_rb.py 65536 4096 > $GRAFT_REPO_ROOT/gpurun_out/tr_$TAG.log 2>&1 \
  || { tail -5 $GRAFT_REPO_ROOT/gpurun_out/tr_$TAG.log; exit 1; }
cd $GRAFT_REPO_ROOT && python tools/timeline.py gpurun_out/tr_$TAG decode_g1 60 > gpurun_out/tl_$TAG.txt && cat gpurun_out/tl_$TAG.txt
