#!/bin/bash
# Round-6 iteration: GPU suite, then the randomized line under the new prologue (order 2) at
# several sub-batch sizes against round 5's order 0 at B = 32 (same box), then a kernel trace
# of one clean 2^16 randomized call.  Usage: tools/gpu_r06b.sh TAG [sizes]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
TAG=${1:-r06b}; SIZES=${2:-8,16,32,64}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/ -x -v -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread \
  > gpurun_out/gpu_tests_$TAG.log 2>&1 || { tail -30 gpurun_out/gpu_tests_$TAG.log; exit 1; }
tail -1 gpurun_out/gpu_tests_$TAG.log
summ() {
python - "$1" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().splitlines()[-1])
print(sys.argv[1], "default", round(d["value"]), {k: round(v, 2) for k, v in d["roofline"]["kernel_avg_ms"].items()})
r = d.get("c2_randomized_batch")
if r:
    for k, v in (r.get("by_sub_batch") or {r["sub_batch"]: r}).items():
        print("  B=%s" % k, {n: (round(v[n]["verifications_per_s"]), round(v[n]["ms_per_step"], 2), v[n]["failed_sub_batches"],
                               v[n]["verified_singly"]) for n in ("clean", "tampered_1_in_16")})
PY
}
for o in 2 0 2; do
  BLS381_RB_ORDER=$o timeout -k 10 500 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-aggregate --no-secondary \
    --sections randomized --rb-batch $([ $o = 2 ] && echo $SIZES || echo 32) > gpurun_out/rb_${TAG}_o$o.json 2> gpurun_out/rb_${TAG}_o$o.err \
    || { tail -5 gpurun_out/rb_${TAG}_o$o.err; exit 1; }
  summ gpurun_out/rb_${TAG}_o$o.json
done
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_$TAG -o run -- python3 tools/prof_rb.py 65536 32 \
  > gpurun_out/prof_$TAG.log 2>&1 || { tail -5 gpurun_out/prof_$TAG.log; exit 1; }
python tools/timeline.py gpurun_out/prof_$TAG rb_decode_g1 40 > gpurun_out/timeline_$TAG.txt && cat gpurun_out/timeline_$TAG.txt
