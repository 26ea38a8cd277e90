#!/bin/bash
# Round-6 iteration 3: GPU suite; the bench's new lines (host buffers, randomized roofline) with the
# sums' loop priority on and off (A/B, same box); a kernel trace of the C2 headline steps for the
# prologue's overlap.  Usage: tools/gpu_r06c.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
TAG=${1:-r06c}
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
h = d.get("c2_host_buffers")
if h: print("  host buffers", round(h["verifications_per_s"]), round(h["ms_per_step"], 2))
r = d.get("c2_randomized_batch")
if r:
    for k, v in (r.get("by_sub_batch") or {r["sub_batch"]: r}).items():
        print("  B=%s" % k, {n: (round(v[n]["verifications_per_s"]), round(v[n]["ms_per_step"], 2), v[n]["failed_sub_batches"],
                               v[n]["verified_singly"]) for n in ("clean", "tampered_1_in_16")})
        if "roofline" in v: print("   roofline", json.dumps(v["roofline"])[:900])
PY
}
for p in 1 0 1; do
  BLS381_RB_SIGPRIO=$p timeout -k 10 500 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-aggregate --no-secondary \
    --sections host,randomized --rb-batch $([ $p = 1 ] && echo 64,8 || echo 64) > gpurun_out/b_${TAG}_p$p.json 2> gpurun_out/b_${TAG}_p$p.err \
    || { tail -5 gpurun_out/b_${TAG}_p$p.err; exit 1; }
  summ gpurun_out/b_${TAG}_p$p.json
done
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_c2_$TAG -o run -- python3 bench.py --steps 3 --warmup 1 \
  --no-cpu-baseline --no-secondary --no-aggregate > gpurun_out/prof_c2_$TAG.log 2>&1 || { tail -5 gpurun_out/prof_c2_$TAG.log; exit 1; }
python tools/timeline.py gpurun_out/prof_c2_$TAG hash_cand 12 > gpurun_out/timeline_c2_$TAG.txt && cat gpurun_out/timeline_c2_$TAG.txt
