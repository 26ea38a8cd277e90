#!/bin/bash
# Round-6 iteration 4: GPU suite, then the fused one-lane prologue (k_prologue_1) against three
# streams, alternating on one box (C2 headline + randomized B = 64), and a kernel trace of the
# fused C2 steps.  Usage: tools/gpu_r06d.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
TAG=${1:-r06d}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/ -x -v -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread \
  > gpurun_out/gpu_tests_$TAG.log 2>&1 || { tail -30 gpurun_out/gpu_tests_$TAG.log; exit 1; }
tail -1 gpurun_out/gpu_tests_$TAG.log
summ() {
python - "$1" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().splitlines()[-1])
print(sys.argv[1], "default", round(d["value"]), d["ms_per_step"], {k: round(v, 2) for k, v in d["roofline"]["kernel_avg_ms"].items()})
r = d.get("c2_randomized_batch")
if r:
    for k, v in (r.get("by_sub_batch") or {r["sub_batch"]: r}).items():
        print("  B=%s" % k, {n: (round(v[n]["verifications_per_s"]), round(v[n]["ms_per_step"], 2)) for n in ("clean", "tampered_1_in_16")})
PY
}
for f in 1 0 1 0; do
  BLS381_FUSED_PROLOGUE=$f timeout -k 10 400 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-aggregate \
    --no-secondary --sections randomized --rb-batch 64 > gpurun_out/b_${TAG}_f$f.json 2> gpurun_out/b_${TAG}_f$f.err \
    || { tail -5 gpurun_out/b_${TAG}_f$f.err; exit 1; }
  summ gpurun_out/b_${TAG}_f$f.json
done
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_c2_$TAG -o run -- python3 bench.py --steps 3 --warmup 1 \
  --no-cpu-baseline --no-secondary --no-aggregate > gpurun_out/prof_c2_$TAG.log 2>&1 || { tail -5 gpurun_out/prof_c2_$TAG.log; exit 1; }
python tools/timeline.py gpurun_out/prof_c2_$TAG prologue 8 > gpurun_out/timeline_c2_$TAG.txt && cat gpurun_out/timeline_c2_$TAG.txt
