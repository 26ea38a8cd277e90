#!/bin/bash
# Same-box A/B of library variants on the C3 committee aggregation line (and C4 with --sections c4):
# base (lib/libbls381.so) and variants/<name>/libbls381.so, alternating, REPS rounds.
# Usage: bash tools/ab_agg.sh TAG REPS name...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
TAG=$1; REPS=$2; shift 2
mkdir -p gpurun_out
for r in $(seq 1 $REPS); do
  for v in base "$@"; do
    if [ "$v" = base ]; then LIBV=$PWD/consensus-specs_amd/lib/libbls381.so; else LIBV=$PWD/variants/$v/libbls381.so; fi
    BLS381_LIB=$LIBV timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --sections c4 > gpurun_out/abagg_${TAG}_${v}_$r.json 2> gpurun_out/abagg_${TAG}_${v}_$r.err || { echo "variant $v failed"; tail -3 gpurun_out/abagg_${TAG}_${v}_$r.err; exit 1; }
    python - <<PY
import json
d = json.loads(open("gpurun_out/abagg_${TAG}_${v}_$r.json").read().splitlines()[-1])
a = d["aggregation"]; c = d.get("c4_aggregate") or {}
print("$v", $r, "C2", round(d["value"]), "C3 aggs/s", round(a["committee_aggregations_per_s"]),
      {k: round(x, 3) for k, x in a["roofline"]["kernel_avg_ms"].items()},
      "C4 keys/s", round(c.get("pubkeys_aggregated_per_s", 0)), {k: round(x, 3) for k, x in (c.get("roofline") or {}).get("kernel_avg_ms", {}).items()})
PY
  done
done
