#!/bin/bash
# Same-box A/B of one build variant against the in-tree library: the C2 headline (tools/ab_variants.sh,
# 3 alternating pairs), then the randomized, latency, C3 and C5 lines twice each.
#   bash tools/ab_variants_full.sh TAG VARIANT   (summary: python tools/ab2_summary.py TAG base VARIANT)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
TAG=$1; V=$2
bash tools/ab_variants.sh $TAG 3 $V || exit 1
for rep in 1 2; do for v in base $V; do
  if [ "$v" = base ]; then unset BLS381_LIB; else export BLS381_LIB=variants/$v/libbls381.so; fi
  timeout -k 10 400 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-aggregate --sections randomized,latency,c3,c5 > gpurun_out/ab2_${TAG}_${v}_$rep.json 2> gpurun_out/ab2_${TAG}_${v}_$rep.err || { echo "$v failed"; tail -5 gpurun_out/ab2_${TAG}_${v}_$rep.err; exit 1; }
  echo "$v $rep done"
done; done
