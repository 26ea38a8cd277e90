#!/bin/bash
# Extra rocprofv3 --pmc passes over tools/prof_workload.py, one run per pass (argument = one pass's
# counters, space separated, quoted).  Usage: bash tools/pmc_custom.sh TAG N "CTRS1" ["CTRS2" ...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
TAG=$1; N=$2; shift 2
OUT=gpurun_out/pmcx_$TAG
mkdir -p $OUT
i=0
for P in "$@"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $OUT/p$i -o p$i -- python3 tools/prof_workload.py $N > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
  echo "pass $i ok"
done
