#!/bin/bash
# rocprofv3 PMC passes over tools/prof_workload.py (each pass its own run; no
# --sys-trace / --runtime-trace with --pmc).  Usage: bash tools/pmc_passes.sh TAG [n]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
TAG=${1:-r01}
N=${2:-65536}
OUT=gpurun_out/pmc_$TAG
mkdir -p $OUT
P1="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_FLAT SQ_INSTS_LDS SQ_WAVES SQ_INSTS_SMEM"
P2="SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY"
P3="FETCH_SIZE GRBM_GUI_ACTIVE"
P4="WRITE_SIZE"
i=0
for P in "$P1" "$P2" "$P3" "$P4"; do
  i=$((i+1))
  timeout -k 10 600 rocprofv3 --pmc $P --output-format csv -d $OUT/p$i -o p$i -- python3 tools/prof_workload.py $N > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
  echo "pass $i ok"
done
# kernel durations of the same workload (kernel trace only; no counters in this run)
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- python3 tools/prof_workload.py $N > $OUT/kt.log 2>&1 || { echo "kernel-trace pass failed"; tail -5 $OUT/kt.log; exit 1; }
echo "kernel-trace pass ok"
