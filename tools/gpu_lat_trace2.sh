#!/bin/bash
# Kernel traces of single calls at 8 and 16 copies (per-kernel duration spread against lanes in use).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
TAG=${1:-r05v}
mkdir -p gpurun_out
export TMPDIR=/tmp
for p in 8 16; do
  BLS381_LAT_PAD=$p timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/lattrace_${TAG}_pad$p -o kt -- python3 tools/lat_ab.py 40 > gpurun_out/lattrace_${TAG}_pad$p.log 2>&1 || { tail -5 gpurun_out/lattrace_${TAG}_pad$p.log; exit 1; }
  echo "trace pad $p ok: $(tail -1 gpurun_out/lattrace_${TAG}_pad$p.log)"
done
