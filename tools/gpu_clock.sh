#!/bin/bash
# Shader clock under light load (the latency path's one-wave launches) against full load.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
O=gpurun_out/clock_${1:-r05g}.txt
: > $O
for cfg in "1 64 0 6" "1 64 5 6" "4 64 5 4" "32 64 5 4" "1 256 5 4" "16384 256 0 3" "1 64 0 6"; do
  echo "# clock_probe $cfg" >> $O
  timeout -k 5 60 ./tools/clock_probe $cfg >> $O || exit 1
done
cat $O
