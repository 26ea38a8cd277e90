#!/bin/bash
# Retry a gpurun call ONLY while the pool had no box for it (nothing ran, nothing charged):
# exit code 3, or a "transient" verdict with "run 0.0s".  Any run that started -- pass or
# fail -- is returned as is and never repeated.  Usage: tools/gpurun_when_free.sh OUT TIMEOUT CMD
OUT=$1; TO=$2; shift 2
for attempt in 1 2 3 4 5 6 7 8; do
  /usr/local/graft/bin/gpurun --timeout "$TO" -- "$@" > "$OUT" 2>&1
  rc=$?
  if [ $rc -eq 3 ] || { grep -q "status=transient" "$OUT" && grep -q "run 0.0s" "$OUT"; }; then
    echo "[when_free] attempt $attempt: no box (rc $rc); waiting" >> "$OUT.attempts"
    sleep 150
    continue
  fi
  exit $rc
done
exit 3
