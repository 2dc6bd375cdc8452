#!/bin/bash
# gpurun with waiting for a free box: re-submits ONLY when gpurun reports that no box / slot was
# available (nothing ran, nothing charged). Any run that started is never repeated.
# usage: scripts/gpurun_retry.sh <log> <timeout_s> '<command>'
LOG=$1; TO=$2; CMD=$3
for i in $(seq 1 12); do
  /usr/local/graft/bin/gpurun --timeout "$TO" -- "$CMD" > "$LOG" 2>&1
  rc=$?
  if grep -q "status=transient rc=None" "$LOG"; then
    echo "no box (try $i), waiting" >> "$LOG.retries"
    sleep 90
    continue
  fi
  exit $rc
done
exit 3
