#!/bin/bash
# Submit one gpurun call, waiting for a free box: re-submits only while gpurun answers 3 ("no box or slot free
# right now", nothing ran, nothing charged), at most 20 times, 2 minutes apart.  Any other outcome ends it.
#   bash scripts/gpurun_wait.sh <timeout-seconds> '<command>'  > log
for i in $(seq 1 20); do
  /usr/local/graft/bin/gpurun --timeout "$1" -- "$2"
  rc=$?
  [ $rc -ne 3 ] && exit $rc
  echo "[gpurun_wait] no box free (try $i), waiting" >&2
  sleep 120
done
exit 3
