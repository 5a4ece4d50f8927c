#!/bin/bash
# Runs one gpurun call; re-submits only when no box was available (exit 3: nothing ran, nothing charged).
T=$1; shift
for i in 1 2 3 4; do
  /usr/local/graft/bin/gpurun --timeout "$T" -- "$@"
  rc=$?
  [ $rc -ne 3 ] && exit $rc
  sleep 45
done
exit $rc
