#!/bin/bash
# queue helper (runs here, not on the GPU box): re-submit a gpurun call while the pool reports no free slot (nothing ran).
# usage: gpuq.sh <log> <timeout> <command>
log=$1; to=$2; cmd=$3
for i in $(seq 1 12); do
  /usr/local/graft/bin/gpurun --timeout $to -- "$cmd" > $log 2>&1
  rc=$?
  if grep -q "status=transient" $log && grep -q "run 0.0s\|run Nones" $log; then sleep 60; continue; fi
  exit $rc
done
exit 3
