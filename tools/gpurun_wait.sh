#!/bin/bash
# Run one gpurun command; if the infrastructure could not provide a box (status "transient",
# nothing ran on a GPU: run time 0), wait and submit it again, at most 6 times.
# Any outcome in which the command actually ran is returned as is (never re-run).
#   bash tools/gpurun_wait.sh <timeout_s> '<command>'
TO=$1; shift
for i in $(seq 1 ${GPURUN_TRIES:-6}); do
  /usr/local/graft/bin/gpurun --timeout "$TO" -- "$@" > gpurun_out/call.log 2>&1
  rc=$?
  tail -3 gpurun_out/call.log
  if grep -q "status=transient\|backing off" gpurun_out/call.log && ! grep -q "run [1-9]" gpurun_out/call.log; then
    echo "[gpurun_wait] no box (attempt $i); waiting"; sleep 150; continue
  fi
  exit $rc
done
exit 3
