#!/bin/bash
# Run one gpurun call; re-submit only when the box could not be prepared (status=transient /
# no box free: nothing ran, nothing charged). A command that ran and failed is never retried.
for i in 1 2 3 4 5 6 7 8 9 10; do
  out=$(/usr/local/graft/bin/gpurun --timeout "${GPU_TIMEOUT:-1200}" -- "$@" 2>&1); rc=$?
  echo "$out" | tail -4
  if echo "$out" | grep -q "status=transient\|no box\|slot free"; then sleep 90; continue; fi
  exit $rc
done
exit 3
