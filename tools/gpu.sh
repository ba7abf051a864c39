#!/bin/bash
# gpurun wrapper: re-submits ONLY when the pool reports an infrastructure
# "transient" status (the command never ran, nothing charged).  A command that
# ran and failed is never re-run.
TO=${GPU_TIMEOUT:-600}
for attempt in $(seq 1 ${GPU_ATTEMPTS:-4}); do
  out=$(/usr/local/graft/bin/gpurun --timeout "$TO" -- "$@" 2>&1)
  rc=$?
  if echo "$out" | grep -q "status=transient\|backing off\|no box or slot"; then
    echo "[gpu.sh] transient infrastructure failure, attempt $attempt; waiting" >&2
    sleep ${GPU_RETRY_SLEEP:-40}
    continue
  fi
  echo "$out"
  exit $rc
done
echo "$out"
exit 3
