#!/bin/bash
# gpurun wrapper: re-submits ONLY when the infrastructure reports a transient failure before
# anything ran (status "transient" / exit 3); every other outcome, success or failure, is final.
#   bash tools/gpu.sh TIMEOUT 'command'
T=$1; shift
for attempt in 1 2 3; do
  /usr/local/graft/bin/gpurun --timeout "$T" -- "$@"
  rc=$?
  st=$(python3 -c "import json; print(json.load(open('gpurun_out/.last_call.json')).get('status',''))" 2>/dev/null)
  if [ "$rc" != "3" ] && [ "$st" != "transient" ]; then exit $rc; fi
  echo "[gpu.sh] transient infrastructure failure (attempt $attempt); waiting to resubmit"
  sleep 90
done
exit $rc
