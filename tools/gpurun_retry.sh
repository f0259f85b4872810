#!/bin/bash
# Runs one gpurun call, retrying only while the pool has no free box (exit 3 / transient, nothing
# charged).  Any other outcome — success, a failing command, a refusal — ends it.
# Usage: tools/gpurun_retry.sh TIMEOUT 'command'  (output: the last attempt's gpurun output)
T=$1; shift
for i in 1 2 3 4 5 6 7 8 9 10 11 12; do
  /usr/local/graft/bin/gpurun --timeout "$T" -- "$@"
  rc=$?
  [ $rc -ne 3 ] && exit $rc
  grep -q '"status": "transient"' /root/repo/gpurun_out/.last_call.json 2>/dev/null || exit $rc
  echo "[retry] no box (attempt $i); waiting 150 s"
  sleep 150
done
exit 3
