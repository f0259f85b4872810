#!/bin/bash
# Round-4 multi-GPU projection on one GPU (tools/shard_projection.py) for $CONFIGS, with a heartbeat
# under gpurun_out/ (a C4 projection runs for minutes between lines).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
( while true; do date >> gpurun_out/heartbeat.log; sleep 60; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
for c in ${CONFIGS:-C2}; do
  lc=$(echo "$c" | tr 'A-Z' 'a-z')
  S=3; [ "$c" = C4 ] && S=1
  timeout -k 10 600 python -u tools/shard_projection.py --config "$c" --steps $S --json "gpurun_out/r4_shard_$lc.json" \
      >> gpurun_out/shards.log 2>&1 || { echo "shard projection $c failed"; tail -5 gpurun_out/shards.log; exit 1; }
  tail -4 gpurun_out/shards.log
done
