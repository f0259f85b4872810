#!/bin/bash
# Round-6 shard projections on the in-tree build: the -m gpu suite, then the multi-GPU shard projections
# (bench.py's tiles, frames in batches as bench.py's timed window) for $CONFIGS.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
( while true; do date >> gpurun_out/heartbeat.log; sleep 60; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
if [ -z "${NOTESTS:-}" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
  rc=$?; tail -3 gpurun_out/gpu_tests.log
  if [ $rc -ne 0 ]; then echo "tests rc=$rc: stopping"; exit $rc; fi
fi
for cfg in ${CONFIGS:-C2}; do
  lc=$(echo "$cfg" | tr 'A-Z' 'a-z')
  S=3; [ "$cfg" = C4 ] && S=1
  timeout -k 10 600 python -u tools/shard_projection.py --config $cfg --steps $S --batch ${BATCH:-5} --json gpurun_out/shard_$lc.json > gpurun_out/shard_$lc.log 2>&1 || exit 5
  grep -v amdgpu.ids gpurun_out/shard_$lc.log
done
