#!/bin/bash
# Lanes under queued vs host-synchronised frames: timings, then kernel traces of
# queued frames at 3 and 4 lanes (rocprofv3 --kernel-trace: per dispatch its queue, start and end).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/lanes
CFG=${CONFIG:-C2}
for L in 3 4 2; do
  for M in "" "--sync" "--default-stream"; do
    timeout -k 10 120 python -u tools/r5_lanes_trace.py --config $CFG --lanes $L --frames ${FRAMES:-12} $M || exit 4
  done
done
for HQ in 8; do
  GPU_MAX_HW_QUEUES=$HQ timeout -k 10 120 python -u tools/r5_lanes_trace.py --config $CFG --lanes 4 --frames ${FRAMES:-12} && \
  GPU_MAX_HW_QUEUES=$HQ timeout -k 10 120 python -u tools/r5_lanes_trace.py --config $CFG --lanes 3 --frames ${FRAMES:-12} || exit 4
done
cd /tmp && export TMPDIR=/tmp
for L in 3 4; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/lanes/trace$L" -o run -- \
      python3 "$GRAFT_REPO_ROOT/tools/r5_lanes_trace.py" --config $CFG --lanes $L --frames 6 > "$GRAFT_REPO_ROOT/gpurun_out/lanes/trace$L.log" 2>&1 || exit 5
  echo "trace $L ok"
done
