#!/bin/bash
# Kernel trace of C3 and C5 frames (one lane, so per-kernel durations are not inflated by overlap).
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd /tmp && export TMPDIR=/tmp
for C in ${CONFIGS:-C3 C5}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/tr_$C" -o run -- \
      python3 "$ROOT/tools/tune_wavefront.py" --config $C --steps 1 PBR_LANES=1 > "$ROOT/gpurun_out/tr_$C.log" 2>&1 || exit 1
done
