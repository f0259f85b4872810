#!/bin/bash
# rocprofv3 kernel statistics of one C3 and one C5 frame (tools/tune_wavefront.py: 1 warm-up + 1
# timed frame) and of one single-lane C2 frame (PBR_LANES=1: kernels do not overlap, so each
# kernel's time is its own).  Kernel-trace only, no counters.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=$ROOT/gpurun_out/profcfg
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for C in C3 C5; do
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$C" -o run -- \
      python3 "$ROOT/tools/tune_wavefront.py" --config $C --steps 1 > "$OUT/$C.log" 2>&1 || exit $?
done
PBR_LANES=1 timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/C2_1lane" -o run -- \
    python3 "$ROOT/tools/tune_wavefront.py" --config C2 --steps 1 > "$OUT/C2_1lane.log" 2>&1
