#!/bin/bash
# Kernel traces for the per-level breakdown: C2 full frame on one lane (no overlap, so kernel
# durations are not inflated by a co-running lane) and a 1/8 shard.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$ROOT/gpurun_out/tr_full1" -o run -- \
    python3 "$ROOT/tools/tune_wavefront.py" --steps 1 PBR_LANES=1 > "$ROOT/gpurun_out/tr_full1.log" 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$ROOT/gpurun_out/tr_shard" -o run -- \
    python3 "$ROOT/tools/tune_wavefront.py" --steps 1 --shard 7/8 "" > "$ROOT/gpurun_out/tr_shard.log" 2>&1 || exit 1
