#!/bin/bash
# Kernel trace of one GPU's C2 shard (rank 1 of 8) frames, for the per-frame launch chain.
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $ROOT/gpurun_out/r3_shardtrace -o run -- python3 $ROOT/tools/tune_wavefront.py --config ${CONFIG:-C2} --steps 5 --shard ${SHARD:-1/8} > $ROOT/gpurun_out/r3_shardtrace.log 2>&1
