#!/bin/bash
# L2 hit/miss and L1→L2 request counters over one frame of $CONFIG (tools/tune_wavefront.py), one pass.
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
CONFIG="${CONFIG:-C5}"
OUT="$ROOT/gpurun_out/pmc_l2_$(echo $CONFIG | tr 'A-Z' 'a-z')"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum \
    --output-format csv -d "$OUT" -o run -- python3 $ROOT/tools/tune_wavefront.py --config $CONFIG --steps 1 > "$OUT.log" 2>&1
