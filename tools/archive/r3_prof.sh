#!/bin/bash
# rocprofv3 kernel stats of bench.py for $CONFIG (default C2) + PMC passes (SQ stall/issue counters,
# FETCH_SIZE, WRITE_SIZE) of one frame of the same build.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
C=${CONFIG:-C2}; c=$(echo $C | tr A-Z a-z)
OUT=$ROOT/gpurun_out/r3prof_$c
mkdir -p $OUT
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- python3 $ROOT/bench.py --config $C --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline) > $OUT/stats.log 2>&1 || { echo "stats failed"; exit 1; }
echo "stats ok"
[ -n "${NOPMC:-}" ] && exit 0
CONFIG=$C PMC_OUT=$OUT SQ_COUNTERS="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD" bash $ROOT/tools/pmc.sh
