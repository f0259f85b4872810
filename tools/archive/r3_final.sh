#!/bin/bash
# Round-3 measurement set for $CONFIGS: rocprofv3 kernel stats of bench.py (timed frames + profile
# windows) and the PMC passes (SQ, FETCH_SIZE, WRITE_SIZE) of one tune_wavefront frame, same build.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
for C in ${CONFIGS:-C2}; do
  c=$(echo $C | tr A-Z a-z)
  OUT=$ROOT/gpurun_out/r3f_$c
  mkdir -p $OUT
  S=3; [ $C = C4 ] && S=1
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- python3 $ROOT/bench.py --config $C --steps $S --warmup 1 --no-cpu-baseline --no-model) > $OUT/stats.log 2>&1 || { echo "$C stats failed"; exit 1; }
  echo "$C stats ok"
  CONFIG=$C PMC_OUT=$OUT bash $ROOT/tools/pmc.sh || exit 1
done
