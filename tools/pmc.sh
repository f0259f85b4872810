#!/bin/bash
# PMC passes over one frame of $CONFIG (default C2) (separate runs: FETCH_SIZE and WRITE_SIZE do not fit one pass;
# the SQ pass gives VALU instructions and wave-cycle shares, the TCC pass the L2 hit rate).
# Kernel-trace + counters only (no sys/runtime trace domains with --pmc).
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
CONFIG="${CONFIG:-C2}"
OUT="${PMC_OUT:-$ROOT/gpurun_out/pmc}"
mkdir -p "$OUT"
CMD="python3 $ROOT/tools/tune_wavefront.py --config $CONFIG --steps 1 ${TUNE_VARIANT:-}"
cd /tmp && export TMPDIR=/tmp
run() {   # name counters...
  local name=$1; shift
  timeout -k 10 600 rocprofv3 --kernel-trace --pmc "$@" --output-format csv -d "$OUT/$name" -o run -- $CMD \
      > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "pmc $name rc=$rc"
  return $rc
}
run sq ${SQ_COUNTERS:-SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD} &&
run fetch FETCH_SIZE &&
run write WRITE_SIZE &&
run tcc TCC_HIT_sum TCC_MISS_sum
