#!/bin/bash
# FETCH_SIZE / WRITE_SIZE passes of one $CONFIG frame for each library in $LIBS (same frame, same
# counters), so two builds' HBM bytes per kernel can be compared.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
C=${CONFIG:-C5}; c=$(echo $C | tr A-Z a-z)
i=0
for L in ${LIBS:-pysicalbasedraytracer_amd/libpbr_hip.so}; do
  CONFIG=$C PMC_OUT=$ROOT/gpurun_out/r3pl_${c}_$i TUNE_VARIANT="--lib $ROOT/$L" \
    SQ_COUNTERS="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_ANY SQ_WAVE_CYCLES" \
    bash $ROOT/tools/pmc.sh || exit 1
  i=$((i+1))
done
