#!/bin/bash
# Round-3 traversal diagnosis on C3: L2 hit/miss + L1->L2 requests (base build), WRITE_SIZE of the base
# build and of the parent-link (no scratch stack) build — does k_wf_extend's excess write traffic come
# from the traversal stack's scratch entries?
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
CONFIG=${CONFIG:-C3} bash tools/pmc_l2.sh; echo "l2 rc=$?"
[ -s gpurun_out/pmc_l2_$(echo ${CONFIG:-C3} | tr A-Z a-z)/run_counter_collection.csv ] || ls -R gpurun_out | head -30
CONFIG=${CONFIG:-C3} PMC_OUT=$ROOT/gpurun_out/r3w_base SQ_COUNTERS="SQ_WAVES SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_SMEM" bash tools/pmc.sh || exit 1
CONFIG=${CONFIG:-C3} PMC_OUT=$ROOT/gpurun_out/r3w_bt TUNE_VARIANT="--lib $ROOT/xso/bt.so" SQ_COUNTERS="SQ_WAVES SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_SMEM" bash tools/pmc.sh || exit 1
echo done
