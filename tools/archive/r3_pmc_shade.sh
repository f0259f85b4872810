#!/bin/bash
# PMC passes over one C5 (or $CONFIG) frame: stall/issue counters, instruction mix, HBM traffic.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
C=${CONFIG:-C5}; c=$(echo $C | tr A-Z a-z)
CONFIG=$C PMC_OUT=$ROOT/gpurun_out/r3pmc_$c SQ_COUNTERS="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD" bash $ROOT/tools/pmc.sh || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_RD --output-format csv -d $ROOT/gpurun_out/r3pmc_$c/sq2 -o run -- python3 $ROOT/tools/tune_wavefront.py --config $C --steps 1 > $ROOT/gpurun_out/r3pmc_$c/sq2.log 2>&1
echo "sq2 rc=$?"
