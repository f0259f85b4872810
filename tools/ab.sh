#!/bin/bash
# A/B timing of library builds on C2 (+ optional $CONFIGS), bit-identity checked against the first.
#   LIBS="xso/base.so pysicalbasedraytracer_amd/libpbr_hip.so" CONFIGS="C2 C3" bash tools/ab.sh
set -o pipefail
mkdir -p gpurun_out
for C in ${CONFIGS:-C2}; do
  REF=${REFDIR:-/tmp}/ref_$C.npy; rm -f $REF
  for L in $LIBS; do
    timeout -k 10 300 python -u tools/tune_wavefront.py --config $C --steps ${STEPS:-5} --lib $L --ref-file $REF ${TUNE_ARGS:-} $VARIANTS || exit 1
  done
done
