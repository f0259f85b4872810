#!/bin/bash
# Round 6 A/B: per config, every library of $LIBS under the default and the serial schedule, with
# per-family ms/frame (HIP events) and a bit-identity check against the first library's frame.
#   LIBS="xlib/base.so xlib/x.so" CONFIGS="C4 C5" STEPS=2 bash tools/r6_ab.sh
set -o pipefail
mkdir -p gpurun_out
OUT=${OUT:-gpurun_out/r6_ab.log}
: > "$OUT"
for C in ${CONFIGS:-C4}; do
  REF=/tmp/ref_$C.npy; rm -f $REF
  for L in $LIBS; do
    timeout -k 10 ${TMO:-300} python -u tools/tune_wavefront.py --config $C --steps ${STEPS:-2} --lib $L --ref-file $REF \
      --profile "" ${VARIANTS:-"serial=1"} >> "$OUT" 2>&1 || { echo "FAILED $C $L" >> "$OUT"; exit 1; }
  done
done
grep -v "^build" "$OUT"
