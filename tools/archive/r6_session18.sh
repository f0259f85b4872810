set -o pipefail
O=gpurun_out/r6_dyn3_ab.log
for C in C3 C5; do
  for L in xlib/final.so xlib/dyn3.so xlib/final.so xlib/dyn3.so; do
    timeout -k 10 300 python -u tools/tune_wavefront.py --config $C --steps 2 --batch 5 --user-stream --lib $L --ref-file /tmp/ref_$C.npy "" >> $O 2>&1 || exit 1
  done
done
for L in xlib/final.so xlib/dyn3.so; do
  timeout -k 10 400 python -u tools/tune_wavefront.py --config C4 --steps 1 --batch 2 --user-stream --lib $L --ref-file /tmp/ref_C4.npy "" >> $O 2>&1 || exit 1
done
LIBS="xlib/final.so xlib/dyn3.so" CONFIGS="C4" STEPS=1 OUT=gpurun_out/r6_ab_dyn3_fam.log tools/r6_ab.sh > /dev/null || exit 1
