set -o pipefail
O=gpurun_out/r6_wpix_ab.log
for C in C2; do
  for L in xlib/final.so xlib/wpix.so xlib/final.so xlib/wpix.so xlib/final.so xlib/wpix.so; do
    timeout -k 10 300 python -u tools/tune_wavefront.py --config $C --steps 4 --batch 5 --user-stream --lib $L --ref-file /tmp/ref_$C.npy "" >> $O 2>&1 || exit 1
  done
done
for C in C3; do
  for L in xlib/final.so xlib/wpix.so xlib/final.so xlib/wpix.so; do
    timeout -k 10 300 python -u tools/tune_wavefront.py --config $C --steps 2 --batch 5 --user-stream --lib $L --ref-file /tmp/ref_$C.npy "" >> $O 2>&1 || exit 1
  done
done
LIBS="xlib/final.so xlib/wpix.so" CONFIGS="C2 C4" STEPS=2 OUT=gpurun_out/r6_ab_wpix_fam.log tools/r6_ab.sh > /dev/null || exit 1
