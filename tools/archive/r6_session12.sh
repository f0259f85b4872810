set -o pipefail
O=gpurun_out/r6_dyn_ab.log
for C in C3 C5; do
  for L in xlib/membud.so xlib/dyn.so xlib/membud.so xlib/dyn.so; do
    timeout -k 10 400 python -u tools/tune_wavefront.py --config $C --steps 2 --batch 5 --lib $L --ref-file /tmp/ref_$C.npy "" >> $O 2>&1 || exit 1
  done
done
for L in xlib/membud.so xlib/dyn.so xlib/membud.so xlib/dyn.so; do
  timeout -k 10 400 python -u tools/tune_wavefront.py --config C4 --steps 1 --batch 2 --lib $L --ref-file /tmp/ref_C4.npy "" >> $O 2>&1 || exit 1
done
LIBS="xlib/membud.so xlib/dyn.so" CONFIGS="C4" STEPS=1 OUT=gpurun_out/r6_ab_dyn_fam.log tools/r6_ab.sh > /dev/null || exit 1
OUT=gpurun_out/r6_gpu_tests_dyn.log TMO=1100 bash tools/r6_tests.sh
