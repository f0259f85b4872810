set -o pipefail
O=gpurun_out/r6_wsr_ab.log
for L in xlib/final.so xlib/wsr.so xlib/final.so xlib/wsr.so xlib/final.so xlib/wsr.so; do
  timeout -k 10 300 python -u tools/tune_wavefront.py --config C2 --steps 4 --batch 5 --user-stream --lib $L --ref-file /tmp/ref_C2.npy "" >> $O 2>&1 || exit 1
done
LIBS="xlib/final.so xlib/wsr.so" CONFIGS="C2" STEPS=3 OUT=gpurun_out/r6_ab_wsr_fam.log tools/r6_ab.sh > /dev/null || exit 1
