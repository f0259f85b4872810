set -o pipefail
LIBS="xlib/segw.so xlib/slab.so" CONFIGS="C2 C3 C5 C4" STEPS=3 OUT=gpurun_out/r6_ab_slab.log tools/r6_ab.sh > /dev/null || exit 1
for C in C5 C4; do
  timeout -k 10 400 python -u tools/tune_wavefront.py --config $C --steps 2 --lib xlib/slab.so "" lanes=4 chunk_log2=24 chunk_log2=23 >> gpurun_out/r6_sched_sweep.log 2>&1 || exit 1
done
