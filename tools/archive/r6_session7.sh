set -o pipefail
LIBS="xlib/base.so xlib/segw.so" CONFIGS="C2 C3 C5 C4" STEPS=3 OUT=gpurun_out/r6_ab_segw.log tools/r6_ab.sh > /dev/null || exit 1
LIBS="xlib/segw.so xlib/base.so" CONFIGS="C4 C5" STEPS=2 OUT=gpurun_out/r6_ab_segw_rev.log tools/r6_ab.sh > /dev/null || exit 1
