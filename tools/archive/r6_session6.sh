set -o pipefail
LIBS="xlib/lam.so xlib/fold2.so" CONFIGS="C2" STEPS=5 OUT=gpurun_out/r6_ab_fold3.log tools/r6_ab.sh > /dev/null || exit 1
FILES="tests/test_bench_frames.py" K="c2" OUT=gpurun_out/r6_t_fold2.log TMO=600 tools/r6_tests.sh
