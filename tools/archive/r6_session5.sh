set -o pipefail
LIBS="xlib/lam.so xlib/fold.so" CONFIGS="C2" STEPS=5 OUT=gpurun_out/r6_ab_fold.log tools/r6_ab.sh > /dev/null || exit 1
LIBS="xlib/lam.so xlib/fold.so" CONFIGS="C2" STEPS=5 OUT=gpurun_out/r6_ab_fold2.log tools/r6_ab.sh > /dev/null || exit 1
FILES="tests/test_bench_frames.py tests/test_gpu_batch.py tests/test_ref_fullsize.py" K="c2 or C2 or whitted or shards" OUT=gpurun_out/r6_t_fold.log TMO=600 tools/r6_tests.sh
