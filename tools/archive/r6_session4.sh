set -o pipefail
LIBS="xlib/nf3.so xlib/lam.so" CONFIGS="C4 C5" STEPS=3 OUT=gpurun_out/r6_ab_lam.log tools/r6_ab.sh > /dev/null || exit 1
FILES="tests/test_gpu_materials.py tests/test_infinite_light.py tests/test_gpu_textures.py" OUT=gpurun_out/r6_t_lam.log TMO=600 tools/r6_tests.sh
