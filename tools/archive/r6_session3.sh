set -o pipefail
LIBS="xlib/base.so xlib/nf3.so" CONFIGS="C2 C3 C5 C4" STEPS=3 OUT=gpurun_out/r6_ab_nf3.log tools/r6_ab.sh > /dev/null || exit 1
timeout -k 10 300 python -u tools/shard_projection.py --config C2 --ns 2,4,8 --steps 3 --lib xlib/base.so > gpurun_out/r6_shard_base.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/shard_projection.py --config C2 --ns 2,4,8 --steps 3 --lib xlib/nf3.so > gpurun_out/r6_shard_nf3.log 2>&1 || exit 1
