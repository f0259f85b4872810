set -o pipefail
LIBS="xlib/base.so xlib/nf2.so" CONFIGS="C2 C3 C5 C4" STEPS=3 OUT=gpurun_out/r6_ab_nf2.log tools/r6_ab.sh > /dev/null || exit 1
timeout -k 10 300 python -u tools/shard_projection.py --config C2 --ns 4,8 --steps 3 --lib xlib/nf2.so > gpurun_out/r6_shard_def.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/shard_projection.py --config C2 --ns 4,8 --steps 3 --lib xlib/nf2.so --schedule fuse=on > gpurun_out/r6_shard_fuse.log 2>&1 || exit 1
