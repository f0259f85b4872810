set -o pipefail
O=gpurun_out/r6_c2_lanes_own.log
timeout -k 10 300 python -u tools/tune_wavefront.py --config C2 --steps 3 --batch 5 --user-stream --lib xlib/final.so "" lanes=4 "chunk_log2=24,lanes=4" "" lanes=4 >> $O 2>&1 || exit 1
