set -o pipefail
O=gpurun_out/r6_ch28.log
timeout -k 10 600 python -u tools/tune_wavefront.py --config C4 --steps 1 --batch 2 --user-stream --lib xlib/ch28.so "" "chunk_log2=28,lanes=2" "chunk_log2=28,lanes=3" >> $O 2>&1 || exit 1
timeout -k 10 400 python -u tools/tune_wavefront.py --config C5 --steps 2 --batch 5 --user-stream --lib xlib/ch28.so "" "chunk_log2=28,lanes=2" >> $O 2>&1 || exit 1
