set -o pipefail
O=gpurun_out/r6_lanes4_batch.log
timeout -k 10 400 python -u tools/tune_wavefront.py --config C3 --steps 2 --batch 5 --lib xlib/cur.so "" lanes=4 "" lanes=4 >> $O 2>&1 || exit 1
timeout -k 10 400 python -u tools/tune_wavefront.py --config C5 --steps 2 --batch 5 --lib xlib/cur.so "" lanes=4 "chunk_log2=27,lanes=4" >> $O 2>&1 || exit 1
timeout -k 10 500 python -u tools/tune_wavefront.py --config C4 --steps 1 --batch 2 --lib xlib/cur.so "" lanes=4 "" lanes=4 >> $O 2>&1 || exit 1
