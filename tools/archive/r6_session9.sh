set -o pipefail
O=gpurun_out/r6_sched_sweep2.log
for C in C5 C3 C4; do
  timeout -k 10 500 python -u tools/tune_wavefront.py --config $C --steps 2 --lib xlib/ch27.so "" lanes=4 chunk_log2=27 "chunk_log2=27,lanes=4" >> $O 2>&1 || exit 1
done
for C in C5 C4; do
  GPU_MAX_HW_QUEUES=8 timeout -k 10 500 python -u tools/tune_wavefront.py --config $C --steps 2 --lib xlib/ch27.so "" lanes=4 >> gpurun_out/r6_sched_hwq8.log 2>&1 || exit 1
done
