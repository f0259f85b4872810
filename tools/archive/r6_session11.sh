set -o pipefail
O=gpurun_out/r6_c2_chunk_ab.log
timeout -k 10 400 python -u tools/tune_wavefront.py --config C2 --steps 3 --batch 5 --lib xlib/wh27.so "" chunk_log2=26 chunk_log2=27 "chunk_log2=26,lanes=2" "chunk_log2=26,lanes=4" >> $O 2>&1 || exit 1
timeout -k 10 400 python -u tools/tune_wavefront.py --config C2 --steps 3 --batch 5 --lib xlib/wh27.so "" chunk_log2=26 chunk_log2=27 >> $O 2>&1 || exit 1
FILES="tests/test_gpu_batch.py tests/test_host_cpp.py" OUT=gpurun_out/r6_t_batch.log TMO=600 bash tools/r6_tests.sh
