set -o pipefail
O=gpurun_out/r6_c3_lanes_check.log
timeout -k 10 400 python -u tools/tune_wavefront.py --config C3 --steps 2 --batch 5 "" lanes=3 lanes=4 "" >> $O 2>&1 || exit 1
timeout -k 10 400 python3 bench.py --config C3 --steps 5 --no-cpu-baseline --no-model > gpurun_out/r6_c3_bench_check.log 2>&1 || exit 1
