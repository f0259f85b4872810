#!/bin/bash
# bench.py lines for the four configs on the current build -> gpurun_out/r3_c*_bench.json
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python bench.py > gpurun_out/r3_c2_bench.json 2> gpurun_out/r3_c2_bench.err || exit 1
echo "C2 $(head -c 200 gpurun_out/r3_c2_bench.json)"
timeout -k 10 300 python bench.py --config C3 --no-model > gpurun_out/r3_c3_bench.json 2> gpurun_out/r3_c3_bench.err || exit 1
echo "C3 $(head -c 200 gpurun_out/r3_c3_bench.json)"
timeout -k 10 300 python bench.py --config C5 --no-model --steps 3 > gpurun_out/r3_c5_bench.json 2> gpurun_out/r3_c5_bench.err || exit 1
echo "C5 $(head -c 200 gpurun_out/r3_c5_bench.json)"
timeout -k 10 400 python bench.py --config C4 --no-model --steps 2 --warmup 1 > gpurun_out/r3_c4_bench.json 2> gpurun_out/r3_c4_bench.err || exit 1
echo "C4 $(head -c 200 gpurun_out/r3_c4_bench.json)"
