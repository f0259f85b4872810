#!/bin/bash
# Frame times of C2-C5 on one GPU (wavefront default) and the per-rank C2 shards of 2-, 4- and
# 8-GPU jobs (tools/tune_wavefront.py --shard).
set -o pipefail
mkdir -p gpurun_out
for C in C2 C3 C5; do
  timeout -k 10 300 python -u tools/tune_wavefront.py --config $C --steps 2 || exit 1
done
timeout -k 10 300 python -u tools/tune_wavefront.py --config C4 --steps 1 || exit 1
for N in 2 4 8; do
  for ((r = 0; r < N; r++)); do
    timeout -k 10 120 python -u tools/tune_wavefront.py --config C2 --steps 5 --shard $r/$N || exit 1
  done
done
