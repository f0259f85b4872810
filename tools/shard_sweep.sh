#!/bin/bash
# Per-rank frame time of an N-GPU C2 job rendered on one GPU (tools/tune_wavefront.py --shard),
# for the tile sizes in $TILES, plus the whole frame.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python -u tools/tune_wavefront.py --config C2 --steps 5 || exit 1
for T in ${TILES:-64 32}; do
  for r in 0 1 2 3 4 5 6 7; do
    timeout -k 10 120 python -u tools/tune_wavefront.py --config C2 --steps 5 --shard $r/8 --tile $T || exit 1
  done
done
