set -o pipefail
mkdir -p gpurun_out
for S in 0/2 0/4 0/8; do
  timeout -k 10 200 python -u tools/tune_wavefront.py --config C2 --steps 7 --shard $S "" PBR_CHUNK_LOG2=24 PBR_CHUNK_LOG2=23 PBR_CHUNK_LOG2=22 "PBR_CHUNK_LOG2=23,PBR_LANES=2" "PBR_CHUNK_LOG2=22,PBR_LANES=2" "" || exit 1
done
