set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --config C4 --no-model --steps 2 --warmup 1 > gpurun_out/r3_c4_bench.json 2> gpurun_out/r3_c4_bench.err || exit 1
timeout -k 10 300 python -u tools/shard_projection.py --config C2 --steps 5 --json gpurun_out/r3_shard_c2.json > gpurun_out/shardproj.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/tune_wavefront.py --config C2 --steps 5 PBR_LANES=3 PBR_LANES=2 PBR_LANES=4 "PBR_LANES=4,PBR_CHUNK_LOG2=24" "PBR_LANES=3,PBR_CHUNK_LOG2=24" PBR_LANES=3 > gpurun_out/lanes.log 2>&1 || exit 1
grep -v amdgpu gpurun_out/lanes.log; tail -5 gpurun_out/shardproj.log
LIBS="xso/cur.so xso/mm3.so xso/fo5.so xso/pshadow.so xso/cur.so" CONFIGS=C2 STEPS=5 bash tools/r3_ab.sh > gpurun_out/occ.log 2>&1 || exit 1
grep -v "amdgpu\|^build" gpurun_out/occ.log
