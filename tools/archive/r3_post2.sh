#!/bin/bash
# Kept build: C2 A/B against the previous build (bit-identity), the C2 shard projection, GPU tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
LIBS="xso/cur.so xso/new.so xso/cur.so xso/new.so" CONFIGS=C2 STEPS=5 bash tools/r3_ab.sh > gpurun_out/post2_ab.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/shard_projection.py --config C2 --steps 5 --json gpurun_out/r3_shard_c2.json > gpurun_out/shardproj2.log 2>&1 || exit 1
grep -v "amdgpu\|^build" gpurun_out/post2_ab.log; tail -4 gpurun_out/shardproj2.log
TESTS=1 CONFIGS=C1 STEPS=1 bash tools/r3_ab.sh || exit 1
CONFIGS="C2" bash tools/r3_final.sh > gpurun_out/final_c2b.log 2>&1 || exit 1
cat gpurun_out/final_c2b.log
