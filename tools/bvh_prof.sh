#!/bin/bash
# Kernel trace of the device BVH build (tools/bvh_build_time.py) → gpurun_out/bvhprof
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $ROOT/gpurun_out/bvhprof -o run -- python3 $ROOT/tools/bvh_build_time.py ${SIZES:-660} > $ROOT/gpurun_out/bvhprof.log 2>&1
