#!/bin/bash
# Path/VolPath schedule switches on the final build (bit-identity against the default): lanes and chunk size.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/tune_wavefront.py --config C3 --steps 3 PBR_LANES=3 PBR_LANES=4 PBR_CHUNK_LOG2=25 PBR_CHUNK_LOG2=27 PBR_LANES=3 || exit 1
timeout -k 10 400 python -u tools/tune_wavefront.py --config C5 --steps 2 PBR_LANES=3 PBR_LANES=4 PBR_CHUNK_LOG2=25 PBR_LANES=3 || exit 1
