#!/bin/bash
# A/B of the fused Whitted shade (camera and continuation tracing inside the shade): C2 and its rank
# shards — bit-identity against base.so (LIB), then the fused build with PBR_FUSED_CAMERA=1/0 and
# PBR_CHUNK_BALANCE=0 (no chunk halving for two-chunk frames).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
LIB=${LIB:-xso/fused4.so}
T="timeout -k 10 300 python -u tools/tune_wavefront.py"
rm -f /tmp/ref_C2.npy
$T --config C2 --steps 5 --lib xso/base.so --ref-file /tmp/ref_C2.npy --profile || exit 1
$T --config C2 --steps 5 --lib $LIB --ref-file /tmp/ref_C2.npy --profile PBR_LANES=3 PBR_FUSED_CAMERA=1 PBR_FUSED_CAMERA=0 PBR_LANES=3 || exit 1
$T --config C2 --steps 5 --lib xso/base.so --ref-file /tmp/ref_C2.npy || exit 1
for S in 0/2 0/8; do
  rm -f /tmp/ref_s.npy
  $T --config C2 --steps 7 --shard $S --lib xso/base.so --ref-file /tmp/ref_s.npy || exit 1
  $T --config C2 --steps 7 --shard $S --lib $LIB --ref-file /tmp/ref_s.npy PBR_LANES=3 PBR_CHUNK_BALANCE=0 PBR_FUSED_CAMERA=0 PBR_FUSED_CAMERA=2 PBR_LANES=3 || exit 1
  $T --config C2 --steps 7 --shard $S --lib xso/base.so --ref-file /tmp/ref_s.npy || exit 1
done
