#!/bin/bash
# A/B of the split probe (PBR_PROBE_SPLIT=1) against the one-pass closest-hit probe on C3/C4/C5, bit-identity checked.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
L=${LIB:-xso/probe.so}
timeout -k 10 300 python -u tools/tune_wavefront.py --config C3 --steps 3 --lib $L --profile PBR_PROBE_SPLIT=0 PBR_PROBE_SPLIT=1 PBR_PROBE_SPLIT=0 PBR_PROBE_SPLIT=1 || exit 1
timeout -k 10 300 python -u tools/tune_wavefront.py --config C5 --steps 2 --lib $L --profile PBR_PROBE_SPLIT=0 PBR_PROBE_SPLIT=1 || exit 1
timeout -k 10 300 python -u tools/tune_wavefront.py --config C4 --steps 1 --lib $L PBR_PROBE_SPLIT=0 PBR_PROBE_SPLIT=1 || exit 1
