#!/bin/bash
# A/B of library builds over configs (bit-identity checked against the first library), then optionally
# the GPU test suite.  LIBS, CONFIGS, STEPS, TESTS=1, PROFILE=1.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for C in ${CONFIGS:-C3}; do
  REF=/tmp/ref_$C.npy; rm -f $REF
  for L in ${LIBS:-pysicalbasedraytracer_amd/libpbr_hip.so}; do
    timeout -k 10 ${ABT:-300} python -u tools/tune_wavefront.py --config $C --steps ${STEPS:-3} --lib $L --ref-file $REF ${PROFILE:+--profile} || exit $?
  done
done
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider ${K:+-k "$K"} > gpurun_out/gpu_tests.log 2>&1
  rc=$?
  tail -30 gpurun_out/gpu_tests.log
  exit $rc
fi
