#!/bin/bash
# Round-4 GPU session: all -m gpu tests, then an interleaved A/B of the round-3 build (xso/base.so)
# against the current one on the BASELINE configs ($CONFIGS), bit-identity checked.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
if [ -z "${NOTESTS:-}" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider ${K:+-k "$K"} > gpurun_out/gpu_tests.log 2>&1
  rc=$?
  tail -30 gpurun_out/gpu_tests.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests rc=$rc: stopping"; exit $rc; fi
fi
if [ -n "${AB:-}" ]; then
  timeout -k 10 ${AB_TIMEOUT:-600} python -u tools/ab_libs.py --configs ${CONFIGS:-C2} --rounds ${ROUNDS:-3} --steps ${STEPS:-5} $AB > gpurun_out/ab.log 2>&1
  rc2=$?
  grep -E "RESULT|DIFFERS|Error|error" gpurun_out/ab.log | tail -30
  [ $rc2 -ne 0 ] && { echo "ab rc=$rc2"; tail -5 gpurun_out/ab.log; exit $rc2; }
fi
exit ${rc:-0}
