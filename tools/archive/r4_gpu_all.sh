#!/bin/bash
# Round-4 GPU session: the -m gpu suite (unless NOTESTS), then tools/r4_measure.sh over $CONFIGS.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
if [ -z "${NOTESTS:-}" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
  rc=$?
  tail -8 gpurun_out/gpu_tests.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests rc=$rc: stopping"; exit $rc; fi
fi
bash tools/r4_measure.sh
