#!/bin/bash
# GPU suite (one process, per-test timeout), then the shade probe over $LIBS on $KINDS.  A test run
# that ends other than pass/fail (a fault, a time limit) stops the session.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
if [ -z "${NOTESTS:-}" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider ${K:+-k "$K"} > gpurun_out/gpu_tests.log 2>&1
  rc=$?
  tail -6 gpurun_out/gpu_tests.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests rc=$rc: stopping"; exit $rc; fi
fi
if [ -n "${LIBS:-}" ]; then
  timeout -k 10 600 python -u tools/r5_shade_probe.py ${PROBE_ARGS:-} --libs $LIBS -- ${KINDS:-mixed} > gpurun_out/probe.log 2>&1 || exit 5
  grep -v amdgpu.ids gpurun_out/probe.log | sed -E 's/ [0-9]+\.[0-9]+ ns\/u//g; s/ 0\.0 M//g'
fi
