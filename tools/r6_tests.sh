#!/bin/bash
# Round 6: the GPU tests with -s (the printed parity fractions are the record), optionally a -k
# filter in $K and test files in $FILES; one process, per-test timeout.
set -o pipefail
mkdir -p gpurun_out
LOG=${OUT:-gpurun_out/r6_gpu_tests.log}
unset OUT   # (the Makefiles the tests run read OUT)
timeout -k 10 ${TMO:-1100} python -u -m pytest ${FILES:-tests} -m gpu -v -s --timeout 400 --timeout-method thread \
  -p no:cacheprovider ${K:+-k "$K"} > "$LOG" 2>&1
rc=$?
grep -E "passed|failed|error" "$LOG" | tail -5
exit $rc
