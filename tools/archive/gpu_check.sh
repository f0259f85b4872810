#!/bin/bash
# GPU session: all -m gpu tests (no -x: report every failure), then a short C2 bench.
# A crash/timeout (rc not 0/1) ends the session.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider ${K:+-k "$K"} > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -30 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests rc=$rc: stopping"; exit $rc; fi
if [ -z "${NOBENCH:-}" ]; then
  timeout -k 10 300 python bench.py --steps ${STEPS:-10} --warmup 3 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/bench.log; exit 2; }
  python -c "import json; d=json.loads(open('gpurun_out/bench.log').read().strip().splitlines()[-1]); print('BENCH', d['config']['workload'], d['ms_per_step'], 'ms', d['value'], 'Msamples/s')"
fi
exit $rc
