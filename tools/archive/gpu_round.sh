#!/bin/bash
# One GPU session: parity tests → smoke → bench → rocprofv3 kernel stats.
# Ordinary test failures (pytest rc 1) do not stop the session; a crash, fault or timeout does.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
STEPS="${STEPS:-tests,smoke,bench,prof}"
stop_if_fatal() { local rc=$1 what=$2; echo "$what rc=$rc"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "fatal rc in $what — stopping"; exit $rc; fi; }
if [[ $STEPS == *tests* ]]; then
  timeout -k 10 1200 python -m pytest tests -m gpu -q -p no:cacheprovider ${PYTEST_ARGS:-} > $OUT/gpu_tests.log 2>&1
  stop_if_fatal $? tests
fi
if [[ $STEPS == *smoke* ]]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
  stop_if_fatal $? smoke
fi
if [[ $STEPS == *bench* ]]; then
  timeout -k 10 900 python bench.py ${BENCH_ARGS:-} > $OUT/bench.log 2>&1
  stop_if_fatal $? bench
fi
if [[ $STEPS == *prof* ]]; then
  ROOT=$(pwd)
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv \
      -d $ROOT/$OUT/prof -o run -- python3 $ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline) > $OUT/prof.log 2>&1
  stop_if_fatal $? prof
fi
echo done
