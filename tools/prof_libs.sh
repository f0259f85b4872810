#!/bin/bash
# Kernel traces of one or more library builds (tools/tune_wavefront.py, 2 frames each).
#   bash tools/prof_libs.sh "" exp/libexp4.so ...
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd /tmp && export TMPDIR=/tmp
for lib in "$@"; do
  name=$(basename "${lib:-default}" .so)
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$ROOT/gpurun_out/trace_$name" -o run -- \
      python3 "$ROOT/tools/tune_wavefront.py" --steps 1 ${lib:+--lib $ROOT/$lib} "" > "$ROOT/gpurun_out/trace_$name.log" 2>&1 || exit 1
done
