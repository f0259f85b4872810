#!/bin/bash
# Per-kernel time of library builds on one config (rocprofv3 --kernel-trace --stats), one lane so
# kernels do not overlap:  LIBS="exp_so/base.so pysicalbasedraytracer_amd/libpbr_hip.so" bash tools/prof_ab.sh
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd /tmp && export TMPDIR=/tmp
for lib in $LIBS; do
  name=$(basename "$lib" .so)
  PBR_LANES=${PBR_LANES:-1} timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/pab_$name" -o run -- \
      python3 "$ROOT/tools/tune_wavefront.py" --config ${CONFIG:-C2} --steps ${STEPS:-3} --lib "$ROOT/$lib" "" > "$ROOT/gpurun_out/pab_$name.log" 2>&1 || exit 1
  echo "== $name"
  python3 -c "
import csv,sys
for r in csv.DictReader(open('$ROOT/gpurun_out/pab_$name/run_kernel_stats.csv')):
    n=r['Name'].replace('(anonymous namespace)::','').split('(')[0][:60]
    print(f\"{n:60s} {r['Calls']:>5s} {float(r['TotalDurationNs'])/1e6:9.2f} ms {float(r['AverageNs'])/1e3:9.1f} us\")
"
done
