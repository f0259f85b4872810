#!/bin/bash
# Round-6 measurement (as tools/archive/r5_measure.sh, leaving only the summaries under gpurun_out/: the raw PMC and trace files of four configs exceed what gpurun copies back) of $CONFIGS on one GPU, same build throughout:
#   1. PMC passes (tools/pmc.sh) → gpurun_out/<cfg>_traffic.json (copied to profiles/ so bench.py
#      finds the traffic of this very build);
#   2. rocprofv3 --kernel-trace --stats of `bench.py --serial` (every launch on one stream: each
#      kernel's own duration, the source of the roofline's standalone per-kernel figures);
#   3. bench.py on the default schedule (with the CPU baseline unless NOCPU is set).
# Any failing step ends the session.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
# a line a minute under gpurun_out/: a C4 bench runs for minutes before it prints its one line
( while true; do date >> "$OUT/heartbeat.log"; sleep 60; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
for cfg in ${CONFIGS:-C2}; do
  lc=$(echo "$cfg" | tr 'A-Z' 'a-z')
  S=${STEPS:-5}; [ "$cfg" = C4 ] && S=${STEPS_C4:-2}
  if [ -z "${NOPMC:-}" ]; then
    CONFIG=$cfg PMC_OUT=$OUT/pmc_$lc bash tools/pmc.sh || { echo "pmc $cfg failed"; exit 3; }
    python3 tools/summarize_prof.py - "$OUT/pmc_$lc" --json="$OUT/${lc}_traffic.json" > "$OUT/${lc}_pmc.md" || exit 3
    cp "$OUT/${lc}_traffic.json" profiles/
    rm -rf "$OUT/pmc_$lc"
  fi
  if [ -z "${NOPROF:-}" ]; then
    (cd /tmp && export TMPDIR=/tmp && timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv \
        -d "$OUT/prof_serial_$lc" -o run -- python3 "$ROOT/bench.py" --config "$cfg" --serial --steps $S --warmup 1 \
        --no-cpu-baseline --no-model) > "$OUT/prof_serial_$lc.log" 2>&1 || { echo "rocprof $cfg failed"; exit 4; }
    echo "rocprof serial $cfg ok"
    rm -f "$OUT/prof_serial_$lc/run_kernel_trace.csv"
  fi
  timeout -k 10 1100 python3 bench.py --config "$cfg" --steps $S ${NOCPU:+--no-cpu-baseline} ${BENCH_ARGS:-} > "$OUT/bench_$lc.log" 2>&1 \
      || { echo "bench $cfg failed"; tail -5 "$OUT/bench_$lc.log"; exit 5; }
  tail -1 "$OUT/bench_$lc.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('BENCH', d['config']['workload'], d['ms_per_step'], 'ms', d['value'], 'Msamples/s; dominant', r['kernel'], 'frac', r['frac'], r['ms_per_frame'], 'ms/frame; frame frac', r['frame']['frac'], r['frame'].get('traffic_frac'), 'cpu', (d.get('cpu_baseline') or {}).get('value'))"
done
echo measure done
