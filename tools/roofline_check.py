"""Recompute bench.py's per-family roofline from a committed rocprofv3 kernel-stats CSV.

    python tools/roofline_check.py profiles/r4_c2_bench.json profiles/r4_c2_kernel_stats.csv

bench.py's `roofline.kernels` come from its serial window (one lane, shadow rays on the render
stream: every kernel runs alone) timed with HIP events.  The CSV is `rocprofv3 --kernel-trace
--stats` of `bench.py --serial` on the same build (tools/archive/r4_measure.sh).  For each family this prints
the launches' mean duration from the CSV (all template instances of the family's kernel), the
family's algorithmic bytes per launch from the bench line, the resulting GB/s and fraction of the
8 TB/s peak, and the bench line's own figures beside them."""
import csv
import json
import re
import sys

PEAK = 8000.0


def family(name):
    """bench.py's profile family of a rocprof kernel name (k_wf_shade's fused level-0 instances,
    4th template argument true, are k_wf_shade_l0)."""
    m = re.search(r"(k_\w+?)(<([^()]*)>)?\(", name)
    if not m:
        return None
    fam = m.group(1)
    if fam == "k_wf_shade" and m.group(3):
        targs = [a.strip() for a in m.group(3).split(",")]
        if len(targs) >= 4 and targs[3] == "true":
            fam = "k_wf_shade_l0"
    return fam


def main():
    bench = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
    rows = list(csv.DictReader(open(sys.argv[2])))
    fam_ns, fam_calls = {}, {}
    for r in rows:
        f = family(r["Name"])
        if not f:
            continue
        fam_ns[f] = fam_ns.get(f, 0.0) + float(r["TotalDurationNs"])
        fam_calls[f] = fam_calls.get(f, 0) + int(r["Calls"])
    rl = bench["roofline"]
    print(f"{bench['config']['workload']}: frame {bench['ms_per_step']} ms, build {rl.get('build')}")
    print(f"{'family':22s} {'rocprof avg us':>14s} {'bench avg us':>12s} {'alg MB/launch':>13s} "
          f"{'GB/s (rocprof)':>14s} {'frac':>7s} {'bench frac':>10s}")
    for f, k in rl["kernels"].items():
        if f not in fam_calls:
            continue
        avg_us = fam_ns[f] / fam_calls[f] / 1e3
        alg = k["alg_bytes_per_launch"]
        gbs = alg / (avg_us * 1e-6) / 1e9
        print(f"{f:22s} {avg_us:14.1f} {k['avg_launch_us']:12.1f} {alg / 1e6:13.1f} {gbs:14.1f} "
              f"{gbs / PEAK:7.4f} {k['frac']:10.4f}")
    print(f"dominant family (bench): {rl['kernel']}, {rl['ms_per_frame']} ms/frame standalone, frac {rl['frac']}")


if __name__ == "__main__":
    main()
