"""Summarise rocprofv3 output (kernel stats + the PMC passes of tools/pmc.sh) into a markdown table.

    python tools/summarize_prof.py gpurun_out/prof gpurun_out/pmc [--json=traffic.json] > profiles/rNN_summary.md
    (first argument "-": PMC tables only)

FETCH_SIZE is doubled (gfx950 reports half the bytes of a 16-B/lane streaming read,
MI355X_MICROARCH.md § HBM); WRITE_SIZE is taken as is.  Both are per frame (the PMC runs render
one warm-up frame and one timed frame, so the per-kernel totals are halved).
"""
import collections
import csv
import os
import re
import sys


def short(name):
    name = re.sub(r"\(anonymous namespace\)::", "", name)
    name = re.sub(r"^void ", "", name)
    return re.sub(r"\(.*$", "", name)


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--json=")]
    js = [a[7:] for a in sys.argv[1:] if a.startswith("--json=")]
    prof, pmc = args[0], args[1] if len(args) > 1 else None
    stats = os.path.join(prof, "run_kernel_stats.csv")
    if prof != "-" and os.path.exists(stats):
        rows = list(csv.DictReader(open(stats)))
        print("## Kernel time (rocprofv3 --kernel-trace --stats)\n")
        print("| kernel | calls | total ms | avg µs | % |")
        print("|---|---:|---:|---:|---:|")
        for r in rows:
            print(f"| `{short(r['Name'])}` | {r['Calls']} | {float(r['TotalDurationNs']) / 1e6:.2f} | "
                  f"{float(r['AverageNs']) / 1e3:.1f} | {float(r['Percentage']):.1f} |")
    if not pmc:
        return
    frames = 2.0
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for sub in ("sq", "fetch", "write", "tcc"):
        p = os.path.join(pmc, sub, "run_counter_collection.csv")
        if not os.path.exists(p):
            continue
        for r in csv.DictReader(open(p)):
            agg[short(r["Kernel_Name"])][r["Counter_Name"]] += float(r["Counter_Value"])
    build = None
    for sub in ("sq", "fetch", "write"):
        p = os.path.join(pmc, sub + ".log")
        if os.path.exists(p):
            for line in open(p):
                if line.startswith("build:"):
                    build = line.split("src")[-1].strip()
    rd = sum(2 * d.get("FETCH_SIZE", 0) * 1024 / frames for k, d in agg.items() if "k_" in k)
    wr = sum(d.get("WRITE_SIZE", 0) * 1024 / frames for k, d in agg.items() if "k_" in k)
    print(f"\nBuild `{build}`: HBM traffic per frame = {rd / 1e9:.2f} GB read + {wr / 1e9:.2f} GB written "
          f"= {(rd + wr) / 1e9:.2f} GB\n")
    if js:
        import json
        # per frame: bytes, and the SQ / TCC counts behind bench.py's issue-side roofline (VALU wave-
        # instructions, wave-cycles and their parked / issue-stalled / active shares in quad-cycles,
        # L2 hits and misses)
        keys = {"SQ_INSTS_VALU": "valu_insts", "SQ_WAVES": "waves", "SQ_WAVE_CYCLES": "wave_cycles",
                "SQ_WAIT_ANY": "wait_any", "SQ_WAIT_INST_ANY": "wait_inst_any", "SQ_ACTIVE_INST_ANY": "active_inst_any",
                "SQ_BUSY_CYCLES": "busy_cycles", "TCC_HIT_sum": "tcc_hit", "TCC_MISS_sum": "tcc_miss"}
        per = {}
        for k, d in agg.items():
            if "k_" not in k:
                continue
            e = {"read_bytes": 2 * d.get("FETCH_SIZE", 0) * 1024 / frames, "write_bytes": d.get("WRITE_SIZE", 0) * 1024 / frames}
            for c, n in keys.items():
                if c in d:
                    e[n] = d[c] / frames
            per[k] = e
        json.dump({"build": build, "frame_read_bytes": rd, "frame_write_bytes": wr, "per_kernel": per,
                   "method": "rocprofv3 --pmc FETCH_SIZE (x2, gfx950) and WRITE_SIZE in separate passes, "
                             "2 frames, halved; SQ_* and TCC_HIT/MISS_sum in passes of their own"}, open(js[0], "w"), indent=1)
    print("\n## PMC per frame (separate passes; FETCH_SIZE ×2 gfx950 correction)\n")
    print("| kernel | HBM read GB | HBM write GB | VALU insts/wave | VALU wave-insts (G) | wave-cycles parked (SQ_WAIT_ANY) | issue-stalled | active | L2 hit |")
    print("|---|---:|---:|---:|---:|---:|---:|---:|---:|")
    for k, d in agg.items():
        if "k_" not in k:
            continue
        wc = d.get("SQ_WAVE_CYCLES", 0) or 1
        waves = d.get("SQ_WAVES", 0) or 1
        print(f"| `{k}` | {2 * d.get('FETCH_SIZE', 0) * 1024 / 1e9 / frames:.2f} | "
              f"{d.get('WRITE_SIZE', 0) * 1024 / 1e9 / frames:.2f} | {d.get('SQ_INSTS_VALU', 0) / waves:.0f} | "
              f"{d.get('SQ_INSTS_VALU', 0) / 1e9 / frames:.3f} | "
              f"{d.get('SQ_WAIT_ANY', 0) / wc:.2f} | {d.get('SQ_WAIT_INST_ANY', 0) / wc:.2f} | "
              f"{d.get('SQ_ACTIVE_INST_ANY', 0) / wc:.2f} | "
              f"{d.get('TCC_HIT_sum', 0) / max(1.0, d.get('TCC_HIT_sum', 0) + d.get('TCC_MISS_sum', 0)):.3f} |")


if __name__ == "__main__":
    main()
