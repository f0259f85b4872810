"""Per-family algorithmic vs PMC bytes per frame from bench.py lines (profiles/r3_c*_bench.json)."""
import json
import sys

for path in sys.argv[1:]:
    d = json.load(open(path))
    r = d["roofline"]
    print(f"{path}: {d['ms_per_step']:.2f} ms, {d['value']:.1f} {d['unit']}")
    print("| family | ms/frame | alg GB/frame | PMC GB/frame | PMC/alg |")
    print("|---|---:|---:|---:|---:|")
    for k, v in r["kernels"].items():
        alg = v["alg_bytes_per_launch"] * v["launches_per_frame"] / 1e9
        pmc = (v.get("traffic_per_launch") or 0) * v["launches_per_frame"] / 1e9
        print(f"| `{k}` | {v['ms_per_frame']:.2f} | {alg:.2f} | {pmc:.2f} | {pmc / alg if alg else 0:.2f} |")
    f = r.get("frame") or {}
    if f:
        print(f"| frame | {f['kernel_ms_per_frame']:.1f} (x{f['concurrency']}) | {f['alg_bytes'] / 1e9:.1f} | "
              f"{(f.get('traffic') or 0) / 1e9:.1f} | {(f.get('traffic') or 0) / f['alg_bytes']:.2f} |")
    print()
