"""Per-launch durations of the last device BVH build in gpurun_out/bvhprof (tools/bvh_prof.sh)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/bvhprof/run_kernel_trace.csv")))
emit = [i for i, r in enumerate(rows) if "k_bvh_emit" in r["Kernel_Name"]]
start = emit[-2] + 1 if len(emit) > 1 else 0
tot = {}
for r in rows[start:emit[-1] + 1]:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    name = r["Kernel_Name"].split("(")[0]
    tot[name] = tot.get(name, 0) + d
    print(f"{name:40s} grid {r.get('Grid_Size', r.get('Grid_Size_X', '?')):>10s} {d:9.1f} us")
print({k: round(v, 1) for k, v in tot.items()}, "total", round(sum(tot.values()), 1))
