"""Analyse a rocprofv3 kernel trace of queued frames (tools/r5_lanes.sh): which HIP stream ran on
which hardware queue, and how many render kernels ran at once over the frames."""
import collections
import csv
import sys

for path in sys.argv[1:]:
    rows = [r for r in csv.DictReader(open(path)) if "k_wf" in r["Kernel_Name"]]
    sq = collections.defaultdict(collections.Counter)
    for r in rows:
        sq[r["Stream_Id"]][r["Queue_Id"]] += 1
    print(path)
    print("  stream -> hardware queue (dispatches):", {k: dict(v) for k, v in sorted(sq.items())})
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows)
    pts = sorted([(s, 1) for s, _ in ev] + [(e, -1) for _, e in ev])
    c, last, hist = 0, pts[0][0], collections.Counter()
    for t, d in pts:
        hist[c] += t - last
        last, c = t, c + d
    tot = sum(hist.values())
    print(f"  span {tot / 1e6:.2f} ms; share of time with k kernels running:",
          {k: round(v / tot, 3) for k, v in sorted(hist.items())})
    # finish kernels mark frame ends: time from one frame's last finish to the next frame's first kernel
    fin = sorted(int(r["End_Timestamp"]) for r in rows if "finish" in r["Kernel_Name"])
    print(f"  {len(fin)} finish launches")
