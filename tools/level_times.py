"""Per-level wavefront kernel times from a rocprofv3 kernel trace (the last of N rendered frames).

    python tools/level_times.py gpurun_out/prof/run_kernel_trace.csv [frames=2]
"""
import collections
import csv
import re
import sys


def main():
    frames = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    rows = list(csv.DictReader(open(sys.argv[1])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    wf = [r for r in rows if "k_wf_" in r["Kernel_Name"]]
    seq = [(re.sub(r".*(k_wf_\w+).*", r"\1", r["Kernel_Name"]),
            (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3) for r in wf]
    frame = seq[len(seq) - len(seq) // frames:]
    last = wf[len(wf) - len(wf) // frames:]
    span = (int(last[-1]["End_Timestamp"]) - int(last[0]["Start_Timestamp"])) / 1e3
    lv = collections.defaultdict(list)
    level = -1
    for k, t in frame:
        if k == "k_wf_camera_extend":
            level = 0
        elif k == "k_wf_extend":
            level += 1
        lv[(k, level if k != "k_wf_finish" else -1)].append(t)
    tot = 0.0
    for (k, l), v in sorted(lv.items(), key=lambda x: (x[0][1], x[0][0])):
        tot += sum(v)
        print(f"{k:22s} level {l:2d}  launches {len(v):3d}  avg {sum(v) / len(v):8.1f} us  total {sum(v) / 1e3:7.2f} ms")
    print(f"frame total {tot / 1e3:.2f} ms of kernels, {span / 1e3:.2f} ms first start to last end "
          f"({len(frame)} launches)")


if __name__ == "__main__":
    main()
