"""The committed round-4 measurement artifacts agree with each other (CPU only).

bench.py's top-level roofline is the dominant kernel family's own rate: its algorithmic bytes per
launch over its mean launch duration in a serial window (every kernel running alone).  The same
build's `rocprofv3 --kernel-trace --stats` of `bench.py --serial` is committed next to each bench
line; tools/roofline_check.py recomputes the rates from it.  Here: for every config, the dominant
family's standalone time per frame is below the frame time of the line, and its rate recomputed
from the rocprof stats matches the line's within 2%."""
import csv
import json
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROF = os.path.join(ROOT, "profiles")


def _family_avg_us(stats_csv, family):
    ns = calls = 0
    for r in csv.DictReader(open(stats_csv)):
        m = re.search(r"(k_\w+?)[<(]", r["Name"])
        if m and m.group(1) == family:
            ns += float(r["TotalDurationNs"])
            calls += int(r["Calls"])
    assert calls > 0, f"{family} not in {stats_csv}"
    return ns / calls / 1e3


@pytest.mark.parametrize("cfg", ["c2", "c3", "c4", "c5"])
def test_dominant_family_rate_reproduces_from_rocprof(cfg):
    bench_path = os.path.join(PROF, f"r4_{cfg}_bench.json")
    stats_path = os.path.join(PROF, f"r4_{cfg}_kernel_stats.csv")
    if not (os.path.exists(bench_path) and os.path.exists(stats_path)):
        pytest.skip("round-4 artifacts not present")
    line = json.loads(open(bench_path).read().strip().splitlines()[-1])
    rl = line["roofline"]
    fam = rl["kernel"]
    k = rl["kernels"][fam]
    assert rl["ms_per_frame"] < line["ms_per_step"]   # a kernel's own time, not the lanes' sum
    assert k["ms_per_frame"] == rl["ms_per_frame"]
    avg_us = _family_avg_us(stats_path, fam)
    frac = k["alg_bytes_per_launch"] / (avg_us * 1e-6) / 8000e9
    assert abs(frac - rl["frac"]) <= 0.02 * rl["frac"], (cfg, fam, frac, rl["frac"])
    # bench.py attaches PMC traffic only when it was measured on the very build it loaded
    assert rl.get("traffic") is not None and rl.get("traffic_source")
