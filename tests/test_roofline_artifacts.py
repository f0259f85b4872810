"""The committed measurement artifacts of the latest round agree with each other (CPU only).

bench.py's top-level roofline is the dominant kernel family's own rate: its algorithmic bytes per
launch over its mean launch duration in a serial window (every kernel running alone).  The same
build's `rocprofv3 --kernel-trace --stats` of `bench.py --serial` is committed next to each bench
line; tools/roofline_check.py recomputes the rates from it.  Here: for every config, the dominant
family's standalone time per frame is below the frame time of the line, and its rate recomputed
from the rocprof stats matches the line's within 2%.  Round 6: the issue side — each family's VALU
wave-instructions per frame, its share of parked wave-cycles and its L2 hit rate — comes from the
same build's SQ / TCC passes (profiles/<cfg>_traffic.json); the line's figures reproduce from that
file, and the dominant family carries the bound that binds it (hbm, issue or latency)."""
import csv
import json
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROF = os.path.join(ROOT, "profiles")


def _family_avg_us(stats_csv, family):
    import sys
    sys.path.insert(0, ROOT)
    import bench   # kernel_family: rocprof names → profile families (the fused level 0 is k_wf_shade_l0)
    ns = calls = 0
    for r in csv.DictReader(open(stats_csv)):
        if bench.kernel_family(r["Name"]) == family:
            ns += float(r["TotalDurationNs"])
            calls += int(r["Calls"])
    assert calls > 0, f"{family} not in {stats_csv}"
    return ns / calls / 1e3


def _latest(cfg):
    for rnd in ("r6", "r5", "r4"):
        b, k = os.path.join(PROF, f"{rnd}_{cfg}_bench.json"), os.path.join(PROF, f"{rnd}_{cfg}_kernel_stats.csv")
        if os.path.exists(b) and os.path.exists(k):
            return rnd, b, k
    return None, None, None


@pytest.mark.parametrize("cfg", ["c2", "c3", "c4", "c5"])
def test_dominant_family_rate_reproduces_from_rocprof(cfg):
    rnd, bench_path, stats_path = _latest(cfg)
    if rnd is None:
        pytest.skip("no round's artifacts present")
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


@pytest.mark.parametrize("cfg", ["c2", "c3", "c4", "c5"])
def test_issue_side_reproduces_from_pmc(cfg):
    rnd, bench_path, _ = _latest(cfg)
    if rnd != "r6":
        pytest.skip("the issue-side roofline starts in round 6")
    import sys
    sys.path.insert(0, ROOT)
    import bench
    line = json.loads(open(bench_path).read().strip().splitlines()[-1])
    rl = line["roofline"]
    t = json.load(open(os.path.join(PROF, f"{cfg}_traffic.json")))
    assert rl["build"].endswith(t["build"]), "the PMC passes are of another build"
    for fam, k in rl["kernels"].items():
        cc = bench.family_counts(t, fam)
        assert cc is not None, fam
        assert k["valu_insts_per_frame"] == round(cc["valu_insts"])
        frac = cc["valu_insts"] / (k["ms_per_frame"] * 1e-3) / bench.VALU_ISSUE_PEAK
        assert abs(frac - k["valu_issue_frac"]) <= 0.01 * k["valu_issue_frac"] + 1e-4, (fam, frac, k["valu_issue_frac"])
        assert abs(cc["wait_any"] / cc["wave_cycles"] - k["wait_any_share"]) <= 2e-3
        assert k["bound"] in ("hbm", "issue", "latency")
        assert k["bound"] == bench.binding_bound(k.get("traffic_frac", k["frac"]), k["valu_issue_frac"], k["wait_any_share"])[0]
    b = rl["binding"]
    assert b["bound"] == rl["kernels"][rl["kernel"]]["bound"] and 0 < b["frac"] <= 1
