"""The device's inline transcendental fast paths (csrc/pbr_math.h, namespace fastm) against glibc.

Each `t_f(x)` of the render path is `(float)f((double)x)`.  On the device it is evaluated inline in
fp64 first and accepted only when every value within 2^-40 relative of the approximation rounds to
the same float; otherwise the out-of-line fp64 call is made.  That is exact only if the
approximation really is that close: this test compiles the same header for the host
(tests/cpp/fast_trans_check.cpp, -ffp-contract=off like the device build) and checks, over millions
of arguments incl. the floats nearest the multiples of pi/2 and the ends of asin/acos/log's ranges,
that the worst relative error stays below 2^-48 (measured: 2^-51), that every accepted argument
rounds to exactly `(float)f((double)x)`, and that the check declines rarely.  The device results
themselves are covered by the full-frame bit-identity runs and the parity suite (-m gpu).
"""
import json
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


@pytest.fixture(scope="module")
def report(tmp_path_factory):
    if shutil.which("g++") is None:
        pytest.skip("g++ not available")
    exe = tmp_path_factory.mktemp("fast_trans") / "fast_trans_check"
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-fno-fast-math", "-Wall", "-Werror",
                    "-o", str(exe), str(ROOT / "tests/cpp/fast_trans_check.cpp")], check=True)
    out = subprocess.run([str(exe), "1000000"], check=True, capture_output=True, text=True).stdout
    return json.loads(out)


@pytest.mark.parametrize("fn", ["sin", "cos", "atan2", "asin", "acos", "log", "exp"])
def test_fast_path_is_within_tolerance_and_exact_when_accepted(report, fn):
    r = report[fn]
    assert r["n"] > 500_000
    assert r["worst_log2"] < -48, r
    assert r["mismatched"] == 0, r
    assert r["declined"] < r["n"] * 1e-3, r
