import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
TESTS = os.path.dirname(os.path.abspath(__file__))
if TESTS not in sys.path:
    sys.path.insert(0, TESTS)


import pytest


@pytest.fixture(autouse=True)
def _default_schedule(request):
    """Tests that change a renderer's schedule (pbr_hip_set_schedule) leave the module-scoped `hip`
    fixture on the measured default for the next test."""
    hip = request.getfixturevalue("hip") if "hip" in request.fixturenames else None
    yield
    if hip is not None and getattr(hip, "ctx", None):
        hip.set_schedule()


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")
