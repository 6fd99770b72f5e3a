import os
import sys

import pytest

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

_gpu_tests_ran = []


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs through libvsim_hip.so)")


def pytest_runtest_setup(item):
    if item.get_closest_marker("gpu") is not None:
        _gpu_tests_ran.append(item.nodeid)


@pytest.fixture(scope="session", autouse=True)
def no_spin_timeouts():
    """Session end of a GPU run: no bounded cross-workgroup wait (fused layer tail, barrier-free
    chain GEMV, stream-K finisher) may have given up in this process (vsim_spin_timeouts; the
    model calls already fail with VSIM_ESPIN when one does)."""
    yield
    hip = sys.modules.get("vsim_amd.hip")
    if not _gpu_tests_ran or hip is None or hip._lib is None:
        return
    n = hip.spin_timeouts()
    assert n == 0, f"{n} bounded cross-workgroup wait(s) gave up during the GPU session"
