import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")
    config.addinivalue_line("markers", "slow: long-running statistical test")


@pytest.fixture(scope="session")
def hip_device():
    """Fail loudly (never skip silently) when a gpu test runs without a HIP device."""
    import multigridmc_amd as mg
    mg.load_library()
    import ctypes
    n = ctypes.c_int(0)
    hip = ctypes.CDLL("libamdhip64.so")
    rc = hip.hipGetDeviceCount(ctypes.byref(n))
    if rc != 0 or n.value < 1:
        pytest.fail("gpu test requested but no HIP device is visible")
    return 0
