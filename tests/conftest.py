import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cfd-demo2_amd"))
sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs through the HIP library)")
    config.addinivalue_line("markers", "slow: long CPU test")
    # make sure the native library and the oracle exist (no-op when up to date)
    import __graft_entry__ as g
    g.build_product()
    g.build_oracle()


@pytest.fixture(scope="session")
def gpu_available():
    import ctypes
    try:
        hip = ctypes.CDLL("libamdhip64.so")
        n = ctypes.c_int(0)
        return hip.hipGetDeviceCount(ctypes.byref(n)) == 0 and n.value > 0
    except OSError:
        return False
