import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "deepseek-ocr.rs_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 (MI355X) GPU")
    config.addinivalue_line("markers", "slow: long-running full-size case")


def gpu_available() -> bool:
    try:
        from dsocr._lib import lib
        import ctypes
        n = ctypes.c_int(0)
        return lib().dsocr_device_count(ctypes.byref(n)) == 0 and n.value > 0
    except Exception:
        return False


@pytest.fixture(scope="session")
def gpu():
    if not gpu_available():
        pytest.fail("GPU test requested but no HIP device / libdsocr.so available")
    return True
