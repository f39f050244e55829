import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box via gpurun)")
    config.addinivalue_line("markers", "slow: long-running (full-size) test")


@pytest.fixture(scope="session")
def oracle_lib():
    from oracle import pyoracle
    pyoracle.build()
    return pyoracle


@pytest.fixture(scope="session")
def gwaoi_lib():
    from goworld_amd import build as gbuild
    from goworld_amd import _lib
    if not os.path.exists(_lib.SO_PATH):
        gbuild.build()
    return _lib.load()


@pytest.fixture(scope="session")
def gpu(gwaoi_lib):
    from goworld_amd import _lib
    if _lib.device_count() < 1:
        pytest.fail("GPU test ran without a HIP device")
    return 0
