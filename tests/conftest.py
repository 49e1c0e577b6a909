import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 (MI355X) device")
    config.addinivalue_line("markers", "slow: long-running (full-size) test")


@pytest.fixture(scope="session")
def oracle_lib():
    import oracle
    oracle.build(ref=None)
    return oracle


@pytest.fixture(scope="session")
def kgx():
    from close_kmers_amd import abi, build
    build.build()
    abi.lib()
    return abi


@pytest.fixture(scope="session")
def gpu(kgx):
    """The HIP engine on a real device; fails (never falls back) without one."""
    n = kgx.device_count()
    if n < 1:
        pytest.fail("no gfx950 device visible: the -m gpu tests need an MI355X")
    return kgx
