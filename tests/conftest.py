import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "orb-slam-system_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 GPU (runs the HIP kernels)")
    config.addinivalue_line("markers", "slow: exhaustive checks (tens of seconds)")


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as O
    O.build()
    return O


@pytest.fixture(scope="session")
def orbx_mod():
    import orbx
    return orbx


@pytest.fixture(scope="session")
def gpu(orbx_mod):
    if orbx_mod.device_count() < 1:
        pytest.fail("gpu test selected but no GPU device is visible")
    return orbx_mod
