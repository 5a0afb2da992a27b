"""pytest configuration: the `gpu` marker and import paths.

`-m "not gpu"` tests run in the CPU container (oracle, host logic, ABI
loading); `-m gpu` tests run on an MI355X and call librm through its C-ABI.
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "opengl-raymarching-in-compute-shader_amd")
for p in (ROOT, PKG, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (MI355X); calls librm")


@pytest.fixture(scope="session")
def rm():
    import rmarch
    rmarch.lib()  # fails loudly if librm.so is missing
    return rmarch


@pytest.fixture(scope="session")
def oracle():
    import oracle as O
    O.lib()
    return O


@pytest.fixture(scope="session")
def gpu(rm):
    """Skip-free guard: a gpu-marked test must run on a GPU box."""
    n = rm.device_count()
    assert n > 0, "gpu test selected but no HIP device is visible"
    return n
