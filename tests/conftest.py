import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libtblup_gpu.so on a real device)")


@pytest.fixture(scope="session")
def golden_dir():
    return os.path.join(ROOT, "tests", "golden")


@pytest.fixture(scope="session")
def gpu():
    """The loaded C-ABI library on a machine with a GPU; fails loudly (never skips) otherwise."""
    from tblup_amd import _native
    lib = _native.load()
    n = _native.device_count()
    if n < 1:
        pytest.fail("no HIP device visible: GPU tests must run on an MI355X box")
    return lib
