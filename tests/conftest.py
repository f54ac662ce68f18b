import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP) device")
    config.addinivalue_line("markers", "slow: multi-process / longer CPU tests")


@pytest.fixture(scope="session")
def hip_lib():
    """Build (incrementally) and load the HIP kernel library; GPU tests use it."""
    from nanodiloco_amd.csrc.build import build

    build()
    from nanodiloco_amd.ops import _ext

    return _ext.lib()
