import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "multi-scale-pointcloud-registration_amd")
for p in (PKG, os.path.join(REPO, "oracle"), os.path.join(REPO, "tests", "golden"), REPO):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through liborpcd_hip.so)")


@pytest.fixture(scope="session")
def oracle():
    import oracle as O
    O.lib()
    return O


@pytest.fixture(scope="session")
def ctx():
    from orpcd_amd import _native
    if _native.device_count() == 0:
        pytest.skip("no HIP device")
    return _native.Context(0)
