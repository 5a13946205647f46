import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle"))

GOLDEN = os.path.join(REPO, "tests", "golden")
DATA = os.path.join(GOLDEN, "data")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP engine)")


@pytest.fixture(scope="session")
def oracle():
    import oracle as o
    o.lib()
    return o


@pytest.fixture(scope="session")
def engine():
    import keyhunt_amd
    if keyhunt_amd.device_count() < 1:
        pytest.fail("no GPU visible: -m gpu tests need an MI355X")
    e = keyhunt_amd.Engine(0)
    yield e
    e.close()
