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
def _engine_session():
    import keyhunt_amd
    if keyhunt_amd.device_count() < 1:
        pytest.fail("no GPU visible: -m gpu tests need an MI355X")
    e = keyhunt_amd.Engine(0)
    yield e
    e.close()


@pytest.fixture
def engine(_engine_session):
    """One engine for the whole session (its tables and pad are reused), with the settings a test may
    change put back to the defaults before each test, so no test's meaning depends on test order:
    the blocked layer-1 layout (kh_bsgs_set_layer1 takes effect at the next bsgs_setup) and the
    automatic launch geometry (which also clears a lane calibration)."""
    import keyhunt_amd
    e = _engine_session
    e._chk(keyhunt_amd.lib().kh_bsgs_set_layer1(e._ctx, keyhunt_amd.KH_LAYER1_BLOCKED), "kh_bsgs_set_layer1")
    e.set_geometry(0, 0)
    e.set_rmd_batch(0)
    yield e
