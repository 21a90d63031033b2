import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP engine C-ABI)")


@pytest.fixture(scope="session")
def c1_data():
    from regcm_amd.config import CONFIGS
    from regcm_amd import icbc
    rc = CONFIGS["C1"]
    return rc, icbc.generate(rc)
