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


# Collection order of the GPU suite: the hot-path parity files first (C1/C3 hydrostatic, then
# the NH core), the whole-config and multi-tile files after, so that under `-x` a slow or
# failing late file costs only itself.
_ORDER = ["test_parity_gpu.py", "test_nh_gpu.py", "test_configs_gpu.py", "test_rccl_gpu.py",
          "test_physics_seam_gpu.py", "test_bdyin_gpu.py", "test_tke_gpu.py",
          "test_restart_gpu.py", "test_restart_oracle_gpu.py", "test_fortran_shim.py"]


def pytest_collection_modifyitems(session, config, items):
    def rank(item):
        name = os.path.basename(str(item.fspath))
        return _ORDER.index(name) if name in _ORDER else len(_ORDER)
    items.sort(key=rank)      # stable: the order inside a file is kept
