"""The Fortran ISO_C_BINDING shim (regcm_amd/fortran/mod_gpu_dyn.F90): the host-language
boundary the north star asks for.  CPU: it builds with amdflang and its bind(c) config type has
the C layout's size.  GPU: a Fortran host (test_shim.F90, the RCM_run loop with physics stubbed)
driving the engine through the shim gives bit-identical results to the Python host."""
import ctypes
import os
import subprocess
import tempfile

import numpy as np
import pytest

from regcm_amd.config import FIELD, RcmdynConfig, field_levels

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FDIR = os.path.join(ROOT, "regcm_amd", "fortran")
EXE = os.path.join(FDIR, "test_shim")


def _build():
    subprocess.run(["make", "-s", "-C", FDIR], check=True)


def test_shim_builds_and_layout():
    _build()
    out = subprocess.run([EXE, "--sizeof"], capture_output=True, text=True, check=True).stdout
    assert int(out.split()[0]) == ctypes.sizeof(RcmdynConfig)


@pytest.mark.gpu
def test_fortran_host_matches_python_host(c1_data):
    from regcm_amd.dycore import DynCore
    _build()
    rc, data = c1_data
    nsteps = 5
    eng = DynCore(rc, data["split"])
    eng.put_state(data["state"])
    eng.bdyval()
    for _ in range(nsteps):
        eng.tend()
        eng.bdyval()
    with tempfile.TemporaryDirectory() as d:
        fin, fout = os.path.join(d, "in.bin"), os.path.join(d, "out.bin")
        with open(fin, "wb") as f:
            np.array([rc.jx, rc.iy, rc.kz, rc.nsplit, nsteps], dtype=np.int32).tofile(f)
            f.write(bytes(eng.cfg))
            np.array([len(data["state"])], dtype=np.int32).tofile(f)
            for name, arr in data["state"].items():
                nk = field_levels(name, rc.kz, rc.nsplit)
                np.array([FIELD[name], nk], dtype=np.int32).tofile(f)
                np.ascontiguousarray(arr, dtype=np.float64).tofile(f)
        subprocess.run([EXE, fin, fout], check=True, timeout=300)
        raw = open(fout, "rb").read()
    lcount = np.frombuffer(raw[:8], dtype=np.int64)[0]
    dt, xbc = np.frombuffer(raw[8:24], dtype=np.float64)
    n3 = rc.kz * rc.iy * rc.jx
    body = np.frombuffer(raw[24:], dtype=np.float64)
    t = body[:n3].reshape(rc.kz, rc.iy, rc.jx)
    u = body[n3:2 * n3].reshape(rc.kz, rc.iy, rc.jx)
    ps = body[2 * n3:].reshape(1, rc.iy, rc.jx)
    assert (lcount, dt, xbc) == eng.get_time()
    assert np.array_equal(t, eng.get("ATM1_T"))
    assert np.array_equal(u, eng.get("ATM1_U"))
    assert np.array_equal(ps, eng.get("PSA"))
