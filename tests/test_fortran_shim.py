"""The Fortran ISO_C_BINDING shim (regcm_amd/fortran/mod_gpu_dyn.F90): the host-language
boundary the north star asks for (Main/mod_regcm_interface.F90:172-228 stays Fortran).

A Fortran host (regcm_amd/fortran/test_shim.F90) runs a script of C-ABI calls through the shim
and writes back every result it reads; the Python host (ctypes over the same library) runs the
same script.  The two must agree bit for bit: every state, slice, boundary and diagnostic field,
the clock, the job sums and the error codes and messages of refused calls.

CPU: the shim builds with amdflang, its bind(c) config type has the C layout's size, and the
host-only entry points (set_nproc, tile_extent, exchange_plan, overlap_shares, a refused create)
agree.  GPU: the hydrostatic core (tend + bdyval, rcmdyn_step, synchronize, the sums, tendency
diagnostics, a restart through set_time), the non-hydrostatic core, ipptls = 2, the
pre/post-physics split with non-zero *PHY tendencies put on the interior only, and a bdyin.
"""
import ctypes
import dataclasses
import os
import struct
import subprocess
import tempfile

import numpy as np
import pytest

from regcm_amd import icbc
from regcm_amd.config import (ATMS_FIELDS, CONFIGS, FIELD, NH_PHY_FIELDS, NH_STATE_FIELDS, PHY_FIELDS,
                              QX_ATMS_FIELDS, QX_PHY_FIELDS, QX_STATE_FIELDS, STATE_FIELDS, TWO_D,
                              RcmdynConfig, build_config, field_levels)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FDIR = os.path.join(ROOT, "regcm_amd", "fortran")
EXE = os.path.join(FDIR, "test_shim")

# op codes of test_shim.F90
END, CREATE, DESTROY, PUT, GET, TEND, BDYVAL, STEP, PRE, POST, BDYIN, SYNC = range(12)
SET_TIME, GET_TIME, SET_DIAG, REDUCTIONS, DIAGNOSTICS, LAST_MS, RUNTIME = range(12, 19)
SET_NPROC, TILE_EXTENT, PLAN, SHARES, KTIMES, SOFT, TILE_EXTENT_CFG = range(19, 26)


def _build():
    subprocess.run(["make", "-s", "-C", FDIR], check=True)


class Script:
    """A sequence of C-ABI calls, run by the Python host (ctypes) or the Fortran host."""

    def __init__(self, cfg: RcmdynConfig):
        self.cfg = cfg
        self.ops = []

    def add(self, code, *args):
        self.ops.append((code, args))
        return self

    def soft(self):
        """The next op reports its return code and message instead of failing."""
        return self.add(SOFT)

    def put(self, name, a, j1=1, i1=1, k1=1):
        a = np.ascontiguousarray(a, dtype=np.float64)
        nk, ni, nj = a.shape
        dims = 2 if name in TWO_D and nk == 1 else 3
        return self.add(PUT, dims, FIELD[name], j1, j1 + nj - 1, i1, i1 + ni - 1, k1, k1 + nk - 1, a)

    def get(self, name, rc, j1=1, i1=1):
        nk = field_levels(name, rc.kz, rc.nsplit)
        dims = 2 if name in TWO_D and nk == 1 else 3
        return self.add(GET, dims, FIELD[name], j1, rc.jx, i1, rc.iy, 1, nk)

    # ---- the Python host
    def run_python(self):
        from regcm_amd.dycore import lib
        L = lib()
        dp = ctypes.POINTER(ctypes.c_double)
        h = ctypes.c_void_p()
        out, soft = [], False
        for code, a in self.ops:
            if code == SOFT:
                soft = True
                continue
            res, rc = [], 0
            if code == CREATE:
                rc = L.rcmdyn_create(ctypes.byref(self.cfg), ctypes.byref(h))
            elif code == DESTROY:
                rc = L.rcmdyn_destroy(h)
                h = ctypes.c_void_p()
            elif code == PUT:
                dims, fid, j1, j2, i1, i2, k1, k2, arr = a
                rc = L.rcmdyn_put(h, fid, arr.ctypes.data_as(dp), j1, j2, i1, i2, k1, k2)
            elif code == GET:
                dims, fid, j1, j2, i1, i2, k1, k2 = a
                buf = np.zeros((k2 - k1 + 1, i2 - i1 + 1, j2 - j1 + 1))
                rc = L.rcmdyn_get(h, fid, buf.ctypes.data_as(dp), j1, j2, i1, i2, k1, k2)
                res = [buf]
            elif code in (TEND, BDYVAL, PRE, POST, BDYIN, SYNC):
                fn = {TEND: L.rcmdyn_tend, BDYVAL: L.rcmdyn_bdyval, PRE: L.rcmdyn_tend_pre_physics,
                      POST: L.rcmdyn_tend_post_physics, BDYIN: L.rcmdyn_bdyin, SYNC: L.rcmdyn_synchronize}[code]
                rc = fn(h)
            elif code == STEP:
                rc = L.rcmdyn_step(h, a[0])
            elif code == SET_TIME:
                rc = L.rcmdyn_set_time(h, *a)
            elif code == GET_TIME:
                x, y, z = ctypes.c_int64(), ctypes.c_double(), ctypes.c_double()
                rc = L.rcmdyn_get_time(h, ctypes.byref(x), ctypes.byref(y), ctypes.byref(z))
                res = [(x.value, y.value, z.value)]
            elif code == SET_DIAG:
                rc = L.rcmdyn_set_diagnostics(h, a[0])
            elif code in (REDUCTIONS, DIAGNOSTICS):
                n = 3 if code == REDUCTIONS else 4
                v = (ctypes.c_double * n)()
                rc = (L.rcmdyn_reductions if code == REDUCTIONS else L.rcmdyn_diagnostics)(h, v)
                res = [tuple(v)]
            elif code == LAST_MS:
                v = ctypes.c_double()
                rc = L.rcmdyn_last_step_ms(h, ctypes.byref(v))
                res = [v.value]
            elif code == RUNTIME:
                buf = ctypes.create_string_buffer(1024)
                rc = L.rcmdyn_runtime_info(buf, 1024)
                res = [buf.value.decode()]
            elif code == SET_NPROC:
                cp = (ctypes.c_int32 * 2)()
                rc = L.rcmdyn_set_nproc(*a, cp)
                res = [tuple(cp)]
            elif code == TILE_EXTENT:
                ext, bdy = (ctypes.c_int32 * 8)(), (ctypes.c_int32 * 4)()
                rc = L.rcmdyn_tile_extent(*a, ext, bdy)
                res = [tuple(ext) + tuple(bdy)]
            elif code == TILE_EXTENT_CFG:
                ext, bdy = (ctypes.c_int32 * 8)(), (ctypes.c_int32 * 4)()
                rc = L.rcmdyn_tile_extent_cfg(ctypes.byref(self.cfg), a[0], ext, bdy)
                res = [tuple(ext) + tuple(bdy)]
            elif code == PLAN:
                n = ctypes.c_int64()
                rc = L.rcmdyn_exchange_plan(ctypes.byref(self.cfg), a[0], None, 0, ctypes.byref(n))
                if rc == 0:
                    ops = np.zeros((max(n.value, 1), 7), dtype=np.int64)
                    rc = L.rcmdyn_exchange_plan(ctypes.byref(self.cfg), a[0],
                                                ops.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)), n.value,
                                                ctypes.byref(n))
                    res = [ops[:n.value]]
            elif code == SHARES:
                v = (ctypes.c_int32 * (6 * a[0]))()
                rc = L.rcmdyn_overlap_shares(ctypes.byref(self.cfg), v, a[0])
                res = [tuple(v)]
            elif code == KTIMES:
                cap = 64
                names = ctypes.create_string_buffer(cap * 48)
                launches, avg, n = (ctypes.c_int32 * cap)(), (ctypes.c_double * cap)(), ctypes.c_int32()
                rc = L.rcmdyn_kernel_times(h, a[0], cap, names, launches, avg, ctypes.byref(n))
                nm = [names.raw[q * 48:(q + 1) * 48].split(b"\0", 1)[0].decode() for q in range(n.value)]
                res = [dict(zip(nm, list(launches)[:n.value]))]
            else:
                raise ValueError(code)
            if soft:
                msg = L.rcmdyn_last_error(h if h.value else None).decode() if rc else ""
                out.append((rc, msg))
                soft = False
            else:
                assert rc == 0, (code, L.rcmdyn_last_error(h if h.value else None).decode())
                out.extend(res)
        if h.value:
            L.rcmdyn_destroy(h)
        return out

    # ---- the Fortran host
    def run_fortran(self, timeout=300):
        _build()
        with tempfile.TemporaryDirectory() as d:
            fin, fout = os.path.join(d, "in.bin"), os.path.join(d, "out.bin")
            with open(fin, "wb") as f:
                raw = bytes(self.cfg)
                f.write(struct.pack("<i", len(raw)) + raw)
                for code, a in self.ops:
                    f.write(struct.pack("<i", code))
                    if code == PUT:
                        f.write(struct.pack("<8i", *a[:8]) + a[8].tobytes())
                    elif code == GET:
                        f.write(struct.pack("<8i", *a))
                    elif code == SET_TIME:
                        f.write(struct.pack("<qdd", *a))
                    elif a:
                        f.write(struct.pack(f"<{len(a)}i", *a))
                f.write(struct.pack("<i", END))
            subprocess.run([EXE, fin, fout], check=True, timeout=timeout)
            buf = open(fout, "rb").read()
        return self._parse(buf)

    def _parse(self, buf):
        out, pos, soft = [], 0, False

        def take(fmt):
            nonlocal pos
            v = struct.unpack_from(fmt, buf, pos)
            pos += struct.calcsize(fmt)
            return v

        def arr(n, dtype):
            nonlocal pos
            v = np.frombuffer(buf, dtype=dtype, count=n, offset=pos)
            pos += n * np.dtype(dtype).itemsize
            return v

        for code, a in self.ops:
            if code == SOFT:
                soft = True
                continue
            if soft:
                rc, = take("<i")
                msg = bytes(arr(1024, np.uint8)).split(b"\0", 1)[0].decode()
                out.append((rc, msg))
                soft = False
                continue
            if code == GET:
                dims, fid, j1, j2, i1, i2, k1, k2 = a
                shape = (k2 - k1 + 1, i2 - i1 + 1, j2 - j1 + 1)
                out.append(arr(int(np.prod(shape)), np.float64).reshape(shape))
            elif code == GET_TIME:
                out.append(take("<qdd"))
            elif code == REDUCTIONS:
                out.append(take("<3d"))
            elif code == DIAGNOSTICS:
                out.append(take("<4d"))
            elif code == LAST_MS:
                out.append(take("<d")[0])
            elif code == RUNTIME:
                out.append(bytes(arr(1024, np.uint8)).split(b"\0", 1)[0].decode())
            elif code == SET_NPROC:
                out.append(take("<2i"))
            elif code in (TILE_EXTENT, TILE_EXTENT_CFG):
                out.append(take("<12i"))
            elif code == PLAN:
                n, = take("<q")
                out.append(arr(7 * n, np.int64).reshape(n, 7))
            elif code == SHARES:
                out.append(take(f"<{6 * a[0]}i"))
            elif code == KTIMES:
                n, = take("<i")
                launches = arr(n, np.int32)
                names = bytes(arr(48 * n, np.uint8))
                nm = [names[q * 48:(q + 1) * 48].split(b"\0", 1)[0].decode() for q in range(n)]
                out.append(dict(zip(nm, [int(x) for x in launches])))
        assert pos == len(buf), (pos, len(buf))
        return out


def assert_same(py, fo):
    assert len(py) == len(fo)
    for q, (a, b) in enumerate(zip(py, fo)):
        if isinstance(a, np.ndarray):
            assert a.shape == b.shape and np.array_equal(a, b), q
        else:
            assert tuple(a) == tuple(b) if isinstance(a, (tuple, list)) else a == b, (q, a, b)


def test_shim_builds_and_layout():
    _build()
    out = subprocess.run([EXE, "--sizeof"], capture_output=True, text=True, check=True).stdout
    assert int(out.split()[0]) == ctypes.sizeof(RcmdynConfig)


def test_fortran_host_only_entry_points(c1_data):
    """set_nproc, tile_extent, a rank's exchange plan and the overlap shares through the shim,
    with no GPU, and a refused create (its return code and message), as the Python host."""
    rc, data = c1_data
    from regcm_amd.vmodes import spinit_constants
    c3 = CONFIGS["C3"]
    split3 = spinit_constants(c3.sigma, c3.ptop, c3.kz, c3.dt, c3.nsplit)
    cfg = build_config(c3, split3, 2, 2, tile_first=1, tile_count=1, comm_rank=1, comm_size=4)
    s = Script(cfg)
    for n in (1, 2, 4, 8, 16):
        s.add(SET_NPROC, n, c3.jx, c3.iy)
    for t in range(8):
        s.add(TILE_EXTENT, c3.jx, c3.iy, 2, 4, t)
    s.add(PLAN, 3).add(SHARES, 1)
    py, fo = s.run_python(), s.run_fortran()
    assert_same(py, fo)
    assert py[3] == (2, 4) and py[-2].shape[0] > 0
    # the band-aware extents (i_band = 1: no west/east side, the cross range ends at jx)
    band = build_config(dataclasses.replace(c3, i_band=1), split3, 2, 4, tile_first=0, tile_count=8)
    s = Script(band)
    for t in range(8):
        s.add(TILE_EXTENT_CFG, t)
    py, fo = s.run_python(), s.run_fortran()
    assert_same(py, fo)
    assert py[7][5] == c3.jx and py[7][8:10] == (0, 0), py[7]
    bad = build_config(rc, data["split"])
    bad.i_band = 2
    s = Script(bad).soft().add(CREATE)
    py, fo = s.run_python(), s.run_fortran()
    assert py == fo and py[0][0] != 0 and "i_band" in py[0][1], py


# ------------------------------------------------------------------------------- GPU cases

def _start(s, rc, st, extra=None):
    s.add(CREATE)
    for name, a in st.items():
        s.put(name, a)
    for name, a in (extra or {}).items():
        s.put(name, a)
    return s.add(BDYVAL)


def _gets(s, rc, names):
    for name in names:
        s.get(name, rc)
    return s


@pytest.mark.gpu
def test_fortran_host_hydrostatic(c1_data):
    """C1: tend + bdyval, rcmdyn_step, synchronize, the job sums, the tendency diagnostics (and
    the refused get when they are off), a restart through get / put / set_time."""
    rc, data = c1_data
    s = Script(build_config(rc, data["split"]))
    _start(s, rc, data["state"])
    s.soft().get("TTEN", rc)                    # diagnostics off: refused
    for _ in range(3):
        s.add(TEND).add(BDYVAL)
    s.add(STEP, 4).add(SYNC).add(GET_TIME).add(REDUCTIONS).add(DIAGNOSTICS)
    s.add(SET_DIAG, 1).add(TEND).add(BDYVAL)
    _gets(s, rc, ["TTEN", "UTEN", "QVTEN", "OMEGA", "QDOT", "PSC", "PTEN"])
    _gets(s, rc, STATE_FIELDS)
    # restart from a SAV state: the prognostic fields put back, the clock set
    for name in STATE_FIELDS:
        s.put(name, data["state"][name])
    s.add(SET_TIME, 2, 2.0 * rc.dt, rc.dt).add(STEP, 2).add(GET_TIME)
    _gets(s, rc, STATE_FIELDS)
    s.add(RUNTIME).add(KTIMES, 1).add(DESTROY)
    py, fo = s.run_python(), s.run_fortran()
    # the runtime paths are each process's own (a Python host that imported torch binds torch's
    # libamdhip64 / librccl, the Fortran host /opt/rocm's): the same report, not the same text
    for r in (py[-2], fo[-2]):
        assert r.startswith("hip=") and "; rccl=" in r, r
    py[-2] = fo[-2] = None
    assert_same(py, fo)
    assert py[0][0] != 0 and "diagnostics" in py[0][1]
    assert py[1][0] == 7                         # 3 tend + bdyval, then rcmdyn_step(4)
    assert "k_update" in py[-1] or len(py[-1]) > 3


@pytest.mark.gpu
def test_fortran_host_step_ms(c1_data):
    """rcmdyn_last_step_ms reads back through the shim (a timing, so only its range is checked)."""
    rc, data = c1_data
    s = Script(build_config(rc, data["split"]))
    _start(s, rc, data["state"]).add(STEP, 10).add(LAST_MS).add(DESTROY)
    fo = s.run_fortran()
    assert 0.0 < fo[0] < 1000.0


@pytest.mark.gpu
def test_fortran_host_nonhydrostatic():
    """N1 (idynamic = 2, acoustic sub-stepping) through the shim, tend + bdyval and step."""
    rc = CONFIGS["N1"]
    data = icbc.generate_nh(rc)
    s = Script(build_config(rc, data["split"]))
    _start(s, rc, data["state"])
    for _ in range(2):
        s.add(TEND).add(BDYVAL)
    s.add(STEP, 3).add(GET_TIME).add(REDUCTIONS)
    _gets(s, rc, STATE_FIELDS + NH_STATE_FIELDS)
    py, fo = s.run_python(), s.run_fortran()
    assert_same(py, fo)
    assert py[0][0] == 5 and py[1][2] > 0.0      # the NH CFL of the last sub-step


@pytest.mark.gpu
def test_fortran_host_species(c1_data):
    """ipptls = 2 (nqx = 5): qi, qr, qs put, stepped and read back through the shim."""
    rc, data = c1_data
    rcq = dataclasses.replace(rc, ipptls=2)
    st = {k: v.copy() for k, v in data["state"].items()}
    st.update(icbc.hydrometeor_state(rcq, st, nqx=rcq.nqx))
    s = Script(build_config(rcq, data["split"]))
    _start(s, rcq, st)
    s.add(TEND).add(BDYVAL).add(STEP, 3)
    _gets(s, rcq, STATE_FIELDS + QX_STATE_FIELDS)
    py, fo = s.run_python(), s.run_fortran()
    assert_same(py, fo)


@pytest.mark.gpu
@pytest.mark.parametrize("nh", [False, True], ids=["hydrostatic", "nonhydrostatic"])
def test_fortran_host_physics_split(c1_data, nh):
    """The physics seam: pre_physics, the ATMS_* slices read, non-zero *PHY tendencies put on
    the interior only (the host's jci x ici loops, global bounds 2..jx-2 x 2..iy-2), post_physics,
    bdyval; with ipptls = 2 on the hydrostatic core (the species' qxphy and qxb3d as well)."""
    if nh:
        rc = CONFIGS["N1"]
        data = icbc.generate_nh(rc)
        st = data["state"]
    else:
        rc0, data = c1_data
        rc = dataclasses.replace(rc0, ipptls=2)
        st = {k: v.copy() for k, v in data["state"].items()}
        st.update(icbc.hydrometeor_state(rc, st, nqx=rc.nqx))
    rng = np.random.Generator(np.random.PCG64(17))
    names = PHY_FIELDS + (NH_PHY_FIELDS if nh else QX_PHY_FIELDS)
    s = Script(build_config(rc, data["split"]))
    _start(s, rc, st)
    slices = [n for n in ATMS_FIELDS if not (nh and n in ("ATMS_ZQ", "ATMS_ZA", "ATMS_DZQ"))]
    slices += [] if nh else QX_ATMS_FIELDS
    for _ in range(2):
        s.add(PRE)
        _gets(s, rc, slices)
        for name in names:
            nk = field_levels(name, rc.kz, rc.nsplit)
            x = 1e-7 * np.abs(rng.standard_normal((nk, rc.iy - 3, rc.jx - 3)))
            s.put(name, x, j1=2, i1=2)
        s.add(POST).add(BDYVAL)
    _gets(s, rc, STATE_FIELDS + (NH_STATE_FIELDS if nh else QX_STATE_FIELDS) + names)
    py, fo = s.run_python(), s.run_fortran()
    assert_same(py, fo)


@pytest.mark.gpu
def test_fortran_host_bdyin(c1_data):
    """bdyin after the host's read_icbc: the raw record put into the XxB_B1 fields through the
    shim, b0 / bt formed on the device, then stepped."""
    from tests.test_bdyin_gpu import HBDY, records
    rc, data = c1_data
    rec = records(rc, data, nh=False, n=1)[0]
    s = Script(build_config(rc, data["split"]))
    _start(s, rc, data["state"]).add(STEP, 2)
    for name, a in rec.items():
        s.put(name, a)
    s.add(BDYIN).add(GET_TIME)
    _gets(s, rc, HBDY)
    s.add(STEP, 3)
    _gets(s, rc, STATE_FIELDS)
    py, fo = s.run_python(), s.run_fortran()
    assert_same(py, fo)
    assert py[0][2] == 0.0                      # xbctime restarts at the new interval
