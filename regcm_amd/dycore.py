"""Host API of the MI355X dynamical-core engine (ctypes over include/rcmdyn.h).

``DynCore`` mirrors the calls the reference driver makes on this path
(Main/mod_regcm_interface.F90:172-228): ``tend()`` for ``call tend``, ``bdyval()`` for
``call bdyval``, ``step(n)`` for n iterations of that loop, and ``put``/``get`` for the module
state that ``mod_atm_interface`` holds.  Errors come back as exceptions carrying the engine's
message (the reference calls ``fatal``; e.g. 'CFL VIOLATION', Main/mod_tendency.F90:702).

The engine library is built in-tree (``regcm_amd/librcmdyn.so``); there is no CPU fallback:
if the library or a GPU is missing, construction fails loudly.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional

import numpy as np

from .config import FIELD, RcmdynConfig, build_config, field_levels

_HERE = os.path.dirname(os.path.abspath(__file__))
# RCMDYN_LIB selects an instrumented build (tools/phases.py); default: the in-tree engine
LIB_PATH = os.environ.get("RCMDYN_LIB") or os.path.join(_HERE, "librcmdyn.so")
_lib = None

EXPORTED = [
    "rcmdyn_create", "rcmdyn_destroy", "rcmdyn_last_error", "rcmdyn_set_nproc",
    "rcmdyn_tile_extent", "rcmdyn_tile_extent_cfg", "rcmdyn_put", "rcmdyn_get", "rcmdyn_set_time", "rcmdyn_get_time",
    "rcmdyn_tend", "rcmdyn_bdyval", "rcmdyn_step", "rcmdyn_synchronize", "rcmdyn_diagnostics",
    "rcmdyn_comm_unique_id", "rcmdyn_last_step_ms", "rcmdyn_set_diagnostics", "rcmdyn_kernel_times",
    "rcmdyn_tend_pre_physics", "rcmdyn_tend_post_physics", "rcmdyn_bdyin", "rcmdyn_reductions", "rcmdyn_runtime_info",
    "rcmdyn_exchange_plan", "rcmdyn_overlap_shares",
]


class EngineError(RuntimeError):
    pass


def lib():
    """Load the in-tree engine library (raises if it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise EngineError(f"engine library missing: {LIB_PATH} (run __graft_entry__.build())")
    L = ctypes.CDLL(LIB_PATH)
    P = ctypes.c_void_p
    i32 = ctypes.c_int32
    dp = ctypes.POINTER(ctypes.c_double)
    L.rcmdyn_create.argtypes = [ctypes.POINTER(RcmdynConfig), ctypes.POINTER(P)]
    L.rcmdyn_destroy.argtypes = [P]
    L.rcmdyn_last_error.argtypes = [P]
    L.rcmdyn_last_error.restype = ctypes.c_char_p
    L.rcmdyn_set_nproc.argtypes = [i32, i32, i32, ctypes.POINTER(i32)]
    L.rcmdyn_tile_extent.argtypes = [i32, i32, i32, i32, i32, ctypes.POINTER(i32), ctypes.POINTER(i32)]
    L.rcmdyn_tile_extent_cfg.argtypes = [ctypes.POINTER(RcmdynConfig), i32, ctypes.POINTER(i32), ctypes.POINTER(i32)]
    L.rcmdyn_put.argtypes = [P, i32, dp, i32, i32, i32, i32, i32, i32]
    L.rcmdyn_get.argtypes = [P, i32, dp, i32, i32, i32, i32, i32, i32]
    L.rcmdyn_set_time.argtypes = [P, ctypes.c_int64, ctypes.c_double, ctypes.c_double]
    L.rcmdyn_get_time.argtypes = [P, ctypes.POINTER(ctypes.c_int64), dp, dp]
    L.rcmdyn_tend.argtypes = [P]
    L.rcmdyn_tend_pre_physics.argtypes = [P]
    L.rcmdyn_tend_post_physics.argtypes = [P]
    L.rcmdyn_bdyin.argtypes = [P]
    L.rcmdyn_bdyval.argtypes = [P]
    L.rcmdyn_step.argtypes = [P, i32]
    L.rcmdyn_synchronize.argtypes = [P]
    L.rcmdyn_diagnostics.argtypes = [P, dp]
    L.rcmdyn_comm_unique_id.argtypes = [ctypes.POINTER(ctypes.c_uint8)]
    L.rcmdyn_last_step_ms.argtypes = [P, dp]
    L.rcmdyn_set_diagnostics.argtypes = [P, i32]
    L.rcmdyn_reductions.argtypes = [P, dp]
    L.rcmdyn_runtime_info.argtypes = [ctypes.c_char_p, i32]
    L.rcmdyn_exchange_plan.argtypes = [ctypes.POINTER(RcmdynConfig), i32, ctypes.POINTER(ctypes.c_int64),
                                       ctypes.c_int64, ctypes.POINTER(ctypes.c_int64)]
    L.rcmdyn_overlap_shares.argtypes = [ctypes.POINTER(RcmdynConfig), ctypes.POINTER(i32), i32]
    L.rcmdyn_kernel_times.argtypes = [P, i32, i32, ctypes.c_char_p, ctypes.POINTER(i32), dp, ctypes.POINTER(i32)]
    _lib = L
    return L


def set_nproc(nproc: int, jx: int, iy: int):
    cp = (ctypes.c_int32 * 2)()
    if lib().rcmdyn_set_nproc(nproc, jx, iy, cp):
        raise EngineError("rcmdyn_set_nproc failed")
    return int(cp[0]), int(cp[1])


def tile_extent(jx: int, iy: int, nproc_j: int, nproc_i: int, tile: int, i_band: int = 0, i_crm: int = 0):
    """Index ranges of one tile, ([jde1, jde2, ide1, ide2, jce1, jce2, ice1, ice2],
    [left, right, bottom, top]).  With i_band / i_crm the j / i direction is periodic
    (rcmdyn_tile_extent_cfg): no boundary side there, and the cross range takes every point."""
    ext = (ctypes.c_int32 * 8)()
    bdy = (ctypes.c_int32 * 4)()
    if i_band or i_crm:
        cfg = RcmdynConfig()
        cfg.jx, cfg.iy, cfg.nproc_j, cfg.nproc_i = jx, iy, nproc_j, nproc_i
        cfg.i_band, cfg.i_crm = i_band, i_crm
        if lib().rcmdyn_tile_extent_cfg(ctypes.byref(cfg), tile, ext, bdy):
            raise EngineError("rcmdyn_tile_extent_cfg failed")
    elif lib().rcmdyn_tile_extent(jx, iy, nproc_j, nproc_i, tile, ext, bdy):
        raise EngineError("rcmdyn_tile_extent failed")
    return list(ext), list(bdy)


PLAN_COLUMNS = ("call", "kind", "chan", "dir", "peer", "count", "sig")


def exchange_plan(rc, split, nproc_j: int, nproc_i: int, rank: int, nsteps: int) -> np.ndarray:
    """Host-only communication plan of one rank (rcmdyn_exchange_plan): an (n, 7) int64 array
    with the columns PLAN_COLUMNS, in issue order.  No GPU is touched."""
    cfg = build_config(rc, split, nproc_j, nproc_i, tile_first=rank, tile_count=1, comm_rank=rank,
                       comm_size=nproc_j * nproc_i)
    n = ctypes.c_int64()
    if lib().rcmdyn_exchange_plan(ctypes.byref(cfg), nsteps, None, 0, ctypes.byref(n)):
        raise EngineError(lib().rcmdyn_last_error(None).decode())
    out = np.zeros((n.value, 7), dtype=np.int64)
    if lib().rcmdyn_exchange_plan(ctypes.byref(cfg), nsteps, out.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)),
                                  n.value, ctypes.byref(n)):
        raise EngineError(lib().rcmdyn_last_error(None).decode())
    return out


def runtime_info() -> str:
    """Paths (and RCCL version) of the HIP runtime and librccl the engine is bound to."""
    buf = ctypes.create_string_buffer(1024)
    if lib().rcmdyn_runtime_info(buf, 1024):
        raise EngineError(lib().rcmdyn_last_error(None).decode())
    return buf.value.decode()


def comm_unique_id() -> bytes:
    buf = (ctypes.c_uint8 * 128)()
    if lib().rcmdyn_comm_unique_id(buf):
        raise EngineError(lib().rcmdyn_last_error(None).decode())
    return bytes(buf)


def overlap_shares(rc, split, nproc_j: int, nproc_i: int):
    """Host-only (rcmdyn_overlap_shares): per rank of an nproc_j x nproc_i job, the points of
    k_columns / k_momentum / k_scalars that run beside the prologue exchange (part 1) and their
    totals, as [(col_p1, col, mom_p1, mom, sca_p1, sca), ...]."""
    n = nproc_j * nproc_i
    out = []
    for r in range(n):
        cfg = build_config(rc, split, nproc_j, nproc_i, tile_first=r, tile_count=1, comm_rank=r, comm_size=n)
        v = (ctypes.c_int32 * 6)()
        if lib().rcmdyn_overlap_shares(ctypes.byref(cfg), v, 1):
            raise EngineError(lib().rcmdyn_last_error(None).decode())
        out.append(tuple(v))
    return out


class DynCore:
    """The dynamical core of one process: one or more tiles on one GPU."""

    def __init__(self, rc, split, nproc_j: int = 1, nproc_i: int = 1, tile_first: int = 0,
                 tile_count: Optional[int] = None, comm_rank: int = 0, comm_size: int = 1,
                 device: int = -1, unique_id: Optional[bytes] = None):
        self.rc = rc
        self.cfg = build_config(rc, split, nproc_j, nproc_i, tile_first, tile_count,
                                comm_rank, comm_size, device, unique_id)
        self.h = ctypes.c_void_p()
        if lib().rcmdyn_create(ctypes.byref(self.cfg), ctypes.byref(self.h)):
            raise EngineError(lib().rcmdyn_last_error(None).decode())

    def _check(self, rc):
        if rc:
            raise EngineError(lib().rcmdyn_last_error(self.h).decode())

    def close(self):
        """rcmdyn_destroy: a lazy tend still pending is launched first; its failure raises."""
        if self.h:
            rc = lib().rcmdyn_destroy(self.h)
            self.h = ctypes.c_void_p()
            if rc:
                raise EngineError(lib().rcmdyn_last_error(None).decode())

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def put(self, name: str, arr: np.ndarray, j1: int = 1, i1: int = 1, k1: int = 1):
        a = np.ascontiguousarray(arr, dtype=np.float64)
        nk, ni, nj = a.shape
        self._check(lib().rcmdyn_put(self.h, FIELD[name], a.ctypes.data_as(ctypes.POINTER(ctypes.c_double)),
                                     j1, j1 + nj - 1, i1, i1 + ni - 1, k1, k1 + nk - 1))

    def get(self, name: str) -> np.ndarray:
        nk = field_levels(name, self.rc.kz, self.rc.nsplit)
        out = np.zeros((nk, self.rc.iy, self.rc.jx))
        self._check(lib().rcmdyn_get(self.h, FIELD[name], out.ctypes.data_as(ctypes.POINTER(ctypes.c_double)),
                                     1, self.rc.jx, 1, self.rc.iy, 1, nk))
        return out

    def put_state(self, st: dict):
        for name, arr in st.items():
            self.put(name, arr)

    def set_time(self, lcount: int, dt: float, xbctime: float):
        self._check(lib().rcmdyn_set_time(self.h, lcount, dt, xbctime))

    def get_time(self):
        a, b, c = ctypes.c_int64(), ctypes.c_double(), ctypes.c_double()
        self._check(lib().rcmdyn_get_time(self.h, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c)))
        return a.value, b.value, c.value

    def tend(self):
        self._check(lib().rcmdyn_tend(self.h))

    def tend_pre_physics(self):
        """surface_pressures .. mkslice .. new_pressure: the ATMS_* fields become readable."""
        self._check(lib().rcmdyn_tend_pre_physics(self.h))

    def tend_post_physics(self):
        """The rest of tend, with the *PHY tendencies put since (physics coupling seam)."""
        self._check(lib().rcmdyn_tend_post_physics(self.h))

    def bdyval(self):
        self._check(lib().rcmdyn_bdyval(self.h))

    def bdyin(self):
        """bdyin from read_icbc on: the record put into the XxB_B1 fields becomes b1."""
        self._check(lib().rcmdyn_bdyin(self.h))

    def step(self, n: int = 1):
        self._check(lib().rcmdyn_step(self.h, n))

    def synchronize(self):
        self._check(lib().rcmdyn_synchronize(self.h))

    def diagnostics(self):
        out = (ctypes.c_double * 4)()
        self._check(lib().rcmdyn_diagnostics(self.h, out))
        return list(out)

    def reductions(self):
        """(ptntot, pt2tot, cflmax) of the last step over the whole job (the 3-hourly report,
        Main/mod_tendency.F90:705-725, Main/mod_sound.F90:634-646); collective over ranks."""
        out = (ctypes.c_double * 3)()
        self._check(lib().rcmdyn_reductions(self.h, out))
        return tuple(out)

    def last_step_ms(self) -> float:
        v = ctypes.c_double()
        self._check(lib().rcmdyn_last_step_ms(self.h, ctypes.byref(v)))
        return v.value

    def set_diagnostics(self, on: bool = True):
        self._check(lib().rcmdyn_set_diagnostics(self.h, 1 if on else 0))

    def kernel_times(self, nsteps: int, cap: int = 64) -> dict:
        """{kernel name: (launches, average ms per launch)} over nsteps eager steps."""
        names = ctypes.create_string_buffer(cap * 48)
        launches = (ctypes.c_int32 * cap)()
        avg = (ctypes.c_double * cap)()
        n = ctypes.c_int32()
        self._check(lib().rcmdyn_kernel_times(self.h, nsteps, cap, names, launches, avg, ctypes.byref(n)))
        raw = names.raw
        out = {}
        for q in range(n.value):
            nm = raw[q * 48:(q + 1) * 48].split(b"\0", 1)[0].decode()
            out[nm] = (int(launches[q]), float(avg[q]))
        return out
