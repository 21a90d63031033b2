"""TEST INFRASTRUCTURE ONLY -- ctypes wrapper of the CPU restatement (librcm_oracle.so).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module.
It exposes the same host API as ``regcm_amd.dycore.DynCore`` (tend / bdyval / step / put /
get) so parity tests read like the reference's own driver (Main/mod_regcm_interface.F90:172-228).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

from regcm_amd.config import (FIELD, RcmdynConfig, build_config, field_levels)

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = os.path.join(_HERE, "librcm_oracle.so")
_lib = None

EXCH_FN = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.POINTER(ctypes.c_double),
                           ctypes.c_int, ctypes.c_int, ctypes.c_int)
EXCHB_FN = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.POINTER(ctypes.c_double),
                            ctypes.c_int, ctypes.c_int)


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB):
            build()
        L = ctypes.CDLL(_LIB)
        P = ctypes.c_void_p
        dp = ctypes.POINTER(ctypes.c_double)
        i = ctypes.c_int
        L.orc_create.restype = P
        L.orc_create.argtypes = [ctypes.POINTER(RcmdynConfig)]
        L.orc_destroy.argtypes = [P]
        L.orc_set_exchange.argtypes = [P, EXCH_FN, EXCHB_FN, P]
        L.orc_frame_info.argtypes = [P, ctypes.POINTER(ctypes.c_int)]
        L.orc_put.argtypes = [P, i, dp, i, i, i, i, i, i]
        L.orc_get.argtypes = [P, i, dp, i, i, i, i, i, i]
        L.orc_set_sound_probe.argtypes = [P, i]
        L.orc_set_tend_probe.argtypes = [P, i]
        L.orc_get_work.restype = i
        L.orc_get_work.argtypes = [P, ctypes.c_char_p, dp, ctypes.c_size_t]
        L.orc_set_time.argtypes = [P, ctypes.c_longlong, ctypes.c_double, ctypes.c_double]
        L.orc_get_time.argtypes = [P, ctypes.POINTER(ctypes.c_longlong),
                                   ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double)]
        L.orc_tend.restype = i
        L.orc_tend.argtypes = [P]
        L.orc_bdyval.argtypes = [P]
        L.orc_bdyin.argtypes = [P]
        L.orc_step.restype = i
        L.orc_step.argtypes = [P, i]
        L.orc_diagnostics.argtypes = [P, dp]
        L.orc_par_create.restype = P
        L.orc_par_create.argtypes = [ctypes.POINTER(RcmdynConfig)]
        L.orc_par_destroy.argtypes = [P]
        L.orc_par_put.argtypes = [P, i, dp, i, i, i, i, i, i]
        L.orc_par_get.argtypes = [P, i, dp, i, i, i, i, i, i]
        L.orc_par_set_time.argtypes = [P, ctypes.c_longlong, ctypes.c_double, ctypes.c_double]
        L.orc_par_get_time.argtypes = [P, ctypes.POINTER(ctypes.c_longlong),
                                       ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double)]
        L.orc_par_bdyval.restype = i
        L.orc_par_bdyval.argtypes = [P]
        L.orc_par_step.restype = i
        L.orc_par_step.argtypes = [P, i]
        _lib = L
    return _lib


class OracleCore:
    """One tile of the CPU restatement.  ``tile`` indexes the set_nproc decomposition."""

    def __init__(self, rc, split, nproc_j=1, nproc_i=1, tile=0):
        self.rc = rc
        self.cfg = build_config(rc, split, nproc_j, nproc_i, tile_first=tile, tile_count=1)
        self.h = lib().orc_create(ctypes.byref(self.cfg))
        if not self.h:
            raise RuntimeError("orc_create failed")
        info = (ctypes.c_int * 16)()
        lib().orc_frame_info(self.h, info)
        self.info = list(info)
        self._cb = None

    def close(self):
        if self.h:
            lib().orc_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_exchange(self, fn, bfn):
        self._cb = (EXCH_FN(fn), EXCHB_FN(bfn))
        lib().orc_set_exchange(self.h, self._cb[0], self._cb[1], None)

    def put(self, name, arr):
        a = np.ascontiguousarray(arr, dtype=np.float64)
        nk, ni, nj = a.shape
        rc = lib().orc_put(self.h, FIELD[name], a.ctypes.data_as(ctypes.POINTER(ctypes.c_double)),
                           1, nj, 1, ni, 1, nk)
        if rc:
            raise KeyError(name)

    def get(self, name):
        nk = field_levels(name, self.rc.kz, self.rc.nsplit)
        out = np.zeros((nk, self.rc.iy, self.rc.jx))
        rc = lib().orc_get(self.h, FIELD[name], out.ctypes.data_as(ctypes.POINTER(ctypes.c_double)),
                           1, self.rc.jx, 1, self.rc.iy, 1, nk)
        if rc:
            raise KeyError(name)
        return out

    def put_state(self, st):
        for name, arr in st.items():
            self.put(name, arr)

    def set_sound_probe(self, nsub):
        lib().orc_set_sound_probe(self.h, nsub)

    def set_tend_probe(self, stage):
        lib().orc_set_tend_probe(self.h, stage)

    def get_work(self, name):
        """An internal work array (orc_get_work) on the global (iy, jx) grid of a one-tile
        oracle: [k][i][j], global 1-based (j, i) at [.., i-1, j-1]."""
        info = (ctypes.c_int * 16)()
        lib().orc_frame_info(self.h, info)
        j0, i0, nj, ni = info[0], info[1], info[2], info[3]
        buf = np.zeros((self.rc.kz + 1) * ni * nj)
        nk = lib().orc_get_work(self.h, name.encode(), buf.ctypes.data_as(ctypes.POINTER(ctypes.c_double)),
                                buf.size)
        if not nk:
            raise KeyError(name)
        fr = buf[: nk * ni * nj].reshape(nk, ni, nj)
        return fr[:, 1 - i0: 1 - i0 + self.rc.iy, 1 - j0: 1 - j0 + self.rc.jx].copy()

    def set_time(self, lcount, dt, xbctime):
        lib().orc_set_time(self.h, lcount, dt, xbctime)

    def get_time(self):
        a, b, c = ctypes.c_longlong(), ctypes.c_double(), ctypes.c_double()
        lib().orc_get_time(self.h, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c))
        return a.value, b.value, c.value

    def tend(self):
        if lib().orc_tend(self.h):
            raise FloatingPointError("CFL VIOLATION")

    def bdyval(self):
        lib().orc_bdyval(self.h)

    def bdyin(self):
        lib().orc_bdyin(self.h)

    def step(self, n=1):
        if lib().orc_step(self.h, n):
            raise FloatingPointError("CFL VIOLATION")

    def diagnostics(self):
        out = (ctypes.c_double * 4)()
        lib().orc_diagnostics(self.h, out)
        return list(out)


class OracleParallel:
    """The hydrostatic restatement as set_nproc tiles on OpenMP threads (oracle/orc_par.c):
    the reference's MPI decomposition on host cores, bit-identical to one tile.  Same host
    API as OracleCore for put/get/bdyval/step/set_time/get_time."""

    def __init__(self, rc, split, nthreads=1, dims=None):
        from regcm_amd.config import set_nproc
        cj, ci = dims if dims is not None else set_nproc(int(nthreads), rc.jx, rc.iy)
        self.rc = rc
        self.nthreads = cj * ci
        self.cfg = build_config(rc, split, cj, ci, tile_first=0, tile_count=1)
        self.h = lib().orc_par_create(ctypes.byref(self.cfg))
        if not self.h:
            raise RuntimeError("orc_par_create failed")

    def close(self):
        if self.h:
            lib().orc_par_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def put(self, name, arr):
        a = np.ascontiguousarray(arr, dtype=np.float64)
        nk, ni, nj = a.shape
        if lib().orc_par_put(self.h, FIELD[name], a.ctypes.data_as(ctypes.POINTER(ctypes.c_double)),
                             1, nj, 1, ni, 1, nk):
            raise KeyError(name)

    def get(self, name):
        nk = field_levels(name, self.rc.kz, self.rc.nsplit)
        out = np.zeros((nk, self.rc.iy, self.rc.jx))
        if lib().orc_par_get(self.h, FIELD[name], out.ctypes.data_as(ctypes.POINTER(ctypes.c_double)),
                             1, self.rc.jx, 1, self.rc.iy, 1, nk):
            raise KeyError(name)
        return out

    def put_state(self, st):
        for name, arr in st.items():
            self.put(name, arr)

    def set_time(self, lcount, dt, xbctime):
        lib().orc_par_set_time(self.h, lcount, dt, xbctime)

    def get_time(self):
        a, b, c = ctypes.c_longlong(), ctypes.c_double(), ctypes.c_double()
        lib().orc_par_get_time(self.h, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c))
        return a.value, b.value, c.value

    def bdyval(self):
        if lib().orc_par_bdyval(self.h):
            raise RuntimeError("orc_par_bdyval: could not get one OpenMP thread per tile")

    def step(self, n=1):
        rc = lib().orc_par_step(self.h, n)
        if rc < 0:
            raise RuntimeError("orc_par_step: could not get one OpenMP thread per tile")
        if rc:
            raise FloatingPointError("CFL VIOLATION")
