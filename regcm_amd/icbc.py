"""Synthetic initial and lateral-boundary conditions ("syn-icbc v1").

No DOMAIN/ICBC NetCDF data exists offline, so the benchmark and the parity tests run on a
deterministic synthetic atmosphere (NumPy PCG64, seed 20261015).  The fields are stored
exactly the way the reference stores them after ``param``/``init``/``bdyin``:

* map factors inverted and terrain converted to geopotential (Main/mod_params.F90:1982-2001);
* u, v coupled with dot-point p*, t and qv with cross-point p* (``couple``,
  Main/mod_bdycod.F90:784-795, 4938-4951);
* ``bt = (b1 - b0) / dtbdys`` (``timeint``, Main/mod_bdycod.F90:5087-5113);
* atm1 = atm2 = b0, psa = psb = p* (Main/mod_init.F90:92-171);
* dstor/hstor from atm2 as spinit does (Main/mod_split.F90:186-235).

Every array is global, C-order ``[k][i][j]`` (= Fortran ``(j,i,k)``), shape
``(nk, iy, jx)``; cross-point fields leave their last row/column unused.
"""
from __future__ import annotations

import math

import numpy as np

from . import constants as C
from .config import RunConfig
from .vmodes import spinit_constants

SEED = 20261015


def psc2psd_global(pc: np.ndarray) -> np.ndarray:
    """Cross -> dot p* on the whole domain (Main/mpplib/mod_mppparam.F90:13811-13862)."""
    iy, jx = pc.shape
    pd = np.zeros_like(pc)
    pd[1:iy - 1, 1:jx - 1] = (pc[1:iy - 1, 1:jx - 1] + pc[0:iy - 2, 1:jx - 1] +
                              pc[1:iy - 1, 0:jx - 2] + pc[0:iy - 2, 0:jx - 2]) * 0.25
    pd[iy - 1, 1:jx - 1] = (pc[iy - 2, 1:jx - 1] + pc[iy - 2, 0:jx - 2]) * 0.5
    pd[0, 1:jx - 1] = (pc[0, 1:jx - 1] + pc[0, 0:jx - 2]) * 0.5
    pd[1:iy - 1, 0] = (pc[1:iy - 1, 0] + pc[0:iy - 2, 0]) * 0.5
    pd[1:iy - 1, jx - 1] = (pc[1:iy - 1, jx - 2] + pc[0:iy - 2, jx - 2]) * 0.5
    pd[0, 0] = pc[0, 0]
    pd[iy - 1, 0] = pc[iy - 2, 0]
    pd[0, jx - 1] = pc[0, jx - 2]
    pd[iy - 1, jx - 1] = pc[iy - 2, jx - 2]
    return pd


def _qsat(t: np.ndarray, p_pa: np.ndarray) -> np.ndarray:
    es = 611.2 * np.exp(17.67 * (t - 273.15) / (t - 29.65))
    es = np.minimum(es, 0.5 * p_pa)
    return C.ep2 * es / (p_pa - es)


def generate(rc: RunConfig, seed: int = SEED, hmax: float = None) -> dict:
    """Build the full initial state, statics, boundary data and split constants."""
    rng = np.random.Generator(np.random.PCG64(seed))
    jx, iy, kz = rc.jx, rc.iy, rc.kz
    sigma = rc.sigma
    hsig = (sigma[1:] + sigma[:-1]) * 0.5
    ptop = rc.ptop
    hmax = (800.0 if rc.ds < 10.0 else 1500.0) if hmax is None else hmax

    jj, ii = np.meshgrid(np.arange(1, jx + 1, dtype=np.float64),
                         np.arange(1, iy + 1, dtype=np.float64))
    jc, ic = 0.5 * jx, 0.5 * iy
    r2 = (jj - jc) ** 2 + (ii - ic) ** 2
    ht = hmax * np.exp(-r2 / (2.0 * (0.15 * jx) ** 2)) + rng.normal(0.0, 20.0, (iy, jx))
    ht = np.maximum(ht, 0.0)
    mf = 1.0 + 0.02 * ((ii - ic) / iy) ** 2
    lat = np.deg2rad(30.0 + 30.0 * (ii - 1.0) / max(iy - 1.0, 1.0))
    coriol = 2.0 * C.eomeg * np.sin(lat)

    # surface pressure (cb) from the US-standard hypsometric relation, then p* = ps - ptop
    expo = C.egrav / (C.rgas * 0.0065)
    ps = C.stdpcb * (1.0 - 0.0065 * ht / 288.15) ** expo
    pstar = ps - ptop
    pdot = psc2psd_global(pstar)

    p_pa = (hsig[:, None, None] * pstar[None] + ptop) * 1000.0            # (kz, iy, jx)
    t = np.maximum(288.15 * (p_pa / 101325.0) ** (C.rgas * 0.0065 / C.egrav), 216.65)
    t = t + rng.normal(0.0, 0.5, t.shape)
    u = (10.0 + 15.0 * np.sin(math.pi * hsig)[:, None, None] *
         np.cos(math.pi * (ii - ic) / iy)[None]) + rng.normal(0.0, 0.3, (kz, iy, jx))
    v = (2.0 * np.sin(2.0 * math.pi * jj / jx))[None] + rng.normal(0.0, 0.3, (kz, iy, jx))
    qv = 0.7 * _qsat(t, p_pa)

    # time-level 1 of the boundary data
    pstar1 = pstar + 0.1
    pdot1 = psc2psd_global(pstar1)
    t1, u1, v1, qv1 = t + 1.0, u + 1.0, v + 1.0, qv * 1.02
    rdtbdy = 1.0 / rc.dtbdys

    def cross(a):
        out = a.copy()
        out[..., iy - 1, :] = 0.0
        out[..., :, jx - 1] = 0.0
        return out

    ub0, vb0 = u * pdot[None], v * pdot[None]
    tb0, qb0 = cross(t * pstar[None]), cross(qv * pstar[None])
    ub1, vb1 = u1 * pdot1[None], v1 * pdot1[None]
    tb1, qb1 = cross(t1 * pstar1[None]), cross(qv1 * pstar1[None])
    pb0 = cross(pstar)
    pb1 = cross(pstar1)

    st = {}
    st["MSFX"] = (1.0 / mf)[None].copy()
    st["MSFD"] = (1.0 / mf)[None].copy()
    st["CORIOL"] = coriol[None].copy()
    st["HT"] = (ht * C.egrav)[None].copy()
    st["XUB_B0"], st["XUB_BT"] = ub0, (ub1 - ub0) * rdtbdy
    st["XVB_B0"], st["XVB_BT"] = vb0, (vb1 - vb0) * rdtbdy
    st["XTB_B0"], st["XTB_BT"] = tb0, (tb1 - tb0) * rdtbdy
    st["XQB_B0"], st["XQB_BT"] = qb0, (qb1 - qb0) * rdtbdy
    st["XPSB_B0"], st["XPSB_BT"] = pb0[None].copy(), ((pb1 - pb0) * rdtbdy)[None].copy()
    for lvl in ("ATM1", "ATM2"):
        st[f"{lvl}_U"] = ub0.copy()
        st[f"{lvl}_V"] = vb0.copy()
        st[f"{lvl}_T"] = tb0.copy()
        st[f"{lvl}_QV"] = qb0.copy()
        st[f"{lvl}_QC"] = np.zeros((kz, iy, jx))
    st["PSA"] = pb0[None].copy()
    st["PSB"] = pb0[None].copy()

    split = spinit_constants(sigma, ptop, kz, rc.dt, rc.nsplit)
    dstor, hstor = spinit_storage(rc, split, st)
    st["DSTOR"], st["HSTOR"] = dstor, hstor
    return dict(state=st, split=split)


def spinit_storage(rc: RunConfig, split: dict, st: dict):
    """dstor/hstor from atm2 (Main/mod_split.F90:192-235), single global tile."""
    jx, iy, kz, ns = rc.jx, rc.iy, rc.kz, rc.nsplit
    dx = rc.ds * 1000.0
    rdx2 = 1.0 / (2.0 * dx)
    msfx = st["MSFX"][0]
    msfd = st["MSFD"][0]
    mapf = 1.0 / (msfx * msfx)
    uuu = st["ATM2_U"] * msfd[None]
    vvv = st["ATM2_V"] * msfd[None]
    ce = (slice(0, iy - 1), slice(0, jx - 1))
    dstor = np.zeros((ns, iy, jx))
    hstor = np.zeros((ns, iy, jx))
    zmatxr = split["zmatxr"]
    for l in range(ns):
        d = np.zeros((iy - 1, jx - 1))
        for k in range(kz):
            u, v = uuu[k], vvv[k]
            expr = (((((((-u[1:iy, 0:jx - 1] + u[1:iy, 1:jx]) - u[0:iy - 1, 0:jx - 1]) +
                        u[0:iy - 1, 1:jx]) + v[1:iy, 0:jx - 1]) + v[1:iy, 1:jx]) -
                     v[0:iy - 1, 0:jx - 1]) - v[0:iy - 1, 1:jx])
            d = d + ((zmatxr[l, k] * mapf[ce]) * rdx2) * expr
        dstor[l][ce] = d
    psb = st["PSB"][0][ce]
    sigmah, varpa1, tau, pd, ptop = split["sigmah"], split["varpa1"], split["tau"], split["pd"], rc.ptop
    for l in range(ns):
        pdlog = varpa1[l, kz] * math.log(sigmah[kz] * pd + ptop)
        eps1 = varpa1[l, kz] * sigmah[kz] / (sigmah[kz] * pd + ptop)
        h = pdlog + eps1 * (psb - pd)
        for k in range(kz):
            pdlog = varpa1[l, k] * math.log(sigmah[k] * pd + ptop)
            eps1 = varpa1[l, k] * sigmah[k] / (sigmah[k] * pd + ptop)
            eps = eps1 * (psb - pd)
            h = ((h + pdlog) + (tau[l, k] * st["ATM2_T"][k][ce]) / psb) + eps
        hstor[l][ce] = h
    return dstor, hstor
