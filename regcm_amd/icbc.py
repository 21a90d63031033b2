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


def psc2psd_band(pc: np.ndarray) -> np.ndarray:
    """psc2psd of a band (i_band = 1): periodic in j, so every column takes the interior form and
    the bottom/top rows the two-point means; no west/east lines or corners
    (Main/mpplib/mod_mppparam.F90:13811-13862 with has_bdyleft = has_bdyright = .false.)."""
    iy, jx = pc.shape
    pm = np.roll(pc, 1, axis=1)                          # pc(j-1), periodic
    pd = np.zeros_like(pc)
    pd[1:iy - 1] = (pc[1:iy - 1] + pc[0:iy - 2] + pm[1:iy - 1] + pm[0:iy - 2]) * 0.25
    pd[iy - 1] = (pc[iy - 2] + pm[iy - 2]) * 0.5
    pd[0] = (pc[0] + pm[0]) * 0.5
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
    band = getattr(rc, "i_band", 0) == 1
    p2d = psc2psd_band if band else psc2psd_global
    pdot = p2d(pstar)

    p_pa = (hsig[:, None, None] * pstar[None] + ptop) * 1000.0            # (kz, iy, jx)
    t = np.maximum(288.15 * (p_pa / 101325.0) ** (C.rgas * 0.0065 / C.egrav), 216.65)
    t = t + rng.normal(0.0, 0.5, t.shape)
    u = (10.0 + 15.0 * np.sin(math.pi * hsig)[:, None, None] *
         np.cos(math.pi * (ii - ic) / iy)[None]) + rng.normal(0.0, 0.3, (kz, iy, jx))
    v = (2.0 * np.sin(2.0 * math.pi * jj / jx))[None] + rng.normal(0.0, 0.3, (kz, iy, jx))
    qv = 0.7 * _qsat(t, p_pa)

    # time-level 1 of the boundary data
    pstar1 = pstar + 0.1
    pdot1 = p2d(pstar1)
    t1, u1, v1, qv1 = t + 1.0, u + 1.0, v + 1.0, qv * 1.02
    rdtbdy = 1.0 / rc.dtbdys

    def cross(a):
        out = a.copy()
        out[..., iy - 1, :] = 0.0
        if not band:                     # a band's cross grid takes every j
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


def hydrometeor_state(rc: RunConfig, st: dict, seed: int = SEED + 5, nqx: int = 5) -> dict:
    """Hydrometeors for the moisture-species tests, coupled with p* like the reference stores
    them: cloud water in the lower and middle troposphere, ice aloft, rain near the surface,
    snow in between (peaks 0.2, 0.05, 0.1, 0.08 g/kg), each times a patchy 0/1 mask so that the
    advection of the cloud edges produces negative forecasts (the negative-moisture fix); atm2
    a few per cent off atm1.  nqx = 2 gives qc only; nqx = 5 also qi, qr, qs."""
    rng = np.random.Generator(np.random.PCG64(seed))
    kz, iy, jx = rc.kz, rc.iy, rc.jx
    hsig = (rc.sigma[1:] + rc.sigma[:-1]) * 0.5
    ps = st["PSA"][0]
    prof = {"QC": (2.0e-4, 0.75, 0.15), "QI": (5.0e-5, 0.30, 0.10), "QR": (1.0e-4, 0.92, 0.08),
            "QS": (8.0e-5, 0.55, 0.12)}
    names = ["QC"] if nqx == 2 else ["QC", "QI", "QR", "QS"]
    out = {}
    for nm in names:
        peak, s0, w = prof[nm]
        layer = peak * np.exp(-0.5 * ((hsig - s0) / w) ** 2)
        mask = (rng.uniform(size=(kz, iy, jx)) < 0.6).astype(np.float64)
        q = layer[:, None, None] * mask * rng.uniform(0.5, 1.5, size=(kz, iy, jx))
        q[:, iy - 1, :] = 0.0
        if getattr(rc, "i_band", 0) != 1:       # a band's cross grid takes every j
            q[:, :, jx - 1] = 0.0
        out[f"ATM1_{nm}"] = q * ps[None]
        out[f"ATM2_{nm}"] = q * ps[None] * rng.uniform(0.95, 1.0, size=(kz, iy, jx))
    return out


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
    band = getattr(rc, "i_band", 0) == 1
    if band:
        # periodic in j: the cross grid takes every j, and u, v at j+1 of the last column wrap
        return _spinit_storage_band(rc, split, st, uuu, vvv, mapf, rdx2)
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


def _spinit_storage_band(rc, split, st, uuu, vvv, mapf, rdx2):
    jx, iy, kz, ns = rc.jx, rc.iy, rc.kz, rc.nsplit
    ce = (slice(0, iy - 1), slice(0, jx))
    dstor = np.zeros((ns, iy, jx))
    hstor = np.zeros((ns, iy, jx))
    zmatxr = split["zmatxr"]
    for l in range(ns):
        d = np.zeros((iy - 1, jx))
        for k in range(kz):
            u, v = uuu[k], vvv[k]
            up, vp = np.roll(u, -1, axis=1), np.roll(v, -1, axis=1)     # (j+1), periodic
            expr = (((((((-u[1:iy] + up[1:iy]) - u[0:iy - 1]) + up[0:iy - 1]) + v[1:iy]) + vp[1:iy]) -
                     v[0:iy - 1]) - vp[0:iy - 1])
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


def nhpp(sigma: np.ndarray, t: np.ndarray, tv: np.ndarray, pr0: np.ndarray, t0: np.ndarray,
         ps_cb: np.ndarray, ps0_pa: np.ndarray, ptop: float) -> np.ndarray:
    """Pressure perturbation in hydrostatic balance with t and the p* ps_cb, integrated up from
    the surface (Share/mod_nhinterp.F90:284-350).  Inputs (kz, ...) on cross points; Pa."""
    kz = t.shape[0]
    pp = np.empty_like(t)
    p0surf = ps0_pa + ptop * 1000.0
    psp = ps_cb * 1000.0 - ps0_pa
    k = kz - 1
    delp0 = p0surf - pr0[k]
    tvpot = (tv[k] - t0[k]) / t[k]
    pp[k] = (tvpot * delp0 + psp) / (1.0 + delp0 / pr0[k])
    for k in range(kz - 2, -1, -1):           # Fortran k = kz-1 .. 1
        wtl = (sigma[k + 1] - sigma[k]) / (sigma[k + 2] - sigma[k])
        wtu = 1.0 - wtl
        aa = C.egrav / (pr0[k + 1] - pr0[k])
        bb = C.egrav * wtl / pr0[k + 1] * t0[k + 1] / t[k + 1]
        cc = C.egrav * wtu / pr0[k] * t0[k] / t[k]
        tvpot = wtl * ((tv[k + 1] - t0[k + 1]) / t[k + 1]) + wtu * ((tv[k] - t0[k]) / t[k])
        pp[k] = (C.egrav * tvpot + pp[k + 1] * (aa - bb)) / (aa + cc)
    return pp


def generate_nh(rc: RunConfig, seed: int = SEED, hmax: float = None, w_noise: float = 0.02,
                rest: bool = False) -> dict:
    """Synthetic non-hydrostatic ICBC ("syn-icbc v1", NH variant).

    The reference state comes from the terrain (regcm_amd/nhbase.py); p* is the constant
    reference p* (``sfs%psa = atm0%ps * 1e-3``, Main/mod_init.F90:144-151); t, qv, u, v are
    the hydrostatic synthetic profiles on the NH half levels; the pressure perturbation
    balances them hydrostatically against the US-standard surface pressure (``nhpp``); w is
    zero on the boundary and small seeded noise inside (so every w term is exercised from
    the first step).  Boundary time level 1 adds (1 K, 1 m/s, +2 % qv) as in the hydrostatic
    generator, with its own balanced pp.

    ``rest=True`` builds the resting reference atmosphere instead (flat terrain, t = t0,
    qv = 0, u = v = pp = w = 0, constant boundaries): the balance test of the NH core.
    """
    from . import nhbase
    rng = np.random.Generator(np.random.PCG64(seed + 2))
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
    if rest:
        ht = np.zeros((iy, jx))
    mf = 1.0 + 0.02 * ((ii - ic) / iy) ** 2
    dlat = 30.0 + 30.0 * (ii - 1.0) / max(iy - 1.0, 1.0)
    xlat = 30.0 + 30.0 * (ii - 0.5) / max(iy - 1.0, 1.0)
    xlon = 10.0 + 20.0 * (jj - 0.5) / max(jx - 1.0, 1.0)
    coriol = 2.0 * C.eomeg * np.sin(np.deg2rad(dlat))
    msfx = 1.0 / mf
    msfd = 1.0 / mf
    ht_geo = ht * C.egrav
    ref = nhbase.reference_state(rc, ht_geo, msfx, msfd, xlat, xlon, dlat)
    F = ref["fields"]
    ce = (slice(0, iy - 1), slice(0, jx - 1))
    ps0 = F["ATM0_PS"][0][ce]                         # Pa
    pr0 = F["ATM0_PR"][:, 0:iy - 1, 0:jx - 1]
    t0 = F["ATM0_T"][:, 0:iy - 1, 0:jx - 1]
    pstar = np.zeros((iy, jx))
    pstar[ce] = ps0 * 1.0e-3                          # Main/mod_init.F90:146
    pdot = psc2psd_global(pstar)
    expo = C.egrav / (C.rgas * 0.0065)
    ps_h = (C.stdpcb * (1.0 - 0.0065 * ht / 288.15) ** expo - ptop)[ce]

    t = np.maximum(288.15 * (pr0 / 101325.0) ** (C.rgas * 0.0065 / C.egrav), 216.65)
    t = t + rng.normal(0.0, 0.5, t.shape)
    qv = 0.7 * _qsat(t, pr0)
    pp = nhpp(sigma, t, t * (1.0 + C.ep1 * qv), pr0, t0, ps_h, ps0, ptop)
    t1, qv1 = t + 1.0, qv * 1.02
    pp1 = nhpp(sigma, t1, t1 * (1.0 + C.ep1 * qv1), pr0, t0, ps_h, ps0, ptop)
    u = (10.0 + 15.0 * np.sin(math.pi * hsig)[:, None, None] *
         np.cos(math.pi * (ii - ic) / iy)[None]) + rng.normal(0.0, 0.3, (kz, iy, jx))
    v = (2.0 * np.sin(2.0 * math.pi * jj / jx))[None] + rng.normal(0.0, 0.3, (kz, iy, jx))
    u1, v1 = u + 1.0, v + 1.0
    w = np.zeros((kz + 1, iy, jx))
    w[1:kz, 1:iy - 2, 1:jx - 2] = rng.normal(0.0, w_noise, (kz - 1, iy - 3, jx - 3))
    if rest:
        t, t1 = t0.copy(), t0.copy()
        qv, qv1 = np.zeros_like(t0), np.zeros_like(t0)
        pp, pp1 = np.zeros_like(t0), np.zeros_like(t0)
        u = np.zeros((kz, iy, jx)); v = np.zeros((kz, iy, jx))
        u1, v1 = u, v
        w[:] = 0.0
    rdtbdy = 1.0 / rc.dtbdys

    def cross3(a):
        out = np.zeros((a.shape[0], iy, jx))
        out[:, 0:iy - 1, 0:jx - 1] = a
        return out

    ps3 = pstar[None]
    tb0, tb1 = cross3(t) * ps3, cross3(t1) * ps3
    qb0, qb1 = cross3(qv) * ps3, cross3(qv1) * ps3
    ppb0, ppb1 = cross3(pp) * ps3, cross3(pp1) * ps3
    ub0, ub1 = u * pdot[None], u1 * pdot[None]
    vb0, vb1 = v * pdot[None], v1 * pdot[None]
    st = dict(F)
    st["MSFX"], st["MSFD"] = msfx[None].copy(), msfd[None].copy()
    st["CORIOL"], st["HT"] = coriol[None].copy(), ht_geo[None].copy()
    st["XUB_B0"], st["XUB_BT"] = ub0, (ub1 - ub0) * rdtbdy
    st["XVB_B0"], st["XVB_BT"] = vb0, (vb1 - vb0) * rdtbdy
    st["XTB_B0"], st["XTB_BT"] = tb0, (tb1 - tb0) * rdtbdy
    st["XQB_B0"], st["XQB_BT"] = qb0, (qb1 - qb0) * rdtbdy
    st["XPPB_B0"], st["XPPB_BT"] = ppb0, (ppb1 - ppb0) * rdtbdy
    st["XWWB_B0"], st["XWWB_BT"] = np.zeros((kz + 1, iy, jx)), np.zeros((kz + 1, iy, jx))
    st["XPSB_B0"], st["XPSB_BT"] = pstar[None].copy(), np.zeros((1, iy, jx))
    for lvl in ("ATM1", "ATM2"):
        st[f"{lvl}_U"], st[f"{lvl}_V"] = ub0.copy(), vb0.copy()
        st[f"{lvl}_T"], st[f"{lvl}_QV"] = tb0.copy(), qb0.copy()
        st[f"{lvl}_QC"] = np.zeros((kz, iy, jx))
        st[f"{lvl}_PP"] = ppb0.copy()
        st[f"{lvl}_W"] = w * ps3
    st["PSA"], st["PSB"] = pstar[None].copy(), pstar[None].copy()
    split = spinit_constants(sigma, ptop, kz, rc.dt, rc.nsplit)
    split["nh_dtsmax"] = ref["nh_dtsmax"]
    split["nh_xmsf"] = ref["nh_xmsf"]
    st["DSTOR"] = np.zeros((rc.nsplit, iy, jx))
    st["HSTOR"] = np.zeros((rc.nsplit, iy, jx))
    return dict(state=st, split=split)


def generate_crm(rc: RunConfig, seed: int = SEED) -> dict:
    """Synthetic doubly periodic state of a cloud-resolving run (i_crm = 1 over a band,
    PreProc/CRM/crm_test.in: TOGA-COARE at clat = 0, NORMER projection, ocean).  With
    i_crm = 0 the same fields serve a non-hydrostatic band (periodic in j, relaxing to the
    initial state at its south and north rows).

    Every field is defined on the whole periodic grid: with i_band and i_crm the cross grid
    takes every j and every i (Main/mpplib/mod_mppparam.F90:1340-1360), so no row or column is
    left unset.  Flat terrain and unit map factors make the reference state and the statics
    horizontally uniform (nhbase, Share/mod_nhinterp.F90:74-106, on the whole grid; dpsdxm,
    dpsdym, dprddx, dprddy = 0; f = 0 and the full-Coriolis terms of latitude 0); the
    temperature carries crm_test.in's 0.1 % perturbation (lperturb_t, perturb_frac_t) on a
    standard-atmosphere profile, qv 70 % of saturation, periodic winds u = 5 + 3 sin(2 pi i/iy),
    v = 2 sin(2 pi j/jx) m/s with noise, pp in hydrostatic balance (nhpp), small noise in w and
    a boundary-layer TKE (ibltyp = 2).  The boundary data equal the initial state (the CRM's
    Rayleigh damping relaxes u, v, pp, w toward 0 and damps no t or qv: nothing reads them).
    init_sound's scalars follow Main/mod_sound.F90:120, 143-153 with nicross = iy, njcross = jx."""
    from . import nhbase
    rng = np.random.Generator(np.random.PCG64(seed + 7))
    jx, iy, kz = rc.jx, rc.iy, rc.kz
    sigma = np.asarray(rc.sigma)
    hsig = (sigma[1:] + sigma[:-1]) * 0.5
    ptop = rc.ptop
    dx = rc.ds * 1000.0
    jj, ii = np.meshgrid(np.arange(1, jx + 1, dtype=np.float64), np.arange(1, iy + 1, dtype=np.float64))
    ter = np.zeros((iy, jx))
    args = (ptop, rc.base_state_pressure, rc.logp_lrate, rc.base_state_ts0)
    ps0, pr0, t0, rho0, z0 = nhbase.nhbase(ter, hsig, *args)
    _, pf0, _, rhof0, zf0 = nhbase.nhbase(ter, sigma, *args)
    st = {"ATM0_PS": ps0[None].copy(), "ATM0_PR": pr0, "ATM0_T": t0, "ATM0_RHO": rho0, "ATM0_Z": z0,
          "ATM0_PF": pf0, "ATM0_RHOF": rhof0, "ATM0_ZF": zf0}
    zero2 = np.zeros((1, iy, jx))
    for n in ("DPSDXM", "DPSDYM", "DMDX", "DMDY", "DDY", "CRY", "CORIOL", "HT"):
        st[n] = zero2.copy()
    st["DPRDDX"], st["DPRDDY"] = np.zeros((kz, iy, jx)), np.zeros((kz, iy, jx))
    st["EF"], st["EX"] = np.full((1, iy, jx), nhbase.EOMEG2), np.full((1, iy, jx), nhbase.EOMEG2)
    st["DDX"], st["CRX"] = np.ones((1, iy, jx)), np.ones((1, iy, jx))
    st["MSFX"], st["MSFD"] = np.ones((1, iy, jx)), np.ones((1, iy, jx))
    pstar = ps0 * 1.0e-3                                     # Main/mod_init.F90:146
    t = np.maximum(288.15 * (pr0 / 101325.0) ** (C.rgas * 0.0065 / C.egrav), 216.65)
    t = t * (1.0 + 0.001 * rng.uniform(-1.0, 1.0, t.shape))
    qv = 0.7 * _qsat(t, pr0)
    pp = nhpp(sigma, t, t * (1.0 + C.ep1 * qv), pr0, t0, pstar, ps0, ptop)
    u = (5.0 + 3.0 * np.sin(2.0 * math.pi * ii / iy))[None] + rng.normal(0.0, 0.3, (kz, iy, jx))
    v = (2.0 * np.sin(2.0 * math.pi * jj / jx))[None] + rng.normal(0.0, 0.3, (kz, iy, jx))
    w = np.zeros((kz + 1, iy, jx))
    w[1:kz] = rng.normal(0.0, 0.02, (kz - 1, iy, jx))
    ps3 = pstar[None]
    st["PSA"], st["PSB"] = ps3.copy(), ps3.copy()
    for lvl in ("ATM1", "ATM2"):
        st[f"{lvl}_U"], st[f"{lvl}_V"] = u * ps3, v * ps3           # psdot = p* (uniform)
        st[f"{lvl}_T"], st[f"{lvl}_QV"] = t * ps3, qv * ps3
        st[f"{lvl}_QC"] = np.zeros((kz, iy, jx))
        st[f"{lvl}_PP"] = pp * ps3
        st[f"{lvl}_W"] = w * ps3
    sig = sigma[:, None, None]
    prof = 1.5 * np.exp(-(1.0 - sig) / 0.08)
    for n, name in enumerate(("ATM1_TKE", "ATM2_TKE")):
        st[name] = np.maximum(prof * (1.0 + 0.3 * rng.standard_normal((kz + 1, iy, jx))) + 0.02 * n, rc.tkemin)
    for b, a in (("XUB", "ATM1_U"), ("XVB", "ATM1_V"), ("XTB", "ATM1_T"), ("XQB", "ATM1_QV"),
                 ("XPPB", "ATM1_PP"), ("XWWB", "ATM1_W")):
        st[f"{b}_B0"], st[f"{b}_BT"] = st[a].copy(), np.zeros_like(st[a])
    st["XPSB_B0"], st["XPSB_BT"] = ps3.copy(), np.zeros((1, iy, jx))
    split = spinit_constants(rc.sigma, ptop, kz, rc.dt, rc.nsplit)
    # init_sound: xmsf = sum(msfx(jci1:jci2,ici1:ici2)) * rnpts, rnpts = 1/((nicross-2)*(njcross-2))
    # (:120, 143-145); the global jci / ici take every point of a periodic direction
    njc, nic = (jx if rc.i_band else jx - 1), (iy if rc.i_crm else iy - 1)
    j1, j2 = (1, jx) if rc.i_band else (2, jx - 2)
    i1, i2 = (1, iy) if rc.i_crm else (2, iy - 2)
    rnpts = 1.0 / float((nic - 2) * (njc - 2))
    split["nh_xmsf"] = float(np.sum(st["MSFX"][0][i1 - 1:i2, j1 - 1:j2])) * rnpts
    cs = math.sqrt(nhbase.XGAMMA * C.rgas * float(np.max(t0)))
    split["nh_dtsmax"] = dx / cs / (1.0 + rc.nhxkd)
    st["DSTOR"] = np.zeros((rc.nsplit, iy, jx))
    st["HSTOR"] = np.zeros((rc.nsplit, iy, jx))
    return dict(state=st, split=split)


def tke_state(rc: RunConfig, seed: int = SEED) -> dict:
    """Synthetic UW-PBL turbulent kinetic energy (ibltyp = 2): atm1/atm2 tke on the kz+1 full
    sigma levels (decoupled, m2/s2), a boundary-layer profile of up to ~1.5 m2/s2 decaying
    above sigma ~0.8, with cell-to-cell noise, floored at tkemin; zero on the dot row/column
    jx, iy like every cross-point field."""
    rng = np.random.Generator(np.random.PCG64(seed + 17))
    jx, iy, kz = rc.jx, rc.iy, rc.kz
    sig = np.asarray(rc.sigma, dtype=np.float64)[:, None, None]          # k = 1 (top) .. kz+1
    prof = 1.5 * np.exp(-(1.0 - sig) / 0.08)
    out = {}
    for n, name in enumerate(("ATM1_TKE", "ATM2_TKE")):
        t = prof * (1.0 + 0.3 * rng.standard_normal((kz + 1, iy, jx))) + 0.02 * n
        t = np.maximum(t, rc.tkemin)
        t[:, iy - 1, :] = 0.0
        if getattr(rc, "i_band", 0) != 1:
            t[:, :, jx - 1] = 0.0
        out[name] = t
    return out
