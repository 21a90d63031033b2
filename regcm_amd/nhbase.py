"""Non-hydrostatic reference state and statics (host-side setup, run once).

The reference computes these in ``param`` before the first step and the dyn core only reads
them; across the C-ABI they are inputs (``RCMDYN_ATM0_*``, ``DPSDXM`` ... ``CRY``).  This
module restates, on the whole domain as one tile:

* ``nhbase`` (Share/mod_nhinterp.F90:74-106) for the half (``hsigma``) and full (``sigma``)
  levels, called from ``make_reference_atmosphere`` (Main/mod_params.F90:2614-2694) with
  terrain in metres;
* ``dpsdxm``/``dpsdym`` with their one-sided boundary forms and ``dprddx``/``dprddy``
  (Main/mod_params.F90:2637-2686);
* ``compute_full_coriolis_coefficients`` (Main/mod_params.F90:2696-2741);
* ``init_sound``'s global scalars (Main/mod_sound.F90:115-161): the short-step limit and the
  interior mean map factor.

Arrays are global C-order ``[k][i][j]`` (Fortran ``(j,i,k)``) with 1-based global indices
mapped to ``[i-1, j-1]``; points the reference never sets stay zero (the reference's
``getmem`` arrays start zeroed), which matters for the 4-point means at the east/north edge
(``ex``/``crx``/``cry`` average in the unset boundary dot values).
"""
from __future__ import annotations

import math

import numpy as np

from . import constants as C

TISO = 216.65                                   # Share/mod_constants.F90:198
ROVG = C.rgas / C.egrav                         # :187
GOVR = C.egrav / C.rgas                         # :188
XGAMMA = 1.0 / (1.0 - C.rovcp)                  # Main/mod_sound.F90:77
DEGRAD = math.pi / 180.0
EOMEG2 = 2.0 * C.eomeg


def nhbase(ter_m: np.ndarray, sig: np.ndarray, ptop: float, p0: float, tlp: float, st0: float):
    """Share/mod_nhinterp.F90:74-106 on cross points; ter_m (iy-1, jx-1) metres."""
    ptoppa = ptop * 1000.0
    ac = 0.5 * GOVR * ter_m / tlp
    b = st0 / tlp
    alnp = -b + np.sqrt(b * b - 4.0 * ac)
    ps0 = p0 * np.exp(alnp) - ptoppa
    kx = len(sig)
    pr0 = np.empty((kx,) + ps0.shape)
    t0 = np.empty_like(pr0)
    rho0 = np.empty_like(pr0)
    z0 = np.empty_like(pr0)
    for k in range(kx):
        pr0[k] = ps0 * sig[k] + ptoppa
        t0[k] = np.maximum(st0 + tlp * np.log(pr0[k] / p0), TISO)
        rho0[k] = pr0[k] / C.rgas / t0[k]
        a = np.log(pr0[k] / (ps0 + ptoppa))
        z0[k] = np.maximum(-(0.5 * ROVG * tlp * a * a + ROVG * st0 * a), 0.0)
    return ps0, pr0, t0, rho0, z0


def reference_state(rc, ht_geo: np.ndarray, msfx: np.ndarray, msfd: np.ndarray,
                    xlat: np.ndarray, xlon: np.ndarray, dlat: np.ndarray) -> dict:
    """All NH statics for a single-tile domain.  ht_geo: geopotential (iy, jx) as stored
    after param; msfx/msfd: inverted map factors as stored; xlat/xlon cross-point and dlat
    dot-point latitudes/longitudes in degrees."""
    jx, iy, kz = rc.jx, rc.iy, rc.kz
    sigma = rc.sigma
    hsigma = (sigma[1:] + sigma[:-1]) * 0.5
    dx = rc.ds * 1000.0
    dx8 = 8.0 * dx
    ce = (slice(0, iy - 1), slice(0, jx - 1))
    ter = ht_geo[ce] * C.regrav
    args = (rc.ptop, rc.base_state_pressure, rc.logp_lrate, rc.base_state_ts0)
    ps0, pr, t, rho, z = nhbase(ter, hsigma, *args)
    _, pf, tf, rhof, zf = nhbase(ter, sigma, *args)

    def full2(a):
        out = np.zeros((iy, jx))
        out[ce] = a
        return out

    def full3(a):
        out = np.zeros((a.shape[0], iy, jx))
        out[:, 0:iy - 1, 0:jx - 1] = a
        return out

    out = {"ATM0_PS": full2(ps0)[None], "ATM0_PR": full3(pr), "ATM0_T": full3(t),
           "ATM0_RHO": full3(rho), "ATM0_Z": full3(z), "ATM0_PF": full3(pf),
           "ATM0_RHOF": full3(rhof), "ATM0_ZF": full3(zf)}
    ps = out["ATM0_PS"][0]

    # dpsdxm / dpsdym, Main/mod_params.F90:2637-2674 (j = jci; one-sided at jce1/jce2)
    dpsdxm = np.zeros((iy, jx))
    dpsdym = np.zeros((iy, jx))
    I = np.arange(0, iy - 1)          # ice1..ice2 (0-based)
    J = np.arange(0, jx - 1)
    for j in range(1, jx - 2):        # jci1..jci2
        dpsdxm[I, j] = (ps[I, j + 1] - ps[I, j - 1]) / (ps[I, j] * dx8 * msfx[I, j])
    dpsdxm[I, 0] = (ps[I, 1] - ps[I, 0]) / (ps[I, 0] * dx8 * msfx[I, 0])
    je = jx - 2
    dpsdxm[I, je] = (ps[I, je] - ps[I, je - 1]) / (ps[I, je] * dx8 * msfx[I, je])
    for i in range(1, iy - 2):        # ici1..ici2
        dpsdym[i, J] = (ps[i + 1, J] - ps[i - 1, J]) / (ps[i, J] * dx8 * msfx[i, J])
    dpsdym[0, J] = (ps[1, J] - ps[0, J]) / (ps[0, J] * dx8 * msfx[0, J])
    ie = iy - 2
    dpsdym[ie, J] = (ps[ie, J] - ps[ie - 1, J]) / (ps[ie, J] * dx8 * msfx[ie, J])
    out["DPSDXM"], out["DPSDYM"] = dpsdxm[None], dpsdym[None]

    # dprddx / dprddy on interior dot points, :2676-2686
    prf = out["ATM0_PR"]
    dprddx = np.zeros((kz, iy, jx))
    dprddy = np.zeros((kz, iy, jx))
    di = (slice(1, iy - 1), slice(1, jx - 1))
    a, b_, c_, d_ = prf[:, 1:iy - 1, 1:jx - 1], prf[:, 1:iy - 1, 0:jx - 2], \
        prf[:, 0:iy - 2, 1:jx - 1], prf[:, 0:iy - 2, 0:jx - 2]
    dprddx[:, di[0], di[1]] = a - b_ + c_ - d_
    dprddy[:, di[0], di[1]] = a - c_ + b_ - d_
    out["DPRDDX"], out["DPRDDY"] = dprddx, dprddy

    # compute_full_coriolis_coefficients, :2696-2741 (interior dot points)
    ef = np.zeros((iy, jx)); ddx = np.zeros((iy, jx)); ddy = np.zeros((iy, jx))
    dmdx = np.zeros((iy, jx)); dmdy = np.zeros((iy, jx))
    for i in range(1, iy - 1):
        for j in range(1, jx - 1):
            dl = dlat[i, j]
            dlatdy = 0.5 * (xlat[i, j - 1] + xlat[i, j] - xlat[i - 1, j - 1] - xlat[i - 1, j])
            if abs(dlatdy) < 1.0e-8:
                dlatdy = math.copysign(1.0e-8, dlatdy)
            dlondy = 0.5 * (xlon[i, j - 1] + xlon[i, j] - xlon[i - 1, j - 1] - xlon[i - 1, j])
            if dlondy > 180.0:
                dlondy -= 360.0
            if dlondy < -180.0:
                dlondy += 360.0
            rotang = -math.atan(dlondy / dlatdy * math.cos(DEGRAD * dl))
            if dlatdy < 0.0:
                rotang += math.pi
            ef[i, j] = EOMEG2 * math.cos(DEGRAD * dl)
            ddx[i, j] = math.cos(rotang)
            ddy[i, j] = math.sin(rotang)
            den = dx * msfd[i, j] * msfd[i, j]
            dmdx[i, j] = -0.5 * (msfx[i, j] + msfx[i - 1, j] - msfx[i, j - 1] - msfx[i - 1, j - 1]) / den
            dmdy[i, j] = -0.5 * (msfx[i, j] + msfx[i, j - 1] - msfx[i - 1, j] - msfx[i - 1, j - 1]) / den
    ex = np.zeros((iy, jx)); crx = np.zeros((iy, jx)); cry = np.zeros((iy, jx))
    ci = (slice(1, iy - 2), slice(1, jx - 2))

    def avg4(a):
        return 0.25 * (a[1:iy - 2, 1:jx - 2] + a[2:iy - 1, 1:jx - 2] +
                       a[1:iy - 2, 2:jx - 1] + a[2:iy - 1, 2:jx - 1])

    ex[ci] = avg4(ef)
    crx[ci] = avg4(ddx)
    cry[ci] = avg4(ddy)
    for name, a in (("EF", ef), ("DDX", ddx), ("DDY", ddy), ("DMDX", dmdx), ("DMDY", dmdy),
                    ("EX", ex), ("CRX", crx), ("CRY", cry)):
        out[name] = a[None]

    # init_sound scalars, Main/mod_sound.F90:130-151
    npts = (iy - 3) * (jx - 3)
    xmsf = float(np.sum(msfx[1:iy - 2, 1:jx - 2])) / 1.0 * (1.0 / npts)
    maxt = float(np.max(t))
    cs = math.sqrt(XGAMMA * C.rgas * maxt)
    dtsmax = dx / cs / (1.0 + rc.nhxkd)
    return dict(fields=out, nh_dtsmax=dtsmax, nh_xmsf=xmsf)


def acoustic_substeps(rc, dtsmax: float, dt: float, lcount: int) -> int:
    """istep of sound, Main/mod_sound.F90:201-205."""
    istep = max(int(dt / dtsmax), 2)
    if lcount > 0:
        istep = max(4, istep)
    return istep
