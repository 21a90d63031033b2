"""Independent NumPy restatements of the oracle rows no other check pins.

TEST INFRASTRUCTURE.  Each restatement below is written from the reference's Fortran text
(file:line in its docstring) with NumPy elementwise arithmetic in the Fortran's operation order
(NumPy evaluates a*b + c as two rounded operations, like the reference without FMA contraction;
the scalar logs of splitf use math.log, the C library's), and compared with the C restatement
(oracle/rcm_oracle.c) bit for bit: none of these rows evaluates a transcendental function on a
field.  The oracle is stopped where a row starts and where it ends through its test hook
orc_set_tend_probe (1: every tendency summed and the t / qx forecasts formed, 2: the time
filters applied, the entry of splitf), so each row is checked on its own inputs:

* the forecast of t and qx and the serial negative-moisture fix with dependent clusters
  (Main/mod_tendency.F90:368-393);
* the time filters filter_ra_2d/3d/uv, filter_raw_qv and filter_raw_4d
  (Main/mod_timefilter.F90:58-281, called at Main/mod_tendency.F90:419-449);
* splitf and spstep: the deld/delh projections, the forward and leapfrog sub-steps with the
  boundary extrapolation, the ddsum/dhsum corrections of p*, t, u, v
  (Main/mod_split.F90:243-669, psc2psd Main/mpplib/mod_mppparam.F90:13811-13861);
* bdyval and bdyuv of the hydrostatic core: the integration copies, the time-dependent
  boundary values, the slices with their corner fills, the qv (iboudy = 3/4) and qc
  inflow/outflow (Main/mod_bdycod.F90:896-1094, 1109-1529, 1699-1805, 1809-1950, 2153-2223).

Every row runs on the limited-area domain and on the tropical band (i_band = 1, periodic in j:
Main/mpplib/mod_mppparam.F90:1112-1114, 1131, 1351-1354), whose one tile is its own west and
east neighbour, so ghost columns hold the wrapped values as the exchange leaves them.
"""
import dataclasses
import math

import numpy as np
import pytest

from regcm_amd import icbc
from regcm_amd.config import CONFIGS, build_config

MINQQ = 1.0e-8            # Share/mod_constants.F90:57
BETARAW = 0.53            # Main/mod_timefilter.F90:39


class Grid:
    """The index ranges of a one-tile domain (Main/mod_atm_interface.F90:231-302 with
    Main/mpplib/mod_mppparam.F90:1338-1360; a band has no west/east side and takes every j on
    the cross grid).  Arrays are the rcmdyn get layout a[..., i-1, j-1]."""

    def __init__(self, rc):
        jx, iy = rc.jx, rc.iy
        self.jx, self.iy = jx, iy
        self.band = bool(rc.i_band)
        self.bl = self.br = not self.band
        self.bb = self.bt = True
        self.jde1, self.jde2, self.ide1, self.ide2 = 1, jx, 1, iy
        self.jce1, self.jce2 = 1, (jx if self.band else jx - 1)
        self.ice1, self.ice2 = 1, iy - 1
        self.jdi1, self.jdi2 = (2, jx - 1) if self.bl else (1, jx)
        self.idi1, self.idi2 = 2, iy - 1
        self.jci1 = self.jce1 + (1 if self.bl else 0)
        self.jci2 = self.jce2 - (1 if self.br else 0)
        self.ici1, self.ici2 = 2, iy - 2

    def box(self, j1, j2, i1, i2):
        return np.meshgrid(np.arange(j1, j2 + 1), np.arange(i1, i2 + 1))

    def wrap(self, J):
        return (J - 1) % self.jx + 1 if self.band else J

    def at(self, a, J, I):
        J = self.wrap(J)
        assert J.min() >= 1 and J.max() <= self.jx and I.min() >= 1 and I.max() <= self.iy
        return a[..., I - 1, J - 1]

    def put(self, a, J, I, v):
        a[..., I - 1, self.wrap(J) - 1] = v


def _case(band=False, **kw):
    rc = dataclasses.replace(CONFIGS["C1"], i_band=int(band), **kw)
    data = icbc.generate(rc)
    st = dict(data["state"])
    for a1, a2 in (("ATM1_QC", "ATM1_QV"), ("ATM2_QC", "ATM2_QV")):   # a cloud layer
        qc = np.zeros_like(st[a2])
        qc[3:12] = 0.01 * st[a2][3:12]
        st[a1] = qc
    if rc.nqx > 2:
        st.update(icbc.hydrometeor_state(rc, st, nqx=rc.nqx))
    return rc, data, st


def _oracle(rc, data, st, nsteps=2, phy=None, probe=0):
    """An oracle after the initial bdyval and nsteps steps; phy (put before the probed tend)."""
    from oracle.oracle import OracleCore
    o = OracleCore(rc, data["split"])
    o.put_state(st)
    o.bdyval()
    o.step(nsteps)
    for name, a in (phy or {}).items():
        o.put(name, a)
    o.set_tend_probe(probe)
    return o


def _clusters(rc, seed, amp):
    """Negative p*-coupled tendencies on a few 3x3 .. 5x5 patches of some levels: the forecast
    goes negative on whole patches, so the sweep reads already-fixed predecessors there."""
    rng = np.random.default_rng(seed)
    a = np.zeros((rc.kz, rc.iy, rc.jx))
    for _ in range(8):
        k = int(rng.integers(0, rc.kz))
        i0, j0 = int(rng.integers(1, rc.iy - 7)), int(rng.integers(0, rc.jx - 5))
        a[k, i0:i0 + 3 + int(rng.integers(0, 3)), j0:j0 + 3 + int(rng.integers(0, 3))] = -amp
    # a patch on the first / last interior column: the band's fix reads the wrapped neighbours
    a[3, 10:14, 0:3] = -amp
    a[5, 20:23, rc.jx - 3:] = -amp
    return a


def _species(rc):
    return ["QV", "QC"] + (["QI", "QR", "QS"] if rc.nqx > 2 else [])


# ------------------------------------------------------------------ forecast + negative fix

def _forecast_fix_np(g, a2q, qten, dt):
    """Main/mod_tendency.F90:375-393 for one species: atmc%qx = atm2%qx on the ce box, plus
    dt*qxten on ci, exchanged (a band's ghost columns: the wrapped forecasts), then the serial
    sweep (k, i, j loops, j fastest) replacing each negative value by
    0.01*sum(abs(atmc%qx(j-1:j+1,i-1:i+1)))/9 in the array-element order of SUM."""
    cq = np.zeros_like(a2q)
    J, I = g.box(g.jce1, g.jce2, g.ice1, g.ice2)
    g.put(cq, J, I, g.at(a2q, J, I))
    J, I = g.box(g.jci1, g.jci2, g.ici1, g.ici2)
    g.put(cq, J, I, g.at(cq, J, I) + dt * g.at(qten, J, I))
    ghost = cq.copy()                               # the exchanged values a ghost column holds
    for k in range(cq.shape[0]):
        for i in range(g.ici1, g.ici2 + 1):
            for j in range(g.jci1, g.jci2 + 1):
                if not cq[k, i - 1, j - 1] < 0.0:
                    continue
                s = 0.0
                for ii in (i - 1, i, i + 1):
                    for jj in (j - 1, j, j + 1):
                        if 1 <= jj <= g.jx:
                            s = s + abs(cq[k, ii - 1, jj - 1])
                        else:                       # only a band reads past its columns
                            assert g.band
                            s = s + abs(ghost[k, ii - 1, (jj - 1) % g.jx])
                cq[k, i - 1, j - 1] = 0.01 * s / 9.0
    return cq


@pytest.mark.parametrize("variant", [{}, {"band": True}, {"ipptls": 2}], ids=["lam", "band", "nqx5"])
def test_forecast_and_negative_fix_match_numpy_restatement(variant):
    """The t forecast and each species' forecast with its serial negative fix (dependent
    clusters forced through the physics tendencies) equal the restatement bit for bit."""
    rc, data, st = _case(**variant)
    phy = {"QVPHY": _clusters(rc, 1, 0.05), "QCPHY": _clusters(rc, 2, 0.02)}
    o = _oracle(rc, data, st, phy=phy, probe=1)
    g = Grid(rc)
    before = {f"ATM2_{s}": o.get(f"ATM2_{s}") for s in _species(rc)}
    before["ATM2_T"] = o.get("ATM2_T")
    _, dt, _ = o.get_time()
    o.tend()
    assert o.get_time()[1] == dt                     # the probe returns before the clock moves
    for name, a in before.items():
        assert np.array_equal(o.get(name), a), name  # atm2 untouched before the filters
    # t: Main/mod_tendency.F90:368-374
    J, I = g.box(g.jci1, g.jci2, g.ici1, g.ici2)
    ct = o.get_work("ct")
    assert np.array_equal(g.at(ct, J, I), g.at(before["ATM2_T"], J, I) + dt * g.at(o.get("TTEN"), J, I))
    ten = {"QV": o.get("QVTEN"), "QC": o.get("QCTEN")}
    if rc.nqx > 2:
        ten.update(QI=o.get_work("qteni"), QR=o.get_work("qtenr"), QS=o.get_work("qtens"))
    nfixed = 0
    for s in _species(rc):
        want = _forecast_fix_np(g, before[f"ATM2_{s}"], ten[s], dt)
        got = o.get_work("c" + s.lower())
        Jc, Ic = g.box(g.jce1, g.jce2, g.ice1, g.ice2)
        assert np.array_equal(g.at(got, Jc, Ic), g.at(want, Jc, Ic)), s
        neg = g.at(before[f"ATM2_{s}"], J, I) + dt * g.at(ten[s], J, I) < 0.0
        nfixed += int(neg.sum())
    assert nfixed > 100                              # the clusters were fixed, serially


# ------------------------------------------------------------------------------ time filters

def _filters_np(g, s, dt, gnu1, gnu2):
    """Main/mod_tendency.F90:419-449 with Main/mod_timefilter.F90: filter_ra_2d of p*
    (:58-73), filter_ra_3d of t (:92-110), filter_raw_qv of qv with the new psa/psb (:257-278),
    filter_raw_4d of the hydrometeors with low = 0 (:231-255), then the u, v forecasts and
    filter_ra_uv (:132-156).  s: the state and forecasts at probe 1; returns the new state."""
    out = {k: v.copy() for k, v in s.items()}
    J, I = g.box(g.jci1, g.jci2, g.ici1, g.ici2)
    at = g.at
    psa, psb, psc = at(s["PSA"], J, I), at(s["PSB"], J, I), at(s["PSC"], J, I)
    d = gnu1 * (psc + psb - 2.0 * psa)
    g.put(out["PSB"], J, I, psa + d)
    g.put(out["PSA"], J, I, psc)
    a1, a2, c = at(s["ATM1_T"], J, I), at(s["ATM2_T"], J, I), at(s["ct"], J, I)
    d = gnu1 * (c + a2 - 2.0 * a1)
    g.put(out["ATM2_T"], J, I, a1 + d)
    g.put(out["ATM1_T"], J, I, c)
    npsa, npsb = at(out["PSA"], J, I), at(out["PSB"], J, I)
    for sp in [x for x in ("QV", "QC", "QI", "QR", "QS") if f"ATM1_{x}" in s]:
        a1, a2, c = at(s[f"ATM1_{sp}"], J, I), at(s[f"ATM2_{sp}"], J, I), at(s["c" + sp.lower()], J, I)
        if sp == "QV":
            d = gnu1 * (c + a2 - 2.0 * a1)
            g.put(out["ATM2_QV"], J, I, np.maximum(a1 + BETARAW * d, MINQQ * npsa))
            g.put(out["ATM1_QV"], J, I, np.maximum(c + (BETARAW - 1.0) * d, MINQQ * npsb))
        else:
            d = gnu2 * (c + a2 - 2.0 * a1)
            m1 = a1 + BETARAW * d
            n1 = c + (BETARAW - 1.0) * d
            g.put(out[f"ATM2_{sp}"], J, I, np.where(m1 < 0.0, 0.0, m1))
            g.put(out[f"ATM1_{sp}"], J, I, np.where(n1 < 0.0, 0.0, n1))
    J, I = g.box(g.jdi1, g.jdi2, g.idi1, g.idi2)
    for f in ("U", "V"):
        a1, a2 = at(s[f"ATM1_{f}"], J, I), at(s[f"ATM2_{f}"], J, I)
        c = a2 + dt * at(s[f"{f}TEN"], J, I)                   # :433-440
        d = gnu1 * (c + a2 - 2.0 * a1)
        g.put(out[f"ATM2_{f}"], J, I, a1 + d)
        g.put(out[f"ATM1_{f}"], J, I, c)
    return out


PROG = ["PSA", "PSB", "ATM1_U", "ATM1_V", "ATM1_T", "ATM2_U", "ATM2_V", "ATM2_T"]


@pytest.mark.parametrize("variant", [{}, {"band": True}, {"ipptls": 2}], ids=["lam", "band", "nqx5"])
def test_time_filters_match_numpy_restatement(variant):
    """From the forecasts (probe 1) the RA / RAW filters give the state splitf starts from
    (probe 2) bit for bit; every point the filters do not visit is unchanged."""
    rc, data, st = _case(**variant)
    phy = {"QVPHY": _clusters(rc, 3, 0.05), "QCPHY": _clusters(rc, 4, 0.02)}
    a = _oracle(rc, data, st, phy=phy, probe=1)
    b = _oracle(rc, data, st, phy=phy, probe=2)
    g = Grid(rc)
    _, dt, _ = a.get_time()
    a.tend()
    b.tend()
    sp = _species(rc)
    names = PROG + [f"ATM{n}_{s}" for n in (1, 2) for s in sp]
    s = {n: a.get(n) for n in names + ["PSC", "UTEN", "VTEN"]}
    s["ct"] = a.get_work("ct")
    for x in sp:
        s["c" + x.lower()] = a.get_work("c" + x.lower())
    want = _filters_np(g, s, dt, rc.gnu1, rc.gnu2)
    for n in names:
        assert np.array_equal(b.get(n), want[n]), n


# ------------------------------------------------------------------------- splitf + spstep

def _psc2psd_np(g, pc):
    """psc2psd, Main/mpplib/mod_mppparam.F90:13811-13861 (a band: no west/east lines)."""
    pd = np.zeros_like(pc)
    J, I = g.box(g.jdi1, g.jdi2, g.idi1, g.idi2)
    g.put(pd, J, I, (g.at(pc, J, I) + g.at(pc, J, I - 1) + g.at(pc, J - 1, I) + g.at(pc, J - 1, I - 1)) * 0.25)
    J, I = g.box(g.jdi1, g.jdi2, g.ide2, g.ide2)
    g.put(pd, J, I, (g.at(pc, J, I - 1) + g.at(pc, J - 1, I - 1)) * 0.5)      # top: pc(j,ice2)
    J, I = g.box(g.jdi1, g.jdi2, g.ide1, g.ide1)
    g.put(pd, J, I, (g.at(pc, J, I) + g.at(pc, J - 1, I)) * 0.5)              # bottom: pc(j,ice1)
    if g.bl:
        J, I = g.box(g.jde1, g.jde1, g.idi1, g.idi2)
        g.put(pd, J, I, (g.at(pc, J, I) + g.at(pc, J, I - 1)) * 0.5)
        g.put(pd, np.array([[g.jde1]]), np.array([[g.ide1]]), pc[g.ice1 - 1, g.jce1 - 1])
        g.put(pd, np.array([[g.jde1]]), np.array([[g.ide2]]), pc[g.ice2 - 1, g.jce1 - 1])
    if g.br:
        J, I = g.box(g.jde2, g.jde2, g.idi1, g.idi2)
        g.put(pd, J, I, (g.at(pc, J - 1, I) + g.at(pc, J - 1, I - 1)) * 0.5)  # pc(jce2, ...)
        g.put(pd, np.array([[g.jde2]]), np.array([[g.ide1]]), pc[g.ice1 - 1, g.jce2 - 1])
        g.put(pd, np.array([[g.jde2]]), np.array([[g.ide2]]), pc[g.ice2 - 1, g.jce2 - 1])
    return pd


def _splitf_np(g, cfg, s, msfx, msfd):
    """splitf + spstep, Main/mod_split.F90:243-669, on the state s at splitf's entry.  Returns
    the corrected state with dstor, hstor and psdota."""
    at, put = g.at, g.put
    kz, nsp = cfg.kz, cfg.nsplit
    dx2 = 2.0 * (cfg.ds * 1000.0)                     # Main/mod_params.F90:1763-1764
    rdx2 = 1.0 / dx2
    ptop, pd_ = cfg.ptop, cfg.pd
    out = {k: v.copy() for k, v in s.items()}
    psa, psb = s["PSA"][0], s["PSB"][0]
    psdota = _psc2psd_np(g, psa)
    mapc = np.zeros_like(psa)                         # map = 1/(msfx*msfx) on ce (:100)
    Jc, Ic = g.box(g.jce1, g.jce2, g.ice1, g.ice2)
    put(mapc, Jc, Ic, 1.0 / (at(msfx, Jc, Ic) * at(msfx, Jc, Ic)))
    shape = (nsp, g.iy, g.jx)
    deld = {n: np.zeros(shape) for n in (1, 2, 3)}
    delh = {n: np.zeros(shape) for n in (1, 2, 3)}
    deld[1][:] = s["DSTOR"]
    delh[1][:] = s["HSTOR"]

    def project_div(u, v, slot):                      # :271-295 / :307-330
        uuu, vvv = u * msfd, v * msfd                 # on jde/ide (exchange_rt: a band wraps)
        for l in range(nsp):
            acc = np.zeros((g.ice2 - g.ice1 + 1, g.jce2 - g.jce1 + 1))
            mp = at(mapc, Jc, Ic)
            for k in range(kz):
                U, V = uuu[k], vvv[k]
                br = (-at(U, Jc, Ic + 1) + at(U, Jc + 1, Ic + 1) - at(U, Jc, Ic) + at(U, Jc + 1, Ic) +
                      at(V, Jc, Ic + 1) + at(V, Jc + 1, Ic + 1) - at(V, Jc, Ic) - at(V, Jc + 1, Ic))
                acc = acc + cfg.zmatxr[l][k] * rdx2 * mp * br
            deld[slot][l][:] = 0.0
            put(deld[slot][l], Jc, Ic, acc)

    def project_geo(ps, t, slot):                     # :342-362 / :374-394
        for l in range(nsp):
            sh, va = cfg.sigmah[kz], cfg.varpa1[l][kz]
            pdlog = va * math.log(sh * pd_ + ptop)
            eps1 = va * sh / (sh * pd_ + ptop)
            p = at(ps, Jc, Ic)
            acc = pdlog + eps1 * (p - pd_)
            for k in range(kz):
                sh, va = cfg.sigmah[k], cfg.varpa1[l][k]
                pdlog = va * math.log(sh * pd_ + ptop)
                eps1 = va * sh / (sh * pd_ + ptop)
                acc = acc + pdlog + cfg.tau[l][k] * at(t[k], Jc, Ic) / p + eps1 * (p - pd_)
            delh[slot][l][:] = 0.0
            put(delh[slot][l], Jc, Ic, acc)

    project_div(s["ATM1_U"], s["ATM1_V"], 3)
    deld[3] = deld[3] - deld[1]
    project_div(s["ATM2_U"], s["ATM2_V"], 2)
    deld[1] = deld[1] - deld[2]
    project_geo(psa, s["ATM1_T"], 3)
    delh[3] = delh[3] - delh[1]
    project_geo(psb, s["ATM2_T"], 2)
    delh[1] = delh[1] - delh[2]
    out["DSTOR"] = deld[2].copy()
    out["HSTOR"] = delh[2].copy()
    # spstep, :463-669
    ddsum, dhsum = np.zeros(shape), np.zeros(shape)
    Jd, Id = g.box(g.jdi1, g.jdi2, g.idi1, g.idi2)
    Ji, Ii = g.box(g.jci1, g.jci2, g.ici1, g.ici2)

    def divergence(h):                                # :498-534 on delh(slot); returns work3 on ci
        fac = dx2 * at(msfx, Jd, Id)
        w1 = (at(h, Jd, Id) + at(h, Jd, Id - 1) - at(h, Jd - 1, Id) - at(h, Jd - 1, Id - 1)) / fac
        w2 = (at(h, Jd, Id) + at(h, Jd - 1, Id) - at(h, Jd, Id - 1) - at(h, Jd - 1, Id - 1)) / fac
        w1 = w1 * at(psdota, Jd, Id)
        w2 = w2 * at(psdota, Jd, Id)
        uu, vv = np.zeros_like(psa), np.zeros_like(psa)
        put(uu, Jd, Id, w1 * at(msfd, Jd, Id))
        put(vv, Jd, Id, w2 * at(msfd, Jd, Id))
        return rdx2 * at(mapc, Ji, Ii) * (-at(uu, Ji, Ii + 1) + at(uu, Ji + 1, Ii + 1) - at(uu, Ji, Ii) +
                                          at(uu, Ji + 1, Ii) + at(vv, Ji, Ii + 1) + at(vv, Ji + 1, Ii + 1) -
                                          at(vv, Ji, Ii) - at(vv, Ji + 1, Ii))

    def boundary_lines(l, new, f):                    # "not in Madala (1987)", :547-567 / :632-651
        if g.bl:
            J, I = g.box(g.jce1, g.jce1, g.ici1, g.ici2)
            put(delh[new][l], J, I, f(J, I))
        if g.br:
            J, I = g.box(g.jce2, g.jce2, g.ici1, g.ici2)
            put(delh[new][l], J, I, f(J, I))
        J, I = g.box(g.jce1, g.jce2, g.ice1, g.ice1)
        put(delh[new][l], J, I, f(J, I))
        J, I = g.box(g.jce1, g.jce2, g.ice2, g.ice2)
        put(delh[new][l], J, I, f(J, I))

    for l in range(nsp):
        n0, n1 = 1, 2
        n2 = n0
        aam, dtau, hbar = cfg.aam[l], cfg.dtau[l], cfg.hbar[l]
        m2 = int(aam) * 2
        dtau2 = dtau * 2.0
        put(ddsum[l], Jc, Ic, at(deld[n0][l], Jc, Ic))
        put(dhsum[l], Jc, Ic, at(delh[n0][l], Jc, Ic))
        w3 = divergence(delh[n0][l])
        pa = at(psa, Ji, Ii)
        put(deld[n1][l], Ji, Ii, at(deld[n0][l], Ji, Ii) - dtau * w3 + at(deld[3][l], Ji, Ii) / m2)
        put(delh[n1][l], Ji, Ii, at(delh[n0][l], Ji, Ii) - dtau * hbar * at(deld[n0][l], Ji, Ii) / pa +
            at(delh[3][l], Ji, Ii) / m2)
        fac = (aam - 1.0) / aam
        boundary_lines(l, n1, lambda J, I: at(delh[n0][l], J, I) * fac)
        put(ddsum[l], Jc, Ic, at(ddsum[l], Jc, Ic) + at(deld[n1][l], Jc, Ic))
        put(dhsum[l], Jc, Ic, at(dhsum[l], Jc, Ic) + at(delh[n1][l], Jc, Ic))
        for _ in range(2, m2 + 1):
            w3 = divergence(delh[n1][l])
            put(deld[n2][l], Ji, Ii, at(deld[n0][l], Ji, Ii) - dtau2 * w3 + at(deld[3][l], Ji, Ii) / aam)
            put(delh[n2][l], Ji, Ii, at(delh[n0][l], Ji, Ii) - dtau2 * hbar * at(deld[n1][l], Ji, Ii) / pa +
                at(delh[3][l], Ji, Ii) / aam)
            a, b = n0, n1
            boundary_lines(l, n2, lambda J, I: 2.0 * at(delh[b][l], J, I) - at(delh[a][l], J, I))
            put(ddsum[l], Jc, Ic, at(ddsum[l], Jc, Ic) + at(deld[n2][l], Jc, Ic))
            put(dhsum[l], Jc, Ic, at(dhsum[l], Jc, Ic) + at(delh[n2][l], Jc, Ic))
            n0, n1 = n1, n2
            n2 = n0
    # corrections, :417-457
    gnu1 = cfg.gnu1
    pa, pb = out["PSA"][0], out["PSB"][0]
    for l in range(nsp):
        an = cfg.an[l]
        gnuan = gnu1 * an
        put(pa, Ji, Ii, at(pa, Ji, Ii) - an * at(ddsum[l], Ji, Ii))
        put(pb, Ji, Ii, at(pb, Ji, Ii) - gnuan * at(ddsum[l], Ji, Ii))
    for l in range(nsp):
        for k in range(kz):
            am = cfg.am[l][k]
            gnuam = gnu1 * am
            put(out["ATM1_T"][k], Ji, Ii, at(out["ATM1_T"][k], Ji, Ii) + am * at(ddsum[l], Ji, Ii))
            put(out["ATM2_T"][k], Ji, Ii, at(out["ATM2_T"][k], Ji, Ii) + gnuam * at(ddsum[l], Ji, Ii))
    for l in range(nsp):
        h = dhsum[l]
        for k in range(kz):
            zm = cfg.zmatx[l][k]
            gnuzm = gnu1 * zm
            fac = at(psdota, Jd, Id) / (dx2 * at(msfd, Jd, Id))
            x = fac * (at(h, Jd, Id) + at(h, Jd, Id - 1) - at(h, Jd - 1, Id) - at(h, Jd - 1, Id - 1))
            y = fac * (at(h, Jd, Id) - at(h, Jd, Id - 1) + at(h, Jd - 1, Id) - at(h, Jd - 1, Id - 1))
            put(out["ATM1_U"][k], Jd, Id, at(out["ATM1_U"][k], Jd, Id) - zm * x)
            put(out["ATM1_V"][k], Jd, Id, at(out["ATM1_V"][k], Jd, Id) - zm * y)
            put(out["ATM2_U"][k], Jd, Id, at(out["ATM2_U"][k], Jd, Id) - gnuzm * x)
            put(out["ATM2_V"][k], Jd, Id, at(out["ATM2_V"][k], Jd, Id) - gnuzm * y)
    out["PSDOTA"] = psdota[None]
    return out


@pytest.mark.parametrize("variant", [{}, {"band": True}, {"nsplit": 3}, {"nsplit": 1}],
                         ids=["lam", "band", "nsplit3", "nsplit1"])
def test_splitf_spstep_match_numpy_restatement(variant):
    """From the state at splitf's entry (probe 2), the NumPy splitf/spstep gives the state the
    whole tend leaves (p*, t, u, v corrected; dstor, hstor; psdota) bit for bit."""
    variant = dict(variant)
    band = variant.pop("band", False)
    rc, data, st = _case(band=band, **variant)
    a = _oracle(rc, data, st, probe=2)
    b = _oracle(rc, data, st)
    a.tend()
    b.tend()
    names = PROG + ["DSTOR", "HSTOR"]
    s = {n: a.get(n) for n in names}
    cfg = build_config(rc, data["split"])
    g = Grid(rc)
    want = _splitf_np(g, cfg, s, a.get("MSFX")[0], a.get("MSFD")[0])
    for n in names + ["PSDOTA"]:
        assert np.array_equal(b.get(n), want[n]), n
    for n in ("ATM1_T", "ATM1_U", "PSA"):           # the corrections did something
        assert not np.array_equal(want[n], s[n]), n


# ------------------------------------------------------------------------------ bdyval

def _bdyval_np(g, rc, s, b, lcount, dt, xbctime):
    """bdyval + bdyuv of the hydrostatic core, iboudy /= 0 (time-dependent values), bdyflow,
    not present_qc: Main/mod_bdycod.F90:1125-1310 (integration copies), 1426-1451 (p*),
    1493-1526 (p*u, p*v), 896-1094 (bdyuv: the slices, zero where never written, their corner
    fills and, on a band, the periodic neighbours exchange_bdy_lr gives them), 1699-1792 (p*t,
    p*qv), 1809-1950 (qv inflow/outflow, iboudy = 3/4), 2153-2223 (qc inflow/outflow)."""
    at, put = g.at, g.put
    kz = rc.kz
    out = {k: v.copy() for k, v in s.items()}
    xt = xbctime + dt
    psa, psb = out["PSA"][0], out["PSB"][0]
    if lcount > 0:                                               # rcmtimer%integrating()
        lines_d, lines_c = [], []
        if g.bl:
            lines_d.append(g.box(g.jde1, g.jde1, g.idi1, g.idi2)); lines_c.append(g.box(g.jce1, g.jce1, g.ici1, g.ici2))
        if g.br:
            lines_d.append(g.box(g.jde2, g.jde2, g.idi1, g.idi2)); lines_c.append(g.box(g.jce2, g.jce2, g.ici1, g.ici2))
        lines_d.append(g.box(g.jde1, g.jde2, g.ide1, g.ide1)); lines_c.append(g.box(g.jce1, g.jce2, g.ice1, g.ice1))
        lines_d.append(g.box(g.jde1, g.jde2, g.ide2, g.ide2)); lines_c.append(g.box(g.jce1, g.jce2, g.ice2, g.ice2))
        for (Jd, Id), (Jc, Ic) in zip(lines_d, lines_c):
            for f in ("U", "V"):
                put(out[f"ATM2_{f}"], Jd, Id, at(out[f"ATM1_{f}"], Jd, Id))
            for f in ["T"] + _species(rc):
                put(out[f"ATM2_{f}"], Jc, Ic, at(out[f"ATM1_{f}"], Jc, Ic))
            put(psb, Jc, Ic, at(psa, Jc, Ic))
    pc_lines = ([g.box(g.jce1, g.jce1, g.ici1, g.ici2)] if g.bl else []) + \
               ([g.box(g.jce2, g.jce2, g.ici1, g.ici2)] if g.br else []) + \
               [g.box(g.jce1, g.jce2, g.ice1, g.ice1), g.box(g.jce1, g.jce2, g.ice2, g.ice2)]
    for J, I in pc_lines:                                        # :1430-1450
        put(psa, J, I, at(b["XPSB_B0"][0], J, I) + xt * at(b["XPSB_BT"][0], J, I))
    pd_lines = ([g.box(g.jde1, g.jde1, g.idi1, g.idi2)] if g.bl else []) + \
               ([g.box(g.jde2, g.jde2, g.idi1, g.idi2)] if g.br else []) + \
               [g.box(g.jde1, g.jde2, g.ide1, g.ide1), g.box(g.jde1, g.jde2, g.ide2, g.ide2)]
    for J, I in pd_lines:                                        # :1493-1525
        put(out["ATM1_U"], J, I, at(b["XUB_B0"], J, I) + xt * at(b["XUB_BT"], J, I))
        put(out["ATM1_V"], J, I, at(b["XVB_B0"], J, I) + xt * at(b["XVB_BT"], J, I))
    # bdyuv (:896-1094): slices indexed [k-1, i-1] (west/east) or [k-1, j-1] (south/north)
    u1, v1 = out["ATM1_U"], out["ATM1_V"]
    zi, zj = np.zeros((kz, g.iy + 2)), np.zeros((kz, g.jx + 2))     # ide1ga:ide2ga, zero-allocated
    sl = {n: zi.copy() for n in ("wue", "wui", "wve", "wvi", "eue", "eui", "eve", "evi")}
    sl.update({n: zj.copy() for n in ("sue", "sui", "sve", "svi", "nue", "nui", "nve", "nvi")})
    ub = lambda J, I: b["XUB_B0"][:, I - 1, J - 1] + xt * b["XUB_BT"][:, I - 1, J - 1]   # noqa: E731
    vb = lambda J, I: b["XVB_B0"][:, I - 1, J - 1] + xt * b["XVB_BT"][:, I - 1, J - 1]   # noqa: E731
    ri = np.arange(g.idi1, g.idi2 + 1)
    rj = np.arange(g.jdi1, g.jdi2 + 1)
    re = np.arange(g.jde1, g.jde2 + 1)
    if g.bl:
        sl["wui"][:, ri] = u1[:, ri - 1, g.jdi1 - 1]; sl["wvi"][:, ri] = v1[:, ri - 1, g.jdi1 - 1]
        sl["wue"][:, ri] = ub(g.jde1, ri); sl["wve"][:, ri] = vb(g.jde1, ri)
    if g.br:
        sl["eui"][:, ri] = u1[:, ri - 1, g.jdi2 - 1]; sl["evi"][:, ri] = v1[:, ri - 1, g.jdi2 - 1]
        sl["eue"][:, ri] = ub(g.jde2, ri); sl["eve"][:, ri] = vb(g.jde2, ri)
    sl["sui"][:, rj] = u1[:, g.idi1 - 1, rj - 1]; sl["svi"][:, rj] = v1[:, g.idi1 - 1, rj - 1]
    sl["nui"][:, rj] = u1[:, g.idi2 - 1, rj - 1]; sl["nvi"][:, rj] = v1[:, g.idi2 - 1, rj - 1]
    sl["sue"][:, re] = ub(re, g.ide1); sl["sve"][:, re] = vb(re, g.ide1)
    sl["nue"][:, re] = ub(re, g.ide2); sl["nve"][:, re] = vb(re, g.ide2)
    if g.bl:                                                     # the corner fills, :1030-1061
        sl["wui"][:, g.ide2] = sl["nue"][:, g.jdi1]; sl["wvi"][:, g.ide2] = sl["nve"][:, g.jdi1]
        sl["nui"][:, g.jde1] = sl["wue"][:, g.idi2]; sl["nvi"][:, g.jde1] = sl["wve"][:, g.idi2]
        sl["wui"][:, g.ide1] = sl["sue"][:, g.jdi1]; sl["wvi"][:, g.ide1] = sl["sve"][:, g.jdi1]
        sl["sui"][:, g.jde1] = sl["wue"][:, g.idi1]; sl["svi"][:, g.jde1] = sl["wve"][:, g.idi1]
    if g.br:
        sl["eui"][:, g.ide2] = sl["nue"][:, g.jdi2]; sl["evi"][:, g.ide2] = sl["nve"][:, g.jdi2]
        sl["nui"][:, g.jde2] = sl["eue"][:, g.idi2]; sl["nvi"][:, g.jde2] = sl["eve"][:, g.idi2]
        sl["eui"][:, g.ide1] = sl["sue"][:, g.jdi2]; sl["evi"][:, g.ide1] = sl["sve"][:, g.jdi2]
        sl["sui"][:, g.jde2] = sl["eue"][:, g.idi1]; sl["svi"][:, g.jde2] = sl["eve"][:, g.idi1]
    if g.band:                                                   # exchange_bdy_lr around the period
        for n in ("sue", "sui", "sve", "svi", "nue", "nui", "nve", "nvi"):
            sl[n][:, 0] = sl[n][:, g.jx]
            sl[n][:, g.jx + 1] = sl[n][:, 1]
    for J, I in pc_lines:                                        # :1699-1790
        put(out["ATM1_T"], J, I, at(b["XTB_B0"], J, I) + xt * at(b["XTB_BT"], J, I))
        put(out["ATM1_QV"], J, I, at(b["XQB_B0"], J, I) + xt * at(b["XQB_BT"], J, I))
    q = out["ATM1_QV"]
    if rc.iboudy in (3, 4):                                      # :1883-1947
        for k in range(kz):
            if g.bl:
                for i in range(g.ici1, g.ici2 + 1):
                    qext = q[k, i - 1, g.jce1 - 1] / psa[i - 1, g.jce1 - 1]
                    qint = q[k, i - 1, g.jci1 - 1] / psa[i - 1, g.jci1 - 1]
                    w = sl["wue"][k, i] + sl["wue"][k, i + 1] + sl["wui"][k, i] + sl["wui"][k, i + 1]
                    q[k, i - 1, g.jce1 - 1] = (qext if w > 0.0 else qint) * psa[i - 1, g.jce1 - 1]
            if g.br:
                for i in range(g.ici1, g.ici2 + 1):
                    qext = q[k, i - 1, g.jce2 - 1] / psa[i - 1, g.jce2 - 1]
                    qint = q[k, i - 1, g.jci2 - 1] / psa[i - 1, g.jci2 - 1]
                    w = sl["eue"][k, i] + sl["eue"][k, i + 1] + sl["eui"][k, i] + sl["eui"][k, i + 1]
                    q[k, i - 1, g.jce2 - 1] = (qext if w < 0.0 else qint) * psa[i - 1, g.jce2 - 1]
        for k in range(kz):
            for (row, rin, sv, vi, inflow) in ((g.ice1, g.ici1, "sve", "svi", lambda w: w > 0.0),
                                              (g.ice2, g.ici2, "nve", "nvi", lambda w: w < 0.0)):
                for j in range(g.jce1, g.jce2 + 1):
                    qext = q[k, row - 1, j - 1] / psa[row - 1, j - 1]
                    qint = q[k, rin - 1, j - 1] / psa[rin - 1, j - 1]
                    w = sl[sv][k, j] + sl[sv][k, j + 1] + sl[vi][k, j] + sl[vi][k, j + 1]
                    q[k, row - 1, j - 1] = (qext if inflow(w) else qint) * psa[row - 1, j - 1]
    for sp in _species(rc)[1:]:                                  # :2155-2223 (n = iqfrst..iqlst)
        qx = out[f"ATM1_{sp}"]
        for k in range(kz):
            if g.bl:
                for i in range(g.ice1, g.ice2 + 1):
                    qxint = qx[k, i - 1, g.jci1 - 1] / psa[i - 1, g.jci1 - 1]
                    w = sl["wue"][k, i] + sl["wue"][k, i + 1] + sl["wui"][k, i] + sl["wui"][k, i + 1]
                    qx[k, i - 1, g.jce1 - 1] = 0.0 if w > 0.0 else qxint * psa[i - 1, g.jce1 - 1]
            if g.br:
                for i in range(g.ice1, g.ice2 + 1):
                    qxint = qx[k, i - 1, g.jci2 - 1] / psa[i - 1, g.jci2 - 1]
                    w = sl["eue"][k, i] + sl["eue"][k, i + 1] + sl["eui"][k, i] + sl["eui"][k, i + 1]
                    qx[k, i - 1, g.jce2 - 1] = 0.0 if w < 0.0 else qxint * psa[i - 1, g.jce2 - 1]
            for (row, rin, sv, vi, inflow) in ((g.ice1, g.ici1, "sve", "svi", lambda w: w > 0.0),
                                              (g.ice2, g.ici2, "nve", "nvi", lambda w: w < 0.0)):
                for j in range(g.jci1, g.jci2 + 1):
                    qxint = qx[k, rin - 1, j - 1] / psa[rin - 1, j - 1]
                    w = sl[sv][k, j] + sl[sv][k, j + 1] + sl[vi][k, j] + sl[vi][k, j + 1]
                    qx[k, row - 1, j - 1] = 0.0 if inflow(w) else qxint * psa[row - 1, j - 1]
    return out


BDY = ["XUB_B0", "XUB_BT", "XVB_B0", "XVB_BT", "XTB_B0", "XTB_BT", "XQB_B0", "XQB_BT", "XPSB_B0", "XPSB_BT"]


@pytest.mark.parametrize("variant", [{}, {"iboudy": 4}, {"iboudy": 3}, {"band": True},
                                     {"band": True, "iboudy": 4}, {"ipptls": 2, "iboudy": 4}],
                         ids=["lam", "iboudy4", "iboudy3", "band", "band-iboudy4", "nqx5-iboudy4"])
def test_bdyval_matches_numpy_restatement(variant):
    """After a tend (the integrating branch) and at the start (lcount = 0), bdyval equals the
    NumPy bdyval bit for bit on every prognostic field, and advances xbctime by dtsec."""
    from oracle.oracle import OracleCore
    variant = dict(variant)
    band = variant.pop("band", False)
    rc, data, st = _case(band=band, **variant)
    g = Grid(rc)
    names = PROG + [f"ATM{n}_{s}" for n in (1, 2) for s in _species(rc)]
    o = OracleCore(rc, data["split"])
    o.put_state(st)
    for start in (True, False):
        if not start:
            o.step(3)
            o.tend()
        lc, dt, xbc = o.get_time()
        s = {n: o.get(n) for n in names}
        b = {n: o.get(n) for n in BDY}
        want = _bdyval_np(g, rc, s, b, lc, dt, xbc)
        o.bdyval()
        for n in names:
            assert np.array_equal(o.get(n), want[n]), (n, start)
        assert o.get_time() == (lc, dt, xbc + rc.dt)
    # the branches acted: the qc lines took inflow zeros and outflow values, and with
    # iboudy = 3/4 some qv boundary values are the interior mixing ratio instead of b0 + xt bt
    assert not np.array_equal(want["ATM1_QC"], s["ATM1_QC"])
    if rc.iboudy in (3, 4):
        plain = _bdyval_np(g, dataclasses.replace(rc, iboudy=5), s, b, lc, dt, xbc)
        assert not np.array_equal(want["ATM1_QV"], plain["ATM1_QV"])


# ------------------------------------------------------------------- semi-Lagrangian pass

def _sladvection_np(g, rc, u1, v1, psa, msfx, msfd, a2q, a1q, dt):
    """One semi-Lagrangian pass of the moisture species (isladvec = 1,
    Main/mod_tendency.F90:1361-1363, 1378-1380): ua = atmx%umd = (atm1%u/psdota)*msfd
    (decouple :889, :999-1000; psdota = psc2psd of the step's p*), adv_velocity (.false.)
    (Main/mod_sladvection.F90:91-114, vadym1 reads va(j+1,i) twice as written), trajcalc_x
    (:134-222: the departure point to third order in dt, dtsq/dtcb of Main/mod_tendency.F90:
    614-615, the fatal check, the indices clamped to the boundary lines), slhadv_x4d (:425-470:
    bilinear outer rows, cubic inner rows, the cubic in y, the quasi-monotone clamp when
    iqmsl = 1, the dlowval test) and hdvg_x4d (:621-657).  Returns {species: tendency}."""
    psdota = _psc2psd_np(g, psa)
    rps = np.zeros_like(psdota)
    Jd, Id = g.box(g.jde1, g.jde2, g.ide1, g.ide2)
    g.put(rps, Jd, Id, 1.0 / g.at(psdota, Jd, Id))
    ua, va = u1 * rps * msfd, v1 * rps * msfd
    dx = rc.ds * 1000.0
    ddx = ddy = dx
    dtsq, dtcb = dt * dt, dt * dt * dt
    out = {n: np.zeros_like(q) for n, q in a2q.items()}

    def U(k, j, i):
        return ua[k, i - 1, g.wrap(np.array(j)) - 1]

    def Va(k, j, i):
        return va[k, i - 1, g.wrap(np.array(j)) - 1]

    def mx(j, i):
        return msfx[i - 1, g.wrap(np.array(j)) - 1]

    def md(j, i):
        return msfd[i - 1, g.wrap(np.array(j)) - 1]

    for k in range(rc.kz):
        for i in range(g.ici1, g.ici2 + 1):
            for j in range(g.jci1, g.jci2 + 1):
                uadvx = 0.25 * (U(k, j, i) + U(k, j, i + 1) + U(k, j + 1, i + 1) + U(k, j + 1, i)) / mx(j, i)
                uadxp1 = 0.25 * (U(k, j + 1, i) + U(k, j + 1, i + 1) + U(k, j + 2, i + 1) + U(k, j + 2, i)) / mx(j + 1, i)
                uadxm1 = 0.25 * (U(k, j, i) + U(k, j, i + 1) + U(k, j - 1, i + 1) + U(k, j - 1, i)) / mx(j - 1, i)
                vadvy = 0.25 * (Va(k, j, i) + Va(k, j, i + 1) + Va(k, j + 1, i + 1) + Va(k, j + 1, i)) / mx(j, i)
                vadyp1 = 0.25 * (Va(k, j, i + 1) + Va(k, j + 1, i + 1) + Va(k, j + 1, i + 2) + Va(k, j, i + 2)) / mx(j, i + 1)
                vadym1 = 0.25 * (Va(k, j, i) + Va(k, j, i - 1) + Va(k, j + 1, i) + Va(k, j + 1, i)) / mx(j, i - 1)
                ux = 0.5 * (uadxp1 - uadxm1) / ddx
                uxx = (uadxp1 - 2.0 * uadvx + uadxm1) / (ddx * ddx)
                xdis = -uadvx * dt + 0.5 * (dtsq * uadvx * ux) - (dtcb * uadvx) * (ux * ux + uadvx * uxx) / 6.0
                xn = xdis / ddx
                xnp = int(xn)
                assert abs(xnp) <= 1                              # else fatal('SLADVECTION')
                alfax = abs((xnp * ddx - xdis) / ddx)
                xsn = int(math.copysign(1.0, xn))
                xnd = j + xnp
                xm1 = xnd + xsn
                xm2 = xm1 + xsn
                xp1 = xnd - xsn
                if g.bl:
                    xnd, xm1, xm2, xp1 = (max(x, g.jce1) for x in (xnd, xm1, xm2, xp1))
                if g.br:
                    xnd, xm1, xm2, xp1 = (min(x, g.jce2) for x in (xnd, xm1, xm2, xp1))
                vy = 0.5 * (vadyp1 - vadym1) / ddy
                vyy = (vadyp1 - 2.0 * vadvy + vadym1) / (ddy * ddy)
                ydis = -vadvy * dt + 0.5 * (dtsq * vadvy * vy) - (dtcb * vadvy) * (vy * vy + vadvy * vyy) / 6.0
                yn = ydis / ddy
                ynp = int(yn)
                assert abs(ynp) <= 1
                betay = abs((ynp * ddy - ydis) / ddy)
                ysn = int(math.copysign(1.0, yn))
                ynd = i + ynp
                ym1 = ynd + ysn
                ym2 = ym1 + ysn
                yp1 = ynd - ysn
                ynd, ym1, ym2, yp1 = (min(max(y, g.ice1), g.ice2) for y in (ynd, ym1, ym2, yp1))
                alfm2 = -(alfax * (1.0 - alfax * alfax)) / 6.0
                alfm1 = (alfax * (1.0 + alfax) * (2.0 - alfax)) / 2.0
                alf0 = ((1.0 - alfax * alfax) * (2.0 - alfax)) / 2.0
                alfp1 = -(alfax * (1.0 - alfax) * (2.0 - alfax)) / 6.0
                betm2 = -(betay * (1.0 - betay * betay)) / 6.0
                betm1 = (betay * (1.0 + betay) * (2.0 - betay)) / 2.0
                bet0 = ((1.0 - betay * betay) * (2.0 - betay)) / 2.0
                betp1 = -(betay * (1.0 - betay) * (2.0 - betay)) / 6.0
                ucapf = (U(k, j + 1, i + 1) * md(j + 1, i + 1) + U(k, j + 1, i) * md(j + 1, i)) * 0.5
                ucapi = (U(k, j, i + 1) * md(j, i + 1) + U(k, j, i) * md(j, i)) * 0.5
                vcapf = (Va(k, j + 1, i + 1) * md(j + 1, i + 1) + Va(k, j, i + 1) * md(j, i + 1)) * 0.5
                vcapi = (Va(k, j + 1, i) * md(j + 1, i) + Va(k, j, i) * md(j, i)) * 0.5
                hdvg = ((ucapf - ucapi) / dx + (vcapf - vcapi) / dx) / (mx(j, i) * mx(j, i))
                for n, q in a2q.items():
                    def Q(jj, ii):
                        return q[k, ii - 1, g.wrap(np.array(jj)) - 1]
                    bl1 = alfax * Q(xm1, yp1) + (1.0 - alfax) * Q(xnd, yp1)
                    bl2 = alfax * Q(xm1, ym2) + (1.0 - alfax) * Q(xnd, ym2)
                    cb1 = alfm2 * Q(xm2, ynd) + alfm1 * Q(xm1, ynd) + alf0 * Q(xnd, ynd) + alfp1 * Q(xp1, ynd)
                    cb2 = alfm2 * Q(xm2, ym1) + alfm1 * Q(xm1, ym1) + alf0 * Q(xnd, ym1) + alfp1 * Q(xp1, ym1)
                    tbadp = betm2 * bl2 + betm1 * cb2 + bet0 * cb1 + betp1 * bl1
                    tsla = tbadp
                    if rc.iqmsl == 1:
                        four = (Q(xnd, ynd), Q(xnd, ym1), Q(xm1, ynd), Q(xm1, ym1))
                        tbmax, tbmin = max(four), min(four)
                        tsla = tbmax if tbadp > tbmax else (tbmin if tbadp < tbmin else tbadp)
                    ften = 0.0
                    if abs(tsla - Q(j, i)) > 1.0e-20:                # dlowval, Share/mod_constants.F90:68
                        ften = ften + (tsla - Q(j, i)) / dt
                    a1 = a1q[n][k, i - 1, j - 1]
                    tatot = a1 * hdvg if a1 > np.finfo(np.float64).eps else 0.0
                    out[n][k, i - 1, j - 1] = ften - tatot
    return out


@pytest.mark.parametrize("variant", [{}, {"iqmsl": 0}, {"band": True}], ids=["qmsl", "plain", "band"])
def test_semi_lagrangian_pass_matches_numpy_restatement(variant):
    """The qv / qc semi-Lagrangian terms of one tend (the oracle stopped right after the pass,
    probe 3) equal the NumPy trajcalc_x + slhadv_x4d + hdvg_x4d bit for bit."""
    variant = dict(variant)
    band = variant.pop("band", False)
    rc, data, st = _case(band=band, isladvec=1, **variant)
    o = _oracle(rc, data, st, probe=3)
    g = Grid(rc)
    s = {n: o.get(n) for n in ("ATM1_U", "ATM1_V", "PSA", "MSFX", "MSFD", "ATM1_QV", "ATM1_QC", "ATM2_QV", "ATM2_QC")}
    _, dt, _ = o.get_time()
    o.tend()
    want = _sladvection_np(g, rc, s["ATM1_U"], s["ATM1_V"], s["PSA"][0], s["MSFX"][0], s["MSFD"][0],
                           {"v": s["ATM2_QV"], "c": s["ATM2_QC"]}, {"v": s["ATM1_QV"], "c": s["ATM1_QC"]}, dt)
    J, I = g.box(g.jci1, g.jci2, g.ici1, g.ici2)
    for n in ("v", "c"):
        got = o.get_work("qdyn" + n)
        assert np.array_equal(g.at(got, J, I), g.at(want[n], J, I)), n
        assert np.abs(g.at(want[n], J, I)).max() > 0.0
