"""CPU tests: synthetic inputs, host-side init, the oracle restatement against the committed
fixtures, and oracle invariants.  No GPU needed."""
import json
import os

import numpy as np
import pytest

from regcm_amd.config import CONFIGS, STATE_FIELDS, set_nproc
from regcm_amd import icbc
from regcm_amd.vmodes import vmodes, spinit_constants

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "c1_oracle.json")


def _fp_match(arr, fp):
    flat = np.ascontiguousarray(arr).ravel()
    assert list(arr.shape) == fp["shape"]
    got = [float(flat[i]).hex() for i in fp["samples_idx"]]
    assert got == fp["samples"]
    assert float(np.sum(flat)) == fp["sum"]
    assert float(np.sum(np.abs(flat))) == fp["abssum"]


@pytest.fixture(scope="module")
def golden():
    with open(GOLDEN) as f:
        return json.load(f)


def test_syn_icbc_fingerprint(golden, c1_data):
    rc, data = c1_data
    for name, fp in golden["inputs"].items():
        _fp_match(data["state"][name], fp)
    for key, vals in golden["split"].items():
        assert [float(x).hex() for x in np.ravel(data["split"][key])] == vals


def test_vmodes_structure():
    """vmodes/spinit invariants (Main/mod_vmodes.F90:358-426, Main/mod_split.F90:86-175)."""
    for kz in (18, 23, 41):
        rc = dict(C1=CONFIGS["C1"], C2=CONFIGS["C2"])["C1" if kz == 18 else "C2"]
        sig = np.array(__import__("regcm_amd.config", fromlist=["SIGMA_TABLES"]).SIGMA_TABLES[kz])
        vm = vmodes(sig, 5.0, kz)
        hb = vm["hbar"]
        assert np.all(hb > 0) and np.all(np.diff(hb) <= 0)
        z = vm["zmatx"]
        ds = np.diff(sig)
        # vnorml: mass-weighted unit columns, largest component positive
        assert np.allclose(np.sum(ds[:, None] * z * z, axis=0), 1.0, atol=1e-12)
        assert np.all(z[np.argmax(np.abs(z), axis=0), np.arange(kz)] > 0)
        assert np.allclose(vm["zmatxr"] @ z, np.eye(kz), atol=1e-9)
        # tau z = z diag(hbar)
        assert np.allclose(vm["tau"] @ z, z * hb[None, :], rtol=1e-8, atol=1e-6 * hb[0])
    sp = spinit_constants(CONFIGS["C3"].sigma, 5.0, 23, 150.0, 2)
    assert list(sp["aam"]) == [4.0, 2.0]                     # m2 = 8 and 4 sub-steps
    assert list(sp["dtau"]) == [37.5, 75.0]


def test_set_nproc_rule():
    """set_nproc, Main/mpplib/mod_mppparam.F90:1152-1186."""
    assert set_nproc(1, 192, 192) == (1, 1)
    assert set_nproc(2, 192, 192) == (2, 1)
    assert set_nproc(4, 192, 192) == (2, 2)
    assert set_nproc(8, 192, 192) == (2, 4)
    assert set_nproc(8, 400, 100) == (4, 2)
    assert set_nproc(6, 60, 200) == (1, 6)


def test_oracle_matches_golden(golden, c1_data):
    from oracle.oracle import OracleCore
    rc, data = c1_data
    o = OracleCore(rc, data["split"])
    o.put_state(data["state"])
    o.bdyval()
    done = 0
    for n in (1, 10, 40):
        o.step(n - done)
        done = n
        ref = golden["steps"][str(n)]
        for name in STATE_FIELDS:
            _fp_match(o.get(name), ref[name])
        assert list(o.get_time()) == ref["_time"]
        assert [float(x).hex() for x in o.diagnostics()[:2]] == ref["_diag"]


def test_oracle_leapfrog_schedule(c1_data):
    """First two steps use dt = dtsec, then 2*dtsec (Main/mod_tendency.F90:608-616);
    xbctime advances by dtsec per bdyval (Main/mod_bdycod.F90:2566)."""
    from oracle.oracle import OracleCore
    rc, data = c1_data
    o = OracleCore(rc, data["split"])
    o.put_state(data["state"])
    o.bdyval()
    assert o.get_time() == (0, rc.dt, rc.dt)
    o.step(1)
    assert o.get_time() == (1, rc.dt, 2 * rc.dt)
    o.step(1)
    assert o.get_time() == (2, 2 * rc.dt, 3 * rc.dt)


def test_oracle_stability_and_mass(c1_data):
    """100 steps of the restatement stay finite and bounded; boundary-forced p* stays in range."""
    from oracle.oracle import OracleCore
    rc, data = c1_data
    o = OracleCore(rc, data["split"])
    o.put_state(data["state"])
    o.bdyval()
    o.step(100)
    psa = o.get("PSA")[0, : rc.iy - 1, : rc.jx - 1]
    assert np.all(np.isfinite(psa)) and psa.min() > 50.0 and psa.max() < 110.0
    t = o.get("ATM1_T")[:, : rc.iy - 1, : rc.jx - 1] / psa[None]
    assert t.min() > 150.0 and t.max() < 340.0
    qv = o.get("ATM1_QV")[:, 1: rc.iy - 2, 1: rc.jx - 2]
    assert qv.min() >= 0.0


def test_oracle_zero_state_fixed_point():
    """A resting, horizontally uniform isothermal atmosphere with matching boundaries and no
    terrain is a fixed point of advection/diffusion: winds stay zero after a step."""
    from oracle.oracle import OracleCore
    rc = CONFIGS["C1"]
    data = icbc.generate(rc)
    st = data["state"]
    kz, iy, jx = rc.kz, rc.iy, rc.jx
    ps = np.full((1, iy, jx), 95.0)
    for lvl in ("ATM1", "ATM2"):
        st[f"{lvl}_U"][:] = 0.0
        st[f"{lvl}_V"][:] = 0.0
        st[f"{lvl}_T"][:] = 260.0 * 95.0
        st[f"{lvl}_QV"][:] = 0.0
        st[f"{lvl}_QC"][:] = 0.0
    for n in ("XUB", "XVB", "XQB"):
        st[n + "_B0"][:] = 0.0
        st[n + "_BT"][:] = 0.0
    st["XTB_B0"][:] = 260.0 * 95.0
    st["XTB_BT"][:] = 0.0
    st["XPSB_B0"][:] = 95.0
    st["XPSB_BT"][:] = 0.0
    st["PSA"][:] = ps
    st["PSB"][:] = ps
    st["HT"][:] = 0.0
    st["CORIOL"][:] = 0.0
    st["MSFX"][:] = 1.0
    st["MSFD"][:] = 1.0
    st["DSTOR"], st["HSTOR"] = icbc.spinit_storage(rc, data["split"], st)
    o = OracleCore(rc, data["split"])
    o.put_state(st)
    o.bdyval()
    o.step(2)
    u = o.get("ATM1_U")
    assert np.max(np.abs(u)) < 1e-9


def test_oracle_option_variants_change_the_solution(c1_data):
    """Each implemented namelist variant runs stably and actually changes the state."""
    import dataclasses
    from oracle.oracle import OracleCore
    rc, data = c1_data
    base = OracleCore(rc, data["split"])
    base.put_state(data["state"])
    base.bdyval()
    base.step(10)
    ref = base.get("ATM1_T")
    refq = base.get("ATM1_QV")
    for variant in ({"iboudy": 4}, {"iboudy": 3}, {"iboudy": 2}, {"ipgf": 1}, {"idiffu": 2}, {"idiffu": 3}, {"isladvec": 1},
                    {"upstream_mode": 0}, {"stability_enhance": 0}, {"diffu_hgtf": 0}):
        rcv = dataclasses.replace(rc, **variant)
        o = OracleCore(rcv, data["split"])
        o.put_state(data["state"])
        o.bdyval()
        o.step(10)
        t, q = o.get("ATM1_T"), o.get("ATM1_QV")
        assert np.isfinite(t).all() and np.isfinite(q).all(), variant
        assert not (np.array_equal(t, ref) and np.array_equal(q, refq)), variant


# ---- non-hydrostatic core (idynamic = 2) ---------------------------------------------------

def _nh_oracle(rest=False, **kw):
    from oracle.oracle import OracleCore
    rc = CONFIGS["N1"]
    data = icbc.generate_nh(rc, rest=rest, **kw)
    o = OracleCore(rc, data["split"])
    o.put_state(data["state"])
    o.bdyval()
    return rc, data, o


def test_nh_reference_state_consistency():
    """nhbase (Share/mod_nhinterp.F90:74-106): hydrostatic, monotone reference profiles;
    init_sound short-step limit from max t0; istep rule of sound (:201-205)."""
    from regcm_amd import nhbase
    rc = CONFIGS["N1"]
    d = icbc.generate_nh(rc)
    st = d["state"]
    ce = (slice(None), slice(0, rc.iy - 1), slice(0, rc.jx - 1))
    pr, t0, rho, z = st["ATM0_PR"][ce], st["ATM0_T"][ce], st["ATM0_RHO"][ce], st["ATM0_Z"][ce]
    assert np.all(np.diff(pr, axis=0) > 0) and np.all(np.diff(z, axis=0) < 0)
    assert np.allclose(rho * 287.0 * t0 / pr, 1.0, atol=2e-3)
    assert np.all(t0 >= nhbase.TISO)
    # hydrostatic: dp/dz = -rho g between half levels (centred estimate), below the levels
    # where t0 is clamped to tiso (z0 keeps the unclamped log-linear profile there); z0
    # integrates from the local surface pressure while t0 uses p0, a ~1 % offset in the
    # reference's own formulas
    dpdz = (pr[1:] - pr[:-1]) / (z[1:] - z[:-1])
    rhom = 0.5 * (rho[1:] + rho[:-1])
    warm = (t0[1:] > nhbase.TISO + 1.0) & (t0[:-1] > nhbase.TISO + 1.0)
    assert warm.sum() > warm.size // 2
    assert np.allclose((dpdz / (-rhom * 9.80665))[warm], 1.0, atol=3e-2)
    assert 7.0 < d["split"]["nh_dtsmax"] < 9.0
    assert nhbase.acoustic_substeps(rc, d["split"]["nh_dtsmax"], 2 * rc.dt, 5) == 4
    assert nhbase.acoustic_substeps(rc, d["split"]["nh_dtsmax"], rc.dt, 0) == 2


def test_nh_oracle_rest_state_stays_at_rest():
    """A resting atmosphere equal to the reference state over flat terrain is a fixed point
    of the NH step up to the minqq floor: buoyancy, acoustic pressure gradient and the
    semi-implicit w/pp solve balance (Main/mod_sound.F90, Main/mod_tendency.F90:1639-1671)."""
    rc, data, o = _nh_oracle(rest=True)
    o.step(10)
    ps = o.get("PSA")[0][None, :-1, :-1]
    for n, lim in (("ATM1_U", 1e-4), ("ATM1_V", 1e-4), ("ATM1_W", 1e-4), ("ATM1_PP", 0.05)):
        assert np.abs(o.get(n)[:, :-1, :-1] / ps).max() < lim, n
    t = o.get("ATM1_T")[:, :-1, :-1] / ps
    assert np.abs(t - data["state"]["ATM0_T"][:, :-1, :-1]).max() < 1e-4


def test_nh_oracle_stable_and_active():
    """N1 at dt = 3 ds: 40 steps without a CFL stop, bounded w and pp; every NH prognostic
    moves, p* stays constant (the NH core keeps p* = ps0, Main/mod_tendency.F90:836-848)."""
    rc, data, o = _nh_oracle()
    st = data["state"]
    o.step(40)
    assert o.get_time()[0] == 40
    ps = o.get("PSA")[0]
    assert np.array_equal(ps, st["PSA"][0])
    psn = ps[None, :-1, :-1]
    w = o.get("ATM1_W")[:, :-1, :-1] / psn
    pp = o.get("ATM1_PP")[:, :-1, :-1] / psn
    assert np.all(np.isfinite(w)) and np.abs(w).max() < 5.0
    assert np.abs(pp - st["ATM1_PP"][:, :-1, :-1] / psn).max() < 2000.0
    for n in ("ATM1_U", "ATM1_V", "ATM1_T", "ATM1_QV", "ATM1_PP", "ATM1_W", "ATM2_W"):
        assert not np.array_equal(o.get(n), st[n]), n


def test_oracle_physics_seam_sums_and_slices(c1_data):
    """Physics coupling seam on the restatement: zero pc_physic tendencies leave the step
    bit-identical, non-zero ones act linearly at first order, and the mkslice export obeys
    the reference's own identities (za = mid-point of zq, dzq = zq difference, tv3d from
    tb3d and the moistures, rhb3d inside [rhmin, rhmax])."""
    from oracle.oracle import OracleCore
    from regcm_amd.config import PHY_FIELDS, STATE_FIELDS
    rc, data = c1_data
    runs = []
    for amp in (0.0, 1e-3, 2e-3):
        o = OracleCore(rc, data["split"])
        o.put_state(data["state"])
        o.bdyval()
        if amp or len(runs) == 0:
            for name in PHY_FIELDS:
                o.put(name, np.full((rc.kz, rc.iy, rc.jx), amp if name in ("TPHY", "UPHY") else 0.0))
        o.tend()
        runs.append(o)
    base = OracleCore(rc, data["split"])
    base.put_state(data["state"])
    base.bdyval()
    base.tend()
    for name in STATE_FIELDS:
        assert np.array_equal(runs[0].get(name), base.get(name)), name
    # one tend: the forecast is linear in the tendency (t: dt * tphy exactly up to rounding)
    t0, t1, t2 = (r.get("ATM1_T")[:, 1:rc.iy - 2, 1:rc.jx - 2] for r in runs)
    d1, d2 = t1 - t0, t2 - t0
    assert np.max(np.abs(d1)) > 0
    assert np.allclose(d2, 2.0 * d1, rtol=1e-6, atol=1e-12)
    o = runs[0]
    zq, za, dzq = o.get("ATMS_ZQ"), o.get("ATMS_ZA"), o.get("ATMS_DZQ")
    sl = (slice(None), slice(0, rc.iy - 1), slice(0, rc.jx - 1))
    assert np.allclose(za[sl], 0.5 * (zq[:-1][sl] + zq[1:][sl]), rtol=1e-14, atol=0)
    assert np.allclose(dzq[sl], zq[:-1][sl] - zq[1:][sl], rtol=1e-14, atol=0)
    assert np.all(dzq[sl] > 0)
    tb, qv, qc, tv = (o.get(n) for n in ("ATMS_TB3D", "ATMS_QVB3D", "ATMS_QCB3D", "ATMS_TV3D"))
    from regcm_amd import constants as C
    assert np.allclose(tv[sl], tb[sl] * (1.0 + C.ep1 * qv[sl] - qc[sl]), rtol=1e-15)
    rh = o.get("ATMS_RHB3D")[:, 1:rc.iy - 2, 1:rc.jx - 2]
    assert rh.min() >= rc.rhmin and rh.max() <= rc.rhmax


def test_oracle_bdyin_matches_numpy_restatement(c1_data):
    """orc_bdyin against an independent NumPy restatement of bdyin (Main/mod_bdycod.F90:
    654-889): p* = ps*d_r10 - ptop, psc2psd, couple, timeint -- bit for bit."""
    from oracle.oracle import OracleCore
    from regcm_amd import icbc
    from test_bdyin_gpu import records
    rc, data = c1_data
    recs = records(rc, data, False)
    o = OracleCore(rc, data["split"])
    o.put_state(data["state"])
    for rec in recs[:2]:
        for name, a in rec.items():
            o.put(name, a)
        o.bdyin()
    iy, jx = rc.iy, rc.jx
    ce = (slice(None), slice(0, iy - 1), slice(0, jx - 1))

    def coupled(rec):
        ps = np.zeros((iy, jx))
        ps[:iy - 1, :jx - 1] = rec["XPSB_B1"][0][:iy - 1, :jx - 1] * 0.1 - rc.ptop
        pd = icbc.psc2psd_global(ps)
        out = {"U": rec["XUB_B1"] * pd[None], "V": rec["XVB_B1"] * pd[None], "P": ps[None]}
        for n, f in (("T", "XTB_B1"), ("Q", "XQB_B1")):
            a = np.zeros_like(rec[f])
            a[ce] = (rec[f] * ps[None])[ce]
            out[n] = a
        return out

    b0, b1 = coupled(recs[0]), coupled(recs[1])
    rdt = 1.0 / rc.dtbdys
    for n, f in (("U", "XUB"), ("V", "XVB"), ("T", "XTB"), ("Q", "XQB"), ("P", "XPSB")):
        assert np.array_equal(o.get(f + "_B0"), b0[n]), f
        assert np.array_equal(o.get(f + "_BT"), (b1[n] - b0[n]) * rdt), f
    assert o.get_time()[2] == 0.0


def test_nh_oracle_sladvection_changes_moisture():
    """isladvec = 1 on the non-hydrostatic core: the semi-Lagrangian qv/qc advection replaces
    the flux form (Main/mod_tendency.F90:1361-1380), stays finite, and changes only moisture
    in the first step (temperature and winds see qv only through later steps)."""
    import dataclasses
    from oracle.oracle import OracleCore
    rc, data, base = _nh_oracle()
    o = OracleCore(dataclasses.replace(rc, isladvec=1), data["split"])
    o.put_state(data["state"])
    o.bdyval()
    base.step(1)
    o.step(1)
    assert np.isfinite(o.get("ATM1_QV")).all()
    assert not np.array_equal(o.get("ATM1_QV"), base.get("ATM1_QV"))
    assert np.array_equal(o.get("ATM1_U"), base.get("ATM1_U"))
    o.step(2)
    assert np.isfinite(o.get("ATM1_T")).all() and np.isfinite(o.get("ATM1_PP")).all()


def test_oracle_tke_bounds_and_independence(c1_data):
    """ibltyp = 2: the oracle's TKE stays finite and >= tkemin on every cross point it owns,
    its boundary lines follow bdyval's inflow/outflow rule (tkemin at level 1), and the rest of
    the state is bit-identical to the run without TKE (nothing in the dyn step reads it)."""
    import dataclasses
    from oracle.oracle import OracleCore
    rc0, data = c1_data
    rc = dataclasses.replace(rc0, ibltyp=2)
    o = OracleCore(rc, data["split"])
    o.put_state(data["state"])
    for name, a in icbc.tke_state(rc).items():
        o.put(name, a)
    o.bdyval()
    b = OracleCore(rc0, data["split"])
    b.put_state(data["state"])
    b.bdyval()
    o.step(4)
    b.step(4)
    t = o.get("ATM1_TKE")[:, : rc.iy - 1, : rc.jx - 1]
    assert np.isfinite(t).all() and t.min() >= rc.tkemin
    assert np.all(t[0, 0, :] == rc.tkemin) and np.all(t[0, :, 0] == rc.tkemin)
    for name in ("ATM1_U", "ATM1_T", "ATM1_QV", "PSA"):
        assert np.array_equal(o.get(name), b.get(name)), name


def _nh_tend_restatement(extra=(), cloud=False):
    """One oracle tend of the N1 NH case with no diffusion (ckh = adyndif = 0, so xkc = 0) and
    no Rayleigh damping, plus the NumPy restatement's shared pieces: the interior points
    outside the relaxation band, the horizontal wind averages of start_advect, qdot of
    compute_omega NH (Main/mod_tendency.F90:1157-1191) and the mass divergence cr."""
    import dataclasses
    from oracle.oracle import OracleCore
    rc = dataclasses.replace(CONFIGS["N1"], ckh=0.0, adyndif=0.0, ifrayd=0)
    data = icbc.generate_nh(rc)
    o = OracleCore(rc, data["split"])
    state = dict(data["state"])
    if cloud:       # a cloud layer: qc = 1 % of qv on levels 4..12, none elsewhere (both vadv4d branches)
        for a1, a2 in (("ATM1_QC", "ATM1_QV"), ("ATM2_QC", "ATM2_QV")):
            qc = np.zeros_like(state[a2])
            qc[3:12] = 0.01 * state[a2][3:12]
            state[a1] = qc
    o.put_state(state)
    o.bdyval()
    g = {n: o.get(n) for n in ("ATM1_U", "ATM1_V", "ATM1_T", "ATM1_PP", "ATM1_W", "PSA", "MSFX", "MSFD",
                                "ATM0_PR", "ATM0_PS", "ATM0_RHOF", "DPSDXM", "DPSDYM") + tuple(extra)}
    o.tend()
    r = {"rc": rc, "g": g, "out": {n: o.get(n) for n in ("TTEN", "QVTEN", "QCTEN", "QDOT", "UTEN", "VTEN")},
         "dtsmax": data["split"]["nh_dtsmax"]}
    o.close()
    kz, nsp = rc.kz, rc.nspgx
    sig = rc.sigma
    hsig = (sig[1:] + sig[:-1]) * 0.5
    dsig = sig[1:] - sig[:-1]
    twt1 = np.zeros(kz + 1); twt2 = np.zeros(kz + 1)
    for k in range(2, kz + 1):                                   # Main/mod_params.F90:2212-2213
        twt1[k] = (sig[k - 1] - hsig[k - 2]) / (hsig[k - 1] - hsig[k - 2])
        twt2[k] = 1.0 - twt1[k]
    dx = rc.ds * 1000.0
    # interior cross points outside the relaxation band (1-based global j, i)
    J = np.arange(nsp + 1, rc.jx - nsp)
    I = np.arange(nsp + 1, rc.iy - nsp)

    def at(a, dj=0, di=0):                                      # a[k][i][j] at (J+dj, I+di)
        return a[:, (I + di - 1)[:, None], (J + dj - 1)[None, :]]

    ps = at(g["PSA"])[0]
    msfx, msfd = at(g["MSFX"])[0], g["MSFD"]
    umc = g["ATM1_U"] * msfd[0][None]
    vmc = g["ATM1_V"] * msfd[0][None]
    # compute_omega NH: qdot from w and the reference-p* slopes (decoupled dot winds umd)
    pa = g["PSA"][0]
    psd = np.zeros_like(pa)
    psd[1:, 1:] = (pa[1:, 1:] + pa[:-1, 1:] + pa[1:, :-1] + pa[:-1, :-1]) * 0.25
    rpsd = np.divide(1.0, psd, out=np.zeros_like(psd), where=psd > 0)
    umd = g["ATM1_U"] * rpsd[None] * msfd[0][None]
    vmd = g["ATM1_V"] * rpsd[None] * msfd[0][None]
    ucc = at(umd) + at(umd, 0, 1) + at(umd, 1, 0) + at(umd, 1, 1)
    vcc = at(vmd) + at(vmd, 0, 1) + at(vmd, 1, 0) + at(vmd, 1, 1)
    pinv = np.divide(1.0, g["PSA"][0], out=np.zeros_like(g["PSA"][0]), where=g["PSA"][0] > 0)
    xw = g["ATM1_W"] * pinv[None]
    egrav = 9.80665
    qdot = np.zeros((kz + 1,) + ps.shape)
    for k in range(2, kz + 1):
        qdot[k - 1] = (-at(g["ATM0_RHOF"])[k - 1] * egrav * at(xw)[k - 1] / at(g["ATM0_PS"])[0] -
                       sig[k - 1] * (at(g["DPSDXM"])[0] * (twt1[k] * ucc[k - 1] + twt2[k] * ucc[k - 2]) +
                                     at(g["DPSDYM"])[0] * (twt1[k] * vcc[k - 1] + twt2[k] * vcc[k - 2])))
    a = at(umc, 1, 1) + at(umc, 1, 0) - at(umc, 0, 1) - at(umc)
    b = at(vmc, 1, 1) + at(vmc, 0, 1) - at(vmc, 1, 0) - at(vmc)
    dummy = 1.0 / (2.0 * dx * msfx * msfx)
    cr = (a + b) * dummy[None] + (qdot[1:] - qdot[:-1]) * ps[None] / dsig[:, None, None]
    # start_advect's wind averages (Main/mod_advection.F90:114-119) and hadv's f1, f2, xmapf
    u1 = at(umc, 0, 1) + at(umc)
    u2 = at(umc, 1, 1) + at(umc, 1, 0)
    v1 = at(vmc, 1, 0) + at(vmc)
    v2 = at(vmc, 1, 1) + at(vmc, 0, 1)
    ul = rc.uoffc * 0.5 * rc.dt / dx                             # Main/mod_advection.F90:106
    f1 = 0.5 * ul * (u2 + u1) / ps[None]
    f2 = 0.5 * ul * (v2 + v1) / ps[None]
    xmsf = 1.0 / (msfx * msfx * (4.0 * dx))                      # Main/mod_params.F90:1993-2001

    def hadv(c, w, e, s_, n):                                    # the upstream flux form
        fx1 = (1.0 + f1) * w + (1.0 - f1) * c
        fx2 = (1.0 + f1) * c + (1.0 - f1) * e
        fy1 = (1.0 + f2) * s_ + (1.0 - f2) * c
        fy2 = (1.0 + f2) * c + (1.0 - f2) * n
        return -xmsf[None] * (u2 * fx2 - u1 * fx1 + v2 * fy2 - v1 * fy1)

    r.update(kz=kz, sig=sig, hsig=hsig, dsig=dsig, twt1=twt1, twt2=twt2, at=at, ps=ps, pinv=pinv,
             qdot=qdot, cr=cr, hadv=hadv)
    return r


def test_nh_theta_advection_matches_numpy_restatement():
    """The NH temperature tendency of the restatement against an independent NumPy
    restatement of the reference's ithadv = 1 path (Main/mod_tendency.F90:98,128-129: ithadv
    stays 1 for idynamic = 2; :1347-1356, 1594-1600): th = atmx%t*(p00/atm1%pr)**rovcp,
    tha = th*p*, thten = hadvt(th) + vadv3d ind 0 (tha) + th*cr, tdyn = atm1%t*thten/tha.
    Also restates qdot of compute_omega NH (:1157-1191).  With ckh = adyndif = 0 (xkc = 0,
    no diffusion) and ifrayd = 0, tten at points outside the relaxation band is exactly that
    tdyn.  The comparison is at 1e-13 relative (numpy and the C restatement both call libm
    pow/division in the same order, so it is usually bit-exact)."""
    r = _nh_tend_restatement()
    rc, g, at, ps, kz = r["rc"], r["g"], r["at"], r["ps"], r["kz"]
    qdot, cr, dsig, twt1, twt2 = r["qdot"], r["cr"], r["dsig"], r["twt1"], r["twt2"]
    np.testing.assert_allclose(qdot, at(r["out"]["QDOT"]), rtol=1e-13, atol=1e-13 * np.abs(qdot).max())
    from regcm_amd import constants as C
    rgas = C.rgas
    cpd = 3.5 * rgas
    rovcp = rgas * (1.0 / cpd)                                   # Share/mod_constants.F90:183-184
    rps = r["pinv"]
    with np.errstate(divide="ignore", invalid="ignore"):
        thf = (g["ATM1_T"] * rps[None]) * (1.0e5 / (g["ATM0_PR"] + g["ATM1_PP"] * rps[None])) ** rovcp
    th, thw, the, ths, thn = at(thf), at(thf, -1), at(thf, 1), at(thf, 0, -1), at(thf, 0, 1)
    fg = r["hadv"](th, thw, the, ths, thn)
    for (p, m) in ((thn, ths), (the, thw)):                      # hadvt limiter :359-386
        big = np.abs(p + m - 2.0 * th) / ps[None] > rc.t_extrema
        fg = np.where(big & (th > p) & (th > m), np.minimum(fg, 0.0), fg)
        fg = np.where(big & (th < p) & (th < m), np.maximum(fg, 0.0), fg)
    tha = th * ps[None]
    thten = 0.0 + fg
    for k in range(2, kz + 1):                                   # vadv3d ind = 0, nk = kz
        fx = qdot[k - 1] * (twt1[k] * tha[k - 1] + twt2[k] * tha[k - 2])
        thten[k - 2] = thten[k - 2] - fx * (1.0 / dsig[k - 2])
        thten[k - 1] = thten[k - 1] + fx * (1.0 / dsig[k - 1])
    thten = thten + th * cr
    tdyn = at(g["ATM1_T"]) * thten / tha
    got = at(r["out"]["TTEN"])
    assert np.abs(tdyn).max() > 1e-6
    np.testing.assert_allclose(got, tdyn, rtol=1e-12, atol=1e-13 * np.abs(tdyn).max())


def test_nh_moisture_advection_matches_numpy_restatement():
    """The NH qv and qc tendencies against an independent NumPy restatement of the reference
    (no diffusion, no Rayleigh damping, points outside the band, as above): qv = hadvqv of
    atmx%qx (upstream form with the q_rel_extrema limiter, Main/mod_advection.F90:517-603) +
    vadvqv of atm1%qx (the qcon power form, :811-836) + atmx%qx*cr (Main/mod_tendency.F90:1616);
    qc = hadvqx (:607-662) + vadv4d ind 1 (the upwind-thresholded twt form, :873-894) +
    atmx%qx*cr, with atmx%qx = max(atm1%qx/p*, minqq) for qv and max(atm1%qx/p*, 0) for qc
    (decouple).  minqq = 1e-8, dlowval = 1e-20 (Share/mod_constants.F90:57, 68)."""
    r = _nh_tend_restatement(extra=("ATM1_QV", "ATM1_QC"), cloud=True)
    rc, g, at, ps, kz = r["rc"], r["g"], r["at"], r["ps"], r["kz"]
    qdot, cr, dsig, sig, hsig = r["qdot"], r["cr"], r["dsig"], r["sig"], r["hsig"]
    twt1, twt2 = r["twt1"], r["twt2"]
    minqq, dlowval = 1.0e-8, 1.0e-20
    xds = 1.0 / dsig
    qcon = np.zeros(kz + 1)
    for k in range(2, kz + 1):                                   # Main/mod_params.F90:2214
        qcon[k] = (sig[k - 1] - hsig[k - 1]) / (hsig[k - 2] - hsig[k - 1])
    rps = r["pinv"]
    for name, clip in (("ATM1_QV", minqq), ("ATM1_QC", 0.0)):
        q1 = g[name]
        xq = np.maximum(q1 * rps[None], clip)
        c, w, e, s_, n = at(xq), at(xq, -1), at(xq, 1), at(xq, 0, -1), at(xq, 0, 1)
        fg = r["hadv"](c, w, e, s_, n)
        if name == "ATM1_QV":                   # hadvqv limiter :569-596 (stability_enhance on)
            den = np.maximum(c, dlowval)
            for (p, m) in ((n, s_), (e, w)):
                big = np.abs(p + m - 2.0 * c) / den > rc.q_rel_extrema
                fg = np.where(big & (c > p) & (c > m), np.minimum(fg, 0.0), fg)
                fg = np.where(big & (c < p) & (c < m), np.maximum(fg, 0.0), fg)
        ten = 0.0 + fg
        f = at(q1)
        for k in range(2, kz + 1):
            fk, fkm, svv = f[k - 1], f[k - 2], qdot[k - 1]
            if name == "ATM1_QV":                                # vadvqv
                ok = (fk > minqq * ps) & (fkm > minqq * ps)
                with np.errstate(divide="ignore", invalid="ignore"):
                    fgk = np.where(ok, fk * (fkm / fk) ** qcon[k], 0.0)
                flux = svv * fgk
            else:                                                # vadv4d ind = 1
                thr = minqq * minqq * ps
                ok = np.where(svv > 0.0, fkm > thr, fk > thr)
                flux = np.where(ok, svv * (twt1[k] * fk + twt2[k] * fkm), 0.0)
            ten[k - 2] = ten[k - 2] - flux * xds[k - 2]
            ten[k - 1] = ten[k - 1] + flux * xds[k - 1]
        ten = ten + c * cr
        got = at(r["out"]["QVTEN" if name == "ATM1_QV" else "QCTEN"])
        assert np.abs(ten).max() > 0.0
        np.testing.assert_allclose(got, ten, rtol=1e-11, atol=1e-12 * np.abs(ten).max(), err_msg=name)


def test_nh_wind_tendency_matches_numpy_restatement():
    """The NH u, v tendencies of the first step against an independent NumPy restatement of
    the reference (no diffusion, no Rayleigh damping, dot points outside the band): hadvuv's
    NH upstream branch of atmx%ud, vd with the divergence term (Main/mod_advection.F90:235-264;
    dmapf = 1/(msfd^2 16 dx), Main/mod_params.F90:1996), vadvuv of atmx%uc, vc (:271-303), the NH curvature and
    Coriolis terms (Main/mod_tendency.F90:1839-1879), the decoupling by 1/psdota (:466-499)
    and sound's scaling by the acoustic step dts = dt/istep (Main/mod_sound.F90:229-245;
    istep = max(int(dt/dtsmax), 2) on the first step).  Shifted whole-domain arrays; only
    the interior is compared."""
    r = _nh_tend_restatement(extra=("CORIOL", "EF", "DDX", "DDY", "DMDX", "DMDY"))
    rc, g, kz = r["rc"], r["g"], r["kz"]
    sig, dsig, twt1, twt2 = r["sig"], r["dsig"], r["twt1"], r["twt2"]
    dx = rc.ds * 1000.0
    ul = rc.uoffc * 0.5 * rc.dt / dx
    xds = 1.0 / dsig

    def sh(a, dj, di):                                           # sh(a)[k, i, j] = a[k, i+di, j+dj]
        return np.roll(a, shift=(-di, -dj), axis=(-2, -1))

    u1, v1, w1 = g["ATM1_U"], g["ATM1_V"], g["ATM1_W"]
    msfd, msfx = g["MSFD"][0], g["MSFX"][0]
    pa = g["PSA"][0]
    psd = np.zeros_like(pa)
    psd[1:, 1:] = (pa[1:, 1:] + pa[:-1, 1:] + pa[1:, :-1] + pa[:-1, :-1]) * 0.25
    rpsd = np.divide(1.0, psd, out=np.zeros_like(psd), where=psd > 0)
    pinv = np.divide(1.0, pa, out=np.zeros_like(pa), where=pa > 0)
    umc, vmc = u1 * msfd, v1 * msfd
    ud, vd = u1 * rpsd, v1 * rpsd
    umd, vmd = ud * msfd, vd * msfd
    # compute_omega NH over the whole domain (cross point (j, i): dots j..j+1, i..i+1)
    ucc = umd + sh(umd, 0, 1) + sh(umd, 1, 0) + sh(umd, 1, 1)
    vcc = vmd + sh(vmd, 0, 1) + sh(vmd, 1, 0) + sh(vmd, 1, 1)
    qdot = np.zeros_like(w1)
    with np.errstate(divide="ignore", invalid="ignore"):
        for k in range(2, kz + 1):
            qdot[k - 1] = (-g["ATM0_RHOF"][k - 1] * 9.80665 * (w1[k - 1] * pinv) / g["ATM0_PS"][0] -
                           sig[k - 1] * (g["DPSDXM"][0] * (twt1[k] * ucc[k - 1] + twt2[k] * ucc[k - 2]) +
                                         g["DPSDYM"][0] * (twt1[k] * vcc[k - 1] + twt2[k] * vcc[k - 2])))
        a = sh(umc, 1, 1) + sh(umc, 1, 0) - sh(umc, 0, 1) - umc
        b = sh(vmc, 1, 1) + sh(vmc, 0, 1) - sh(vmc, 1, 0) - vmc
        cr = (a + b) / (2.0 * dx * msfx * msfx) + (qdot[1:] - qdot[:-1]) * pa / dsig[:, None, None]
        dm = 1.0 / (msfd * msfd * 16.0 * dx)
    # hadvuv, NH upstream branch
    divd = 0.25 * (cr + sh(cr, 0, -1) + sh(cr, -1, 0) + sh(cr, -1, -1))
    ucmona = sh(umc, 0, 1) + 2.0 * umc + sh(umc, 0, -1)
    ucmonb = sh(umc, 1, 1) + 2.0 * sh(umc, 1, 0) + sh(umc, 1, -1)
    ucmonc = sh(umc, -1, 1) + 2.0 * sh(umc, -1, 0) + sh(umc, -1, -1)
    vcmona = sh(vmc, 1, 0) + 2.0 * vmc + sh(vmc, -1, 0)
    vcmonb = sh(vmc, 1, 1) + 2.0 * sh(vmc, 0, 1) + sh(vmc, -1, 1)
    vcmonc = sh(vmc, 1, -1) + 2.0 * sh(vmc, 0, -1) + sh(vmc, -1, -1)
    diag = divd - dm * ((ucmonb - ucmonc) + (vcmonb - vcmonc))
    ff1, ff2 = ul * (sh(ud, 1, 0) + ud), ul * (sh(ud, -1, 0) + ud)
    ff3, ff4 = ul * (sh(vd, 0, 1) + vd), ul * (sh(vd, 0, -1) + vd)
    ucb = (1.0 + ff1) * ucmona + (1.0 - ff1) * ucmonb
    ucc_ = (1.0 + ff2) * ucmonc + (1.0 - ff2) * ucmona
    vcb = (1.0 + ff3) * vcmona + (1.0 - ff3) * vcmonb
    vcc_ = (1.0 + ff4) * vcmonc + (1.0 - ff4) * vcmona
    udyn = ud * diag - dm * (sh(ud, 1, 0) * ucb - sh(ud, -1, 0) * ucc_ + sh(ud, 0, 1) * vcb - sh(ud, 0, -1) * vcc_)
    vdyn = vd * diag - dm * (sh(vd, 1, 0) * ucb - sh(vd, -1, 0) * ucc_ + sh(vd, 0, 1) * vcb - sh(vd, 0, -1) * vcc_)
    # vadvuv of the coupled winds atmx%uc, vc = atm1 u, v (Main/mod_tendency.F90:1304)
    for k in range(2, kz + 1):
        qq = 0.25 * (qdot[k - 1] + sh(qdot, 0, -1)[k - 1] + sh(qdot, -1, 0)[k - 1] + sh(qdot, -1, -1)[k - 1])
        uu = qq * (twt1[k] * u1[k - 1] + twt2[k] * u1[k - 2])
        vv = qq * (twt1[k] * v1[k - 1] + twt2[k] * v1[k - 2])
        udyn[k - 2] = udyn[k - 2] - uu * xds[k - 2]
        udyn[k - 1] = udyn[k - 1] + uu * xds[k - 1]
        vdyn[k - 2] = vdyn[k - 2] - vv * xds[k - 2]
        vdyn[k - 1] = vdyn[k - 1] + vv * xds[k - 1]
    # curvature NH
    wad = 0.125 * (sh(w1, -1, -1) + sh(w1, -1, 0) + sh(w1, 0, -1) + w1)
    wabar = wad[:-1] + wad[1:]
    amfac = wabar * rpsd * (1.0 / 6.371229e6)
    duv = u1 * g["DMDY"][0] - v1 * g["DMDX"][0]
    cor, ef = g["CORIOL"][0], g["EF"][0]
    udyn = udyn + cor * v1 - ef * g["DDX"][0] * wabar + vmd * duv - u1 * amfac
    vdyn = vdyn - cor * u1 + ef * g["DDY"][0] * wabar - umd * duv - v1 * amfac
    istep = max(int(rc.dt / r["dtsmax"]), 2)
    dts = rc.dt / istep
    nsp = rc.nspgx
    J = np.arange(nsp + 2, rc.jx - nsp)                          # dot points off the band
    I = np.arange(nsp + 2, rc.iy - nsp)
    sl = (slice(None), (I - 1)[:, None], (J - 1)[None, :])
    for name, dyn in (("UTEN", udyn), ("VTEN", vdyn)):
        want = (dyn * rpsd * dts)[sl]
        got = r["out"][name][sl]
        assert np.abs(want).max() > 0.0
        np.testing.assert_allclose(got, want, rtol=1e-11, atol=1e-12 * np.abs(want).max(), err_msg=name)


def _cross_band(rc):
    """{(j, i): ibnd} of the cross-point relaxation band, restating setup_boundaries
    (Main/mod_atm_interface.F90:383-512) for a domain that is neither a channel (bandflag) nor
    a CRM: the south/north rows, then the west/east columns, with the corner rules."""
    jx, iy, nsp = rc.jx, rc.iy, rc.nspgx
    icx = icy = 1
    igbb1, igbb2, jgbl1, jgbl2 = 2, nsp - 1, 2, nsp - 1
    igbt1, igbt2 = iy - icy - nsp + 2, iy - icy - 1
    jgbr1, jgbr2 = jx - icx - nsp + 2, jx - icx - 1
    ib = {}
    for i in range(1, iy + 1):                                   # south
        if igbb1 <= i <= igbb2:
            for j in range(1, jx + 1):
                if jgbl1 <= j <= jgbr2:
                    if j <= jgbl2 and i >= j:
                        continue
                    if j >= jgbr1 and i >= (jgbr2 - j + 2):
                        continue
                    ib[(j, i)] = i - igbb1 + 2
    for i in range(1, iy + 1):                                   # north
        if igbt1 <= i <= igbt2:
            for j in range(1, jx + 1):
                if jgbl1 <= j <= jgbr2:
                    if j <= jgbl2 and (igbt2 - i + 2) >= j:
                        continue
                    if j >= jgbr1 and (igbt2 - i) >= (jgbr2 - j):
                        continue
                    ib[(j, i)] = igbt2 - i + 2
    for i in range(1, iy + 1):                                   # west
        if i < igbb1 or i > igbt2:
            continue
        for j in range(1, jx + 1):
            if jgbl1 <= j <= jgbl2:
                if i < igbb2 and j > i:
                    continue
                if i > igbt1 and j > (igbt2 - i + 2):
                    continue
                ib[(j, i)] = j - jgbl1 + 2
    for i in range(1, iy + 1):                                   # east
        if i < igbb1 or i > igbt2:
            continue
        for j in range(1, jx + 1):
            if jgbr1 <= j <= jgbr2:
                if i < igbb2 and (jgbr2 - j + 2) > i:
                    continue
                if i > igbt1 and (jgbr2 - j) > (igbt2 - i):
                    continue
                ib[(j, i)] = jgbr2 - j + 2
    # the nudging loops run over the interior cross points only (jci, ici)
    return {(j, i): n for (j, i), n in ib.items() if 2 <= j <= jx - 2 and 2 <= i <= iy - 2}


def test_hydrostatic_temperature_tendency_matches_numpy_restatement():
    """The hydrostatic t, qv and qc tendencies of the first step against an independent NumPy restatement
    of the reference (C1 with no diffusion, points off the relaxation band): compute_omega's
    cr, pten and the qdot scan and omega (Main/mod_tendency.F90:1118-1215), hadvt of atmx%t in
    the upstream form with the t_extrema limiter (Main/mod_advection.F90:311-393; upstream_mode
    and stability_enhance are on for idynamic < 3, Main/mod_params.F90:645-647), vadv3d ind 1
    of atm1%t with the (pf/pb)**c287 interpolation on mkslice's b-level pressures
    (:767-779, Main/mod_slice.F90:233-239) and the adiabatic term
    omega*rgas/cpmf(qv)*tv/(ptop/p* + hsigma) (Main/mod_tendency.F90:1565-1575; cpmf =
    cpd*(1 + 0.8 qv), Share/cpmf.inc); qv = hadvqv + vadvqv and qc = hadvqx + vadv4d ind 1
    (on a cloud layer) as in the NH check."""
    import dataclasses
    from oracle.oracle import OracleCore
    from regcm_amd import constants as C
    rc = dataclasses.replace(CONFIGS["C1"], ckh=0.0, adyndif=0.0)
    data = icbc.generate(rc)
    o = OracleCore(rc, data["split"])
    state = dict(data["state"])
    for a1, a2 in (("ATM1_QC", "ATM1_QV"), ("ATM2_QC", "ATM2_QV")):   # a cloud layer for the qc check
        qc = np.zeros_like(state[a2])
        qc[3:12] = 0.01 * state[a2][3:12]
        state[a1] = qc
    o.put_state(state)
    o.bdyval()
    g = {n: o.get(n) for n in ("ATM1_U", "ATM1_V", "ATM1_T", "ATM1_QV", "ATM1_QC", "PSA", "PSB", "MSFX",
                                "MSFD", "ATM2_T", "XTB_B0", "XTB_BT")}
    _, dt0, xbc = o.get_time()
    o.tend()
    tten, qvten, qcten = o.get("TTEN"), o.get("QVTEN"), o.get("QCTEN")
    o.close()
    kz = rc.kz
    sig = rc.sigma
    hsig = (sig[1:] + sig[:-1]) * 0.5
    dsig = sig[1:] - sig[:-1]
    twt1 = np.zeros(kz + 1); twt2 = np.zeros(kz + 1)
    for k in range(2, kz + 1):
        twt1[k] = (sig[k - 1] - hsig[k - 2]) / (hsig[k - 1] - hsig[k - 2])
        twt2[k] = 1.0 - twt1[k]
    dx = rc.ds * 1000.0
    ul = rc.uoffc * 0.5 * rc.dt / dx
    rgas = C.rgas
    cpd = 3.5 * rgas
    c287 = rgas / 1000.0                                         # Share/mod_constants.F90:132-134
    ep1 = 28.96454 / 18.01528 - 1.0                              # amd/amw - 1 (:303)
    minqq = 1.0e-8

    def sh(a, dj, di):                                           # sh(a)[k, i, j] = a[k, i+di, j+dj]
        return np.roll(a, shift=(-di, -dj), axis=(-2, -1))

    u1, v1, t1, q1 = g["ATM1_U"], g["ATM1_V"], g["ATM1_T"], g["ATM1_QV"]
    pa, pb = g["PSA"][0], g["PSB"][0]
    msfx, msfd = g["MSFX"][0], g["MSFD"][0]
    psd = np.zeros_like(pa)
    psd[1:, 1:] = (pa[1:, 1:] + pa[:-1, 1:] + pa[1:, :-1] + pa[:-1, :-1]) * 0.25
    rpsd = np.divide(1.0, psd, out=np.zeros_like(psd), where=psd > 0)
    rpsa = np.divide(1.0, pa, out=np.zeros_like(pa), where=pa > 0)
    umc, vmc = u1 * msfd, v1 * msfd
    ud, vd = u1 * rpsd, v1 * rpsd
    with np.errstate(divide="ignore", invalid="ignore"):
        cr = ((sh(umc, 1, 1) + sh(umc, 1, 0) - sh(umc, 0, 1) - umc) +
              (sh(vmc, 1, 1) + sh(vmc, 0, 1) - sh(vmc, 1, 0) - vmc)) / (2.0 * dx * msfx * msfx)
        pten = np.zeros_like(pa)
        for k in range(kz):
            pten = pten - cr[k] * dsig[k]
        qdot = np.zeros((kz + 1,) + pa.shape)
        for k in range(2, kz + 1):
            qdot[k - 1] = qdot[k - 2] - (pten + cr[k - 2]) * dsig[k - 2] * rpsa
    xt = t1 * rpsa
    xq = np.maximum(q1 * rpsa, minqq)
    tv = xt * (1.0 + ep1 * xq)
    # upstream hadvt of atmx%t with the t_extrema limiter (frame-edge values, never compared,
    # may be inf/nan: p* is zero outside the frame)
    old_err = np.seterr(divide="ignore", invalid="ignore")
    u1a = sh(umc, 0, 1) + umc
    u2a = sh(umc, 1, 1) + sh(umc, 1, 0)
    v1a = sh(vmc, 1, 0) + vmc
    v2a = sh(vmc, 1, 1) + sh(vmc, 0, 1)
    f1 = 0.5 * ul * (u2a + u1a) / pa
    f2 = 0.5 * ul * (v2a + v1a) / pa
    c, w, e, s_, n = xt, sh(xt, -1, 0), sh(xt, 1, 0), sh(xt, 0, -1), sh(xt, 0, 1)
    fx1 = (1.0 + f1) * w + (1.0 - f1) * c
    fx2 = (1.0 + f1) * c + (1.0 - f1) * e
    fy1 = (1.0 + f2) * s_ + (1.0 - f2) * c
    fy2 = (1.0 + f2) * c + (1.0 - f2) * n
    xmsf = 1.0 / (msfx * msfx * (4.0 * dx))
    fg = -xmsf * (u2a * fx2 - u1a * fx1 + v2a * fy2 - v1a * fy1)
    for (p_, m_) in ((n, s_), (e, w)):
        big = np.abs(p_ + m_ - 2.0 * c) / pa > rc.t_extrema
        fg = np.where(big & (c > p_) & (c > m_), np.minimum(fg, 0.0), fg)
        fg = np.where(big & (c < p_) & (c < m_), np.maximum(fg, 0.0), fg)
    tdyn = 0.0 + fg
    # vadv3d ind 1 (idynamic = 1) on mkslice's b-level pressures
    pbh = (hsig[:, None, None] * pb + rc.ptop) * 1000.0
    pbf = (sig[:, None, None] * pb + rc.ptop) * 1000.0
    for k in range(2, kz + 1):
        dq = qdot[k - 1] * (twt1[k] * t1[k - 1] * (pbf[k - 1] / pbh[k - 1]) ** c287 +
                            twt2[k] * t1[k - 2] * (pbf[k - 1] / pbh[k - 2]) ** c287)
        tdyn[k - 2] = tdyn[k - 2] - dq * (1.0 / dsig[k - 2])
        tdyn[k - 1] = tdyn[k - 1] + dq * (1.0 / dsig[k - 1])
    nsp = rc.nspgx
    J = np.arange(nsp + 1, rc.jx - nsp)
    I = np.arange(nsp + 1, rc.iy - nsp)
    sl = (slice(None), (I - 1)[:, None], (J - 1)[None, :])
    # omega (dummy = 1/(dx8 msfx), dx8 = 8 dx, Main/mod_params.F90:1766) and the adiabatic term
    dummy = 1.0 / (8.0 * dx * msfx)
    om = np.zeros_like(t1)
    for k in range(kz):
        om[k] = (0.5 * (qdot[k + 1] + qdot[k]) * pa + hsig[k] * (
            pten + ((ud[k] + sh(ud, 0, 1)[k] + sh(ud, 1, 1)[k] + sh(ud, 1, 0)[k]) * (sh(pa, 1, 0) - sh(pa, -1, 0)) +
                    (vd[k] + sh(vd, 0, 1)[k] + sh(vd, 1, 1)[k] + sh(vd, 1, 0)[k]) * (sh(pa, 0, 1) - sh(pa, 0, -1))) *
            dummy))
    rovcpm = rgas / (cpd * (1.0 + 0.80 * xq))
    tdyn = tdyn + (om * rovcpm * tv) / (rc.ptop * rpsa + hsig[:, None, None])
    # qv: hadvqv of atmx%qx (q_rel_extrema limiter) + vadvqv of atm1%qx (qcon power form)
    c, w, e, s_, n = xq, sh(xq, -1, 0), sh(xq, 1, 0), sh(xq, 0, -1), sh(xq, 0, 1)
    fx1 = (1.0 + f1) * w + (1.0 - f1) * c
    fx2 = (1.0 + f1) * c + (1.0 - f1) * e
    fy1 = (1.0 + f2) * s_ + (1.0 - f2) * c
    fy2 = (1.0 + f2) * c + (1.0 - f2) * n
    fq = -xmsf * (u2a * fx2 - u1a * fx1 + v2a * fy2 - v1a * fy1)
    den = np.maximum(c, 1.0e-20)
    for (p_, m_) in ((n, s_), (e, w)):
        big = np.abs(p_ + m_ - 2.0 * c) / den > rc.q_rel_extrema
        fq = np.where(big & (c > p_) & (c > m_), np.minimum(fq, 0.0), fq)
        fq = np.where(big & (c < p_) & (c < m_), np.maximum(fq, 0.0), fq)
    qdyn = 0.0 + fq
    for k in range(2, kz + 1):
        qcon = (sig[k - 1] - hsig[k - 1]) / (hsig[k - 2] - hsig[k - 1])   # Main/mod_params.F90:2214
        fk, fkm = q1[k - 1], q1[k - 2]
        ok = (fk > minqq * pa) & (fkm > minqq * pa)
        flux = qdot[k - 1] * np.where(ok, fk * (fkm / fk) ** qcon, 0.0)
        qdyn[k - 2] = qdyn[k - 2] - flux * (1.0 / dsig[k - 2])
        qdyn[k - 1] = qdyn[k - 1] + flux * (1.0 / dsig[k - 1])
    # qc: hadvqx of atmx%qc + vadv4d ind 1 of atm1%qc (no relaxation of qc: every interior point)
    qc1 = g["ATM1_QC"]
    xc = np.maximum(qc1 * rpsa, 0.0)
    c, w, e, s_, n = xc, sh(xc, -1, 0), sh(xc, 1, 0), sh(xc, 0, -1), sh(xc, 0, 1)
    fx1 = (1.0 + f1) * w + (1.0 - f1) * c
    fx2 = (1.0 + f1) * c + (1.0 - f1) * e
    fy1 = (1.0 + f2) * s_ + (1.0 - f2) * c
    fy2 = (1.0 + f2) * c + (1.0 - f2) * n
    cdyn = 0.0 - xmsf * (u2a * fx2 - u1a * fx1 + v2a * fy2 - v1a * fy1)
    for k in range(2, kz + 1):
        fk, fkm, svv = qc1[k - 1], qc1[k - 2], qdot[k - 1]
        thr = minqq * minqq * pa
        ok = np.where(svv > 0.0, fkm > thr, fk > thr)
        flux = np.where(ok, svv * (twt1[k] * fk + twt2[k] * fkm), 0.0)
        cdyn[k - 2] = cdyn[k - 2] - flux * (1.0 / dsig[k - 2])
        cdyn[k - 1] = cdyn[k - 1] + flux * (1.0 / dsig[k - 1])
    np.seterr(**old_err)
    # the band: relaxation of t toward the boundary data (iboudy = 5), at every interior point
    band = _cross_band(rc)
    fnudge, gnudge = 0.1 / rc.dt, 1.0 / (rc.dt * 50.0)           # Main/mod_bdycod.F90:204-215
    anudge = np.where(hsig < 0.4, rc.high_nudge, np.where(hsig < 0.8, rc.medium_nudge, rc.low_nudge))
    fg = (g["XTB_B0"] + (xbc + dt0) * g["XTB_BT"]) - g["ATM2_T"]  # nudge3d, :4242-4245
    relax = np.zeros_like(tdyn)
    lap = sh(fg, -1, 0) + sh(fg, 1, 0) + sh(fg, 0, -1) + sh(fg, 0, 1) - 4.0 * fg
    for (jj, ii), ib in band.items():
        xfun = np.exp(-((ib - 2) / anudge))                      # hefc, hegc (:258-267)
        relax[:, ii - 1, jj - 1] = (fnudge * xfun) * fg[:, ii - 1, jj - 1] - (gnudge * xfun) * lap[:, ii - 1, jj - 1]
    tall = tdyn + relax
    Jc = np.arange(2, rc.jx - 1)
    Ic = np.arange(2, rc.iy - 1)
    sc = (slice(None), (Ic - 1)[:, None], (Jc - 1)[None, :])
    assert len(band) > 0
    np.testing.assert_allclose(tten[sc], tall[sc], rtol=1e-10, atol=1e-11 * np.abs(tall[sc]).max(),
                               err_msg="t with the band")
    assert np.abs(cdyn[sc]).max() > 0.0
    np.testing.assert_allclose(qcten[sc], cdyn[sc], rtol=1e-10, atol=1e-11 * np.abs(cdyn[sc]).max(),
                               err_msg="qc")
    for name, want, got in (("t", tdyn[sl], tten[sl]), ("qv", qdyn[sl], qvten[sl])):
        assert np.abs(want).max() > 0.0
        np.testing.assert_allclose(got, want, rtol=1e-10, atol=1e-11 * np.abs(want).max(), err_msg=name)


def _uw_kpbl(rc, seed=5):
    """A PBL-top field for iuwvadv = 1: every value 1..kz, most columns >= 4 (the rule acts)."""
    rng = np.random.default_rng(seed)
    k = rng.integers(1, rc.kz + 1, size=(1, rc.iy, rc.jx)).astype(np.float64)
    return k


def _uw_qc_state(rc, state, seed=6):
    """A cloud layer with level-to-level structure, so the PBL-top slopes take every branch
    (monotone up, monotone down, mixed) across the columns."""
    rng = np.random.default_rng(seed)
    st = dict(state)
    for a1, a2 in (("ATM1_QC", "ATM1_QV"), ("ATM2_QC", "ATM2_QV")):
        st[a1] = state[a2] * rng.uniform(0.0, 0.02, size=state[a2].shape)
    return st


@pytest.mark.parametrize("idynamic", [1, 2])
def test_uw_vertical_flux_matches_numpy_restatement(idynamic):
    """vadv4d ind = 3 (ibltyp = 2 with iuwvadv = 1, Main/mod_tendency.F90:148-154,
    Main/mod_advection.F90:917-961) against an independent NumPy restatement: the first step's
    qc tendency with iuwvadv = 1 minus the one with iuwvadv = 0 is the difference of the two
    vertical fluxes (everything else in the qc chain is the same computation): the
    twt-interpolated interface values, replaced at kpbl - 1 and kpbl by the PBL-top slope rule
    for kpbl >= 4, times qdot, against ind = 1's thresholded form."""
    import dataclasses
    from oracle.oracle import OracleCore
    if idynamic == 1:
        rc = dataclasses.replace(CONFIGS["C1"], ibltyp=2)
        data = icbc.generate(rc)
    else:
        rc = dataclasses.replace(CONFIGS["N1"], ibltyp=2)
        data = icbc.generate_nh(rc)
    st = _uw_qc_state(rc, data["state"])
    st.update(icbc.tke_state(rc))
    kpbl = _uw_kpbl(rc)
    out = {}
    for uw in (0, 1):
        o = OracleCore(dataclasses.replace(rc, iuwvadv=uw), data["split"])
        o.put_state(st)
        o.put("KPBL", kpbl)
        o.bdyval()
        f = o.get("ATM1_QC")
        psa = o.get("PSA")[0]
        o.tend()
        out[uw] = o.get("QCTEN")
        qdot = o.get("QDOT")
        o.close()
    kz = rc.kz
    sig = np.asarray(rc.sigma)
    hsig = (sig[1:] + sig[:-1]) * 0.5
    dsig = sig[1:] - sig[:-1]
    xds = 1.0 / dsig
    twt1 = np.zeros(kz + 1); twt2 = np.zeros(kz + 1)
    for k in range(2, kz + 1):
        twt1[k] = (sig[k - 1] - hsig[k - 2]) / (hsig[k - 1] - hsig[k - 2])
        twt2[k] = 1.0 - twt1[k]
    F = lambda k: f[k - 1]                        # noqa: E731  (1-based level, [i, j] plane)
    H = lambda k: hsig[k - 1]                     # noqa: E731
    S = lambda k: sig[k - 1]                      # noqa: E731
    # ind = 1
    fg1 = np.zeros((kz + 1,) + psa.shape)
    thr = 1.0e-8 * 1.0e-8 * psa
    for k in range(2, kz + 1):
        svv = qdot[k - 1]
        lin = svv * (twt1[k] * F(k) + twt2[k] * F(k - 1))
        fg1[k] = np.where(svv > 0.0, np.where(F(k - 1) > thr, lin, 0.0), np.where(F(k) > thr, lin, 0.0))
    # ind = 3, column by column as the reference loops
    fg3 = np.zeros_like(fg1)
    for k in range(2, kz + 1):
        fg3[k] = twt1[k] * F(k) + twt2[k] * F(k - 1)
    kp = kpbl[0].astype(int)
    ni, nj = psa.shape
    for i in range(ni):
        for j in range(nj):
            kpb = kp[i, j]
            if kpb < 4:
                continue
            col = lambda k: F(k)[i, j]            # noqa: E731
            k = kpb - 2
            d1, d0 = col(k + 1) - col(k), col(k) - col(k - 1)
            if d1 > 0.0 and d0 > 0.0:
                slope = min(d1 / (H(k + 1) - H(k)), d0 / (H(k) - H(k - 1)))
            elif d1 < 0.0 and d0 < 0.0:
                slope = max(d1 / (H(k + 1) - H(k)), d0 / (H(k) - H(k - 1)))
            else:
                slope = 0.0
            k = kpb
            fg3[k - 1][i, j] = col(k - 2) + slope * (S(k - 1) - H(k - 2))
            if abs(col(k - 2) + slope * (H(k - 1) - H(k - 2)) - col(k)) > abs(col(k - 1) - col(k)):
                fg3[k][i, j] = col(k)
            else:
                fg3[k][i, j] = col(k - 2) + slope * (S(k) - H(k - 2))
    for k in range(2, kz + 1):
        fg3[k] = fg3[k] * qdot[k - 1]

    def ten(fg):
        t = np.zeros((kz,) + psa.shape)
        for k in range(2, kz + 1):
            t[k - 2] -= fg[k] * xds[k - 2]
            t[k - 1] += fg[k] * xds[k - 1]
        return t
    want = ten(fg3) - ten(fg1)
    got = out[1] - out[0]
    sc = (slice(None), slice(1, rc.iy - 2), slice(1, rc.jx - 2))     # ici x jci
    assert np.abs(want[sc]).max() > 0.0
    changed = np.abs(want[sc]) > 0.0
    assert changed.any() and not changed.all()
    np.testing.assert_allclose(got[sc], want[sc], rtol=1e-9, atol=1e-12 * np.abs(out[0][sc]).max())


def _nh_tend_pair(base, on):
    """The N1 NH oracle's first-step tendencies for two option sets (the state after bdyval,
    and TTEN/QVTEN/QCTEN of each run)."""
    import dataclasses
    from oracle.oracle import OracleCore
    res = []
    for opts in (base, on):
        rc = dataclasses.replace(CONFIGS["N1"], **opts)
        data = icbc.generate_nh(rc)
        o = OracleCore(rc, data["split"])
        o.put_state(data["state"])
        o.bdyval()
        g = {n: o.get(n) for n in ("ATM2_U", "ATM2_V", "ATM2_T", "ATM2_QV", "ATM2_W", "ATM2_PP", "PSA", "PSB", "HT",
                                    "ATM0_Z", "ATM0_ZF", "XTB_B0", "XTB_BT", "XQB_B0", "XQB_BT", "XPPB_B0",
                                    "XPPB_BT", "XUB_B0", "XUB_BT", "XVB_B0", "XVB_BT")}
        g["time"] = o.get_time()
        o.tend()
        g["out"] = {n: o.get(n) for n in ("TTEN", "QVTEN", "QCTEN")}
        # u, v, pp, w tendencies as tend leaves them for sound: decoupled (x 1/p*) and scaled by
        # the acoustic step dts (Main/mod_tendency.F90:478-499, Main/mod_sound.F90:229-245)
        g["work"] = {n: o.get_work(n) for n in ("uten", "vten", "ppten", "wten")}
        lc, dt, _ = g["time"]
        istep = max(2, int(dt / data["split"]["nh_dtsmax"]))
        if lc > 0:
            istep = max(istep, 4)
        g["dts"] = dt / istep
        o.close()
        res.append((rc, g))
    return res


def test_nh_diffusion_matches_numpy_restatement():
    """The NH horizontal diffusion of t and qv (Main/mod_tendency.F90:1514-1527) against an
    independent NumPy restatement: calc_coeff's NH Smagorinsky coefficient with the dw/dz term
    and the topographic background (Main/mod_diffusion.F90:100-140, 168-251: xkhz = ckh dx,
    xkhmax = 2 dx^2/(64 dt), dydc = adyndif vonkar^2 dx/4, the b-level winds ubd3d/vbd3d =
    atm2/psdotb and wb3d = atm2%w/psb of mkslice, Main/mod_slice.F90:176-181, 261-263), scaled
    by rdxsq psb, then diffu_x3d of tb3d and diffu_x4d3d of qxb3d (:658-790, 805-): the
    fourth-order interior operator and the second-order rows on the boundary ring (the corners
    take both rows).  Checked as the difference of the first-step tendencies with ckh =
    adyndif = 1 and with both 0 (xkc = 0); everything else is the same computation."""
    from regcm_amd import constants as C
    (rc, g0), (_, g1) = _nh_tend_pair({"ckh": 0.0, "adyndif": 0.0, "ifrayd": 0}, {"ifrayd": 0})
    kz, jx, iy = rc.kz, rc.jx, rc.iy
    dx = rc.ds * 1000.0
    dxsq = dx * dx
    xkhz = 1.0 * dx
    xkhmax = 2.0 * (dxsq / (64.0 * rc.dt))
    dydc = 1.0 * 0.4 * 0.4 * dx * 0.25
    pb = g1["PSB"][0]
    rpsb = np.divide(1.0, pb, out=np.zeros_like(pb), where=pb > 0)
    # interior dot points' psdotb (4-point mean; calc_coeff at ci points reads only those)
    psd = np.zeros_like(pb)
    psd[1:, 1:] = (pb[1:, 1:] + pb[:-1, 1:] + pb[1:, :-1] + pb[:-1, :-1]) * 0.25
    rpsd = np.divide(1.0, psd, out=np.zeros_like(psd), where=psd > 0)
    ud, vd = g1["ATM2_U"] * rpsd[None], g1["ATM2_V"] * rpsd[None]
    wx = g1["ATM2_W"] * rpsb[None]
    ht = g1["HT"][0]
    J = np.arange(2, jx - 1)          # jci (1-based)
    I = np.arange(2, iy - 1)

    def at(a, dj=0, di=0):
        return a[..., (I + di - 1)[:, None], (J + dj - 1)[None, :]]
    if rc.diffu_hgtf == 1:
        hg = [np.abs((at(ht) - at(ht, 0, -1)) / dx), np.abs((at(ht) - at(ht, 0, 1)) / dx),
              np.abs((at(ht) - at(ht, -1, 0)) / dx), np.abs((at(ht) - at(ht, 1, 0)) / dx)]
        hgmax = np.maximum(np.maximum(hg[0], hg[1]), np.maximum(hg[2], hg[3])) * C.regrav * 1.0e3
        hgfact = xkhz / (1.0 + hgmax * hgmax)
    else:                          # the NH default (dynparam, Main/mod_params.F90:648-652)
        hgfact = np.full(at(ht).shape, xkhz)
    dudx = at(ud, 1, 0) + at(ud, 1, 1) - at(ud) - at(ud, 0, 1)
    dvdx = at(vd, 1, 0) + at(vd, 1, 1) - at(vd) - at(vd, 0, 1)
    dudy = at(ud, 0, 1) + at(ud, 1, 1) - at(ud) - at(ud, 1, 0)
    dvdy = at(vd, 0, 1) + at(vd, 1, 1) - at(vd) - at(vd, 1, 0)
    dwdz = at(wx)[:kz] - at(wx)[1:kz + 1]
    duv = np.sqrt(np.maximum((dudx - dvdy) * (dudx - dvdy) + (dvdx + dudy) * (dvdx + dudy) - dwdz * dwdz, 0.0))
    xkc = np.minimum(hgfact[None] + dydc * duv, xkhmax) * (1.0 / dxsq) * at(pb)[None]

    def diffu(f, xk):
        """diffu_x3d / diffu_x4d3d / diffu_x3df (fac = 1) on the jci x ici points with the
        coefficient xk of nk levels."""
        out = np.zeros((xk.shape[0], len(I), len(J)))
        f = f[: xk.shape[0]]
        c1, c2, c3 = 1.0, -4.0, 12.0
        inner = (slice(None), slice(1, -1), slice(1, -1))
        four = (c1 * (at(f, 2, 0) + at(f, -2, 0) + at(f, 0, 2) + at(f, 0, -2)) +
                c2 * (at(f, 1, 0) + at(f, -1, 0) + at(f, 0, 1) + at(f, 0, -1)) + c3 * at(f))
        out[inner] = out[inner] - xk[inner] * four[inner]
        two = c1 * (at(f, 1, 0) + at(f, -1, 0) + at(f, 0, 1) + at(f, 0, -1)) + c2 * at(f)
        for sl in ((slice(None), slice(None), 0), (slice(None), slice(None), -1),
                   (slice(None), 0, slice(None)), (slice(None), -1, slice(None))):
            out[sl] = out[sl] + xk[sl] * two[sl]
        return out
    tb = g1["ATM2_T"] * rpsb[None]
    qb = np.maximum(g1["ATM2_QV"] * rpsb[None], 1.0e-8)
    for name, f in (("QVTEN", qb), ("TTEN", tb)):
        want = diffu(f, xkc)
        got = at(g1["out"][name]) - at(g0["out"][name])
        scale = np.abs(at(g1["out"][name])).max()
        assert np.abs(want).max() > 1e-6 * scale, name
        np.testing.assert_allclose(got, want, rtol=1e-9, atol=1e-12 * scale, err_msg=name)
    # pp: diffu_x3d of ppb3d = atm2%pp/psb with xkc; w: diffu_x3df of wb3d with xkcf, kz+1
    # levels (Main/mod_diffusion.F90:523-656): xkcf(1) = xkc(1), xkcf(k+1) = xkc(k)
    # (:232-235), scaled the same way; both then x 1/psa x dts as tend and sound leave them
    fac = (1.0 / at(g1["PSA"])[0]) * g1["dts"]
    xkcf = np.concatenate([xkc[:1], xkc], axis=0)
    for name, f, xk in (("ppten", g1["ATM2_PP"] * rpsb[None], xkc), ("wten", wx, xkcf)):
        want = diffu(f, xk) * fac[None]
        got = at(g1["work"][name]) - at(g0["work"][name])
        scale = np.abs(at(g1["work"][name])).max()
        assert np.abs(want).max() > 1e-6 * scale, name
        np.testing.assert_allclose(got, want, rtol=1e-9, atol=1e-12 * scale, err_msg=name)


def test_nh_rayleigh_damping_matches_numpy_restatement():
    """raydamp of t, qv, u, v, pp and w (ifrayd = 1, Main/mod_tendency.F90:356-364, 466-477; raydamp3 / raydampqv,
    Main/mod_bdycod.F90:5021-5085 with tau, :5108-5116) against an independent NumPy
    restatement: on levels 1..rayndamp, tau(za(k), za(1)) = rayalpha0 sin^2(pi/2 (1 - (za(1) -
    za(k))/rayhd)) above za(1) - rayhd, else 0, times (b0 + (xbctime + dt) bt - atm2) (za =
    atm0%z, Main/mod_atm_interface.F90:975).  Checked as the difference of the first-step
    tendencies with ifrayd = 1 and 0."""
    (rc, g0), (_, g1) = _nh_tend_pair({"ifrayd": 0}, {"ifrayd": 1})
    kz, jx, iy = rc.kz, rc.jx, rc.iy
    _, dt, xbc = g1["time"]
    xt = xbc + dt
    z = g1["ATM0_Z"]
    ztop = z[0]
    halfpi = np.pi * 0.5                                       # Share/mod_constants.F90 halfpi = mathpi/2
    sl = (slice(None), slice(1, iy - 2), slice(1, jx - 2))     # ici x jci
    for name, b0, bt, var in (("TTEN", "XTB_B0", "XTB_BT", "ATM2_T"), ("QVTEN", "XQB_B0", "XQB_BT", "ATM2_QV")):
        want = np.zeros((kz, iy, jx))
        for k in range(min(kz, rc.rayndamp)):
            zk = z[k]
            tau = np.where(zk > ztop - rc.rayhd,
                           rc.rayalpha0 * np.sin(halfpi * (1.0 - (ztop - zk) / rc.rayhd)) ** 2, 0.0)
            want[k] = tau * ((g1[b0][k] + xt * g1[bt][k]) - g1[var][k])
        got = g1["out"][name] - g0["out"][name]
        scale = np.abs(g1["out"][name][sl]).max()
        # (the synthetic qv is near minqq on the damped top levels: a small but non-zero term)
        assert np.abs(want[sl]).max() > (1e-6 * scale if name == "TTEN" else 0.0), name
        np.testing.assert_allclose(got[sl], want[sl], rtol=1e-9, atol=1e-12 * np.abs(want[sl]).max(),
                                   err_msg=name)
    # pp toward its boundary data (raydamp3), w toward 0 on the full levels with zq = atm0%zf
    # (raydamp3f, :5005-5019), both x 1/psa x dts; u, v at dot points with z averaged from the
    # four cross neighbours (raydampuv, :4953-4983), x 1/psdota x dts
    fac = np.divide(1.0, g1["PSA"][0], out=np.zeros_like(g1["PSA"][0]), where=g1["PSA"][0] > 0) * g1["dts"]
    zf = g1["ATM0_ZF"]
    for name, nk, zz, bval, var in (
            ("ppten", kz, z, g1["XPPB_B0"] + xt * g1["XPPB_BT"], g1["ATM2_PP"]),
            ("wten", kz + 1, zf, 0.0 * g1["ATM2_W"], g1["ATM2_W"])):
        want = np.zeros((nk, iy, jx))
        for k in range(min(nk, rc.rayndamp)):
            tau = np.where(zz[k] > zz[0] - rc.rayhd,
                           rc.rayalpha0 * np.sin(halfpi * (1.0 - (zz[0] - zz[k]) / rc.rayhd)) ** 2, 0.0)
            want[k] = tau * (bval[k] - var[k]) * fac
        got = g1["work"][name] - g0["work"][name]
        scale = np.abs(g1["work"][name][sl]).max()
        assert np.abs(want[sl]).max() > 1e-6 * scale, name
        np.testing.assert_allclose(got[sl], want[sl], rtol=1e-9, atol=1e-12 * scale, err_msg=name)
    pa = g1["PSA"][0]
    psd = np.zeros_like(pa)
    psd[1:, 1:] = (pa[1:, 1:] + pa[:-1, 1:] + pa[1:, :-1] + pa[:-1, :-1]) * 0.25
    dfac = np.divide(1.0, psd, out=np.zeros_like(psd), where=psd > 0) * g1["dts"]
    zd = np.zeros_like(z)
    zd[:, 1:, 1:] = 0.25 * (z[:, 1:, 1:] + z[:, 1:, :-1] + z[:, :-1, 1:] + z[:, :-1, :-1])
    dl = (slice(None), slice(1, iy - 1), slice(1, jx - 1))     # idi x jdi
    for name, b0, bt, var in (("uten", "XUB_B0", "XUB_BT", "ATM2_U"), ("vten", "XVB_B0", "XVB_BT", "ATM2_V")):
        want = np.zeros((kz, iy, jx))
        for k in range(min(kz, rc.rayndamp)):
            tau = np.where(zd[k] > zd[0] - rc.rayhd,
                           rc.rayalpha0 * np.sin(halfpi * (1.0 - (zd[0] - zd[k]) / rc.rayhd)) ** 2, 0.0)
            want[k] = tau * ((g1[b0][k] + xt * g1[bt][k]) - g1[var][k]) * dfac
        got = g1["work"][name] - g0["work"][name]
        scale = np.abs(g1["work"][name][dl]).max()
        assert np.abs(want[dl]).max() > 1e-6 * scale, name
        np.testing.assert_allclose(got[dl], want[dl], rtol=1e-9, atol=1e-12 * scale, err_msg=name)


def test_hydrostatic_wind_tendency_matches_numpy_restatement():
    """The hydrostatic u, v tendencies of the first step against an independent NumPy
    restatement of the reference (C1, no diffusion, dot points off the band): hadvuv's
    hydrostatic upstream branch (Main/mod_advection.F90:203-233), vadvuv of atmx%uc, vc
    (:271-303), the Coriolis term (Main/mod_tendency.F90:1830-1838) and the pressure-gradient
    force with ipgf = 0 (:1886-2119): the log-p* term with rtbar from atmx%tv, the geopotential
    of the hydrostatic column integral (td = atm1%t (1 + ep1 qv) since alpha_hyd = 0,
    Share/mod_constants.F90:319-320; tvfac = 1/(1 + qc/(1 + qv))) and its gradient."""
    import dataclasses
    from oracle.oracle import OracleCore
    from regcm_amd import constants as C
    rc = dataclasses.replace(CONFIGS["C1"], ckh=0.0, adyndif=0.0)
    assert rc.ipgf == 0
    data = icbc.generate(rc)
    o = OracleCore(rc, data["split"])
    o.put_state(data["state"])
    o.bdyval()
    g = {n: o.get(n) for n in ("ATM1_U", "ATM1_V", "ATM1_T", "ATM1_QV", "ATM1_QC", "PSA", "MSFX", "MSFD",
                                "CORIOL", "HT")}
    o.tend()
    uten, vten = o.get("UTEN"), o.get("VTEN")
    o.close()
    kz = rc.kz
    sig = rc.sigma
    hsig = (sig[1:] + sig[:-1]) * 0.5
    dsig = sig[1:] - sig[:-1]
    twt1 = np.zeros(kz + 1); twt2 = np.zeros(kz + 1)
    for k in range(2, kz + 1):
        twt1[k] = (sig[k - 1] - hsig[k - 2]) / (hsig[k - 1] - hsig[k - 2])
        twt2[k] = 1.0 - twt1[k]
    dx = rc.ds * 1000.0
    ul = rc.uoffc * 0.5 * rc.dt / dx
    rgas = C.rgas
    ep1 = 28.96454 / 18.01528 - 1.0
    minqq = 1.0e-8
    ptop = rc.ptop

    def sh(a, dj, di):                                           # sh(a)[k, i, j] = a[k, i+di, j+dj]
        return np.roll(a, shift=(-di, -dj), axis=(-2, -1))

    old_err = np.seterr(divide="ignore", invalid="ignore")      # frame edges: never compared
    u1, v1, t1 = g["ATM1_U"], g["ATM1_V"], g["ATM1_T"]
    pa, msfx, msfd = g["PSA"][0], g["MSFX"][0], g["MSFD"][0]
    psd = np.zeros_like(pa)
    psd[1:, 1:] = (pa[1:, 1:] + pa[:-1, 1:] + pa[1:, :-1] + pa[:-1, :-1]) * 0.25
    rpsd = np.divide(1.0, psd, out=np.zeros_like(psd), where=psd > 0)
    rpsa = np.divide(1.0, pa, out=np.zeros_like(pa), where=pa > 0)
    umc, vmc = u1 * msfd, v1 * msfd
    ud, vd = u1 * rpsd, v1 * rpsd
    # compute_omega's qdot (hydrostatic scan) for vadvuv
    cr = ((sh(umc, 1, 1) + sh(umc, 1, 0) - sh(umc, 0, 1) - umc) +
          (sh(vmc, 1, 1) + sh(vmc, 0, 1) - sh(vmc, 1, 0) - vmc)) / (2.0 * dx * msfx * msfx)
    pten = np.zeros_like(pa)
    for k in range(kz):
        pten = pten - cr[k] * dsig[k]
    qdot = np.zeros((kz + 1,) + pa.shape)
    for k in range(2, kz + 1):
        qdot[k - 1] = qdot[k - 2] - (pten + cr[k - 2]) * dsig[k - 2] * rpsa
    # hadvuv, hydrostatic upstream branch
    ucmona = sh(umc, 0, 1) + 2.0 * umc + sh(umc, 0, -1)
    ucmonb = sh(umc, 1, 1) + 2.0 * sh(umc, 1, 0) + sh(umc, 1, -1)
    ucmonc = sh(umc, -1, 1) + 2.0 * sh(umc, -1, 0) + sh(umc, -1, -1)
    vcmona = sh(vmc, 1, 0) + 2.0 * vmc + sh(vmc, -1, 0)
    vcmonb = sh(vmc, 1, 1) + 2.0 * sh(vmc, 0, 1) + sh(vmc, -1, 1)
    vcmonc = sh(vmc, 1, -1) + 2.0 * sh(vmc, 0, -1) + sh(vmc, -1, -1)
    ff1, ff2 = ul * (sh(ud, 1, 0) + ud), ul * (sh(ud, -1, 0) + ud)
    ff3, ff4 = ul * (sh(vd, 0, 1) + vd), ul * (sh(vd, 0, -1) + vd)
    ucb = (1.0 + ff1) * ucmona + (1.0 - ff1) * ucmonb
    ucc_ = (1.0 + ff2) * ucmonc + (1.0 - ff2) * ucmona
    vcb = (1.0 + ff3) * vcmona + (1.0 - ff3) * vcmonb
    vcc_ = (1.0 + ff4) * vcmonc + (1.0 - ff4) * vcmona
    dm = 1.0 / (msfd * msfd * 16.0 * dx)
    udyn = -dm * ((sh(ud, 1, 0) + ud) * ucb - (ud + sh(ud, -1, 0)) * ucc_ +
                  (sh(ud, 0, 1) + ud) * vcb - (ud + sh(ud, 0, -1)) * vcc_)
    vdyn = -dm * ((sh(vd, 1, 0) + vd) * ucb - (vd + sh(vd, -1, 0)) * ucc_ +
                  (sh(vd, 0, 1) + vd) * vcb - (vd + sh(vd, 0, -1)) * vcc_)
    for k in range(2, kz + 1):                                   # vadvuv of atm1 u, v
        qq = 0.25 * (qdot[k - 1] + sh(qdot, 0, -1)[k - 1] + sh(qdot, -1, 0)[k - 1] + sh(qdot, -1, -1)[k - 1])
        uu = qq * (twt1[k] * u1[k - 1] + twt2[k] * u1[k - 2])
        vv = qq * (twt1[k] * v1[k - 1] + twt2[k] * v1[k - 2])
        udyn[k - 2] = udyn[k - 2] - uu / dsig[k - 2]
        udyn[k - 1] = udyn[k - 1] + uu / dsig[k - 1]
        vdyn[k - 2] = vdyn[k - 2] - vv / dsig[k - 2]
        vdyn[k - 1] = vdyn[k - 1] + vv / dsig[k - 1]
    cor = g["CORIOL"][0]                                         # Coriolis
    udyn = udyn + cor * v1
    vdyn = vdyn - cor * u1
    # pressure-gradient force, ipgf = 0: the log-p* part
    xq = np.maximum(g["ATM1_QV"] * rpsa, minqq)
    xc = np.maximum(g["ATM1_QC"] * rpsa, 0.0)
    tv = (t1 * rpsa) * (1.0 + ep1 * xq)
    rtbar = 0.25 * (sh(tv, -1, -1) + sh(tv, -1, 0) + sh(tv, 0, -1) + tv)
    rtbar = rgas * rtbar * psd
    h = hsig[:, None, None]
    udyn = udyn - rtbar * (np.log(0.5 * (pa + sh(pa, 0, -1)) * h + ptop) -
                           np.log(0.5 * (sh(pa, -1, 0) + sh(pa, -1, -1)) * h + ptop)) / (dx * msfd)
    vdyn = vdyn - rtbar * (np.log(0.5 * (pa + sh(pa, -1, 0)) * h + ptop) -
                           np.log(0.5 * (sh(pa, -1, -1) + sh(pa, 0, -1)) * h + ptop)) / (dx * msfd)
    # geopotential (half levels, cross points) and its gradient
    td = t1 * (1.0 + ep1 * xq)
    tvfac = 1.0 / (1.0 + xc / (1.0 + xq))
    phi = np.zeros_like(t1)
    phi[kz - 1] = g["HT"][0] - rgas * (td[kz - 1] * rpsa * tvfac[kz - 1]) * np.log(
        (hsig[kz - 1] + ptop * rpsa) / (1.0 + ptop * rpsa))
    for lev in range(kz - 1, 0, -1):                             # 1-based lev = kz-1 .. 1
        tvavg = ((td[lev - 1] * dsig[lev - 1] + td[lev] * dsig[lev]) /
                 (pa * (dsig[lev - 1] + dsig[lev]))) * tvfac[lev - 1]
        phi[lev - 1] = phi[lev] - rgas * tvavg * np.log((hsig[lev - 1] + ptop * rpsa) / (hsig[lev] + ptop * rpsa))
    udyn = udyn - psd * (phi + sh(phi, 0, -1) - sh(phi, -1, 0) - sh(phi, -1, -1)) / (2.0 * dx * msfd)
    vdyn = vdyn - psd * (phi + sh(phi, -1, 0) - sh(phi, 0, -1) - sh(phi, -1, -1)) / (2.0 * dx * msfd)
    np.seterr(**old_err)
    nsp = rc.nspgx
    J = np.arange(nsp + 2, rc.jx - nsp)                          # dot points off the band
    I = np.arange(nsp + 2, rc.iy - nsp)
    sl = (slice(None), (I - 1)[:, None], (J - 1)[None, :])
    for name, want, got in (("u", udyn[sl], uten[sl]), ("v", vdyn[sl], vten[sl])):
        assert np.abs(want).max() > 0.0
        np.testing.assert_allclose(got, want, rtol=1e-10, atol=1e-11 * np.abs(want).max(), err_msg=name)


@pytest.mark.parametrize("nthreads", [2, 4, 6])
def test_oracle_threads_match_single_tile(c1_data, nthreads):
    """The all-cores CPU baseline (oracle/orc_par.c: set_nproc tiles on OpenMP threads with
    neighbour-to-neighbour exchanges in shared memory) reproduces the single-tile restatement
    bit for bit, as the reference does across MPI rank counts."""
    from oracle.oracle import OracleCore, OracleParallel
    rc, data = c1_data
    ref = OracleCore(rc, data["split"])
    par = OracleParallel(rc, data["split"], nthreads)
    assert par.nthreads == nthreads
    for o in (ref, par):
        o.put_state(data["state"])
        o.bdyval()
        o.step(3)
    assert par.get_time() == ref.get_time()
    for name in STATE_FIELDS:
        assert np.array_equal(par.get(name), ref.get(name)), name


NH_VARIANTS = [{}, {"isladvec": 1}, {"ibltyp": 2}, {"iboudy": 4}, {"idiffu": 2}]


@pytest.mark.parametrize("variant", NH_VARIANTS, ids=lambda v: ",".join(f"{k}={x}" for k, x in v.items()) or "default")
@pytest.mark.parametrize("nthreads", [2, 4])
def test_nh_oracle_threads_match_single_tile(nthreads, variant):
    """The NH restatement as set_nproc tiles on OpenMP threads (the all-cores NH CPU baseline):
    the reference's exchanges, plus the whole-domain gather of sound's upper radiative
    condition (estore, Main/mod_sound.F90:496-497) and of its day-alarm means, summed in the
    single-tile order -- bit-identical to one tile over 3 steps (istep changes on the first
    two, the radiative mask is built on the first)."""
    import dataclasses
    from oracle.oracle import OracleCore, OracleParallel
    from regcm_amd.config import CONFIGS, NH_STATE_FIELDS
    from regcm_amd import icbc
    rc = dataclasses.replace(CONFIGS["N1"], **variant)
    data = icbc.generate_nh(CONFIGS["N1"])
    st = dict(data["state"])
    if rc.ibltyp == 2:
        st.update(icbc.tke_state(rc))
    ref = OracleCore(rc, data["split"])
    par = OracleParallel(rc, data["split"], nthreads)
    assert par.nthreads == nthreads
    for o in (ref, par):
        o.put_state(st)
        o.bdyval()
        o.step(3)
    assert par.get_time() == ref.get_time()
    names = STATE_FIELDS[:12] + NH_STATE_FIELDS + (["ATM1_TKE", "ATM2_TKE"] if rc.ibltyp == 2 else [])
    for name in names:
        assert np.array_equal(par.get(name), ref.get(name)), name


@pytest.mark.parametrize("ifupr", [0, 1])
def test_nh_sound_substep_matches_numpy_restatement(ifupr):
    """One acoustic sub-step of sound (Main/mod_sound.F90:249-682, the first sub-step of the
    first step) against an independent NumPy restatement, from the state sound starts with (the
    oracle stopped right after sound's set-up, orc_set_sound_probe(0)) to the state after the
    sub-step (probe 1): dp'/dp0, the pressure-gradient update of u and v (:266-296), the lower
    boundary w, the coefficients cc, cdd, cj, ca, g1, g2 and the Ikawa tridiagonal (a, b, c,
    rhs; :322-457), the pp predictor (:459-468), the upward elimination and the downward w
    sweep (:470-479, 566-573), the zero-gradient w on the boundary ring (:577-607), the new pp,
    pi and the dp'/dt temperature correction of atm1 and atm2 t (:661-680).  The lid: w = 0
    (ifupr = 0), or the upper radiative condition (ifupr = 1, :486-562): estore and astore
    from the elimination's top coefficients, the day-alarm means abar and rhon over the
    interior (rnpts of init_sound, :120), the 13 x 13 tmask from the fi, fj, fk, fl weights
    (:126-141, 523-543) and its convolution of estore with the indices clamped to the interior
    (:551-561).  The transcendental terms (the tmask's sin / cos) make it <= 1e-11 relative."""
    import dataclasses
    import math
    from oracle.oracle import OracleCore
    from regcm_amd import constants as C
    rc = dataclasses.replace(CONFIGS["N1"], ifupr=ifupr)
    data = icbc.generate_nh(rc)
    runs = []
    for probe in (0, 1):
        o = OracleCore(rc, data["split"])
        o.put_state(data["state"])
        o.bdyval()
        o.set_sound_probe(probe)
        _, dt, _ = o.get_time()
        o.tend()
        r = {n: o.get_work(n) for n in ("cu", "cv", "cpp", "cw", "pi", "pr1", "rho1", "cqv", "uten", "vten",
                                        "ppten", "wten")}
        r.update({n: o.get(n) for n in ("ATM1_T", "ATM2_T", "ATM0_PR", "ATM0_T", "ATM0_RHO", "ATM0_PS",
                                         "HT", "MSFX", "MSFD", "DPRDDX", "DPRDDY", "PSB")})
        r["dt"] = dt
        o.close()
        runs.append(r)
    a, b = runs
    kz, jx, iy = rc.kz, rc.jx, rc.iy
    kp = kz + 1
    dt = a["dt"]
    istep = max(2, int(dt / data["split"]["nh_dtsmax"]))
    dts = dt / istep
    dx = rc.ds * 1000.0
    sig = np.asarray(rc.sigma)
    dsig = np.concatenate([[0.0], sig[1:] - sig[:-1]])            # dsigma(k) at [k]
    egrav, regrav = C.egrav, C.regrav
    rgas, cpd = C.rgas, 3.5 * C.rgas
    xgamma = 1.0 / (1.0 - rgas * (1.0 / cpd))                      # Main/mod_sound.F90:77
    bet = rc.nhbet
    bp, bm = (1.0 + bet) * 0.5, (1.0 - bet) * 0.5
    bpxbp, bpxbm = bp * bp, bp * bm

    def F(x):                                                      # 1-based [k][i][j] views
        return lambda k, i, j: x[k - 1][i - 1][j - 1]
    u = a["cu"].copy(); v = a["cv"].copy(); pp = a["cpp"].copy(); w = a["cw"].copy()
    pr0, t0, rho0 = a["ATM0_PR"], a["ATM0_T"], a["ATM0_RHO"]
    ps0 = a["ATM0_PS"][0]
    pr1, rho1 = a["pr1"], a["rho1"]
    ht, msfx, msfd = a["HT"][0], a["MSFX"][0], a["MSFD"][0]
    psb = a["PSB"][0]
    rpsb = np.divide(1.0, psb, out=np.zeros_like(psb), where=psb > 0)
    a2t = a["ATM2_T"]
    JE, IE = slice(0, jx - 1), slice(0, iy - 1)                   # jce, ice (0-based)
    # dp'/dp0 on the cross points (atmc%t as sound's scratch, :258-263)
    cdt = np.zeros_like(pp)
    for k in range(1, kz + 1):
        km1, kp1 = max(1, k - 1), min(kz, k + 1)
        cdt[k - 1][IE, JE] = (pp[km1 - 1][IE, JE] - pp[kp1 - 1][IE, JE]) / (pr0[km1 - 1][IE, JE] - pr0[kp1 - 1][IE, JE])
    # u, v on jdi x idi (:266-296)
    D = (slice(None), slice(1, iy - 1), slice(1, jx - 1))

    def sh(x, dj, di):                                             # x at (j+dj, i+di), on D
        return x[:, 1 + di: iy - 1 + di, 1 + dj: jx - 1 + dj]
    rho = 0.25 * (sh(rho1, 0, 0) + sh(rho1, -1, 0) + sh(rho1, 0, -1) + sh(rho1, -1, -1))
    dpp = 0.25 * (sh(cdt, 0, 0) + sh(cdt, -1, 0) + sh(cdt, 0, -1) + sh(cdt, -1, -1))
    chh = 0.5 * dts / (rho * dx) / msfd[1:iy - 1, 1:jx - 1][None]
    u[D] = u[D] - chh * (sh(pp, 0, 0) - sh(pp, -1, 0) + sh(pp, 0, -1) - sh(pp, -1, -1) - a["DPRDDX"][D] * dpp)
    v[D] = v[D] - chh * (sh(pp, 0, 0) - sh(pp, 0, -1) + sh(pp, -1, 0) - sh(pp, -1, -1) - a["DPRDDY"][D] * dpp)
    u[D] = u[D] + a["uten"][D]
    v[D] = v[D] + a["vten"][D]
    np.testing.assert_allclose(b["cu"][D], u[D], rtol=1e-13, atol=1e-13 * np.abs(u[D]).max(), err_msg="u")
    np.testing.assert_allclose(b["cv"][D], v[D], rtol=1e-13, atol=1e-13 * np.abs(v[D]).max(), err_msg="v")
    # the semi-implicit w / pp solve, column by column on jci x ici
    U, V, P, W, R0, R1, P0, P1, T0 = F(u), F(v), F(pp), F(w), F(rho0), F(rho1), F(pr0), F(pr1), F(t0)
    wnew = w.copy()
    ppnew = pp.copy()
    pinew = np.zeros_like(pp)
    a1t, a2tn = a["ATM1_T"].copy(), a["ATM2_T"].copy()
    cols = {}
    for i in range(2, iy - 1):
        for j in range(2, jx - 1):
            wo = [None] + [W(k, i, j) for k in range(1, kp + 1)]
            e = [0.0] * (kp + 1); f = [0.0] * (kp + 1)
            cc = [0.0] * (kz + 1); cdd = [0.0] * (kz + 1); cj = [0.0] * (kz + 1); ca = [0.0] * (kz + 1)
            g1 = [0.0] * (kz + 1); g2 = [0.0] * (kz + 1); aa = [0.0] * (kz + 1); bb = [0.0] * (kz + 1)
            cq = [0.0] * (kz + 1); tk = [0.0] * (kz + 1); px = [0.0] * (kz + 1); py = [0.0] * (kz + 1)
            pt = [0.0] * (kz + 1); rhs = [0.0] * (kz + 1)
            wk = list(wo)
            wk[kp] = 0.5 * 0.25 * regrav * (
                (V(kz, i + 1, j) + V(kz, i, j) + V(kz, i + 1, j + 1) + V(kz, i, j + 1)) * (ht[i, j - 1] - ht[i - 2, j - 1]) +
                (U(kz, i + 1, j) + U(kz, i, j) + U(kz, i + 1, j + 1) + U(kz, i, j + 1)) * (ht[i - 1, j] - ht[i - 1, j - 2])
            ) / (dx * msfx[i - 1, j - 1])
            e[kz] = 0.0
            f[kz] = wk[kp]
            mx = msfx[i - 1, j - 1]
            md = lambda jj, ii: msfd[ii - 1, jj - 1]                  # noqa: E731
            for k in range(1, kz + 1):
                km1, kp1 = max(1, k - 1), min(k + 1, kz)
                tk[k] = (0.5 * ps0[i - 1, j - 1] * T0(k, i, j)) / (xgamma * P0(k, i, j) * a2t[k - 1][i - 1][j - 1] *
                                                                   rpsb[i - 1, j - 1])
                cc[k] = xgamma * P1(k, i, j) * dts / (dx * mx)
                cdd[k] = xgamma * P1(k, i, j) * R0(k, i, j) * egrav * dts / (ps0[i - 1, j - 1] * dsig[k])
                cj[k] = 0.5 * R0(k, i, j) * egrav * dts
                if k == 1:
                    px[k] = 0.0625 * (P0(1, i, j + 1) - P0(1, i, j - 1)) * (
                        U(1, i, j) + U(1, i, j + 1) + U(1, i + 1, j) + U(1, i + 1, j + 1) -
                        U(2, i, j) - U(2, i, j + 1) - U(2, i + 1, j) - U(2, i + 1, j + 1)) / (P0(1, i, j) - P0(2, i, j))
                    py[k] = 0.0625 * (P0(1, i + 1, j) - P0(1, i - 1, j)) * (
                        V(1, i, j) + V(1, i, j + 1) + V(1, i + 1, j) + V(1, i + 1, j + 1) -
                        V(2, i, j) - V(2, i, j + 1) - V(2, i + 1, j) - V(2, i + 1, j + 1)) / (P0(1, i, j) - P0(2, i, j))
                    continue
                rofac = (dsig[km1] * R0(k, i, j) + dsig[k] * R0(km1, i, j)) / (dsig[km1] * R1(k, i, j) + dsig[k] * R1(km1, i, j))
                ca[k] = egrav * dts / (P0(k, i, j) - P0(km1, i, j)) * rofac
                g1[k] = 1.0 - dsig[km1] * tk[k]
                g2[k] = 1.0 + dsig[k] * tk[km1]
                cq[k] = -ca[k] * (cdd[km1] - cj[km1]) * g2[k] * bpxbp
                bb[k] = 1.0 + ca[k] * (g1[k] * (cdd[k] - cj[k]) + g2[k] * (cdd[km1] + cj[km1])) * bpxbp
                aa[k] = -ca[k] * (cdd[k] + cj[k]) * g1[k] * bpxbp
                py[k] = 0.125 * (P0(k, i + 1, j) - P0(k, i - 1, j)) * (
                    V(km1, i, j) + V(km1, i, j + 1) + V(km1, i + 1, j) + V(km1, i + 1, j + 1) -
                    V(kp1, i, j) - V(kp1, i, j + 1) - V(kp1, i + 1, j) - V(kp1, i + 1, j + 1)) / (P0(km1, i, j) - P0(kp1, i, j))
                px[k] = 0.125 * (P0(k, i, j + 1) - P0(k, i, j - 1)) * (
                    U(km1, i, j) + U(km1, i, j + 1) + U(km1, i + 1, j) + U(km1, i + 1, j + 1) -
                    U(kp1, i, j) - U(kp1, i, j + 1) - U(kp1, i + 1, j) - U(kp1, i + 1, j + 1)) / (P0(km1, i, j) - P0(kp1, i, j))
            py[kz] = py[kz] * 0.5
            px[kz] = px[kz] * 0.5
            for k in range(1, kz + 1):
                div = (V(k, i + 1, j) * md(j, i + 1) - V(k, i, j) * md(j, i) + V(k, i + 1, j + 1) * md(j + 1, i + 1) -
                       V(k, i, j + 1) * md(j + 1, i) + U(k, i, j + 1) * md(j + 1, i) - U(k, i, j) * md(j, i) +
                       U(k, i + 1, j + 1) * md(j + 1, i + 1) - U(k, i + 1, j) * md(j, i + 1))
                pt[k] = a["ppten"][k - 1][i - 1][j - 1] - 0.5 * cc[k] * (div / mx - 2.0 * (py[k] + px[k]))
            for k in range(2, kz + 1):
                rhs[k] = wk[k] + a["wten"][k - 1][i - 1][j - 1] + ca[k] * (
                    bpxbm * ((cdd[k - 1] - cj[k - 1]) * g2[k] * wo[k - 1] -
                             ((cdd[k - 1] + cj[k - 1]) * g2[k] + (cdd[k] - cj[k]) * g1[k]) * wo[k] +
                             (cdd[k] + cj[k]) * g1[k] * wo[k + 1]) +
                    (P(k, i, j) * g1[k] - P(k - 1, i, j) * g2[k]) + (g1[k] * pt[k] - g2[k] * pt[k - 1]) * bp)
            pold = [None] + [P(k, i, j) for k in range(1, kz + 1)]
            pc = [None] + [pold[k] + pt[k] + (cj[k] * (wo[k + 1] + wo[k]) + cdd[k] * (wo[k + 1] - wo[k])) * bm
                           for k in range(1, kz + 1)]
            for k in range(kz, 1, -1):
                den = aa[k] * e[k] + bb[k]
                e[k - 1] = -cq[k] / den
                f[k - 1] = (rhs[k] - f[k] * aa[k]) / den
            cols[(j, i)] = (wo, e, f, cj, cdd, wk, pold, pc)
    wpval = {c: 0.0 for c in cols}
    if ifupr:
        # :486-493: estore, astore at every interior column (pc[1]: the predicted pp at k = 1)
        est, ast = {}, {}
        for (j, i), (wo, e, f, cj, cdd, wk, pold, pc) in cols.items():
            den = (cdd[1] + cj[1]) * bp
            est[(j, i)] = pc[1] + f[1] * den
            ast[(j, i)] = den * e[1] + (cj[1] - cdd[1]) * bp
        # :506-543, the day alarm on the first step: the means and the mask
        atot = rhontot = 0.0
        for i in range(2, iy - 1):
            for j in range(2, jx - 1):
                atot = atot + ast[(j, i)]
                ensq = egrav * egrav / cpd / (a2t[0][i - 1][j - 1] * rpsb[i - 1, j - 1])
                rhontot = rhontot + rho1[0][i - 1][j - 1] * math.sqrt(ensq)
        rnpts = 1.0 / float(((iy - 1) - 2) * ((jx - 1) - 2))
        abar, rhon = atot * rnpts, rhontot * rnpts
        dxmsfb = 2.0 / (dx * dx) / data["split"]["nh_xmsf"]
        fk = [1.0] + [2.0] * 5 + [1.0]
        fw = {n: (0.5 if abs(n) == 6 else 1.0) for n in range(-6, 7)}
        tmask = {(jj, ii): 0.0 for ii in range(-6, 7) for jj in range(-6, 7)}
        for kk in range(7):
            for ll in range(7):
                xkeff = dxmsfb * math.sin(math.pi * kk / 12.0) * math.cos(math.pi * ll / 12.0)
                xleff = dxmsfb * math.sin(math.pi * ll / 12.0) * math.cos(math.pi * kk / 12.0)
                xkleff = math.sqrt(xkeff * xkeff + xleff * xleff)
                for ii in range(-6, 7):
                    for jj in range(-6, 7):
                        tmask[(jj, ii)] = tmask[(jj, ii)] + (fw[ii] * fw[jj] * fk[kk] * fk[ll]) / 144.0 * \
                            math.cos(2.0 * math.pi * kk * ii / 12.0) * math.cos(2.0 * math.pi * ll * jj / 12.0) * \
                            xkleff / (rhon - abar * xkleff)
        # :551-561: the convolution, indices clamped to icross1+1 .. icross2-1
        for (j, i) in cols:
            acc = 0.0
            for ii in range(-6, 7):
                inn = min(max(2, i + ii), (iy - 1) - 1)
                for jj in range(-6, 7):
                    jnn = min(max(2, j + jj), (jx - 1) - 1)
                    acc = acc + est[(jnn, inn)] * tmask[(jj, ii)]
            wpval[(j, i)] = acc
        assert max(abs(x) for x in wpval.values()) > 1e-6      # the lid moves
    for (j, i), (wo, e, f, cj, cdd, wk, pold, pc) in cols.items():
            wk[1] = wpval[(j, i)]
            for k in range(1, kz + 1):
                wk[k + 1] = e[k] * wk[k] + f[k]
            for k in range(1, kp + 1):
                wnew[k - 1][i - 1][j - 1] = wk[k]
            for k in range(1, kz + 1):
                cddt = xgamma * P1(k, i, j) * R0(k, i, j) * egrav * dts / (ps0[i - 1, j - 1] * dsig[k])
                cjt = R0(k, i, j) * egrav * dts * 0.5
                pn = pc[k] + (cjt * (wk[k + 1] + wk[k]) + cddt * (wk[k + 1] - wk[k])) * bp
                ppnew[k - 1][i - 1][j - 1] = pn
                pinew[k - 1][i - 1][j - 1] = pn - pold[k] - a["ppten"][k - 1][i - 1][j - 1]
                cpm = cpd * (1.0 + 0.80 * a["cqv"][k - 1][i - 1][j - 1])
                dpterm = psb[i - 1, j - 1] * (pn - pold[k]) / (cpm * R1(k, i, j))
                a2tn[k - 1][i - 1][j - 1] = a2tn[k - 1][i - 1][j - 1] + rc.gnu1 * dpterm
                a1t[k - 1][i - 1][j - 1] = a1t[k - 1][i - 1][j - 1] + dpterm
    # zero-gradient w on the boundary ring (:577-607): bottom/top rows, then left/right columns
    wnew[:, 0, 1:jx - 2] = wnew[:, 1, 1:jx - 2]
    wnew[:, 0, 0] = wnew[:, 1, 1]
    wnew[:, 0, jx - 2] = wnew[:, 1, jx - 3]
    wnew[:, iy - 2, 1:jx - 2] = wnew[:, iy - 3, 1:jx - 2]
    wnew[:, iy - 2, 0] = wnew[:, iy - 3, 1]
    wnew[:, iy - 2, jx - 2] = wnew[:, iy - 3, jx - 3]
    wnew[:, 1:iy - 2, 0] = wnew[:, 1:iy - 2, 1]
    wnew[:, 1:iy - 2, jx - 2] = wnew[:, 1:iy - 2, jx - 3]
    CI = (slice(None), slice(1, iy - 2), slice(1, jx - 2))
    CE = (slice(None), slice(0, iy - 1), slice(0, jx - 1))
    for name, want, got, sl in (("w", wnew, b["cw"], CE), ("pp", ppnew, b["cpp"], CI), ("pi", pinew, b["pi"], CI),
                                ("atm1 t", a1t, b["ATM1_T"], CI), ("atm2 t", a2tn, b["ATM2_T"], CI)):
        assert np.abs(want[sl]).max() > 0.0, name
        np.testing.assert_allclose(got[sl], want[sl], rtol=1e-11, atol=1e-12 * np.abs(want[sl]).max(), err_msg=name)
    assert not np.array_equal(b["cpp"][CI], a["cpp"][CI]) and not np.array_equal(b["cw"][CE], a["cw"][CE])


# ---- idiffu = 3: the sixth-order flux-limited column scheme ---------------------------------

def _psc2psd_np(pc):
    """psc2psd on the global grid, Main/mpplib/mod_mppparam.F90:13811-13862 (pc[i-1, j-1])."""
    iy, jx = pc.shape
    pd = np.empty_like(pc)
    P = lambda j, i: pc[i - 1, j - 1]  # noqa: E731
    for i in range(1, iy + 1):
        for j in range(1, jx + 1):
            jin, iin = 2 <= j <= jx - 1, 2 <= i <= iy - 1
            if jin and iin:
                v = (P(j, i) + P(j, i - 1) + P(j - 1, i) + P(j - 1, i - 1)) * 0.25
            elif jin and i == iy:
                v = (P(j, iy - 1) + P(j - 1, iy - 1)) * 0.5
            elif jin and i == 1:
                v = (P(j, 1) + P(j - 1, 1)) * 0.5
            elif iin and j == 1:
                v = (P(1, i) + P(1, i - 1)) * 0.5
            elif iin and j == jx:
                v = (P(jx - 1, i) + P(jx - 1, i - 1)) * 0.5
            else:
                v = P(1 if j == 1 else jx - 1, 1 if i == 1 else iy - 1)
            pd[i - 1, j - 1] = v
    return pd


def _diffu6_np(fv, lv, j, i, jmax, imax):
    """The bracket of Main/mod_diffusion.F90:428-470 / 618-648 at 1-based (j, i); fv, lv
    index [i-1, j-1]."""
    F = lambda jj, ii: fv[ii - 1, jj - 1]  # noqa: E731
    L = lambda jj, ii: lv[ii - 1, jj - 1]  # noqa: E731
    jm = [max(j - d, 1) for d in (1, 2, 3)]
    jp = [min(j + d, jmax) for d in (1, 2, 3)]
    im = [max(i - d, 1) for d in (1, 2, 3)]
    ip = [min(i + d, imax) for d in (1, 2, 3)]
    x0 = 10.0 * (F(j, i) - F(jm[0], i)) + -5.0 * (F(jp[0], i) - F(jm[1], i)) + 1.0 * (F(jp[1], i) - F(jm[2], i))
    x0 = 0.0 if x0 * (L(j, i) - L(jm[0], i)) <= 0.0 else x0
    x1 = 10.0 * (F(jp[0], i) - F(j, i)) + -5.0 * (F(jp[1], i) - F(jm[0], i)) + 1.0 * (F(jp[2], i) - F(jm[1], i))
    x1 = 0.0 if x1 * (L(jp[0], i) - L(j, i)) <= 0.0 else x1
    y0 = 10.0 * (F(j, i) - F(j, im[0])) + -5.0 * (F(j, ip[0]) - F(j, im[1])) + 1.0 * (F(j, ip[1]) - F(j, im[2]))
    y0 = 0.0 if y0 * (L(j, i) - L(j, im[0])) <= 0.0 else y0
    y1 = 10.0 * (F(j, ip[0]) - F(j, i)) + -5.0 * (F(j, ip[1]) - F(j, im[0])) + 1.0 * (F(j, ip[2]) - F(j, im[1]))
    y1 = 0.0 if y1 * (L(j, ip[0]) - L(j, i)) <= 0.0 else y1
    return (x1 - x0) + (y1 - y0)


def test_oracle_idiffu3_column_restatement(c1_data):
    """idiffu = 3 in the oracle against a NumPy restatement of Main/mod_diffusion.F90:412-516
    (diffu_d) and calc_coeff's :174-183: the u, v tendencies of one tend differ from a run
    whose diffusion is zero (idiffu = 1 with ckh = adyndif = 0) by diff_6th_coef * p*dotb *
    the bracket of u / msfd, on the column j = jdi2 only; and the qv forecast by the same for
    qxb3d (limiter on qxb3d / msfd) times the forecast's time step, on j = jci2 only."""
    import dataclasses
    from oracle.oracle import OracleCore
    rc, data = c1_data
    r3 = dataclasses.replace(rc, idiffu=3)
    r0 = dataclasses.replace(rc, idiffu=1, ckh=0.0, adyndif=0.0)
    out = {}
    for key, r in (("d6", r3), ("zero", r0)):
        o = OracleCore(r, data["split"])
        o.put_state(data["state"])
        o.bdyval()
        st = {n: o.get(n) for n in ("ATM2_U", "ATM2_V", "ATM2_QV", "PSB")}
        o.tend()
        out[key] = {n: o.get_work(n) for n in ("uten", "vten", "cqv")}
    jx, iy, kz = rc.jx, rc.iy, rc.kz
    coef = 0.12 * 0.015625 / (2.0 * rc.dt)
    psb = st["PSB"][0]
    psd = _psc2psd_np(psb)
    msfd = data["state"]["MSFD"][0]
    jd, jc = jx - 1, jx - 2                       # jdi2, jci2 of one tile
    for name, a2 in (("uten", st["ATM2_U"]), ("vten", st["ATM2_V"])):
        d = out["d6"][name] - out["zero"][name]
        assert not np.any(np.delete(d, jd - 1, axis=2)), name
        worst = 0.0
        for k in range(kz):
            um = (a2[k] * (1.0 / psd)) / msfd
            for i in range(2, iy):
                term = (coef * psd[i - 1, jd - 1]) * _diffu6_np(um, um, jd, i, jx, iy)
                worst = max(worst, abs(d[k, i - 1, jd - 1] - term) / max(abs(term), 1e-30))
        assert worst < 1e-8, (name, worst)
    d = out["d6"]["cqv"] - out["zero"]["cqv"]
    assert not np.any(np.delete(d, jc - 1, axis=2))
    ratios = []
    for k in range(kz):
        with np.errstate(divide="ignore", invalid="ignore"):     # p*b is 0 on the dot-only row/column
            qb = np.maximum(st["ATM2_QV"][k] * (1.0 / psb), 1e-8)
        for i in range(2, iy - 1):
            term = (coef * psb[i - 1, jc - 1]) * _diffu6_np(qb, qb / msfd, jc, i, jx - 1, iy - 1)
            if abs(term) > 1e-14:
                ratios.append(d[k, i - 1, jc - 1] / term)
    ratios = np.array(ratios)
    assert ratios.size > 10
    dt2 = ratios.mean()
    assert any(abs(dt2 - x) < 1e-6 * x for x in (rc.dt, 2.0 * rc.dt)), dt2
    assert np.max(np.abs(ratios - dt2)) < 1e-6 * dt2


@pytest.mark.parametrize("core", ["hydrostatic", "nh"])
def test_centred_advection_equals_upstream_without_offcentring(core, c1_data):
    """upstream_mode = .false. (the centred branches of Main/mod_advection.F90:141-201, 322-335,
    409-460, 532-545, 624-637, restated as written in the oracle) is bit for bit the upstream
    form with uoffc = 0: the identity the engine's centred mode (ul = 0) rests on."""
    import dataclasses
    from oracle.oracle import OracleCore
    from regcm_amd.config import CONFIGS, NH_STATE_FIELDS, STATE_FIELDS
    from regcm_amd import icbc
    if core == "hydrostatic":
        rc, data = c1_data
        names = STATE_FIELDS
    else:
        rc = CONFIGS["N1"]
        data = icbc.generate_nh(rc)
        names = list(STATE_FIELDS) + list(NH_STATE_FIELDS)
    runs = []
    for kw in ({"upstream_mode": 0}, {"uoffc": 0.0}, {}):
        o = OracleCore(dataclasses.replace(rc, **kw), data["split"])
        o.put_state(data["state"])
        o.bdyval()
        o.step(4)
        runs.append({n: o.get(n) for n in names})
    for n in names:
        assert np.array_equal(runs[0][n], runs[1][n]), n
    assert any(not np.array_equal(runs[0][n], runs[2][n]) for n in names)


def _species_run(rc, data, st, nsteps):
    from oracle.oracle import OracleCore
    o = OracleCore(rc, data["split"])
    o.put_state(st)
    o.bdyval()
    o.step(nsteps)
    return o


@pytest.mark.parametrize("core", ["hydrostatic", "nh"])
def test_oracle_species_follow_qc_chain(c1_data, core):
    """nqx = 5 (ipptls = 2): every hydrometeor n = iqfrst..iqlst runs qc's chain of the dyn step
    (hadvqx, vadv4d, diffu_x4d, the NH + atmx%qx*cr, the fix, filter_raw_4d's zero floor,
    bdyval's copies and inflow/outflow), Main/mod_tendency.F90:331-335, 375-393, 426-427,
    1378-1388, 1526, 1615-1617; Main/mod_bdycod.F90:1143-1284, 2153-2220.  With qi = qr = qs = qc
    at the start, the four stay bit-identical over the steps (the restatement's species loop
    against its qc code)."""
    import dataclasses
    if core == "nh":
        rc = dataclasses.replace(CONFIGS["N1"], ipptls=2)
        data = icbc.generate_nh(rc)
    else:
        rc = dataclasses.replace(c1_data[0], ipptls=2)
        data = c1_data[1]
    st = dict(data["state"])
    st.update(icbc.hydrometeor_state(rc, st, nqx=5))
    for lev in ("ATM1", "ATM2"):
        for sp in ("QI", "QR", "QS"):
            st[f"{lev}_{sp}"] = st[f"{lev}_QC"].copy()
    o = _species_run(rc, data, st, 3)
    for lev in ("ATM1", "ATM2"):
        qc = o.get(f"{lev}_QC")
        assert np.abs(qc - st[f"{lev}_QC"]).max() > 0.0
        for sp in ("QI", "QR", "QS"):
            assert np.array_equal(o.get(f"{lev}_{sp}"), qc), (lev, sp)


@pytest.mark.parametrize("core", ["hydrostatic", "nh"])
def test_oracle_species_water_load(c1_data, core):
    """The total water load of decouple, qcd = ((qc + qi) + qr) + qs (Main/mod_tendency.F90:
    1107-1115), is what tvfac (:2037, hydrostatic) and the NH water loading of w (:1662-1671) read:
    an ipptls = 2 start with qi = qc, qr = qs = 0 loads 2 qc exactly, so its first step's
    winds, temperature, p* (and NH pp, w) equal those of an ipptls = 1 start with qc doubled."""
    import dataclasses
    if core == "nh":
        rc1 = CONFIGS["N1"]
        data = icbc.generate_nh(rc1)
        dyn = ["ATM1_U", "ATM1_V", "ATM1_T", "ATM1_QV", "PSA", "ATM1_PP", "ATM1_W"]
    else:
        rc1, data = c1_data
        dyn = ["ATM1_U", "ATM1_V", "ATM1_T", "ATM1_QV", "PSA"]
    rc2 = dataclasses.replace(rc1, ipptls=2)
    st = dict(data["state"])
    st.update(icbc.hydrometeor_state(rc2, st, nqx=5))
    st2 = dict(st)
    st1 = {k: v for k, v in st.items() if k[5:] not in ("QI", "QR", "QS")}
    for lev in ("ATM1", "ATM2"):
        st2[f"{lev}_QI"] = st[f"{lev}_QC"].copy()
        st2[f"{lev}_QR"] = np.zeros_like(st[f"{lev}_QC"])
        st2[f"{lev}_QS"] = np.zeros_like(st[f"{lev}_QC"])
        st1[f"{lev}_QC"] = 2.0 * st[f"{lev}_QC"]
    o2 = _species_run(rc2, data, st2, 1)
    o1 = _species_run(rc1, data, st1, 1)
    for name in dyn:
        assert np.array_equal(o2.get(name), o1.get(name)), name
    # and the load matters: the same start without the species differs
    st0 = {k: v for k, v in st1.items()}
    for lev in ("ATM1", "ATM2"):
        st0[f"{lev}_QC"] = st[f"{lev}_QC"]
    o0 = _species_run(rc1, data, st0, 1)
    assert not np.array_equal(o0.get("ATM1_U"), o1.get("ATM1_U"))
