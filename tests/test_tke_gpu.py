"""GPU parity of the UW-PBL TKE in the dyn step (ibltyp = 2).

The reference advects atm1%tke (hadv3d ind = 1, vadv3d of tke*p*), diffuses atm2%tke with nuk,
forecasts with the tkemin floor and Robert-Asselin filters it (Main/mod_tendency.F90:515-544,
1414-1425, 1545-1548), and bounds it in bdyval (Main/mod_bdycod.F90:1166-1306, 2415-2530).
Tolerances: the TKE kernels have no transcendental function; they read qdot and the
diffusion coefficients of the step, whose ulps follow the step's own bounds
(tests/test_parity_gpu.py), so the TKE is held to the same 1e-12 (one step) and 1e-11
(three steps) relative max-norm; decompositions are bit-identical; the TKE leaves every other
field bit-identical.
"""
import dataclasses

import numpy as np
import pytest

from regcm_amd import icbc
from regcm_amd.config import CONFIGS, NH_STATE_FIELDS, STATE_FIELDS, TKE_STATE_FIELDS

pytestmark = pytest.mark.gpu

CROSS = {"ATM1_TKE", "ATM2_TKE"}


def relerr(a, b, rc, name):
    if name in CROSS:
        a = a[:, : rc.iy - 1, : rc.jx - 1]
        b = b[:, : rc.iy - 1, : rc.jx - 1]
    den = max(np.max(np.abs(b)), 1e-300)
    return float(np.max(np.abs(a - b)) / den)


def start(c, rc, data, tke=True):
    c.put_state(data["state"])
    if tke:
        for name, a in icbc.tke_state(rc).items():
            c.put(name, a)
    c.bdyval()
    return c


@pytest.fixture(scope="module")
def tke_c1(c1_data):
    rc, data = c1_data
    return dataclasses.replace(rc, ibltyp=2), data


@pytest.fixture(scope="module")
def tke_n1():
    rc = dataclasses.replace(CONFIGS["N1"], ibltyp=2)
    return rc, icbc.generate_nh(rc)


def pair(rc, data, nproc=(1, 1)):
    from oracle.oracle import OracleCore
    from regcm_amd.dycore import DynCore
    o = start(OracleCore(rc, data["split"]), rc, data)
    e = start(DynCore(rc, data["split"], nproc_j=nproc[0], nproc_i=nproc[1]), rc, data)
    return o, e


def test_tke_init_bdyval_exact(tke_c1):
    rc, data = tke_c1
    o, e = pair(rc, data)
    for name in TKE_STATE_FIELDS:
        assert np.array_equal(e.get(name), o.get(name)), name


@pytest.mark.parametrize("variant", [{}, {"idiffu": 2}, {"idiffu": 3}, {"iboudy": 4}, {"iboudy": 3}, {"upstream_mode": 0}],
                         ids=lambda v: ",".join(f"{k}={x}" for k, x in v.items()) or "default")
def test_tke_parity(tke_c1, variant):
    rc, data = tke_c1
    rc = dataclasses.replace(rc, **variant)
    o, e = pair(rc, data)
    for nsteps, tol in ((1, 1e-12), (2, 1e-11)):
        o.step(nsteps)
        e.step(nsteps)
        for name in TKE_STATE_FIELDS:
            err = relerr(e.get(name), o.get(name), rc, name)
            assert err < tol, (name, err, nsteps)
    t = e.get("ATM1_TKE")[:, : rc.iy - 1, : rc.jx - 1]
    assert t.min() >= rc.tkemin
    assert not np.array_equal(e.get("ATM1_TKE"), icbc.tke_state(rc)["ATM1_TKE"])


def test_tke_leaves_the_state_alone(tke_c1, c1_data):
    from regcm_amd.dycore import DynCore
    rc, data = tke_c1
    rc0, _ = c1_data
    a = start(DynCore(rc, data["split"]), rc, data)
    b = start(DynCore(rc0, data["split"]), rc0, data, tke=False)
    a.step(4)
    b.step(4)
    for name in STATE_FIELDS:
        assert np.array_equal(a.get(name), b.get(name)), name


@pytest.mark.parametrize("nproc", [(2, 2), (1, 3)])
def test_tke_decomposition_invariance(tke_c1, nproc):
    from regcm_amd.dycore import DynCore
    rc, data = tke_c1
    a = start(DynCore(rc, data["split"]), rc, data)
    b = start(DynCore(rc, data["split"], nproc_j=nproc[0], nproc_i=nproc[1]), rc, data)
    a.step(5)
    b.step(5)
    for name in TKE_STATE_FIELDS + STATE_FIELDS:
        assert np.array_equal(a.get(name), b.get(name)), name


def test_tke_physics_tendency(tke_c1):
    """The UW scheme's tendency (TKEPHY) enters tketen after the dyn part (:530-531)."""
    rc, data = tke_c1
    o, e = pair(rc, data)
    rng = np.random.Generator(np.random.PCG64(3))
    phy = 1e-4 * rng.standard_normal((rc.kz + 1, rc.iy, rc.jx))
    for c in (o, e):
        c.put("TKEPHY", phy)
        c.step(3)
    for name in TKE_STATE_FIELDS:
        assert relerr(e.get(name), o.get(name), rc, name) < 1e-11, name
    assert np.array_equal(e.get("TKEPHY"), phy)


def test_nh_tke_parity(tke_n1):
    rc, data = tke_n1
    o, e = pair(rc, data)
    for nsteps, tol in ((1, 1e-11), (2, 1e-10)):
        o.step(nsteps)
        e.step(nsteps)
        for name in TKE_STATE_FIELDS:
            err = relerr(e.get(name), o.get(name), rc, name)
            assert err < tol, (name, err, nsteps)
    from regcm_amd.dycore import DynCore
    til = start(DynCore(rc, data["split"], nproc_j=2, nproc_i=2), rc, data)
    ref = start(DynCore(rc, data["split"]), rc, data)
    til.step(4)
    ref.step(4)
    for name in TKE_STATE_FIELDS + NH_STATE_FIELDS:
        assert np.array_equal(til.get(name), ref.get(name)), name


@pytest.mark.parametrize("core", ["hydrostatic", "nh"])
def test_tke_idiffu3_tiles_match_oracle_tiles(tke_c1, tke_n1, core):
    """idiffu = 3 with the TKE (diffu_x3df of atm2 tke with nuk on each tile's column j = jci2,
    Main/mod_diffusion.F90:602-651) on 2 x 2 tiles against the oracle run as the same tiles."""
    from oracle.oracle import OracleParallel
    from regcm_amd.dycore import DynCore
    rc, data = tke_c1 if core == "hydrostatic" else tke_n1
    rc = dataclasses.replace(rc, idiffu=3)
    o = start(OracleParallel(rc, data["split"], nthreads=4), rc, data)
    e = start(DynCore(rc, data["split"], nproc_j=2, nproc_i=2), rc, data)
    tol = 1e-11 if core == "hydrostatic" else 1e-10
    o.step(2)
    e.step(2)
    for name in TKE_STATE_FIELDS:
        err = relerr(e.get(name), o.get(name), rc, name)
        assert err < tol, (name, err)


def test_tke_errors(c1_data, tke_c1):
    from regcm_amd.dycore import DynCore, EngineError
    rc, data = c1_data
    e = DynCore(rc, data["split"])
    with pytest.raises(EngineError, match="ibltyp=2"):
        e.put("ATM1_TKE", np.zeros((rc.kz + 1, rc.iy, rc.jx)))
    rc2, _ = tke_c1
    e2 = DynCore(rc2, data["split"])
    with pytest.raises(EngineError, match="no TKE tendency"):
        e2.get("TKEPHY")


def test_tke_restart_bit_identical(tke_c1):
    """SAV restart with the UW TKE (mod_savefile writes atm1/atm2 tke for ibltyp = 2): the
    continued run equals the uninterrupted one bit for bit, also on another decomposition."""
    from regcm_amd.dycore import DynCore
    rc, data = tke_c1
    ref = start(DynCore(rc, data["split"]), rc, data)
    ref.step(6)
    run = start(DynCore(rc, data["split"]), rc, data)
    run.step(3)
    names = STATE_FIELDS + TKE_STATE_FIELDS
    sav = {n: run.get(n) for n in names}
    clock = run.get_time()
    run.close()
    rst = DynCore(rc, data["split"], nproc_j=2, nproc_i=2)
    rst.put_state(data["state"])                  # statics and boundary data
    for n, a in sav.items():
        rst.put(n, a)
    rst.set_time(*clock)
    rst.step(3)
    for n in names:
        assert np.array_equal(rst.get(n), ref.get(n)), n


def _uw(rc, data):
    """iuwvadv = 1 state: a structured cloud layer and a PBL-top field (tests/test_oracle_cpu.py)."""
    from tests.test_oracle_cpu import _uw_kpbl, _uw_qc_state
    return dataclasses.replace(rc, iuwvadv=1), _uw_qc_state(rc, data["state"]), _uw_kpbl(rc)


@pytest.mark.parametrize("core", ["hydrostatic", "nh"])
def test_uw_vertical_flux_parity(tke_c1, tke_n1, core):
    """iuwvadv = 1 (vadv4d ind = 3 of qc with the host's kpbl, Main/mod_advection.F90:917-961):
    the engine against the oracle, both cores, with a new kpbl put between the steps as the UW
    scheme does; the qc tendency differs from iuwvadv = 0's.  One step within 1e-11.  Later
    steps are held to the oracle's own spread under a 1e-14 perturbation of t: the rule's
    overshoot test at kpbl compares |f(kpb-2) + slope dh - f(kpb)| with |f(kpb-1) - f(kpb)|,
    which are the same number whenever the min/max picks the upper layer's gradient, so an
    ulp of input difference (the log/pow of the PGF reach qdot) decides that branch."""
    from oracle.oracle import OracleCore
    from regcm_amd.dycore import DynCore
    rc, data = tke_c1 if core == "hydrostatic" else tke_n1
    rcu, st, kpbl = _uw(rc, data)
    kpbl2 = np.roll(kpbl, 3, axis=-1)

    def start(cls, state):
        c = cls(rcu, data["split"])
        c.put_state(state)
        for name, a in icbc.tke_state(rcu).items():
            c.put(name, a)
        c.put("KPBL", kpbl)
        c.bdyval()
        return c
    o, e = start(OracleCore, st), start(DynCore, st)
    stp = dict(st)
    stp["ATM1_T"] = st["ATM1_T"] * (1.0 + 1e-14)
    p = start(OracleCore, stp)
    for n, c in enumerate((o, e, p)):
        c.step(1)
        if n < 2:
            for name in STATE_FIELDS:
                err = relerr(e.get(name), o.get(name), rcu, name) if n == 1 else 0.0
                assert err < 1e-11, (name, err)
    for c in (o, e, p):
        c.put("KPBL", kpbl2)
        c.step(3)
    for name in STATE_FIELDS:
        err = relerr(e.get(name), o.get(name), rcu, name)
        spread = relerr(p.get(name), o.get(name), rcu, name)
        assert err <= max(1e-10, 100.0 * spread), (name, err, spread)
    base = DynCore(rc, data["split"])
    base.put_state(st)
    for name, a in icbc.tke_state(rc).items():
        base.put(name, a)
    base.bdyval()
    base.step(4)
    assert not np.array_equal(base.get("ATM1_QC"), e.get("ATM1_QC"))


def test_uw_decomposition_and_refusal(tke_c1):
    """iuwvadv = 1 is bit-identical on 2 x 2 tiles; a kpbl above kz is refused at the put
    ('kpbl is greater than kz', Main/mod_advection.F90:923-925)."""
    from regcm_amd.dycore import DynCore, EngineError
    rc, data = tke_c1
    rcu, st, kpbl = _uw(rc, data)
    runs = []
    for nproc in ((1, 1), (2, 2)):
        e = DynCore(rcu, data["split"], nproc_j=nproc[0], nproc_i=nproc[1])
        e.put_state(st)
        for name, a in icbc.tke_state(rcu).items():
            e.put(name, a)
        e.put("KPBL", kpbl)
        e.bdyval()
        e.step(4)
        runs.append(e)
    for name in STATE_FIELDS:
        assert np.array_equal(runs[0].get(name), runs[1].get(name)), name
    bad = kpbl.copy()
    bad[0, 5, 5] = rcu.kz + 1
    with pytest.raises(EngineError, match="kpbl is greater than kz"):
        runs[0].put("KPBL", bad)
