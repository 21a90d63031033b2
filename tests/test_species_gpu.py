"""nqx = 5 (physicsparam ipptls = 2, Main/mod_params.F90:1358-1366): the hydrometeors qi, qr, qs
go through qc's chain of the dyn step (hadvqx, vadv4d, diffu_x4d, the sums with qxphy, the
forecast and negative-moisture fix, filter_raw_4d, bdyval's copies and inflow/outflow lines) and
the total water load enters tvfac (hydrostatic) and the water loading (NH).  The HIP engine is
checked against the oracle's restatement through the C-ABI, on one tile and decomposed.

Tolerances as tests/test_parity_gpu.py: the hydrometeor chain has no transcendental function,
so after one step the species are bit-identical to the oracle; later steps inherit the ulps of
the PGF / vadv3d powers through qdot and the winds (< 1e-11 after 3 steps)."""
import dataclasses

import numpy as np
import pytest

from regcm_amd import icbc
from regcm_amd.config import CONFIGS, QX_ATMS_FIELDS, QX_STATE_FIELDS, QX_PHY_FIELDS, STATE_FIELDS

pytestmark = pytest.mark.gpu

ALL = list(STATE_FIELDS) + QX_STATE_FIELDS
CROSS = {"ATM1_T", "ATM1_QV", "ATM1_QC", "ATM2_T", "ATM2_QV", "ATM2_QC", "PSA", "PSB", "DSTOR", "HSTOR"} | \
    set(QX_STATE_FIELDS)


def relerr(a, b, rc, name):
    if name in CROSS:
        a = a[:, : rc.iy - 1, : rc.jx - 1]
        b = b[:, : rc.iy - 1, : rc.jx - 1]
    den = max(np.max(np.abs(b)), 1e-300)
    return float(np.max(np.abs(a - b)) / den)


def species_state(rc, data):
    st = {k: v.copy() for k, v in data["state"].items()}
    st.update(icbc.hydrometeor_state(rc, st, nqx=rc.nqx))
    return st


def start(cls, rc, data, st, nproc=(1, 1), extra=None):
    if cls.__name__ == "DynCore":
        c = cls(rc, data["split"], nproc_j=nproc[0], nproc_i=nproc[1])
    else:
        c = cls(rc, data["split"])
    c.put_state(st)
    for name, a in (extra or {}).items():
        c.put(name, a)
    c.bdyval()
    return c


@pytest.fixture(scope="module")
def qx_c1(c1_data):
    rc, data = c1_data
    rcq = dataclasses.replace(rc, ipptls=2)
    return rcq, data, species_state(rcq, data)


VARIANTS = [{}, {"isladvec": 1}, {"idiffu": 2}, {"idiffu": 3}, {"iboudy": 4}, {"iboudy": 3},
            {"upstream_mode": 0}]


def _vid(v):
    return ",".join(f"{k}={x}" for k, x in v.items()) or "default"


@pytest.mark.parametrize("variant", VARIANTS, ids=_vid)
def test_species_parity(qx_c1, variant):
    """ipptls = 2 against the oracle: the species bit-identical after one step (their chain has
    no transcendental; qdot, the mass fluxes and xkc are exact), every field < 1e-11 after 3."""
    from oracle.oracle import OracleCore
    from regcm_amd.dycore import DynCore
    rc, data, st = qx_c1
    rcv = dataclasses.replace(rc, **variant)
    o, e = start(OracleCore, rcv, data, st), start(DynCore, rcv, data, st)
    o.step(1)
    e.step(1)
    # the interior bit-identical (the boundary lines take p* of the split corrections, which
    # carry the powers' ulps through delh)
    for name in QX_STATE_FIELDS:
        a, b = e.get(name)[:, 1:rcv.iy - 2, 1:rcv.jx - 2], o.get(name)[:, 1:rcv.iy - 2, 1:rcv.jx - 2]
        ndiff = int((a != b).sum())
        assert ndiff == 0, (name, ndiff)
    for name in ALL:
        err = relerr(e.get(name), o.get(name), rcv, name)
        assert err < 1e-12, (name, err)
    o.step(2)
    e.step(2)
    for name in ALL:
        err = relerr(e.get(name), o.get(name), rcv, name)
        assert err < 1e-11, (name, err)


def test_species_change_the_step(qx_c1, c1_data):
    """The species are advected and their load reaches the geopotential: qi moves, and the
    temperature of an ipptls = 2 run differs from ipptls = 1 with the same qv, qc."""
    from regcm_amd.dycore import DynCore
    rc, data, st = qx_c1
    e = start(DynCore, rc, data, st)
    e.step(3)
    assert not np.array_equal(e.get("ATM1_QI"), st["ATM1_QI"])
    rc1 = c1_data[0]
    st1 = {k: v for k, v in st.items() if k not in QX_STATE_FIELDS}
    e1 = start(DynCore, rc1, data, st1)
    e1.step(3)
    assert not np.array_equal(e.get("ATM1_U"), e1.get("ATM1_U"))


def test_species_negative_fix(qx_c1):
    """The patchy cloud edges make negative species forecasts, some with negative sweep
    predecessors (the serial sweep); the fix is bit-identical to the oracle's serial loop."""
    from oracle.oracle import OracleCore
    from regcm_amd.dycore import DynCore
    from tests.test_parity_gpu import _dependent_negatives
    rc, data, st = qx_c1
    o, e = start(OracleCore, rc, data, st), start(DynCore, rc, data, st)
    o.tend()
    e.tend()
    dt = o.get_time()[1]
    dep = 0
    for nm, sp in (("qteni", "QI"), ("qtenr", "QR"), ("qtens", "QS")):
        # the forecast before the fix: atm2 + dt * qxten on the interior
        dep += _dependent_negatives(st[f"ATM2_{sp}"] + dt * o.get_work(nm), rc)
    # the fix rewrote the negatives: compare the filtered state after tend
    for name in QX_STATE_FIELDS:
        a, b = e.get(name)[:, 1:rc.iy - 2, 1:rc.jx - 2], o.get(name)[:, 1:rc.iy - 2, 1:rc.jx - 2]
        ndiff = int((a != b).sum())
        assert ndiff == 0, (name, ndiff)
    assert dep > 0


@pytest.mark.parametrize("nthreads", [2, 3, 4, 7])
def test_species_tiles_match_oracle_tiles(qx_c1, monkeypatch, nthreads):
    """Decomposed: against the oracle run as the same set_nproc tiles (oracle/orc_par.c).  The
    reference exchanges atmc%qx before its negative-moisture fix (Main/mod_tendency.F90:381-393),
    so a tile's first interior column reads its neighbour's unfixed forecast where one tile reads
    the fixed value: with negative hydrometeor forecasts at a tile edge the reference itself
    depends on the decomposition, and so does the engine, tile for tile.  1 x 7 tiles are
    narrower than the split step's halo (its per-sub-step exchanges and the exchange of atmc%qx
    run as the reference's).  Species interior bit-identical after one step; < 1e-11 after 3."""
    from oracle.oracle import OracleParallel
    from regcm_amd.config import set_nproc
    from regcm_amd.dycore import DynCore
    rc, data, st = qx_c1
    cj, ci = set_nproc(nthreads, rc.jx, rc.iy)
    o = OracleParallel(rc, data["split"], nthreads=nthreads)
    o.put_state(st)
    o.bdyval()
    e = start(DynCore, rc, data, st, (cj, ci))
    o.step(1)
    e.step(1)
    for name in QX_STATE_FIELDS:
        a, b = e.get(name)[:, 1:rc.iy - 2, 1:rc.jx - 2], o.get(name)[:, 1:rc.iy - 2, 1:rc.jx - 2]
        ndiff = int((a != b).sum())
        assert ndiff == 0, (name, ndiff)
    o.step(2)
    e.step(2)
    for name in ALL:
        err = relerr(e.get(name), o.get(name), rc, name)
        assert err < 1e-11, (name, err)


@pytest.mark.parametrize("nthreads", [2, 4])
def test_qc_tiles_match_oracle_tiles(c1_data, nthreads):
    """nqx = 2 with cloud water: the qc chain on decomposed tiles against the oracle's tiles
    (the fix's decomposition dependence above applies to qc as well)."""
    from oracle.oracle import OracleParallel
    from regcm_amd.config import set_nproc
    from regcm_amd.dycore import DynCore
    rc, data = c1_data
    st = species_state(rc, data)
    cj, ci = set_nproc(nthreads, rc.jx, rc.iy)
    o = OracleParallel(rc, data["split"], nthreads=nthreads)
    o.put_state(st)
    o.bdyval()
    e = start(DynCore, rc, data, st, (cj, ci))
    o.step(1)
    e.step(1)
    a, b = e.get("ATM1_QC")[:, 1:rc.iy - 2, 1:rc.jx - 2], o.get("ATM1_QC")[:, 1:rc.iy - 2, 1:rc.jx - 2]
    assert int((a != b).sum()) == 0
    o.step(2)
    e.step(2)
    for name in STATE_FIELDS:
        err = relerr(e.get(name), o.get(name), rc, name)
        assert err < 1e-11, (name, err)


@pytest.mark.parametrize("nproc", [(2, 2), (1, 7)], ids=str)
def test_species_rccl_transport(qx_c1, monkeypatch, nproc):
    """The same tiles with their halos sent over RCCL (one-rank self send/receive) are
    bit-identical to the device-copy exchange."""
    from regcm_amd.dycore import DynCore
    rc, data, st = qx_c1
    ref = start(DynCore, rc, data, st, nproc)
    monkeypatch.setenv("RCMDYN_FORCE_RCCL", "1")
    til = start(DynCore, rc, data, st, nproc)
    for e in (ref, til):
        e.step(4)
    for name in ALL:
        same = np.array_equal(ref.get(name), til.get(name))
        assert same, name


@pytest.mark.parametrize("env", ["RCMDYN_NO_QFUSE", "RCMDYN_NO_FUSE_BDY", "RCMDYN_NO_GRAPH"])
def test_species_step_forms(qx_c1, monkeypatch, env):
    """The step forms (qfuse, the fused bdyval, graph replay) and the drop-in call sequence agree
    bit for bit with species."""
    from regcm_amd.dycore import DynCore
    rc, data, st = qx_c1
    ref = start(DynCore, rc, data, st)
    monkeypatch.setenv(env, "1")
    alt = start(DynCore, rc, data, st)
    ref.step(5)
    for _ in range(5):
        alt.tend()
        alt.bdyval()
    for name in ALL:
        same = np.array_equal(ref.get(name), alt.get(name))
        assert same, name


@pytest.mark.parametrize("name", ["C1", "C3"])
def test_negfix_wavefront_equals_row_sweep(name, monkeypatch):
    """The serial fix of a dense plane two ways (qxcommon.hpp): the skewed wavefront (default)
    and the row sweep in the reference's order (RCMDYN_NEGFIX_MODE=1) give the same state bit for
    bit, on the patchy hydrometeor fields whose qi / qr / qs and qc planes hold chains of
    dependent negatives (at C3, the grid of tools/species_bench.py, hundreds of links deep)."""
    from regcm_amd.dycore import DynCore
    rc = dataclasses.replace(CONFIGS[name], ipptls=2)
    data = icbc.generate(CONFIGS[name])
    st = species_state(rc, data)
    runs = []
    for mode in ("0", "1"):
        monkeypatch.setenv("RCMDYN_NEGFIX_MODE", mode)
        e = start(DynCore, rc, data, st)
        e.step(4)
        runs.append(e)
    for name_ in ALL:
        assert np.array_equal(runs[0].get(name_), runs[1].get(name_)), name_


def test_species_physics_seam(qx_c1):
    """qxphy of qi, qr, qs enter the sums as the reference adds them (:332-335), against the
    oracle; pre + post physics is the whole tend."""
    from oracle.oracle import OracleCore
    from regcm_amd.dycore import DynCore
    rc, data, st = qx_c1
    rng = np.random.default_rng(11)
    phy = {n: rng.normal(0.0, 1e-9, (rc.kz, rc.iy, rc.jx)) * st["PSA"][0][None] for n in QX_PHY_FIELDS}
    o, e = start(OracleCore, rc, data, st, extra=phy), start(DynCore, rc, data, st, extra=phy)
    o.step(1)
    e.tend_pre_physics()
    e.tend_post_physics()
    e.bdyval()
    for name in QX_STATE_FIELDS:
        a, b = e.get(name)[:, 1:rc.iy - 2, 1:rc.jx - 2], o.get(name)[:, 1:rc.iy - 2, 1:rc.jx - 2]
        ndiff = int((a != b).sum())
        assert ndiff == 0, (name, ndiff)
        err = relerr(e.get(name), o.get(name), rc, name)
        assert err < 1e-12, (name, err)
    for name in QX_PHY_FIELDS:
        same = np.array_equal(e.get(name), phy[name])
        assert same, name
    # the mkslice export qxb3d of the species (Main/mod_slice.F90:193-195), as the physics reads it
    for name in QX_ATMS_FIELDS:
        same = np.array_equal(e.get(name), o.get(name))
        assert same, name


def test_species_restart(qx_c1):
    """A restart from the species' SAV fields (get / put) continues bit-identically."""
    from regcm_amd.dycore import DynCore
    rc, data, st = qx_c1
    ref = start(DynCore, rc, data, st)
    ref.step(3)
    sav = {n: ref.get(n) for n in ALL}
    t = ref.get_time()
    rst = DynCore(rc, data["split"])
    for n in ("MSFX", "MSFD", "CORIOL", "HT", "XUB_B0", "XUB_BT", "XVB_B0", "XVB_BT", "XTB_B0", "XTB_BT",
              "XQB_B0", "XQB_BT", "XPSB_B0", "XPSB_BT"):
        rst.put(n, st[n])
    for n, a in sav.items():
        rst.put(n, a)
    rst.set_time(*t)
    ref.step(3)
    rst.step(3)
    for n in ALL:
        same = np.array_equal(rst.get(n), ref.get(n))
        assert same, n


def test_species_fields_refused_for_nqx2(c1_data):
    from regcm_amd.dycore import DynCore, EngineError
    rc, data = c1_data
    e = DynCore(rc, data["split"])
    with pytest.raises(EngineError, match="nqx = 5"):
        e.put("ATM1_QI", np.zeros((rc.kz, rc.iy, rc.jx)))
    with pytest.raises(EngineError, match="nqx = 5"):
        e.get("ATM2_QS")


# ----------------------------------------------------------------- non-hydrostatic core
# The NH chain of the species (k_nh_qx_tend): hadvqx, vadv4d, + atmx%qx * cr of adiabatic
# (Main/mod_tendency.F90:1615-1617), diffu_x4d, the sums, the forecast, the exchange of atmc%qx,
# the fix and filter_raw_4d in place; the total load enters the water loading of w
# (:1662-1671).  Tolerances as tests/test_nh_gpu.py (the NH step is transcendental almost
# everywhere: 1e-11 after one step, 1e-10 after three).
NH_ALL = ["ATM1_U", "ATM1_V", "ATM1_T", "ATM1_QV", "ATM1_QC", "ATM2_U", "ATM2_V", "ATM2_T", "ATM2_QV", "ATM2_QC",
          "PSA", "PSB", "ATM1_PP", "ATM2_PP", "ATM1_W", "ATM2_W"] + QX_STATE_FIELDS
NH_CROSS = CROSS | {"ATM1_PP", "ATM2_PP", "ATM1_W", "ATM2_W"}


def nh_relerr(a, b, rc, name):
    if name in NH_CROSS:
        a = a[:, : rc.iy - 1, : rc.jx - 1]
        b = b[:, : rc.iy - 1, : rc.jx - 1]
    den = max(np.max(np.abs(b)), 1e-300)
    return float(np.max(np.abs(a - b)) / den)


@pytest.fixture(scope="module")
def qx_n1():
    rc = dataclasses.replace(CONFIGS["N1"], ipptls=2)
    data = icbc.generate_nh(rc)
    return rc, data, species_state(rc, data)


NH_VARIANTS = [{}, {"isladvec": 1}, {"idiffu": 2}, {"idiffu": 3}, {"iboudy": 4}]


@pytest.mark.parametrize("variant", NH_VARIANTS, ids=_vid)
def test_nh_species_parity(qx_n1, variant):
    from oracle.oracle import OracleCore
    from regcm_amd.dycore import DynCore
    rc, data, st = qx_n1
    rcv = dataclasses.replace(rc, **variant)
    o, e = start(OracleCore, rcv, data, st), start(DynCore, rcv, data, st)
    for nsteps, tol in ((1, 1e-11), (2, 1e-10)):
        o.step(nsteps)
        e.step(nsteps)
        for name in NH_ALL:
            err = nh_relerr(e.get(name), o.get(name), rcv, name)
            assert err < tol, (name, err, nsteps)


def test_nh_species_change_the_step(qx_n1):
    """The species' load reaches w through the water loading: an ipptls = 2 run differs from
    ipptls = 1 with the same qv, qc."""
    from regcm_amd.dycore import DynCore
    rc, data, st = qx_n1
    e = start(DynCore, rc, data, st)
    e.step(2)
    assert not np.array_equal(e.get("ATM1_QR"), st["ATM1_QR"])
    rc1 = dataclasses.replace(rc, ipptls=1)
    st1 = {k: v for k, v in st.items() if k not in QX_STATE_FIELDS}
    e1 = start(DynCore, rc1, data, st1)
    e1.step(2)
    assert not np.array_equal(e.get("ATM1_W"), e1.get("ATM1_W"))


@pytest.mark.parametrize("nthreads", [2, 4])
def test_nh_species_tiles_match_oracle_tiles(qx_n1, nthreads):
    """The NH core decomposed, against the oracle's same tiles (the fix's decomposition
    dependence as test_species_tiles_match_oracle_tiles)."""
    from oracle.oracle import OracleParallel
    from regcm_amd.config import set_nproc
    from regcm_amd.dycore import DynCore
    rc, data, st = qx_n1
    cj, ci = set_nproc(nthreads, rc.jx, rc.iy)
    o = OracleParallel(rc, data["split"], nthreads=nthreads)
    o.put_state(st)
    o.bdyval()
    e = start(DynCore, rc, data, st, (cj, ci))
    for nsteps, tol in ((1, 1e-11), (2, 1e-10)):
        o.step(nsteps)
        e.step(nsteps)
        for name in NH_ALL:
            err = nh_relerr(e.get(name), o.get(name), rc, name)
            assert err < tol, (name, err, nsteps)


@pytest.mark.parametrize("env", ["RCMDYN_NO_GRAPH", "RCMDYN_NO_OVERLAP", "RCMDYN_FORCE_RCCL"])
def test_nh_species_step_forms(qx_n1, monkeypatch, env):
    """2 x 2 tiles: graph replay, the overlapped exchanges and the RCCL transport against the
    drop-in call sequence with none of them, bit for bit."""
    from regcm_amd.dycore import DynCore
    rc, data, st = qx_n1
    ref = start(DynCore, rc, data, st, (2, 2))
    monkeypatch.setenv(env, "1")
    alt = start(DynCore, rc, data, st, (2, 2))
    ref.step(4)
    if env == "RCMDYN_NO_GRAPH":
        for _ in range(4):
            alt.tend()
            alt.bdyval()
    else:
        alt.step(4)
    for name in NH_ALL:
        same = np.array_equal(ref.get(name), alt.get(name))
        assert same, name


@pytest.mark.parametrize("core", ["hydrostatic", "nh"])
def test_species_smooth_decomposition_bit_identical(c1_data, core):
    """With smooth hydrometeor layers (no cloud edges, so no negative forecast reaches the fix
    at a tile edge) a 2 x 2 decomposition with nqx = 5 is bit-identical to one tile, as the
    reference's decompositions are; with cloud edges the fix itself depends on the tiles
    (test_species_tiles_match_oracle_tiles)."""
    from regcm_amd.dycore import DynCore
    if core == "nh":
        rc = dataclasses.replace(CONFIGS["N1"], ipptls=2)
        data = icbc.generate_nh(rc)
    else:
        rc = dataclasses.replace(c1_data[0], ipptls=2)
        data = c1_data[1]
    st = dict(data["state"])
    hsig = (rc.sigma[1:] + rc.sigma[:-1]) * 0.5
    ps = st["PSA"][0]
    for nm, (peak, s0, w) in {"QC": (2e-4, 0.75, 0.15), "QI": (5e-5, 0.3, 0.1), "QR": (1e-4, 0.92, 0.08),
                              "QS": (8e-5, 0.55, 0.12)}.items():
        layer = peak * (0.2 + np.exp(-0.5 * ((hsig - s0) / w) ** 2))    # positive everywhere
        st[f"ATM1_{nm}"] = layer[:, None, None] * ps[None]
        st[f"ATM2_{nm}"] = 0.98 * st[f"ATM1_{nm}"]
    one = start(DynCore, rc, data, st)
    til = start(DynCore, rc, data, st, (2, 2))
    one.step(4)
    til.step(4)
    names = (NH_ALL if core == "nh" else ALL)
    for name in names:
        assert np.array_equal(one.get(name), til.get(name)), name
