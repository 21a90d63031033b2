"""GPU parity of the non-hydrostatic core (idynamic = 2): the HIP engine through the C-ABI
against the CPU restatement (oracle/rcm_oracle.c, nh_tend / nh_sound).

Tolerances: the NH step's dataflow contains transcendental functions almost everywhere
(exp/log of the NH vertical temperature flux, x**y of vadvqv, sin of the Rayleigh damping
profile, sin/cos/sqrt of the upper radiative coefficients), evaluated by OCML on the device
and by libm on the host, so the bound is a relative max-norm: 1e-11 after one step, 1e-10
after three; after twenty the engine-oracle difference must stay inside the oracle's own
spread under a 1e-14 perturbation of the initial temperature (the acoustic sub-steps and the
extrema limiters amplify ulp differences like any other perturbation).  The initial boundary
pass is transcendental-free and must match exactly.
"""
import dataclasses

import numpy as np
import pytest

from regcm_amd.config import CONFIGS, NH_STATE_FIELDS, QX_STATE_FIELDS
from regcm_amd import icbc
from tests.test_parity_gpu import with_species

pytestmark = pytest.mark.gpu

NH_FIELDS = ["ATM1_U", "ATM1_V", "ATM1_T", "ATM1_QV", "ATM1_QC", "ATM2_U", "ATM2_V", "ATM2_T",
             "ATM2_QV", "ATM2_QC", "PSA", "PSB"] + NH_STATE_FIELDS
CROSS = {"ATM1_T", "ATM1_QV", "ATM1_QC", "ATM2_T", "ATM2_QV", "ATM2_QC", "PSA", "PSB",
         "ATM1_PP", "ATM2_PP", "ATM1_W", "ATM2_W"} | set(QX_STATE_FIELDS)


def relerr(a, b, rc, name):
    if name in CROSS:
        a = a[:, : rc.iy - 1, : rc.jx - 1]
        b = b[:, : rc.iy - 1, : rc.jx - 1]
    den = max(np.max(np.abs(b)), 1e-300)
    return float(np.max(np.abs(a - b)) / den)


@pytest.fixture(scope="module")
def nh_data():
    rc = CONFIGS["N1"]
    return rc, icbc.generate_nh(rc)


def make_pair(rc, data):
    from oracle.oracle import OracleCore
    from regcm_amd.dycore import DynCore
    o = OracleCore(rc, data["split"])
    e = DynCore(rc, data["split"])
    st = with_species(rc, data["state"])
    o.put_state(st)
    e.put_state(st)
    o.bdyval()
    e.bdyval()
    return o, e


def test_nh_init_bdyval_exact(nh_data):
    rc, data = nh_data
    o, e = make_pair(rc, data)
    for name in NH_FIELDS:
        assert relerr(e.get(name), o.get(name), rc, name) == 0.0, name
    assert e.get_time() == o.get_time()


def test_nh_parity_and_envelope(nh_data):
    from oracle.oracle import OracleCore
    rc, data = nh_data
    o, e = make_pair(rc, data)
    for nsteps, tol in ((1, 1e-11), (2, 1e-10)):
        o.step(nsteps)
        e.step(nsteps)
        assert e.get_time() == o.get_time()
        for name in NH_FIELDS:
            err = relerr(e.get(name), o.get(name), rc, name)
            assert err < tol, (name, err, nsteps)
    o.step(17)
    e.step(17)
    st = {k: v.copy() for k, v in data["state"].items()}
    st["ATM1_T"] = st["ATM1_T"] * (1.0 + 1e-14)
    p = OracleCore(rc, data["split"])
    p.put_state(st)
    p.bdyval()
    p.step(20)
    for name in NH_FIELDS:
        err = relerr(e.get(name), o.get(name), rc, name)
        spread = relerr(p.get(name), o.get(name), rc, name)
        assert err <= max(1e-9, 100.0 * spread), (name, err, spread)


def test_nh_graph_replay_equals_eager(nh_data):
    """rcmdyn_step replays a captured graph from the third step on; the result must be
    bit-identical to eager tend + bdyval calls."""
    from regcm_amd.dycore import DynCore
    rc, data = nh_data
    a = DynCore(rc, data["split"])
    b = DynCore(rc, data["split"])
    for x in (a, b):
        x.put_state(data["state"])
        x.bdyval()
    a.step(8)
    for _ in range(8):
        b.tend()
        b.bdyval()
    for name in NH_FIELDS:
        assert np.array_equal(a.get(name), b.get(name)), name


def test_nh_rest_state():
    """The resting reference atmosphere stays at rest on the device, as in the oracle."""
    from regcm_amd.dycore import DynCore
    rc = CONFIGS["N1"]
    data = icbc.generate_nh(rc, rest=True)
    e = DynCore(rc, data["split"])
    e.put_state(data["state"])
    e.bdyval()
    e.step(10)
    ps = e.get("PSA")[0][None, :-1, :-1]
    for n, lim in (("ATM1_U", 1e-4), ("ATM1_V", 1e-4), ("ATM1_W", 1e-4), ("ATM1_PP", 0.05)):
        assert np.abs(e.get(n)[:, :-1, :-1] / ps).max() < lim, n


def test_nh_dprddx_formed_from_pr(nh_data):
    """The acoustic u, v update forms atm0%dprddx / dprddy from atm0%pr
    (Main/mod_params.F90:2676-2686); the host's put of the reference's values passes the
    engine's check, and a put that is not those four-point sums is refused at the next call
    instead of being silently replaced."""
    from regcm_amd.dycore import DynCore, EngineError
    rc, data = nh_data
    e = DynCore(rc, data["split"])
    e.put_state(data["state"])
    e.bdyval()
    e.step(1)
    bad = data["state"]["DPRDDX"].copy()
    bad[3, 10, 10] += 1e-9
    e.put("DPRDDX", bad)
    with pytest.raises(EngineError, match="DPRDDX/DPRDDY differ"):
        e.step(1)
    e.put("DPRDDX", data["state"]["DPRDDX"])
    e.step(1)


NH_VARIANTS = [{"iboudy": 4}, {"iboudy": 3}, {"iboudy": 2}, {"idiffu": 2}, {"idiffu": 3}, {"ifupr": 0}, {"ifrayd": 0}, {"isladvec": 1},
               {"upstream_mode": 0}, {"stability_enhance": 0}, {"ipptls": 2}]
# idiffu = 3 depends on the decomposition as the reference's does (test_nh_idiffu3_tiles), and
# so does the fix of negative forecasts at tile edges (ipptls = 2: tests/test_species_gpu.py)
NH_DECOMP_VARIANTS = [v for v in NH_VARIANTS if v.get("idiffu") != 3 and "ipptls" not in v]


@pytest.mark.parametrize("variant", NH_VARIANTS, ids=lambda v: ",".join(f"{k}={x}" for k, x in v.items()))
def test_nh_variant_parity(nh_data, variant):
    rc, data = nh_data
    rcv = dataclasses.replace(rc, **variant)
    o, e = make_pair(rcv, data)
    fields = NH_FIELDS + (QX_STATE_FIELDS if rcv.nqx > 2 else [])
    for nsteps, tol in ((1, 1e-11), (2, 1e-10)):
        o.step(nsteps)
        e.step(nsteps)
        for name in fields:
            err = relerr(e.get(name), o.get(name), rcv, name)
            assert err < tol, (name, err, nsteps)


@pytest.mark.parametrize("nproc", [(2, 1), (2, 2), (1, 3)])
def test_nh_decomposition_invariance(nh_data, nproc):
    """The NH step on a decomposed domain (local tiles, the RCCL staging layout) is
    bit-identical to one tile: same kernels per point, exact halos, the 6-deep estore halo of
    the radiative condition, and the day-alarm means summed in the global order."""
    from regcm_amd.dycore import DynCore
    rc, data = nh_data
    ref = DynCore(rc, data["split"])
    til = DynCore(rc, data["split"], nproc_j=nproc[0], nproc_i=nproc[1])
    for e in (ref, til):
        e.put_state(data["state"])
        e.bdyval()
        e.step(8)
    for name in NH_FIELDS:
        assert np.array_equal(ref.get(name), til.get(name)), name


@pytest.mark.parametrize("mode", ["dropin", "serial"])
def test_nh_overlap_modes(nh_data, monkeypatch, mode):
    """The NH halo/compute overlap (cr/qdot/xkcr beside k_nh_tend_c, cqv/cqc beside
    k_nh_tend_d, dp'/dp0 and pp beside part 1 of k_nh_sound_uv, the strip after the join) is
    bit-identical to one tile through the drop-in pair (tend's exchanges on the first stream,
    the sound loop's overlapped) and with it off (RCMDYN_NO_OVERLAP=1); the default is
    test_nh_decomposition_invariance."""
    from regcm_amd.dycore import DynCore
    rc, data = nh_data
    ref = DynCore(rc, data["split"])
    if mode == "serial":
        monkeypatch.setenv("RCMDYN_NO_OVERLAP", "1")
    til = DynCore(rc, data["split"], nproc_j=2, nproc_i=2)
    for e in (ref, til):
        e.put_state(data["state"])
        e.bdyval()
    ref.step(6)
    if mode == "dropin":
        for _ in range(6):
            til.tend()
            til.bdyval()
    else:
        til.step(6)
    for name in NH_FIELDS:
        assert np.array_equal(ref.get(name), til.get(name)), name


TFUSE_CASES = [({}, (1, 1)), ({}, (2, 2)), ({"isladvec": 1}, (1, 1)), ({"iboudy": 4}, (2, 1)),
               ({"ipptls": 2}, (1, 1)), ({"idiffu": 3}, (1, 1))]


@pytest.mark.parametrize("variant,nproc", TFUSE_CASES, ids=lambda x: str(x))
def test_nh_fused_time_filters_bit_identical(nh_data, monkeypatch, variant, nproc):
    """The time filters of t, qv, qc fused into k_nh_tend_c and the negative-moisture fix
    (into the other parity, Tile::tq) equal the in-place filter pass (RCMDYN_NH_NO_TFUSE=1)
    bit for bit: eager and graph-replayed steps, the drop-in pair, an odd step count (the
    state read from the second parity) and a put between steps."""
    from regcm_amd.dycore import DynCore
    rc, data = nh_data
    rcv = dataclasses.replace(rc, **variant)
    st = with_species(rcv, data["state"])
    fused = DynCore(rcv, data["split"], nproc_j=nproc[0], nproc_i=nproc[1])
    monkeypatch.setenv("RCMDYN_NH_NO_TFUSE", "1")
    inplace = DynCore(rcv, data["split"], nproc_j=nproc[0], nproc_i=nproc[1])
    fields = NH_FIELDS + (QX_STATE_FIELDS if rcv.nqx > 2 else [])
    for e in (fused, inplace):
        e.put_state(st)
        e.bdyval()
        e.step(5)
        for _ in range(2):
            e.tend()
            e.bdyval()
        e.tend_pre_physics()
        e.tend_post_physics()
        e.bdyval()
        e.put("ATM1_T", e.get("ATM1_T") * (1.0 + 1e-12))
        e.step(2)
    for name in fields:
        assert np.array_equal(fused.get(name), inplace.get(name)), name


@pytest.mark.parametrize("variant", NH_DECOMP_VARIANTS, ids=lambda v: ",".join(f"{k}={x}" for k, x in v.items()))
def test_nh_variant_decomposition(nh_data, variant):
    from regcm_amd.dycore import DynCore
    rc, data = nh_data
    rcv = dataclasses.replace(rc, **variant)
    ref = DynCore(rcv, data["split"])
    til = DynCore(rcv, data["split"], nproc_j=2, nproc_i=2)
    for e in (ref, til):
        e.put_state(data["state"])
        e.bdyval()
        e.step(6)
    for name in NH_FIELDS:
        assert np.array_equal(ref.get(name), til.get(name)), name


@pytest.mark.parametrize("nthreads", [2, 4])
def test_nh_idiffu3_tiles(nh_data, nthreads):
    """NH idiffu = 3 on set_nproc tiles against the oracle run as the same tiles: the
    sixth-order terms of u, v, t, qv, qc, pp and w (kz + 1 levels) on every tile's own column."""
    from oracle.oracle import OracleParallel
    from regcm_amd.config import set_nproc
    from regcm_amd.dycore import DynCore
    rc, data = nh_data
    rcv = dataclasses.replace(rc, idiffu=3)
    cj, ci = set_nproc(nthreads, rc.jx, rc.iy)
    o = OracleParallel(rcv, data["split"], nthreads=nthreads)
    e = DynCore(rcv, data["split"], nproc_j=cj, nproc_i=ci)
    for x in (o, e):
        x.put_state(data["state"])
        x.bdyval()
    for nsteps, tol in ((1, 1e-11), (2, 1e-10)):
        o.step(nsteps)
        e.step(nsteps)
        for name in NH_FIELDS:
            err = relerr(e.get(name), o.get(name), rcv, name)
            assert err < tol, (name, err, nsteps)


def test_nh_negative_moisture_list(nh_data):
    """Clusters of negative NH qc forecasts: k_nh_tend_c lists them, k_nh_negfix fixes the
    independent ones from the list and the serial sweep the dependent ones, reproducing the
    reference's order-dependent fix (Main/mod_tendency.F90:382-393) bit for bit."""
    from oracle.oracle import OracleCore
    from regcm_amd.dycore import DynCore
    from tests.test_parity_gpu import _dependent_negatives
    rc, data = nh_data
    st = {k: v.copy() for k, v in data["state"].items()}
    rng = np.random.default_rng(11)
    ps = st["PSA"][0]
    pat = rng.uniform(0.0, 2.0e-5, size=st["ATM1_QC"].shape) * (rng.uniform(size=st["ATM1_QC"].shape) < 0.5)
    st["ATM1_QC"] = pat * ps[None]
    st["ATM2_QC"] = np.zeros_like(pat)
    o = OracleCore(rc, data["split"])
    e = DynCore(rc, data["split"])
    e.set_diagnostics(True)
    for c in (o, e):
        c.put_state(st)
        c.bdyval()
        c.tend()
    dt = o.get_time()[1]
    assert _dependent_negatives(dt * o.get("QCTEN"), rc) > 0
    assert int((dt * o.get("QCTEN")[:, 1:rc.iy - 2, 1:rc.jx - 2] < 0).sum()) > 1000
    for name in ("ATM1_QC", "ATM2_QC", "QCTEN"):
        a, b = e.get(name), o.get(name)
        assert np.array_equal(a[:, 1:rc.iy - 2, 1:rc.jx - 2], b[:, 1:rc.iy - 2, 1:rc.jx - 2]), name
