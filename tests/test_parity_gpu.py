"""GPU parity: the HIP engine (through the C-ABI) against the CPU restatement (oracle).

Tolerances: fields whose dataflow contains no transcendental function must match
bit-for-bit (same operation order, -ffp-contract=off on both sides).  Fields downstream of
log/pow (PGF, vadv3d, vadvqv, phi) may differ by libm-vs-OCML ulps; the bound is a relative
max-norm of 1e-12 after one step, growing with the step count as stated per test.
"""
import numpy as np
import pytest

from regcm_amd.config import CONFIGS, QX_STATE_FIELDS, STATE_FIELDS
from regcm_amd import icbc

pytestmark = pytest.mark.gpu

CROSS = {"ATM1_T", "ATM1_QV", "ATM1_QC", "ATM2_T", "ATM2_QV", "ATM2_QC", "PSA", "PSB",
         "DSTOR", "HSTOR", "PSC", "PTEN", "TTEN", "QVTEN", "QCTEN", "OMEGA", "QDOT", "XKC", "PHI"} | \
    set(QX_STATE_FIELDS)


def relerr(a, b, rc, name):
    if name in CROSS:
        a = a[:, : rc.iy - 1, : rc.jx - 1]
        b = b[:, : rc.iy - 1, : rc.jx - 1]
    den = max(np.max(np.abs(b)), 1e-300)
    return float(np.max(np.abs(a - b)) / den)


def with_species(rc, state):
    """ipptls = 2: the state with patchy qi, qr, qs layers (icbc.hydrometeor_state)."""
    if rc.nqx <= 2:
        return state
    st = dict(state)
    st.update(icbc.hydrometeor_state(rc, st, nqx=rc.nqx))
    return st


def state_fields(rc):
    return list(STATE_FIELDS) + (QX_STATE_FIELDS if rc.nqx > 2 else [])


def make_pair(rc, data, nproc_j=1, nproc_i=1):
    from oracle.oracle import OracleCore
    from regcm_amd.dycore import DynCore
    o = OracleCore(rc, data["split"])
    e = DynCore(rc, data["split"], nproc_j=nproc_j, nproc_i=nproc_i)
    st = with_species(rc, data["state"])
    o.put_state(st)
    e.put_state(st)
    o.bdyval()
    e.bdyval()
    return o, e


def test_init_bdyval_exact(c1_data):
    rc, data = c1_data
    o, e = make_pair(rc, data)
    for name in STATE_FIELDS:
        assert relerr(e.get(name), o.get(name), rc, name) == 0.0, name
    assert e.get_time() == o.get_time()


def test_one_tend_intermediates(c1_data):
    rc, data = c1_data
    o, e = make_pair(rc, data)
    e.set_diagnostics(True)
    o.tend()
    e.tend()
    exact = ["QDOT", "PSDOTA", "XKC", "OMEGA", "PTEN", "PSC", "QCTEN"]
    for name in exact:
        assert relerr(e.get(name), o.get(name), rc, name) == 0.0, name
    for name in ["TTEN", "QVTEN", "UTEN", "VTEN", "PHI"]:
        err = relerr(e.get(name), o.get(name), rc, name)
        assert err < 1e-12, (name, err)
    assert e.get_time() == o.get_time()


def test_one_step_state(c1_data):
    rc, data = c1_data
    o, e = make_pair(rc, data)
    o.step(1)
    e.step(1)
    for name in STATE_FIELDS:
        err = relerr(e.get(name), o.get(name), rc, name)
        assert err < 1e-12, (name, err)


def test_twenty_steps_graph_replay(c1_data):
    rc, data = c1_data
    o, e = make_pair(rc, data)
    o.step(20)
    e.step(20)
    for name in STATE_FIELDS:
        err = relerr(e.get(name), o.get(name), rc, name)
        assert err < 1e-9, (name, err)
    assert e.get_time() == o.get_time()
    do, de = o.diagnostics(), e.diagnostics()
    assert abs(do[0] - de[0]) <= 1e-9 * abs(do[0])


def test_tend_bdyval_equals_step(c1_data):
    rc, data = c1_data
    from regcm_amd.dycore import DynCore
    e1 = DynCore(rc, data["split"])
    e2 = DynCore(rc, data["split"])
    for e in (e1, e2):
        e.put_state(data["state"])
        e.bdyval()
    for _ in range(6):                  # the drop-in sequence: graph per call, both parities
        e1.tend()
        e1.bdyval()
    e2.step(6)
    assert e1.get_time() == e2.get_time()
    for name in STATE_FIELDS:
        assert np.array_equal(e1.get(name), e2.get(name)), name


def test_cfl_violation_stops_within_lag(c1_data):
    """A state that goes NaN stops rcmdyn_step within FLAG_LAG steps of the failing step
    (checked on the host from per-step flag snapshots, no per-step stream sync), reports the
    step the oracle fails at, and clears the flag once reported (Main/mod_tendency.F90:702)."""
    from oracle.oracle import OracleCore
    from regcm_amd.dycore import DynCore, EngineError
    rc, data = c1_data
    st = {k: v.copy() for k, v in data["state"].items()}
    for name in ("ATM1_T", "ATM2_T"):
        st[name][5, 20:24, 20:24] = np.nan
    o = OracleCore(rc, data["split"])
    o.put_state(st)
    o.bdyval()
    fail = None
    for n in range(1, 20):
        try:
            o.step(1)
        except FloatingPointError:
            fail = n
            break
    assert fail is not None
    e = DynCore(rc, data["split"])
    e.put_state(st)
    e.bdyval()
    with pytest.raises(EngineError, match=rf"CFL VIOLATION \(step {fail}\)"):
        e.step(100)
    assert e.get_time()[0] <= fail + 3             # FLAG_LAG = 2 steps in flight at most
    e.set_time(0, rc.dt, 0.0)
    e.put_state(data["state"])
    e.bdyval()
    e.step(2)                                       # the flag was cleared


def test_get_reports_failed_step(c1_data):
    """rcmdyn_get never hands out fields of a failed run: a step that went NaN inside the
    2-step report lag of rcmdyn_tend is reported by the next get (the reference's fatal stops
    before any output, Main/mod_tendency.F90:702)."""
    from regcm_amd.dycore import DynCore, EngineError
    rc, data = c1_data
    st = {k: v.copy() for k, v in data["state"].items()}
    for name in ("ATM1_T", "ATM2_T"):
        st[name][5, 20:24, 20:24] = np.nan
    e = DynCore(rc, data["split"])
    e.put_state(st)
    e.bdyval()
    with pytest.raises(EngineError, match="CFL VIOLATION"):
        for _ in range(6):
            e.tend()
            e.bdyval()
        e.get("ATM1_T")


@pytest.mark.parametrize("nproc", [(2, 1), (2, 2), (1, 3), (1, 7)])
def test_decomposition_invariance(c1_data, nproc):
    """Tiles exchanging halos reproduce the single-tile result bit-for-bit; tiles
    narrower than the split-step halo (1 x 7) take the per-sub-step exchange path."""
    rc, data = c1_data
    from regcm_amd.dycore import DynCore
    ref = DynCore(rc, data["split"])
    til = DynCore(rc, data["split"], nproc_j=nproc[0], nproc_i=nproc[1])
    for e in (ref, til):
        e.put_state(data["state"])
        e.bdyval()
        e.step(6)
    for name in STATE_FIELDS:
        assert np.array_equal(ref.get(name), til.get(name)), name


@pytest.mark.parametrize("nproc", [(2, 1), (2, 2), (2, 4)])
def test_decomposition_invariance_c3(nproc):
    """The headline domain on the set_nproc tilings of 2/4/8 GPUs (local tiles): bit-identical
    to one tile, including the partial blocks the ghost-ring kernels run on 96 x 48 tiles."""
    from regcm_amd.dycore import DynCore
    rc = CONFIGS["C3"]
    data = icbc.generate(rc)
    ref = DynCore(rc, data["split"])
    til = DynCore(rc, data["split"], nproc_j=nproc[0], nproc_i=nproc[1])
    for e in (ref, til):
        e.put_state(data["state"])
        e.bdyval()
        e.step(5)
    for name in STATE_FIELDS:
        assert np.array_equal(ref.get(name), til.get(name)), name


@pytest.mark.parametrize("mode", ["step", "dropin", "serial"])
def test_overlap_parts_bit_identical(monkeypatch, mode):
    """Halo/compute overlap: on a decomposed domain the whole prologue exchange
    runs on the second stream while part 1 of k_columns (and, in rcmdyn_step, of k_momentum
    and k_scalars: the blocks whose staged tile reads no point an exchange writes) computes;
    part 2 follows the join.  C3 on 1 x 2 tiles (192 x 96: k_momentum / k_scalars have part-1
    blocks) is bit-identical to one tile, through rcmdyn_step, through the drop-in
    tend + bdyval pair (k_columns split only) and with the split off (RCMDYN_NO_OVERLAP)."""
    from regcm_amd.dycore import DynCore
    rc = CONFIGS["C3"]
    data = icbc.generate(rc)
    ref = DynCore(rc, data["split"])
    if mode == "serial":
        monkeypatch.setenv("RCMDYN_NO_OVERLAP", "1")
    til = DynCore(rc, data["split"], nproc_j=1, nproc_i=2)
    for e in (ref, til):
        e.put_state(data["state"])
        e.bdyval()
    ref.step(5)
    if mode == "dropin":
        for _ in range(5):
            til.tend()
            til.bdyval()
    else:
        til.step(5)
    for name in STATE_FIELDS:
        assert np.array_equal(ref.get(name), til.get(name)), name
    a, b = ref.reductions(), til.reductions()
    assert np.allclose(a[:2], b[:2], rtol=1e-12, atol=0), (a, b)   # the partials in another order


@pytest.mark.parametrize("nproc", [(2, 1), (2, 2), (2, 4)], ids=str)
def test_overlap_shifted_blocks_bit_identical(nproc):
    """C3 on the tiles of the 2/4/8-GPU runs (96 x 192, 96 x 96, 96 x 48): the block columns of
    k_momentum / k_scalars in parts 1 and 2 start at the origin that puts one 64-wide column
    wholly inside the part-1 rectangle (rcmdyn_overlap_shares: 62 / 56 / 44 % of their points
    beside the exchange, none with the default origin).  Bit-identical to one tile."""
    from regcm_amd.dycore import DynCore
    rc = CONFIGS["C3"]
    data = icbc.generate(rc)
    ref = DynCore(rc, data["split"])
    til = DynCore(rc, data["split"], nproc_j=nproc[0], nproc_i=nproc[1])
    for e in (ref, til):
        e.put_state(data["state"])
        e.bdyval()
        e.step(5)
    for name in STATE_FIELDS:
        assert np.array_equal(ref.get(name), til.get(name)), name


def test_c2_ten_steps():
    rc = CONFIGS["C2"]
    data = icbc.generate(rc)
    o, e = make_pair(rc, data)
    o.step(10)
    e.step(10)
    for name in STATE_FIELDS:
        err = relerr(e.get(name), o.get(name), rc, name)
        assert err < 1e-10, (name, err)


def test_diagnostics_switch_is_transparent(c1_data):
    """Tendency diagnostics on/off give identical prognostic results; off refuses gets."""
    rc, data = c1_data
    from regcm_amd.dycore import DynCore, EngineError
    e1 = DynCore(rc, data["split"])
    e2 = DynCore(rc, data["split"])
    e2.set_diagnostics(True)
    for e in (e1, e2):
        e.put_state(data["state"])
        e.bdyval()
        e.step(4)
    for name in STATE_FIELDS:
        assert np.array_equal(e1.get(name), e2.get(name)), name
    with pytest.raises(EngineError):
        e1.get("TTEN")
    assert np.isfinite(e2.get("TTEN")).all()


def test_kernel_times_hook(c1_data):
    """rcmdyn_kernel_times runs real (eager) steps and reports every kernel of the step."""
    rc, data = c1_data
    from regcm_amd.dycore import DynCore
    e1 = DynCore(rc, data["split"])
    e2 = DynCore(rc, data["split"])
    for e in (e1, e2):
        e.put_state(data["state"])
        e.bdyval()
    kt = e1.kernel_times(3)
    e2.step(3)
    for name in STATE_FIELDS:
        assert np.array_equal(e1.get(name), e2.get(name)), name
    base = {}
    for name, v in kt.items():          # level-marching forms: k_scalars_km<opt> -> k_scalars
        b = name.split("<")[0]
        base[b[:-3] if b.endswith("_km") else b] = v
    # rcmdyn_step's step: bdyval's boundary lines run inside k_split_correct_bdy, k_qfilter's
    # work in k_columns / k_scalars / the extra blocks of k_split_project and k_split_correct;
    # k_momentum and k_scalars share one launch (k_update)
    for k in ("k_update", "k_columns", "k_split_project",
              "k_spstep_fused", "k_split_correct_bdy", "k_bdyval_qc"):
        assert k in base and base[k][0] == 3 and base[k][1] > 0.0, k
    for k in ("k_bdyval_set", "k_split_correct", "k_qfilter", "k_momentum", "k_scalars"):
        assert k not in base, sorted(base)


QFUSE_CASES = [({}, (1, 1)), ({}, (2, 2)), ({}, (1, 3)), ({"iboudy": 4}, (2, 1)), ({"isladvec": 1}, (2, 2)),
               ({"ibltyp": 2}, (1, 1))]


@pytest.mark.parametrize("variant,nproc", QFUSE_CASES, ids=lambda x: str(x))
def test_qfilter_fusion_equals_qfilter(c1_data, monkeypatch, variant, nproc):
    """The step without k_qfilter (qfuse: p*'s RA filter and the copies in k_columns, the RAW
    filter of non-negative moisture in k_scalars, the listed negatives fixed in the extra
    blocks of k_split_project and k_split_correct) is bit-identical to the k_qfilter step
    (RCMDYN_NO_QFUSE), eager and graph-replayed, with a state that forces clusters of dependent
    negative qv (the serial sweep) and on decompositions."""
    import dataclasses
    from regcm_amd.dycore import DynCore
    rc, data = c1_data
    rcv = dataclasses.replace(rc, **variant)
    st = {k: v.copy() for k, v in data["state"].items()}
    # dry columns with alternating signs in the forecast: rows of negative qv on a few levels
    st["ATM1_QV"][5:8, 10:14, 10:30] = -1e-7 * st["PSA"][0][10:14, 10:30]
    st["ATM2_QV"][5:8, 10:14, 10:30] = -2e-7 * st["PSA"][0][10:14, 10:30]
    if rcv.ibltyp == 2:
        st.update(icbc.tke_state(rcv))
    fused = DynCore(rcv, data["split"], nproc_j=nproc[0], nproc_i=nproc[1])
    monkeypatch.setenv("RCMDYN_NO_QFUSE", "1")
    sep = DynCore(rcv, data["split"], nproc_j=nproc[0], nproc_i=nproc[1])
    for e in (fused, sep):
        e.put_state(st)
        e.bdyval()
        e.step(5)
    assert fused.get_time() == sep.get_time()
    for name in state_fields(rcv) + (["ATM1_TKE", "ATM2_TKE"] if rcv.ibltyp == 2 else []):
        assert np.array_equal(fused.get(name), sep.get(name)), name
    assert np.array_equal(fused.reductions(), sep.reductions())


FUSE_CASES = [({}, (1, 1)), ({}, (2, 2)), ({}, (1, 3)), ({"iboudy": 4}, (1, 1)), ({"iboudy": 4}, (2, 2)),
              ({"isladvec": 1}, (2, 1)), ({"ibltyp": 2}, (1, 1)), ({"ibltyp": 2}, (2, 2)),
              ({"ipptls": 2}, (1, 1)), ({"ipptls": 2}, (2, 2)), ({"ipptls": 2, "iboudy": 4}, (2, 1))]


@pytest.mark.parametrize("variant,nproc", FUSE_CASES, ids=lambda x: str(x))
def test_fused_bdyval_equals_separate(c1_data, monkeypatch, variant, nproc):
    """rcmdyn_step runs bdyval's boundary lines inside the split-correct launch
    (k_split_correct_bdy): bit-identical to the separate k_bdyval_set launch of the drop-in
    call sequence (RCMDYN_NO_FUSE_BDY), for eager and graph-replayed steps, with the iboudy = 4
    qv inflow/outflow, semi-Lagrangian and TKE options, on one tile and decomposed."""
    import dataclasses
    from regcm_amd.dycore import DynCore
    rc, data = c1_data
    rcv = dataclasses.replace(rc, **variant)
    st = {k: v.copy() for k, v in data["state"].items()}
    if rcv.ibltyp == 2:
        st.update(icbc.tke_state(rcv))
    st = with_species(rcv, st)     # ipptls = 2: patchy cloud, so the qc inflow/outflow acts
    fused = DynCore(rcv, data["split"], nproc_j=nproc[0], nproc_i=nproc[1])
    monkeypatch.setenv("RCMDYN_NO_FUSE_BDY", "1")
    sep = DynCore(rcv, data["split"], nproc_j=nproc[0], nproc_i=nproc[1])
    for e in (fused, sep):
        e.put_state(st)
        e.bdyval()
        e.step(5)
    assert fused.get_time() == sep.get_time()
    for name in state_fields(rcv) + (["ATM1_TKE", "ATM2_TKE"] if rcv.ibltyp == 2 else []):
        assert np.array_equal(fused.get(name), sep.get(name)), name
    assert np.array_equal(fused.reductions(), sep.reductions())


@pytest.mark.parametrize("nproc", [(1, 1), (2, 2)], ids=str)
def test_deferred_corrections_any_call_order(c1_data, monkeypatch, nproc):
    """rcmdyn_tend leaves its launch to the next call (lazy tend: rcmdyn_bdyval replays
    rcmdyn_step's one-step graph) and, when launched alone, its split corrections to the next
    rcmdyn_bdyval (launched with the boundary lines, rcmdyn_step's k_split_correct_bdy); a get,
    a put, a synchronize or a reductions call in between launches them first.  Every order is
    bit-identical to rcmdyn_step, to tend launching its own graph at once
    (RCMDYN_NO_LAZY_TEND) and to tend launching its corrections itself
    (RCMDYN_NO_DEFER_CORR), and the clock a host reads after tend is the same either way."""
    from regcm_amd.dycore import DynCore
    rc, data = c1_data
    st = with_species(rc, data["state"])
    mk = lambda: DynCore(rc, data["split"], nproc_j=nproc[0], nproc_i=nproc[1])
    ref, a, b = mk(), mk(), mk()
    monkeypatch.setenv("RCMDYN_NO_LAZY_TEND", "1")
    d = mk()                           # tend launches its own graph at once
    monkeypatch.setenv("RCMDYN_NO_DEFER_CORR", "1")
    c = mk()
    for e in (ref, a, b, c, d):
        e.put_state(st)
        e.bdyval()
    ref.step(8)
    for n in range(8):
        a.tend()
        a.bdyval()
        b.tend()
        t_mid = b.get_time()           # the clock after tend, before any launch
        if n % 4 == 0:
            b.get("ATM1_T")            # settles the lazy tend and its corrections before bdyval
        elif n % 4 == 1:
            b.synchronize()
        elif n % 4 == 2:
            b.put("ATM1_QV", b.get("ATM1_QV"))
        else:
            b.reductions()
        assert b.get_time() == t_mid
        b.bdyval()
        for e in (c, d):
            e.tend()
            e.bdyval()
    for name in STATE_FIELDS:
        r = ref.get(name)
        for e in (a, b, c, d):
            assert np.array_equal(e.get(name), r), name
    assert a.get_time() == ref.get_time() == b.get_time() == c.get_time() == d.get_time()
    assert np.array_equal(a.reductions(), ref.reductions())
    assert np.array_equal(d.reductions(), ref.reductions())


def test_lazy_tend_survives_failed_launch(c1_data, monkeypatch):
    """A launch failure between the lazy tend and its launch (injected with
    RCMDYN_INJECT_LAUNCH_FAILURE: the second launch of a lazy tend's graph fails before it is
    issued) leaves the step pending: the clock a host reads stays the tend's, and the next
    bdyval runs the whole step, so the run stays bit-identical to rcmdyn_step.  A
    tend still pending at destroy is launched, not dropped: destroy returns 0."""
    from regcm_amd.dycore import DynCore, EngineError
    rc, data = c1_data
    st = data["state"]
    ref = DynCore(rc, data["split"])
    monkeypatch.setenv("RCMDYN_INJECT_LAUNCH_FAILURE", "2")
    a = DynCore(rc, data["split"])
    monkeypatch.delenv("RCMDYN_INJECT_LAUNCH_FAILURE")
    for e in (ref, a):
        e.put_state(st)
        e.bdyval()
    ref.step(6)
    failed = 0
    for n in range(6):
        a.tend()
        t_mid = a.get_time()
        try:
            a.bdyval()
        except EngineError as x:
            assert "injected" in str(x)
            failed += 1
            assert a.get_time() == t_mid
            a.bdyval()                 # the pending step runs now
    assert failed == 1
    for name in STATE_FIELDS:
        assert np.array_equal(a.get(name), ref.get(name)), name
    assert a.get_time() == ref.get_time()
    a.tend()
    a.close()                          # launches the pending tend; no error


def _dependent_negatives(cq, rc):
    """(k, i, j) cross points of the interior where the reference's serial sweep reads an
    already-fixed predecessor (Main/mod_tendency.F90:382-393)."""
    jci = slice(1, rc.jx - 2)
    ici = slice(1, rc.iy - 2)
    neg = np.zeros_like(cq, dtype=bool)
    neg[:, ici, jci] = cq[:, ici, jci] < 0
    dep = np.zeros_like(neg)
    p = np.pad(neg, ((0, 0), (1, 1), (1, 1)))
    # predecessors (j-1,i) (j-1,i-1) (j,i-1) (j+1,i-1) in padded coordinates (+1)
    pred = p[:, 1:-1, :-2] | p[:, :-2, :-2] | p[:, :-2, 1:-1] | p[:, :-2, 2:]
    dep = neg & pred
    return int(dep.sum())


def test_negative_moisture_serial_sweep(c1_data):
    """A state with clusters of negative qc forecasts: the parallel fix + serial sweep
    reproduce the reference's order-dependent fix bit-for-bit."""
    rc, data = c1_data
    from oracle.oracle import OracleCore
    from regcm_amd.dycore import DynCore
    st = {k: v.copy() for k, v in data["state"].items()}
    rng = np.random.default_rng(7)
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
    cqc = dt * o.get("QCTEN")               # atm2 qc is zero in the interior: cqc = 0 + dt * qcten
    assert _dependent_negatives(cqc, rc) > 0
    for name in ("ATM1_QC", "ATM2_QC", "QCTEN"):
        a, b = e.get(name), o.get(name)
        assert np.array_equal(a[:, 1:rc.iy - 2, 1:rc.jx - 2], b[:, 1:rc.iy - 2, 1:rc.jx - 2]), name


# namelist options beyond the defaults, each against the oracle and under decomposition
VARIANTS = [{"iboudy": 4}, {"iboudy": 3}, {"iboudy": 2}, {"iboudy": 1}, {"ipgf": 1}, {"idiffu": 2}, {"idiffu": 3}, {"isladvec": 1},
            {"isladvec": 1, "iqmsl": 0}, {"upstream_mode": 0}, {"stability_enhance": 0}, {"diffu_hgtf": 0},
            {"ipptls": 2}]
# idiffu = 3 acts on each tile's last interior column, so its result depends on the
# decomposition as the reference's does (test_idiffu3_tiles_match_oracle_tiles); so does the
# moisture fix with negative forecasts at tile edges (ipptls = 2's cloud edges,
# tests/test_species_gpu.py compares those against the oracle's tiles)
DECOMP_VARIANTS = [v for v in VARIANTS if v.get("idiffu") != 3 and "ipptls" not in v]


def _variant_id(v):
    return ",".join(f"{k}={x}" for k, x in v.items())


@pytest.mark.parametrize("variant", VARIANTS, ids=_variant_id)
def test_variant_parity(c1_data, variant):
    """Option variants match the oracle: 1 step < 1e-12, 3 steps < 1e-11.  Over 20 steps the
    engine-oracle difference must stay inside the oracle's own sensitivity to a 1e-14
    perturbation of the initial state (iboudy = 4's inflow/outflow switches flip on
    near-zero boundary winds, so ulp-level differences grow by branch flips, not by error)."""
    import dataclasses
    from oracle.oracle import OracleCore
    rc, data = c1_data
    rcv = dataclasses.replace(rc, **variant)
    o, e = make_pair(rcv, data)
    for nsteps, tol in ((1, 1e-12), (2, 1e-11)):
        o.step(nsteps)
        e.step(nsteps)
        for name in state_fields(rcv):
            err = relerr(e.get(name), o.get(name), rcv, name)
            assert err < tol, (name, err, nsteps)
    o.step(17)
    e.step(17)
    st = {k: v.copy() for k, v in with_species(rcv, data["state"]).items()}
    st["ATM1_T"] = st["ATM1_T"] * (1.0 + 1e-14)
    p = OracleCore(rcv, data["split"])
    p.put_state(st)
    p.bdyval()
    p.step(20)
    for name in state_fields(rcv):
        err = relerr(e.get(name), o.get(name), rcv, name)
        spread = relerr(p.get(name), o.get(name), rcv, name)
        assert err <= max(1e-9, 100.0 * spread), (name, err, spread)


@pytest.mark.parametrize("variant", DECOMP_VARIANTS, ids=_variant_id)
def test_variant_decomposition(c1_data, variant):
    import dataclasses
    from regcm_amd.dycore import DynCore
    rc, data = c1_data
    rcv = dataclasses.replace(rc, **variant)
    ref = DynCore(rcv, data["split"])
    til = DynCore(rcv, data["split"], nproc_j=2, nproc_i=2)
    for e in (ref, til):
        e.put_state(data["state"])
        e.bdyval()
        e.step(6)
    for name in STATE_FIELDS:
        assert np.array_equal(ref.get(name), til.get(name)), name


@pytest.mark.parametrize("nthreads,transport", [(2, "copy"), (3, "copy"), (4, "copy"), (4, "rccl")])
def test_idiffu3_tiles_match_oracle_tiles(c1_data, monkeypatch, nthreads, transport):
    """idiffu = 3 on a decomposed domain: the reference applies the sixth-order term on every
    tile's own column j = jdi2 / jci2 (Main/mod_diffusion.F90:421, 611, 745, 902), so the engine's
    tiles are checked against the oracle run as the same set_nproc tiles (oracle/orc_par.c),
    1 step < 1e-12, 3 steps < 1e-11; the column terms reach the neighbour's ring through their
    own exchange (also over RCCL), and the result differs from one tile."""
    import dataclasses
    from oracle.oracle import OracleParallel
    from regcm_amd.config import set_nproc
    from regcm_amd.dycore import DynCore
    rc, data = c1_data
    rcv = dataclasses.replace(rc, idiffu=3)
    cj, ci = set_nproc(nthreads, rc.jx, rc.iy)
    if transport == "rccl":
        monkeypatch.setenv("RCMDYN_FORCE_RCCL", "1")
    o = OracleParallel(rcv, data["split"], nthreads=nthreads)
    e = DynCore(rcv, data["split"], nproc_j=cj, nproc_i=ci)
    one = DynCore(rcv, data["split"])
    for x in (o, e, one):
        x.put_state(data["state"])
        x.bdyval()
    for nsteps, tol in ((1, 1e-12), (2, 1e-11)):
        o.step(nsteps)
        e.step(nsteps)
        for name in STATE_FIELDS:
            err = relerr(e.get(name), o.get(name), rcv, name)
            assert err < tol, (name, err, nsteps)
    one.step(3)
    if cj > 1:
        assert not np.array_equal(one.get("ATM1_QV"), e.get("ATM1_QV"))


@pytest.mark.parametrize("iy", [300, 560])
def test_bdyval_qc_tall_tile(iy):
    """bdyval's qc inflow/outflow on a tile taller than one 256-thread block: the west/east
    pass must read qc(jci1|jci2, ice1|ice2) before the south/north pass rewrites them
    (Main/mod_bdycod.F90:2153-2220), whichever chunk of the block loop each lands in.  Random
    positive qc everywhere, so the corners carry distinct values; bit-exact after bdyval."""
    import dataclasses
    rc = dataclasses.replace(CONFIGS["C1"], jx=24, iy=iy, nspgx=None, nspgd=None)
    data = icbc.generate(rc)
    st = {k: v.copy() for k, v in data["state"].items()}
    rng = np.random.default_rng(11)
    for name in ("ATM1_QC", "ATM2_QC"):
        st[name] = rng.uniform(1e-6, 1e-4, size=st[name].shape) * st["PSA"][0][None]
    from oracle.oracle import OracleCore
    from regcm_amd.dycore import DynCore
    o, e = OracleCore(rc, data["split"]), DynCore(rc, data["split"])
    for c in (o, e):
        c.put_state(st)
        c.bdyval()
    for name in STATE_FIELDS:
        assert np.array_equal(e.get(name)[..., : rc.iy - 1, : rc.jx - 1],
                              o.get(name)[..., : rc.iy - 1, : rc.jx - 1]), name
    for c in (o, e):
        c.step(2)
    for name in STATE_FIELDS:
        err = relerr(e.get(name), o.get(name), rc, name)
        assert err < 1e-11, (name, err)


def test_sladvection_departure_check(c1_data):
    """A departure point more than one cell away stops the step like the reference's
    fatal('SLADVECTION') (Main/mod_sladvection.F90:149-154), in the engine and the oracle."""
    import dataclasses
    from regcm_amd.dycore import EngineError
    rc, data = c1_data
    rcv = dataclasses.replace(rc, isladvec=1)
    st = {k: v.copy() for k, v in data["state"].items()}
    for name in ("ATM1_U", "ATM2_U"):
        st[name] = st[name] * 60.0               # ~600 m/s: u dt > dx at 60 km, 150 s
    from oracle.oracle import OracleCore
    from regcm_amd.dycore import DynCore
    o, e = OracleCore(rcv, data["split"]), DynCore(rcv, data["split"])
    for c in (o, e):
        c.put_state(st)
        c.bdyval()
    with pytest.raises(FloatingPointError):
        o.tend()
    with pytest.raises(EngineError, match="SLADVECTION"):
        e.tend()            # reported by the call, at the latest by the next synchronize
        e.synchronize()
