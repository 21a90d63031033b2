"""GPU parity of the reference's own non-hydrostatic namelist, PreProc/CRM/crm_test.in (i_band
= 1, i_crm = 1, iboudy = 0, ibltyp = 2, idynamic = 2; 64 x 64 x 23 at 3 km, dt 5 s), and of the
non-hydrostatic band without CRM: the HIP engine through the C-ABI against the oracle.

The grid of a CRM run is periodic in j and i (Main/mpplib/mod_mppparam.F90:1104-1108,
1131-1132; see tests/test_crm_cpu.py for what that changes in the step), so every prognostic
field is compared on the whole domain.  Tolerances as tests/test_nh_gpu.py (the NH step is
transcendental almost everywhere): the initial boundary pass exactly, 1e-11 after one step,
1e-10 after two, and after twenty within the oracle's own spread under a 1e-14 perturbation of
the initial temperature; engine-to-engine properties (tiles, transports, graph replay) bit for
bit.
"""
import dataclasses

import numpy as np
import pytest

from regcm_amd import icbc
from regcm_amd.config import CONFIGS

pytestmark = pytest.mark.gpu

FIELDS = ["ATM1_U", "ATM1_V", "ATM1_T", "ATM1_QV", "ATM1_QC", "ATM2_U", "ATM2_V", "ATM2_T", "ATM2_QV",
          "ATM2_QC", "PSA", "PSB", "ATM1_PP", "ATM2_PP", "ATM1_W", "ATM2_W", "ATM1_TKE", "ATM2_TKE"]


def relerr(a, b):
    return float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-300))


@pytest.fixture(scope="module")
def crm_data():
    rc = CONFIGS["CRM"]
    return rc, icbc.generate_crm(rc)


def engine(rc, data, st=None, nproc=(1, 1)):
    from regcm_amd.dycore import DynCore
    e = DynCore(rc, data["split"], nproc_j=nproc[0], nproc_i=nproc[1])
    e.put_state(st if st is not None else data["state"])
    e.bdyval()
    return e


def oracle(rc, data, st=None):
    from oracle.oracle import OracleCore
    o = OracleCore(rc, data["split"])
    o.put_state(st if st is not None else data["state"])
    o.bdyval()
    return o


def test_crm_matches_oracle(crm_data):
    """crm_test.in's shape against the oracle at 1, 2 and 20 steps."""
    rc, data = crm_data
    o, e = oracle(rc, data), engine(rc, data)
    for name in FIELDS:
        assert relerr(e.get(name), o.get(name)) == 0.0, name
    for nsteps, tol in ((1, 1e-11), (1, 1e-10)):
        o.step(nsteps)
        e.step(nsteps)
        assert e.get_time() == o.get_time()
        for name in FIELDS:
            err = relerr(e.get(name), o.get(name))
            assert err < tol, (name, err, nsteps)
    o.step(18)
    e.step(18)
    st = {k: v.copy() for k, v in data["state"].items()}
    st["ATM1_T"] = st["ATM1_T"] * (1.0 + 1e-14)
    p = oracle(rc, data, st)
    p.step(20)
    for name in FIELDS:
        err, spread = relerr(e.get(name), o.get(name)), relerr(p.get(name), o.get(name))
        assert err <= max(1e-9, 100.0 * spread), (name, err, spread)


CRM_VARIANTS = [{"ipptls": 2}, {"isladvec": 1}, {"idiffu": 2}, {"ifrayd": 0}, {"ifupr": 0}]


@pytest.mark.parametrize("variant", CRM_VARIANTS, ids=lambda v: ",".join(f"{k}={x}" for k, x in v.items()))
def test_crm_variants_match_oracle(variant):
    """crm_test.in's configuration with the options a CRM namelist may change: the hydrometeors
    of ipptls = 2 (their fix and filters on the doubly periodic planes), semi-Lagrangian
    moisture (departure points across both periods), the 9-point diffusion, no Rayleigh damping,
    no radiative upper condition; against the oracle at 1 and 2 steps."""
    from regcm_amd.config import QX_STATE_FIELDS
    rc = dataclasses.replace(CONFIGS["CRM"], **variant)
    data = icbc.generate_crm(rc)
    st = dict(data["state"])
    names = list(FIELDS)
    if rc.ipptls == 2:
        st.update(icbc.hydrometeor_state(rc, st, nqx=rc.nqx))
        names += QX_STATE_FIELDS
    o, e = oracle(rc, data, st), engine(rc, data, st)
    for name in names:
        assert relerr(e.get(name), o.get(name)) == 0.0, name
    for nsteps, tol in ((1, 1e-11), (1, 1e-10)):
        o.step(nsteps)
        e.step(nsteps)
        for name in names:
            err = relerr(e.get(name), o.get(name))
            assert err < tol, (name, err, nsteps)


@pytest.mark.parametrize("nproc", [(2, 2), (2, 1), (1, 2), (1, 3)], ids=str)
def test_crm_tiles_bit_identical(crm_data, nproc):
    """Tiles exchange around both periods (a tile may be its own neighbour in j or in i, and
    two tiles are each other's two neighbours); the day-alarm means are summed in one-tile
    order, so every tiling equals one tile bit for bit."""
    rc, data = crm_data
    one, til = engine(rc, data), engine(rc, data, nproc=nproc)
    one.step(6)
    til.step(6)
    for name in FIELDS:
        assert np.array_equal(one.get(name), til.get(name)), name


@pytest.mark.parametrize("nproc", [(1, 1), (2, 2)], ids=str)
def test_crm_rccl_transport(crm_data, monkeypatch, nproc):
    """The periodic messages through RCCL (a one-rank communicator, self send/receive) equal the
    device-copy transport."""
    rc, data = crm_data
    ref = engine(rc, data, nproc=nproc)
    monkeypatch.setenv("RCMDYN_FORCE_RCCL", "1")
    dec = engine(rc, data, nproc=nproc)
    ref.step(4)
    dec.step(4)
    for name in FIELDS:
        assert np.array_equal(ref.get(name), dec.get(name)), name


def test_crm_graph_replay_and_dropin_equal_eager(crm_data):
    rc, data = crm_data
    a, b = engine(rc, data), engine(rc, data)
    a.step(6)
    for _ in range(6):
        b.tend()
        b.bdyval()
    for name in FIELDS:
        assert np.array_equal(a.get(name), b.get(name)), name


def test_crm_rotation_commutes_with_step():
    """Without the radiative condition (its interior clamp is not translation invariant) the
    doubly periodic step commutes with a rotation of the state in j and i, bit for bit."""
    rc = dataclasses.replace(CONFIGS["CRM"], ifupr=0)
    data = icbc.generate_crm(rc)
    m, n = 13, 7
    rot = {k: np.roll(v, (n, m), axis=(-2, -1)) if v.ndim == 3 and v.shape[-2:] == (rc.iy, rc.jx) else v
           for k, v in data["state"].items()}
    a, b = engine(rc, data), engine(rc, data, rot)
    a.step(5)
    b.step(5)
    for name in FIELDS:
        assert np.array_equal(np.roll(a.get(name), (n, m), axis=(-2, -1)), b.get(name)), name


def test_crm_refusals(crm_data):
    """CRM without the band, on the hydrostatic core, or iboudy = 0 on a limited area are
    refused at create, not run differently."""
    from regcm_amd.dycore import DynCore, EngineError
    rc, data = crm_data
    for bad, msg in ((dict(i_band=0), "i_crm"), (dict(i_crm=0), "iboudy = 0")):
        with pytest.raises(EngineError, match=msg):
            DynCore(dataclasses.replace(rc, **bad), data["split"])


# ---- the non-hydrostatic band (periodic in j, south / north boundaries) --------------------

NHB_CROSS = {"ATM1_T", "ATM1_QV", "ATM1_QC", "ATM2_T", "ATM2_QV", "ATM2_QC", "PSA", "PSB",
             "ATM1_PP", "ATM2_PP", "ATM1_W", "ATM2_W"}
NHB_FIELDS = FIELDS[:16]


def nh_band_case(variant=None):
    """The CRM case's fields as a band (i_crm = 0): periodic in j, the south and north rows
    relax to the boundary data (the initial state) with iboudy = 5 by default."""
    rc = dataclasses.replace(CONFIGS["CRM"], **{"i_crm": 0, "iboudy": 5, "ibltyp": 1, **(variant or {})})
    data = icbc.generate_crm(rc)
    st = {k: v for k, v in data["state"].items() if "TKE" not in k or rc.ibltyp == 2}
    return rc, data, st


def band_relerr(a, b, rc, name):
    if name in NHB_CROSS:
        a, b = a[:, : rc.iy - 1, :], b[:, : rc.iy - 1, :]
    return relerr(a, b)


@pytest.mark.parametrize("variant", [{}, {"iboudy": 1}, {"iboudy": 4}, {"ibltyp": 2}], ids=str)
def test_nh_band_matches_oracle(variant):
    rc, data, st = nh_band_case(variant)
    o, e = oracle(rc, data, st), engine(rc, data, st)
    names = NHB_FIELDS + (["ATM1_TKE", "ATM2_TKE"] if rc.ibltyp == 2 else [])
    for name in names:
        assert band_relerr(e.get(name), o.get(name), rc, name) == 0.0, name
    for nsteps, tol in ((1, 1e-11), (2, 1e-10)):
        o.step(nsteps)
        e.step(nsteps)
        for name in names:
            err = band_relerr(e.get(name), o.get(name), rc, name)
            assert err < tol, (name, err, nsteps)


@pytest.mark.parametrize("nproc", [(2, 1), (2, 2), (3, 1)], ids=str)
def test_nh_band_tiles_bit_identical(nproc):
    rc, data, st = nh_band_case()
    one, til = engine(rc, data, st), engine(rc, data, st, nproc=nproc)
    one.step(5)
    til.step(5)
    for name in NHB_FIELDS:
        assert np.array_equal(one.get(name), til.get(name)), name
