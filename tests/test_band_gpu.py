"""GPU parity of the tropical band (i_band = 1, hydrostatic): the HIP engine through the C-ABI
against the restatement's band (oracle/rcm_oracle.c), and the band's own invariants.

A band is periodic in j (Main/mpplib/mod_mppparam.F90:1112-1114, 1131): one tile in j is its
own west and east neighbour, two tiles in j are each other's west and east neighbour, and the
cross grid takes every j (:1351-1354), so the cross fields are compared on all jx columns.
Only the south and north rows relax to the boundary data (Main/mod_atm_interface.F90:435-457).
Tolerances as tests/test_parity_gpu.py: 1 step < 1e-12 and 3 steps < 1e-11 in relative
max-norm (libm-vs-OCML ulps downstream of log/pow); engine-to-engine properties bit-exact.
"""
import dataclasses

import numpy as np
import pytest

from regcm_amd.config import CONFIGS, QX_STATE_FIELDS, STATE_FIELDS
from regcm_amd import icbc

pytestmark = pytest.mark.gpu

CROSS = {"ATM1_T", "ATM1_QV", "ATM1_QC", "ATM2_T", "ATM2_QV", "ATM2_QC", "PSA", "PSB",
         "DSTOR", "HSTOR", "ATM1_TKE", "ATM2_TKE"} | set(QX_STATE_FIELDS)

# the options of tests/test_band_cpu.py plus the two whose result depends on the tiling
# (idiffu = 3's last-column term and clamped stencil, the moisture fix's j-order sweep)
VARIANTS = [{}, {"isladvec": 1}, {"ibltyp": 2}, {"iboudy": 1}, {"iboudy": 4}, {"idiffu": 2},
            {"idiffu": 3}, {"ipptls": 2}]
TILING_VARIANTS = [{}, {"isladvec": 1, "ibltyp": 2}, {"iboudy": 4}]


def _vid(v):
    return ",".join(f"{k}={x}" for k, x in v.items()) or "default"


def relerr(a, b, rc, name):
    if name in CROSS:                    # the cross grid: every j, rows 1..iy-1
        a = a[:, : rc.iy - 1, :]
        b = b[:, : rc.iy - 1, :]
    den = max(np.max(np.abs(b)), 1e-300)
    return float(np.max(np.abs(a - b)) / den)


def band_case(variant, name="C1"):
    rc = dataclasses.replace(CONFIGS[name], i_band=1, **variant)
    data = icbc.generate(rc)
    st = dict(data["state"])
    if rc.ibltyp == 2:
        st.update(icbc.tke_state(rc))
    if rc.nqx > 2:
        st.update(icbc.hydrometeor_state(rc, st, nqx=rc.nqx))
    return rc, data, st


def fields(rc):
    return (list(STATE_FIELDS) + (QX_STATE_FIELDS if rc.nqx > 2 else []) +
            (["ATM1_TKE", "ATM2_TKE"] if rc.ibltyp == 2 else []))


def engine(rc, data, st, nproc_j=1, nproc_i=1):
    from regcm_amd.dycore import DynCore
    e = DynCore(rc, data["split"], nproc_j=nproc_j, nproc_i=nproc_i)
    e.put_state(st)
    e.bdyval()
    return e


@pytest.mark.parametrize("variant", VARIANTS, ids=_vid)
def test_band_matches_oracle(variant):
    """One tile (its own periodic neighbour through the halo exchange) against the oracle's
    one tile: the initial bdyval exactly, then 1 and 3 steps."""
    from oracle.oracle import OracleCore
    rc, data, st = band_case(variant)
    o = OracleCore(rc, data["split"])
    o.put_state(st)
    o.bdyval()
    e = engine(rc, data, st)
    for name in fields(rc):
        assert relerr(e.get(name), o.get(name), rc, name) == 0.0, name
    for nsteps, tol in ((1, 1e-12), (2, 1e-11)):
        o.step(nsteps)
        e.step(nsteps)
        for name in fields(rc):
            err = relerr(e.get(name), o.get(name), rc, name)
            assert err < tol, (name, err, nsteps)
    assert e.get_time() == o.get_time()


def test_band_twenty_steps_vs_oracle():
    from oracle.oracle import OracleCore
    rc, data, st = band_case({})
    o = OracleCore(rc, data["split"])
    o.put_state(st)
    o.bdyval()
    e = engine(rc, data, st)
    o.step(20)
    e.step(20)
    for name in fields(rc):
        err = relerr(e.get(name), o.get(name), rc, name)
        assert err < 1e-9, (name, err)


@pytest.mark.parametrize("nproc", [(2, 1), (1, 2), (2, 2), (3, 1), (2, 4)], ids=str)
@pytest.mark.parametrize("variant", TILING_VARIANTS, ids=_vid)
def test_band_tiles_bit_identical(variant, nproc):
    """Tiles of a band exchange around the period (with 2 tiles in j one tile is both the west
    and the east neighbour): bit-identical to one tile over 6 steps."""
    rc, data, st = band_case(variant)
    one = engine(rc, data, st)
    til = engine(rc, data, st, *nproc)
    one.step(6)
    til.step(6)
    for name in fields(rc):
        assert np.array_equal(one.get(name), til.get(name)), name


@pytest.mark.parametrize("variant,dims", [({"idiffu": 3}, (2, 2)), ({"idiffu": 3}, (3, 1)),
                                          ({"ipptls": 2}, (2, 2)), ({"ipptls": 2}, (1, 3))], ids=str)
def test_band_tiles_match_oracle_tiles(variant, dims):
    """The tiling-dependent options against the oracle run as the same tiles (orc_par.c)."""
    from oracle.oracle import OracleParallel
    rc, data, st = band_case(variant)
    o = OracleParallel(rc, data["split"], dims=dims)
    o.put_state(st)
    o.bdyval()
    e = engine(rc, data, st, *dims)
    for nsteps, tol in ((1, 1e-12), (2, 1e-11)):
        o.step(nsteps)
        e.step(nsteps)
        for name in fields(rc):
            err = relerr(e.get(name), o.get(name), rc, name)
            assert err < tol, (name, err, nsteps)


def test_band_rotation_commutes_with_step():
    """A rotation of every input by m columns in j commutes with the engine's step, bit for
    bit (no west/east edge; the block and tile boundaries move relative to the data)."""
    rc, data, st = band_case({"isladvec": 1})
    m = 13
    rot = {k: np.roll(v, m, axis=-1) for k, v in st.items()}
    a = engine(rc, data, st)
    b = engine(rc, data, rot)
    a.step(5)
    b.step(5)
    for name in fields(rc):
        assert np.array_equal(np.roll(a.get(name), m, axis=-1), b.get(name)), name


@pytest.mark.parametrize("nproc", [(1, 1), (2, 1), (2, 2)], ids=str)
def test_band_rccl_transport(monkeypatch, nproc):
    """The periodic messages through RCCL (RCMDYN_FORCE_RCCL: a one-rank communicator; one
    tile in j sends to itself) equal the device-copy transport."""
    rc, data, st = band_case({})
    ref = engine(rc, data, st, *nproc)
    monkeypatch.setenv("RCMDYN_FORCE_RCCL", "1")
    dec = engine(rc, data, st, *nproc)
    ref.step(6)
    dec.step(6)
    for name in fields(rc):
        assert np.array_equal(ref.get(name), dec.get(name)), name


def test_band_c3_tiles_bit_identical():
    """The headline domain as a band on the 8-GPU tiling (2 x 4): bit-identical to one tile."""
    rc, data, st = band_case({}, "C3")
    one = engine(rc, data, st)
    til = engine(rc, data, st, 2, 4)
    one.step(4)
    til.step(4)
    for name in fields(rc):
        assert np.array_equal(one.get(name), til.get(name)), name


def test_band_reference_grid_test_009():
    """The reference's own band run, Testing/test_009.in: 720 x 210 x 18 at ds = 55.5994675 km,
    dt = 150 s, i_band = 1, iboudy = 5 (:3-5, 16; a wide, non-square grid) against the oracle
    after 1, 3 and 10 steps, and its 8-GPU tiling (2 x 4) bit-identical to one tile."""
    from oracle.oracle import OracleCore
    rc = dataclasses.replace(CONFIGS["C1"], jx=720, iy=210, kz=18, ds=55.5994675, dt=150.0, i_band=1,
                             name="test_009 band 720x210x18")
    data = icbc.generate(rc)
    st = dict(data["state"])
    o = OracleCore(rc, data["split"])
    o.put_state(st)
    o.bdyval()
    e = engine(rc, data, st)
    til = engine(rc, data, st, 2, 4)
    for name in fields(rc):
        assert relerr(e.get(name), o.get(name), rc, name) == 0.0, name
    for nsteps, tol in ((1, 1e-12), (2, 1e-11), (7, 1e-9)):
        o.step(nsteps)
        e.step(nsteps)
        til.step(nsteps)
        for name in fields(rc):
            err = relerr(e.get(name), o.get(name), rc, name)
            assert err < tol, (name, err, nsteps)
            assert np.array_equal(e.get(name), til.get(name)), name
    assert e.get_time() == o.get_time() == til.get_time()
