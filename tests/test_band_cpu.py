"""CPU tests of the tropical band (i_band = 1): the grid is periodic in j, every tile is its own
or its neighbours' west/east neighbour around the period, and only the south and north rows
relax to the boundary data (Main/mpplib/mod_mppparam.F90:1112-1114, 1131, 1351-1354;
Main/mod_atm_interface.F90:435-457).  The restatement is checked by properties the band has
whatever the state: a rotation in j commutes with the step, and the set_nproc tiles of the
threaded oracle reproduce one tile bit for bit.  No GPU needed."""
import dataclasses

import numpy as np
import pytest

from regcm_amd import icbc
from regcm_amd.config import CONFIGS, STATE_FIELDS

# the options whose arithmetic is the same at every j of a band.  idiffu = 3 clamps its
# stencil to the global 1..jx-1 (Main/mod_diffusion.F90:428-470, no band branch) and acts on
# each tile's last column, and the moisture fix sweeps in j order: both are position- and
# decomposition-dependent in the reference too
BAND_VARIANTS = [{}, {"isladvec": 1}, {"ibltyp": 2}, {"iboudy": 1}, {"iboudy": 4}, {"idiffu": 2}]


def _vid(v):
    return ",".join(f"{k}={x}" for k, x in v.items()) or "default"


def band_case(variant, name="C1"):
    rc = dataclasses.replace(CONFIGS[name], i_band=1, **variant)
    data = icbc.generate(rc)
    st = dict(data["state"])
    if rc.ibltyp == 2:
        st.update(icbc.tke_state(rc))
    return rc, data, st


def fields(rc):
    return list(STATE_FIELDS) + (["ATM1_TKE", "ATM2_TKE"] if rc.ibltyp == 2 else [])


def test_band_generate_is_periodic():
    """The synthetic band state: the cross grid takes every j (no zero column at j = jx), p*
    on the dot grid is the periodic four-point mean, and dstor/hstor cover every j."""
    rc, data, st = band_case({})
    jx, iy = rc.jx, rc.iy
    psa = st["PSA"][0]
    assert np.all(psa[: iy - 1, :] > 0.0)
    pd = icbc.psc2psd_band(psa)
    j = jx - 1
    i = iy // 2
    assert pd[i, 0] == (psa[i, 0] + psa[i - 1, 0] + psa[i, j] + psa[i - 1, j]) * 0.25
    assert np.all(st["DSTOR"][:, : iy - 1, jx - 1] != 0.0)


@pytest.mark.parametrize("variant", BAND_VARIANTS, ids=_vid)
def test_band_rotation_commutes_with_step(variant):
    """Rotating every input by m columns in j and stepping equals stepping and rotating: the
    band has no west or east edge, so each point's arithmetic is the same wherever it sits."""
    from oracle.oracle import OracleCore
    rc, data, st = band_case(variant)
    m = 7
    rot = {k: np.roll(v, m, axis=-1) for k, v in st.items()}
    a = OracleCore(rc, data["split"])
    b = OracleCore(rc, data["split"])
    a.put_state(st)
    b.put_state(rot)
    for o in (a, b):
        o.bdyval()
        o.step(4)
    for name in fields(rc):
        assert np.array_equal(np.roll(a.get(name), m, axis=-1), b.get(name)), name


@pytest.mark.parametrize("dims", [(1, 2), (2, 1), (2, 2), (3, 1), (2, 4)], ids=str)
@pytest.mark.parametrize("variant", BAND_VARIANTS, ids=_vid)
def test_band_tiles_match_single_tile(variant, dims):
    """The band as set_nproc tiles on threads (oracle/orc_par.c): the periodic neighbours wrap
    in j (with 2 tiles in j one tile is both the west and the east neighbour), and the result
    is bit-identical to one tile, which exchanges with itself."""
    from oracle.oracle import OracleCore, OracleParallel
    rc, data, st = band_case(variant)
    ref = OracleCore(rc, data["split"])
    par = OracleParallel(rc, data["split"], dims=dims)
    for o in (ref, par):
        o.put_state(st)
        o.bdyval()
        o.step(4)
    assert par.get_time() == ref.get_time()
    for name in fields(rc):
        assert np.array_equal(par.get(name), ref.get(name)), name


def test_band_stays_bounded():
    """60 steps of the band stay finite with p* in range; the S/N relaxation holds the rows
    next to the boundary near the boundary data."""
    from oracle.oracle import OracleCore
    rc, data, st = band_case({})
    o = OracleCore(rc, data["split"])
    o.put_state(st)
    o.bdyval()
    o.step(60)
    psa = o.get("PSA")[0, : rc.iy - 1, :]
    assert np.all(np.isfinite(psa)) and psa.min() > 50.0 and psa.max() < 110.0
    t = o.get("ATM1_T")[:, : rc.iy - 1, :] / psa[None]
    assert t.min() > 150.0 and t.max() < 340.0


def test_band_bad_values_refused():
    """i_band is 0 or 1 (both cores since round 6); CRM needs the band and the NH core, and
    iboudy = 0 needs CRM (oracle and engine alike: the engine's refusals are checked in
    test_abi_cpu)."""
    from oracle.oracle import OracleCore
    data = icbc.generate_nh(CONFIGS["N1"])
    for bad in (dict(i_crm=1), dict(i_crm=1, i_band=1, idynamic=1), dict(iboudy=0)):
        with pytest.raises(RuntimeError):
            OracleCore(dataclasses.replace(CONFIGS["N1"], **bad), data["split"])
    OracleCore(dataclasses.replace(CONFIGS["N1"], i_band=1), data["split"]).close()
    rc = dataclasses.replace(CONFIGS["C1"], i_band=2)
    with pytest.raises(RuntimeError):
        OracleCore(rc, icbc.generate(CONFIGS["C1"])["split"])
