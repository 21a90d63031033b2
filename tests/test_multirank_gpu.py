"""The engine's multi-rank (remote-peer) path on one GPU: one engine per tile, each its own
"rank" driven by its own host thread, exchanging through the in-process loopback transport
(RCMDYN_LOCAL_COMM, regcm_amd/csrc/comm.hip).  Every halo message goes through the code an
RCCL job runs -- rank-addressed sends/receives per exchange point, two channels (the
overlapped second stream), the job-wide flag and day-alarm collectives -- with a device copy in
place of the xGMI transfer.  The decomposed job must reproduce the single-tile engine
bit-for-bit, as the reference does across MPI rank counts."""
import os
import threading

import numpy as np
import pytest

from regcm_amd.config import CONFIGS, NH_STATE_FIELDS, STATE_FIELDS
from regcm_amd import icbc

pytestmark = pytest.mark.gpu


def run_ranks(rc, data, cj, ci, nsteps, group, per_rank=None):
    """Run nsteps on cj x ci ranks (threads); returns the engines (still open).  per_rank(e, r)
    runs after the state put (a rank's own puts)."""
    import gc
    from regcm_amd.dycore import DynCore
    gc.collect()            # engines of earlier tests are destroyed here, not in a rank thread
    n = cj * ci
    os.environ["RCMDYN_LOCAL_COMM"] = group
    try:
        engs = [DynCore(rc, data["split"], nproc_j=cj, nproc_i=ci, tile_first=r, tile_count=1,
                        comm_rank=r, comm_size=n, device=0) for r in range(n)]
    finally:
        del os.environ["RCMDYN_LOCAL_COMM"]
    errs = []

    def work(e):
        try:
            e.put_state(data["state"])
            if per_rank:
                per_rank(e, engs.index(e))
            e.bdyval()
            e.step(nsteps)
            e.synchronize()
        except Exception as x:          # pragma: no cover - reported below
            errs.append(repr(x))

    th = [threading.Thread(target=work, args=(e,)) for e in engs]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    assert not any(t.is_alive() for t in th), "a rank hung"
    assert not errs, errs
    return engs


def gather(engs, name):
    """Each rank's get fills only its owned points; the tiles partition the domain."""
    return sum(e.get(name) for e in engs)


def single(rc, data, nsteps):
    from regcm_amd.dycore import DynCore
    e = DynCore(rc, data["split"])
    e.put_state(data["state"])
    e.bdyval()
    e.step(nsteps)
    return e


@pytest.mark.parametrize("name,cj,ci", [("C1", 2, 2), ("C1", 1, 3), ("C3", 2, 4)])
def test_hydrostatic_ranks_bit_identical(name, cj, ci):
    rc = CONFIGS[name]
    data = icbc.generate(rc)
    nsteps = 10                     # crosses the 8-step job-wide flag reduction
    engs = run_ranks(rc, data, cj, ci, nsteps, f"h{name}{cj}{ci}")
    ref = single(rc, data, nsteps)
    for f in STATE_FIELDS:
        assert np.array_equal(gather(engs, f), ref.get(f)), f
    assert all(e.get_time() == ref.get_time() for e in engs)


@pytest.mark.parametrize("cj,ci", [(2, 1), (2, 2), (1, 2), (3, 1)], ids=str)
def test_band_ranks_bit_identical(cj, ci):
    """The tropical band (i_band = 1) on ranks: the first and last tile columns are remote
    neighbours across the period, with two tiles in j one rank is both the west and the east
    peer (its messages in the receiver's direction order), and with one tile in j a rank's
    periodic exchange stays inside it.  Bit-identical to one tile."""
    import dataclasses
    rc = dataclasses.replace(CONFIGS["C1"], i_band=1)
    data = icbc.generate(rc)
    nsteps = 10
    engs = run_ranks(rc, data, cj, ci, nsteps, f"band{cj}{ci}")
    ref = single(rc, data, nsteps)
    for f in STATE_FIELDS:
        assert np.array_equal(gather(engs, f), ref.get(f)), f


def test_hydrostatic_ranks_variant_sladv_tke():
    """isladvec = 1 (the widest prologue halos) with UW TKE (its exchange on both channels)."""
    import dataclasses
    rc = dataclasses.replace(CONFIGS["C1"], isladvec=1, ibltyp=2)
    data = icbc.generate(CONFIGS["C1"])
    data = {"split": data["split"], "state": dict(data["state"], **icbc.tke_state(rc))}
    engs = run_ranks(rc, data, 2, 2, 4, "hvar")
    ref = single(rc, data, 4)
    for f in STATE_FIELDS + ["ATM1_TKE", "ATM2_TKE"]:
        assert np.array_equal(gather(engs, f), ref.get(f)), f


def test_nonhydrostatic_ranks_bit_identical():
    """NH on 2 x 2 ranks: the acoustic sub-step exchanges, the 6-deep estore halo and the
    day-alarm all-reduce of the radiative condition (3 steps: istep changes on the first two)."""
    rc = CONFIGS["N1"]
    data = icbc.generate_nh(rc)
    engs = run_ranks(rc, data, 2, 2, 3, "nh")
    ref = single(rc, data, 3)
    for f in STATE_FIELDS[:12] + NH_STATE_FIELDS:
        assert np.array_equal(gather(engs, f), ref.get(f)), f


@pytest.mark.parametrize("cj,ci", [(2, 2), (1, 2), (2, 1)], ids=str)
def test_crm_ranks_bit_identical(cj, ci):
    """PreProc/CRM/crm_test.in's configuration (i_crm = 1: NH, periodic in j and i, UW TKE) on
    ranks: every tile's four sides are remote peers across one of the two periods (with two
    tiles in a direction one rank is both neighbours there, with one tile the periodic exchange
    stays inside the rank), the corner peers wrap in both directions, and the day-alarm sums of
    the radiative condition are all-reduced.  Bit-identical to one tile."""
    from regcm_amd.config import CONFIGS as C
    rc = C["CRM"]
    data = icbc.generate_crm(rc)
    engs = run_ranks(rc, data, cj, ci, 4, f"crm{cj}{ci}")
    ref = single(rc, data, 4)
    for f in STATE_FIELDS[:12] + NH_STATE_FIELDS + ["ATM1_TKE", "ATM2_TKE"]:
        assert np.array_equal(gather(engs, f), ref.get(f)), f


def test_job_reductions_over_ranks():
    """rcmdyn_reductions is collective: every rank gets the job-wide ptntot/pt2tot (sums of the
    tiles' partials) equal to the single tile's within the reordering of one sum."""
    rc = CONFIGS["C1"]
    data = icbc.generate(rc)
    engs = run_ranks(rc, data, 2, 2, 3, "red")
    ref = single(rc, data, 3).reductions()
    out = [None] * len(engs)

    def red(q):
        out[q] = engs[q].reductions()
    th = [threading.Thread(target=red, args=(q,)) for q in range(len(engs))]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=120)
    for o in out:
        assert o is not None and o == out[0]
        assert abs(o[0] - ref[0]) <= 1e-12 * abs(ref[0]) and abs(o[1] - ref[1]) <= 1e-12 * abs(ref[1])


@pytest.mark.parametrize("band", [0, 1], ids=["lam", "band"])
def test_uw_kpbl_put_on_own_points(band):
    """iuwvadv = 1 with each rank putting kpbl on its own cross points only (as the physics
    computes it): vadv4d ind = 3 of the fused step reads kpbl on the ghost ring
    k_scalars computes in place of the cqv/cqc exchange, so the engine exchanges a put kpbl once
    before the next tend.  Bit-identical to the single tile with the global put.  The band's
    ranks take their points from the band-aware extents (rcmdyn_tile_extent_cfg): the last tile
    column's cross range then ends at jx, not jx - 1."""
    import dataclasses
    from regcm_amd.dycore import tile_extent
    rc0 = dataclasses.replace(CONFIGS["C1"], i_band=band)
    rc = dataclasses.replace(rc0, ibltyp=2, iuwvadv=1)
    base = icbc.generate(rc0)
    st = dict(base["state"], **icbc.tke_state(rc))
    st.update(icbc.hydrometeor_state(rc, st, nqx=2))
    rng = np.random.default_rng(5)
    kpbl = rng.integers(1, rc.kz + 1, size=(1, rc.iy, rc.jx)).astype(np.float64)
    cj, ci = 2, 2

    def own_kpbl(e, r):
        ext, _ = tile_extent(rc.jx, rc.iy, cj, ci, r, i_band=band)
        j1, j2, i1, i2 = ext[4], ext[5], ext[6], ext[7]
        assert not band or r // ci < cj - 1 or j2 == rc.jx
        e.put("KPBL", kpbl[:, i1 - 1:i2, j1 - 1:j2], j1=j1, i1=i1)

    data = {"split": base["split"], "state": st}
    engs = run_ranks(rc, data, cj, ci, 4, "uwk", per_rank=own_kpbl)
    # the reference: the same 2 x 2 tiles in one engine with the global put (the moisture fix
    # of the cloud edges depends on the decomposition, as the reference's)
    from regcm_amd.dycore import DynCore
    ref = DynCore(rc, base["split"], nproc_j=cj, nproc_i=ci)
    ref.put_state(dict(st, KPBL=kpbl))
    ref.bdyval()
    ref.step(4)
    for f in STATE_FIELDS:
        assert np.array_equal(gather(engs, f), ref.get(f)), f
