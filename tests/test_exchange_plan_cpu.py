"""The multi-rank communication schedule of the engine, checked on the host for every rank of
2-, 4- and 8-GPU decompositions of the BASELINE configurations (no GPU, no communicator).

rcmdyn_exchange_plan runs the engine's own step sequence (prepare, then tend + bdyval) in a
plan-only mode in which every halo message and collective a rank would issue is logged in
issue order.  An RCCL job needs, for every ordered pair of ranks (A, B) and every channel
(communicator), A's sends to B to be exactly B's receives from A, in the same order, with the
same length and the same box shapes (Main/mpplib/mod_mppparam.F90:6867-7428 posts the matching
irecv/isend pairs of the reference); and every rank to issue the same collectives in the same
order.  Those are asserted here for the remote-peer path the single-GPU tests cannot reach."""
import dataclasses
from collections import defaultdict

import numpy as np
import pytest

from regcm_amd import dycore, icbc
from regcm_amd.config import CONFIGS, set_nproc


def plans(rc, split, cj, ci, nsteps):
    return [dycore.exchange_plan(rc, split, cj, ci, r, nsteps) for r in range(cj * ci)]


def check_plans(pl, cj, ci, band=False):
    n = cj * ci
    sends, recvs = defaultdict(list), defaultdict(list)
    colls = []
    for r, p in enumerate(pl):
        assert len(p) > 0, r
        cl = []
        for call, kind, chan, d, peer, count, sig in p:
            if kind == 1:
                assert 0 <= peer < n and peer != r and count > 0 and chan in (0, 1)
                (sends if d == 0 else recvs)[(r, peer, chan) if d == 0 else (peer, r, chan)].append((count, sig))
            else:
                assert d == -1 and chan == 0
                cl.append((kind, count))
        colls.append(cl)
    for key in set(sends) | set(recvs):
        assert sends.get(key, []) == recvs.get(key, []), ("send/recv mismatch", key)
    assert all(c == colls[0] for c in colls), "collectives differ across ranks"
    # every tile exchanges with each of its (up to 8) neighbours
    for r in range(n):
        lj, li = divmod(r, ci)
        for dj in (-1, 0, 1):
            for di in (-1, 0, 1):
                q = ((lj + dj) % cj if band else lj + dj, li + di)
                if (dj or di) and 0 <= q[0] < cj and 0 <= q[1] < ci and q != (lj, li):
                    assert sends.get((r, q[0] * ci + q[1], 0)), (r, q)
    return sum(len(v) for v in sends.values()), len(colls[0])


@pytest.mark.parametrize("name,nranks", [("C3", 2), ("C3", 4), ("C3", 8), ("C4", 4), ("C4", 8), ("C1", 3)])
def test_hydrostatic_plans_match(name, nranks):
    rc = CONFIGS[name]
    data = icbc.generate(rc)
    cj, ci = set_nproc(nranks, rc.jx, rc.iy)
    pl = plans(rc, data["split"], cj, ci, 3)
    msgs, ncoll = check_plans(pl, cj, ci)
    assert msgs > 0 and ncoll >= 1
    # the overlapped schedule issues every exchange on the engine's stream (channel 0; the
    # kernels that read no ghost point run on the second stream)
    assert all((p[:, 2] == 0).all() for p in pl)


@pytest.mark.parametrize("name,nranks", [("C3", 8), ("C1", 4)])
def test_hydrostatic_plans_match_no_overlap(monkeypatch, name, nranks):
    """RCMDYN_NO_OVERLAP=1 (round 2's schedule): the prologue's atm2 part travels on the second
    stream (channel 1), ordered after the first stream's atm1/p* part on the shared
    communicator; the plans still match rank to rank."""
    monkeypatch.setenv("RCMDYN_NO_OVERLAP", "1")
    rc = CONFIGS[name]
    data = icbc.generate(rc)
    cj, ci = set_nproc(nranks, rc.jx, rc.iy)
    pl = plans(rc, data["split"], cj, ci, 3)
    check_plans(pl, cj, ci)
    assert any((p[:, 2] == 1).any() for p in pl)


@pytest.mark.parametrize("variant", [{"isladvec": 1}, {"ibltyp": 2}, {"iboudy": 4}, {"idiffu": 2}, {"idiffu": 3}],
                         ids=lambda v: ",".join(f"{k}={x}" for k, x in v.items()))
def test_hydrostatic_variant_plans_match(variant):
    rc = dataclasses.replace(CONFIGS["C1"], **variant)
    data = icbc.generate(CONFIGS["C1"])
    check_plans(plans(rc, data["split"], 2, 2, 3), 2, 2)


@pytest.mark.parametrize("name,cj,ci", [("C1", 2, 2), ("C1", 3, 1), ("C1", 1, 3), ("C3", 2, 4), ("C3", 4, 2)], ids=str)
@pytest.mark.parametrize("variant", [{}, {"isladvec": 1, "ibltyp": 2}, {"idiffu": 3}],
                         ids=lambda v: ",".join(f"{k}={x}" for k, x in v.items()) or "default")
def test_band_plans_match(name, cj, ci, variant):
    """A band (i_band = 1) is periodic in j: the tiles of the first and the last tile column
    are neighbours, and with two tiles in j one rank is both the west and the east neighbour,
    so its messages to that rank must be issued in the order the receiver posts them; with one
    tile in j the periodic exchange is the rank's own copy (no message)."""
    rc = dataclasses.replace(CONFIGS[name], i_band=1, **variant)
    data = icbc.generate(rc)
    pl = plans(rc, data["split"], cj, ci, 3)
    msgs, _ = check_plans(pl, cj, ci, band=True)
    assert msgs > 0
    if cj > 1:                       # the wrap-around pair exchanges
        assert any(((p[:, 1] == 1) & (p[:, 4] == (cj - 1) * ci)).any() for p in pl[:ci])


def test_narrow_tiles_per_substep_exchange_plans_match():
    """Tiles narrower than the split-step halo take the per-sub-step exchange path (1 x 7)."""
    rc = CONFIGS["C1"]
    data = icbc.generate(rc)
    check_plans(plans(rc, data["split"], 1, 7, 2), 1, 7)


@pytest.mark.parametrize("name,nranks,nsteps", [("N1", 4, 3), ("N2", 8, 3)])
def test_nonhydrostatic_plans_match(name, nranks, nsteps):
    """NH: the day-alarm all-reduce, the acoustic sub-step exchanges and the 6-deep estore halo
    (3 steps: the first two change istep)."""
    rc = CONFIGS[name]
    data = icbc.generate_nh(rc)
    cj, ci = set_nproc(nranks, rc.jx, rc.iy)
    msgs, ncoll = check_plans(plans(rc, data["split"], cj, ci, nsteps), cj, ci)
    assert ncoll >= 2          # the day-alarm sums and the step-flag reduction


@pytest.mark.parametrize("variant", [{"idiffu": 3}, {"idiffu": 3, "ibltyp": 2}, {"upstream_mode": 0}],
                         ids=lambda v: ",".join(f"{k}={x}" for k, x in v.items()))
def test_nonhydrostatic_variant_plans_match(variant):
    """NH variants with other exchange widths (idiffu = 3: atm2 3 wide, p*b 4 wide)."""
    rc = dataclasses.replace(CONFIGS["N1"], **variant)
    data = icbc.generate_nh(CONFIGS["N1"])
    check_plans(plans(rc, data["split"], 2, 2, 2), 2, 2)


def test_c5_eight_rank_plan_matches():
    """C5 on 2 x 4 tiles (BASELINE's 8-GPU NH configuration).  The plan depends on the split
    constants only through spinit (sigma, ptop, kz, dt, nsplit: N2's are C5's) and istep."""
    rc = CONFIGS["C5"]
    split = icbc.generate_nh(CONFIGS["N2"])["split"]
    cj, ci = set_nproc(8, rc.jx, rc.iy)
    assert (cj, ci) == (2, 4)
    check_plans(plans(rc, split, cj, ci, 2), cj, ci)


def test_plan_refuses_multi_tile_rank():
    rc = CONFIGS["C1"]
    data = icbc.generate(rc)
    cfg_rank = 0
    with pytest.raises(dycore.EngineError):
        from regcm_amd.config import build_config
        import ctypes
        cfg = build_config(rc, data["split"], 2, 2, tile_first=0, tile_count=2, comm_rank=cfg_rank, comm_size=4)
        n = ctypes.c_int64()
        if dycore.lib().rcmdyn_exchange_plan(ctypes.byref(cfg), 1, None, 0, ctypes.byref(n)):
            raise dycore.EngineError(dycore.lib().rcmdyn_last_error(None).decode())
