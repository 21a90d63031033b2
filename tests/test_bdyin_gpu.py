"""GPU parity of the device ICBC boundary pipeline.

rcmdyn_bdyin restates mod_bdycod::bdyin from read_icbc on (Main/mod_bdycod.F90:654-889):
b0 <- b1; the new record converted (p* = ps/10 - ptop), exchanged, coupled with p* (u, v with
its psc2psd), exchanged, time-interpolated (bt = (b1 - b0)/dtbdys); xbctime = 0.  Each value
is one product or difference, so the engine's b0/bt equal the oracle's (orc_bdyin) bit for
bit, on one tile and on decomposed ones.  States stepped across a boundary update stay within
the step's own tolerance (tests/test_parity_gpu.py, tests/test_nh_gpu.py).
"""
import numpy as np
import pytest

from regcm_amd import icbc
from regcm_amd.config import CONFIGS, NH_STATE_FIELDS, STATE_FIELDS

pytestmark = pytest.mark.gpu

BDY = ["XUB_B0", "XUB_BT", "XVB_B0", "XVB_BT", "XTB_B0", "XTB_BT", "XQB_B0", "XQB_BT"]
HBDY = BDY + ["XPSB_B0", "XPSB_BT"]
NHBDY = BDY + ["XPPB_B0", "XPPB_BT", "XWWB_B0", "XWWB_BT"]
CROSS = {"ATM1_T", "ATM1_QV", "ATM1_QC", "ATM2_T", "ATM2_QV", "ATM2_QC", "PSA", "PSB",
         "DSTOR", "HSTOR", "ATM1_PP", "ATM2_PP", "ATM1_W", "ATM2_W"}


def relerr(a, b, rc, name):
    if name in CROSS:
        a = a[:, : rc.iy - 1, : rc.jx - 1]
        b = b[:, : rc.iy - 1, : rc.jx - 1]
    den = max(np.max(np.abs(b)), 1e-300)
    return float(np.max(np.abs(a - b)) / den)


def records(rc, data, nh, n=3, seed=5):
    """n raw ICBC records as read_icbc returns them (u, v m/s on dot points; t K, qv kg/kg on
    cross points; ps hPa; NH pp Pa, w m/s), drifting from the synthetic initial state."""
    st = data["state"]
    rng = np.random.Generator(np.random.PCG64(seed))
    kz, iy, jx = rc.kz, rc.iy, rc.jx
    ps = st["PSA"][0]
    pd = icbc.psc2psd_global(ps)
    ce = (slice(None), slice(0, iy - 1), slice(0, jx - 1))
    pss = np.where(ps > 0.0, ps, 1.0)[None]
    recs = []
    for r in range(n):
        rec = {"XUB_B1": st["XUB_B0"] / pd[None] + 0.5 * r + 0.2 * rng.standard_normal((kz, iy, jx)),
               "XVB_B1": st["XVB_B0"] / pd[None] - 0.3 * r + 0.2 * rng.standard_normal((kz, iy, jx))}
        t = np.zeros((kz, iy, jx))
        q = np.zeros((kz, iy, jx))
        t[ce] = (st["XTB_B0"] / pss)[ce] + 0.4 * r + 0.2 * rng.standard_normal((kz, iy - 1, jx - 1))
        q[ce] = (st["XQB_B0"] / pss)[ce] * (1.0 + 0.01 * r)
        rec["XTB_B1"], rec["XQB_B1"] = t, q
        if nh:
            pp = np.zeros((kz, iy, jx))
            pp[ce] = (st["XPPB_B0"] / pss)[ce] + 5.0 * rng.standard_normal((kz, iy - 1, jx - 1))
            w = np.zeros((kz + 1, iy, jx))
            w[ce] = 0.01 * rng.standard_normal((kz + 1, iy - 1, jx - 1))
            rec["XPPB_B1"], rec["XWWB_B1"] = pp, w
        else:
            p = np.zeros((1, iy, jx))
            p[ce] = ((ps[None] + rc.ptop) * 10.0)[ce] + 0.5 * r
            rec["XPSB_B1"] = p
        recs.append(rec)
    return recs


def feed(c, rec):
    for name, a in rec.items():
        c.put(name, a)
    c.bdyin()


def make_pair(rc, data, nproc=(1, 1)):
    from oracle.oracle import OracleCore
    from regcm_amd.dycore import DynCore
    o = OracleCore(rc, data["split"])
    e = DynCore(rc, data["split"], nproc_j=nproc[0], nproc_i=nproc[1])
    for c in (o, e):
        c.put_state(data["state"])
    return o, e


def check_bdy(o, e, names):
    for name in names:
        assert np.array_equal(e.get(name), o.get(name)), name
    assert e.get_time()[2] == 0.0 and o.get_time()[2] == 0.0


@pytest.fixture(scope="module")
def nh_data():
    rc = CONFIGS["N1"]
    return rc, icbc.generate_nh(rc)


def test_bdyin_init_and_update_exact(c1_data):
    rc, data = c1_data
    recs = records(rc, data, False)
    o, e = make_pair(rc, data)
    for c in (o, e):            # init_bdy: the records at the start and dtbdys later
        feed(c, recs[0])
        feed(c, recs[1])
    check_bdy(o, e, HBDY)
    for c in (o, e):
        c.bdyval()
        c.step(2)
        c.tend()
        feed(c, recs[2])        # alarm_in_bdy: bdyin between tend and bdyval (RCM_run)
    check_bdy(o, e, HBDY)
    for c in (o, e):
        c.bdyval()
        c.step(2)
    for name in STATE_FIELDS:
        err = relerr(e.get(name), o.get(name), rc, name)
        assert err < 1e-11, (name, err)


@pytest.mark.parametrize("nproc", [(2, 2), (1, 3)])
def test_bdyin_decomposition_invariance(c1_data, nproc):
    from regcm_amd.dycore import DynCore
    rc, data = c1_data
    recs = records(rc, data, False)
    cores = [DynCore(rc, data["split"]), DynCore(rc, data["split"], nproc_j=nproc[0], nproc_i=nproc[1])]
    for c in cores:
        c.put_state(data["state"])
        feed(c, recs[0])
        feed(c, recs[1])
        c.bdyval()
        c.step(3)
    for name in HBDY + STATE_FIELDS:
        assert np.array_equal(cores[0].get(name), cores[1].get(name)), name


def test_nh_bdyin_exact(nh_data):
    rc, data = nh_data
    recs = records(rc, data, True)
    o, e = make_pair(rc, data)
    psdot = icbc.psc2psd_global(data["state"]["ATM0_PS"][0])[None]
    for c in (o, e):
        c.put("ATM0_PSDOT", psdot)
        feed(c, recs[0])
        feed(c, recs[1])
    check_bdy(o, e, NHBDY)
    for c in (o, e):
        c.bdyval()
        c.step(2)
    for name in STATE_FIELDS[:12] + NH_STATE_FIELDS:
        err = relerr(e.get(name), o.get(name), rc, name)
        assert err < 1e-10, (name, err)


def test_bdyin_errors(c1_data):
    from regcm_amd.dycore import DynCore, EngineError
    rc, data = c1_data
    e = DynCore(rc, data["split"])
    with pytest.raises(EngineError, match="no ICBC record"):
        e.bdyin()
    with pytest.raises(EngineError, match="non-hydrostatic"):
        e.put("XPPB_B1", np.zeros((rc.kz, rc.iy, rc.jx)))
