"""The RCCL halo transport on one GPU.

RCCL refuses two ranks on one device, so the multi-process path cannot run on a one-GPU
box.  RCMDYN_FORCE_RCCL=1 makes one engine that holds several tiles move every halo
message between them through RCCL instead of device copies: a one-rank communicator whose
grouped ncclSend/ncclRecv go to itself (comm.hip).  That exercises the communicator set-up,
the per-neighbour grouping of the exchange points, the two-stream (halo/compute overlap)
schedule with RCCL on both streams, the RCCL all-reduce of the NH day-alarm sums and the
capture of all of it into the step graphs.  The result must be bit-identical to one tile, as
for the device-copy transport (tests/test_parity_gpu.py) and the reference across rank
counts.
"""
import numpy as np
import pytest

from regcm_amd.config import CONFIGS, NH_STATE_FIELDS, STATE_FIELDS
from regcm_amd import icbc

pytestmark = pytest.mark.gpu

NH_FIELDS = ["ATM1_U", "ATM1_V", "ATM1_T", "ATM1_QV", "ATM1_QC", "ATM2_U", "ATM2_V", "ATM2_T",
             "ATM2_QV", "ATM2_QC", "PSA", "PSB"] + NH_STATE_FIELDS


def _engine(rc, data, nproc_j=1, nproc_i=1):
    from regcm_amd.dycore import DynCore
    e = DynCore(rc, data["split"], nproc_j=nproc_j, nproc_i=nproc_i)
    e.put_state(data["state"])
    e.bdyval()
    return e


def test_runtime_info():
    from regcm_amd.dycore import runtime_info
    info = runtime_info()
    assert info.startswith("hip=") and "librccl" in info and "rccl=" in info, info
    print(info)


@pytest.mark.parametrize("mode", ["graph", "eager", "dropin"])
def test_rccl_transport_hydrostatic(c1_data, monkeypatch, mode):
    rc, data = c1_data
    one = _engine(rc, data)
    monkeypatch.setenv("RCMDYN_FORCE_RCCL", "1")
    if mode == "eager":
        monkeypatch.setenv("RCMDYN_NO_GRAPH", "1")
    dec = _engine(rc, data, 2, 2)
    one.step(6)
    if mode == "dropin":
        for _ in range(6):
            dec.tend()
            dec.bdyval()
    else:
        dec.step(6)
    assert dec.get_time() == one.get_time()
    for name in STATE_FIELDS:
        assert np.array_equal(one.get(name), dec.get(name)), name
    a, b = one.reductions(), dec.reductions()
    assert a[2] == 0.0 and b[2] == 0.0
    assert np.allclose(a[:2], b[:2], rtol=1e-12, atol=0), (a, b)   # tile partials summed in another order


def test_rccl_shared_channel(c1_data, monkeypatch):
    """Both streams on the job's one communicator (RCMDYN_RCCL_CHAN2=one, the only mode), the
    second stream's exchange ordered after the first's.  Bit-identical to one tile."""
    rc, data = c1_data
    one = _engine(rc, data)
    monkeypatch.setenv("RCMDYN_FORCE_RCCL", "1")
    monkeypatch.setenv("RCMDYN_RCCL_CHAN2", "one")
    dec = _engine(rc, data, 2, 2)
    one.step(6)
    dec.step(6)
    for name in STATE_FIELDS:
        assert np.array_equal(one.get(name), dec.get(name)), name


def test_rccl_transport_nonhydrostatic(monkeypatch):
    rc = CONFIGS["N1"]
    data = icbc.generate_nh(rc)
    one = _engine(rc, data)
    monkeypatch.setenv("RCMDYN_FORCE_RCCL", "1")
    dec = _engine(rc, data, 2, 2)
    for e in (one, dec):
        e.step(5)                       # eager steps 1-2 (day alarm: RCCL all-reduce), then graphs
    for name in NH_FIELDS:
        assert np.array_equal(one.get(name), dec.get(name)), name
    a, b = one.reductions(), dec.reductions()
    assert 0.0 < a[2] < 1.0 and a[2] == b[2], (a, b)


def test_reductions_report(c1_data):
    """ptntot/pt2tot of the last step match the oracle's sums (Main/mod_tendency.F90:1449-1459)."""
    from oracle.oracle import OracleCore
    rc, data = c1_data
    e = _engine(rc, data)
    o = OracleCore(rc, data["split"])
    o.put_state(data["state"])
    o.bdyval()
    e.step(3)
    o.step(3)
    r = e.reductions()
    d = o.diagnostics()
    assert np.allclose(r[:2], d[:2], rtol=1e-10, atol=0), (r, d)
    assert r[0] > 0.0 and r[1] > 0.0


def test_rccl_job_wide_cfl_stop(c1_data, monkeypatch):
    """With a communicator the error flags are max-reduced over the ranks every 8 steps
    (GLOBAL_EVERY) and only the reduced word stops the run, so every rank fails at the same
    call, as the reference's fatal aborts the whole job (Main/abort.F90:20-36)."""
    from regcm_amd.dycore import EngineError
    rc, data = c1_data
    st = {k: v.copy() for k, v in data["state"].items()}
    for name in ("ATM1_T", "ATM2_T"):
        st[name][5, 20:24, 20:24] = np.nan
    monkeypatch.setenv("RCMDYN_FORCE_RCCL", "1")
    from regcm_amd.dycore import DynCore
    e = DynCore(rc, data["split"], nproc_j=2, nproc_i=2)
    e.put_state(st)
    e.bdyval()
    with pytest.raises(EngineError, match=r"CFL VIOLATION \(job, by step (8|16)\)"):
        e.step(100)
    assert e.get_time()[0] <= 24


TORCH_FIRST = r"""
import sys
import numpy as np
import torch  # noqa: F401  (loads torch's bundled librccl.so.1 / libamdhip64 before the engine)
sys.path.insert(0, sys.argv[1])
from regcm_amd.config import CONFIGS, STATE_FIELDS
from regcm_amd import icbc
from regcm_amd.dycore import DynCore, runtime_info
print(runtime_info())
rc = CONFIGS["C1"]
data = icbc.generate(rc)
engs = []
for nproc in ((1, 1), (2, 2)):
    e = DynCore(rc, data["split"], nproc_j=nproc[0], nproc_i=nproc[1])
    e.put_state(data["state"])
    e.bdyval()
    e.step(6)
    engs.append(e)
for name in STATE_FIELDS:
    assert np.array_equal(engs[0].get(name), engs[1].get(name)), name
print("torch-first ok")
"""


def test_rccl_graph_under_torch_rccl(tmp_path):
    """A process that imported torch before the engine binds torch's bundled RCCL (2.26, same
    soname as /opt/rocm's 2.27; the pytest run that collects the CPU tests is one).  The
    decomposed, overlapped, graph-captured step over RCCL self-communication must run and stay
    bit-identical there too: every exchange is captured on the origin stream (side_begin in
    engine.hip).  In a child process, so a crash fails this test instead of the run."""
    import os
    import subprocess
    import sys
    script = tmp_path / "torch_first.py"
    script.write_text(TORCH_FIRST)
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, RCMDYN_FORCE_RCCL="1")
    p = subprocess.run([sys.executable, str(script), root], capture_output=True, text=True, timeout=240, env=env)
    print(p.stdout[-2000:], p.stderr[-2000:])
    assert p.returncode == 0, (p.returncode, p.stderr[-2000:])
    assert "torch-first ok" in p.stdout
