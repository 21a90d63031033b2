"""iuwvadv = 1 engine-vs-oracle divergence locator (hydrostatic C1): per step, the worst
ATM1_QC / QCTEN point and its neighbourhood."""
import dataclasses
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
import numpy as np  # noqa: E402
from regcm_amd import icbc  # noqa: E402
from regcm_amd.config import CONFIGS  # noqa: E402
from regcm_amd.dycore import DynCore  # noqa: E402
from oracle.oracle import OracleCore  # noqa: E402
from test_oracle_cpu import _uw_kpbl, _uw_qc_state  # noqa: E402

uw = int(sys.argv[1]) if len(sys.argv) > 1 else 1
rc = dataclasses.replace(CONFIGS["C1"], ibltyp=2, iuwvadv=uw)
data = icbc.generate(rc)
st = _uw_qc_state(rc, data["state"])
kpbl = _uw_kpbl(rc)
cs = []
for cls in (OracleCore, DynCore):
    c = cls(rc, data["split"])
    c.put_state(st)
    for n, a in icbc.tke_state(rc).items():
        c.put(n, a)
    c.put("KPBL", kpbl)
    c.bdyval()
    c.set_diagnostics(True) if hasattr(c, "set_diagnostics") else None
    cs.append(c)
o, e = cs
for s in range(4):
    for c in cs:
        c.tend()
    for name in ("QCTEN", "QVTEN", "TTEN", "QDOT"):
        a, b = e.get(name), o.get(name)
        a = a[:, : rc.iy - 1, : rc.jx - 1]; b = b[:, : rc.iy - 1, : rc.jx - 1]
        d = np.abs(a - b)
        q = np.unravel_index(np.argmax(d), d.shape)
        print(f"step {s} tend {name}: max abs {d.max():.3e} at k,i,j={q} eng {a[q]:.6e} orc {b[q]:.6e} "
              f"scale {np.abs(b).max():.3e} kpbl {kpbl[0][q[1], q[2]]}", flush=True)
    for c in cs:
        c.bdyval()
    for name in ("ATM1_QC", "ATM2_QC", "ATM1_QV"):
        a, b = e.get(name), o.get(name)
        a = a[:, : rc.iy - 1, : rc.jx - 1]; b = b[:, : rc.iy - 1, : rc.jx - 1]
        d = np.abs(a - b)
        q = np.unravel_index(np.argmax(d), d.shape)
        print(f"step {s} state {name}: max abs {d.max():.3e} at {q} eng {a[q]:.6e} orc {b[q]:.6e} "
              f"neg eng {(a < 0).sum()} orc {(b < 0).sum()}", flush=True)
