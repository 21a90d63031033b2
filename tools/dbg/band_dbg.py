"""Debug helper: one tend of a band engine vs the oracle, per-field max difference and where."""
import dataclasses, sys
import numpy as np
from regcm_amd.config import CONFIGS, STATE_FIELDS
from regcm_amd import icbc
from regcm_amd.dycore import DynCore
from oracle.oracle import OracleCore
var = eval(sys.argv[1]) if len(sys.argv) > 1 else {}
nproc = eval(sys.argv[2]) if len(sys.argv) > 2 else (1, 1)
rc = dataclasses.replace(CONFIGS["C1"], i_band=1, **var)
data = icbc.generate(rc)
st = dict(data["state"])
o = OracleCore(rc, data["split"]); o.put_state(st); o.bdyval()
e = DynCore(rc, data["split"], nproc_j=nproc[0], nproc_i=nproc[1]); e.put_state(st); e.bdyval()
e.set_diagnostics(True)
o.tend(); e.tend()
for name in ["PSC", "PTEN", "QDOT", "PSDOTA", "XKC", "OMEGA", "TTEN", "QVTEN", "QCTEN", "UTEN", "VTEN", "PHI"] + list(STATE_FIELDS):
    try:
        a, b = e.get(name), o.get(name)
    except Exception as ex:
        print(name, "ERR", ex); continue
    a = a[:, : rc.iy - 1, :] if a.shape[1] == rc.iy else a
    b = b[:, : rc.iy - 1, :] if b.shape[1] == rc.iy else b
    d = np.abs(a - b)
    d[np.isnan(d)] = np.inf
    if d.max() == 0:
        print(name, "exact"); continue
    k, i, j = np.unravel_index(np.argmax(d), d.shape)
    bad = np.argwhere(d > 1e-12 * max(np.nanmax(np.abs(b)), 1e-300))
    js = sorted(set(bad[:, 2].tolist()))
    is_ = sorted(set(bad[:, 1].tolist()))
    print(f"{name} max {d.max():.3e} at k={k} i={i+1} j={j+1} e={a[k,i,j]} o={b[k,i,j]} nbad={len(bad)} j:{[x+1 for x in js[:12]]} i:{[x+1 for x in is_[:12]]}")
