"""Debug aid: where a decomposed nqx = 5 run departs from one tile (per field, per step)."""
import dataclasses
import sys

import numpy as np

sys.path.insert(0, ".")
from regcm_amd import icbc  # noqa: E402
from regcm_amd.config import CONFIGS, QX_STATE_FIELDS, STATE_FIELDS  # noqa: E402
from regcm_amd.dycore import DynCore  # noqa: E402

ipptls = int(sys.argv[1]) if len(sys.argv) > 1 else 2
nproc = tuple(int(x) for x in sys.argv[2].split("x")) if len(sys.argv) > 2 else (2, 1)
rc = dataclasses.replace(CONFIGS["C1"], ipptls=ipptls)
data = icbc.generate(rc)
st = {k: v.copy() for k, v in data["state"].items()}
st.update(icbc.hydrometeor_state(rc, st, nqx=rc.nqx))
names = list(STATE_FIELDS) + (QX_STATE_FIELDS if rc.nqx == 5 else [])
a = DynCore(rc, data["split"])
b = DynCore(rc, data["split"], nproc_j=nproc[0], nproc_i=nproc[1])
for e in (a, b):
    e.put_state(st)
    e.bdyval()
for n in names:
    x, y = a.get(n), b.get(n)
    if not np.array_equal(x, y):
        idx = np.argwhere(x != y)
        print("after bdyval", n, len(idx), idx[:3].tolist())
for s in range(3):
    for e in (a, b):
        e.tend()
    for n in names:
        x, y = a.get(n), b.get(n)
        if not np.array_equal(x, y):
            idx = np.argwhere(x != y)
            print("step", s + 1, "tend", n, len(idx), idx[:4].tolist(), float(np.max(np.abs(x - y))))
    for e in (a, b):
        e.bdyval()
    for n in names:
        x, y = a.get(n), b.get(n)
        if not np.array_equal(x, y):
            idx = np.argwhere(x != y)
            print("step", s + 1, "bdyval", n, len(idx), idx[:4].tolist())
