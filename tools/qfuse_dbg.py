"""qfuse vs k_qfilter divergence locator (C1, negative qv rows): after each step, the fields
that differ and the first differing point."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np  # noqa: E402
from regcm_amd import icbc  # noqa: E402
from regcm_amd.config import CONFIGS, STATE_FIELDS  # noqa: E402
from regcm_amd.dycore import DynCore  # noqa: E402

rc = CONFIGS["C1"]
data = icbc.generate(rc)
st = {k: v.copy() for k, v in data["state"].items()}
st["ATM1_QV"][5:8, 10:14, 10:30] = -1e-7 * st["PSA"][0][10:14, 10:30]
st["ATM2_QV"][5:8, 10:14, 10:30] = -2e-7 * st["PSA"][0][10:14, 10:30]
os.environ["RCMDYN_NO_GRAPH"] = "1"
a = DynCore(rc, data["split"])
os.environ["RCMDYN_NO_QFUSE"] = "1"
b = DynCore(rc, data["split"])
for e in (a, b):
    e.put_state(st)
    e.bdyval()
for s in range(3):
    for e in (a, b):
        e.tend()
    for n in STATE_FIELDS:
        x, y = a.get(n), b.get(n)
        if not np.array_equal(x, y):
            d = np.argwhere(x != y)
            print(f"step {s} after tend: {n} differs at {len(d)} points, first {tuple(d[0])} "
                  f"{x[tuple(d[0])]:.17g} vs {y[tuple(d[0])]:.17g}", flush=True)
    for e in (a, b):
        e.bdyval()
print("done")
