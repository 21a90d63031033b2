"""Per-kernel times (us) of the C3 step at several points of a long run (the synthetic case
drifts after ~3000 steps): python tools/late_kt.py"""
import os, sys
sys.path.insert(0, os.getcwd())
from regcm_amd import icbc
from regcm_amd.config import CONFIGS
from regcm_amd.dycore import DynCore
rc = CONFIGS["C3"]; data = icbc.generate(rc)
e = DynCore(rc, data["split"]); e.put_state(data["state"]); e.bdyval()
for n in (0, 2000, 3800, 4400):
    while e.get_time()[0] < n:
        e.step(100); e.synchronize()
    kt = e.kernel_times(3)
    print("step", e.get_time()[0], {k: round(v[1] * 1e3, 1) for k, v in sorted(kt.items(), key=lambda kv: -kv[1][1])[:8]}, flush=True)
