"""Per-step device time of the hydrostatic step on a small single-tile domain (the size of one
rank's tile when the driver's scaling runs split C3 over 2/4/8 GPUs): the kernel-latency floor
of a rank's step before any exchange.  python tools/small_tile.py"""
import dataclasses
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

from regcm_amd import icbc  # noqa: E402
from regcm_amd.config import CONFIGS  # noqa: E402
from regcm_amd.dycore import DynCore  # noqa: E402

for jx, iy in ((192, 192), (96, 192), (96, 96), (96, 48)):
    rc = dataclasses.replace(CONFIGS["C3"], jx=jx, iy=iy)
    data = icbc.generate(rc)
    e = DynCore(rc, data["split"])
    e.put_state(data["state"])
    e.bdyval()
    e.step(20)
    e.synchronize()
    t0 = time.perf_counter()
    e.step(200)
    e.synchronize()
    dt = (time.perf_counter() - t0) / 200
    print(f"C3 physics on {jx}x{iy}x{rc.kz}: {dt * 1e3:.4f} ms/step", flush=True)

# per-kernel times (eager, HIP events per launch) on the smallest tile
rc = dataclasses.replace(CONFIGS["C3"], jx=96, iy=48)
data = icbc.generate(rc)
e = DynCore(rc, data["split"])
e.put_state(data["state"])
e.bdyval()
e.step(4)
kt = e.kernel_times(5)
for name, (n, us) in sorted(kt.items(), key=lambda kv: -kv[1][1] * kv[1][0]):
    print(f"  {name:32s} {n / 5:4.1f}/step {us * 1e3:8.2f} us")
