"""Per-step device time of the hydrostatic step on a small single-tile domain (the size of one
rank's tile when the driver's scaling runs split C3 over 2/4/8 GPUs): the kernel-latency floor
of a rank's step before any exchange; then, per rank count, the share of each update kernel
that runs beside the prologue exchange (rcmdyn_overlap_shares, host-only: `--shares` prints
only that and needs no GPU).  python tools/small_tile.py [--shares]"""
import dataclasses
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

from regcm_amd import icbc  # noqa: E402
from regcm_amd.config import CONFIGS  # noqa: E402
from regcm_amd.config import set_nproc  # noqa: E402
from regcm_amd.dycore import DynCore, overlap_shares  # noqa: E402


def shares():
    rc = CONFIGS["C3"]
    data = icbc.generate(rc)
    print("part 1 (beside the prologue exchange), share of each kernel's points over all ranks:")
    for n in (2, 4, 8):
        cj, ci = set_nproc(n, rc.jx, rc.iy)
        sh = overlap_shares(rc, data["split"], cj, ci)
        tot = [sum(x[q] for x in sh) for q in range(6)]
        print(f"  {n} ranks ({cj}x{ci} tiles of {rc.jx // cj}x{rc.iy // ci}): k_columns {tot[0] / tot[1]:.0%}, "
              f"k_momentum {tot[2] / tot[3]:.0%}, k_scalars {tot[4] / tot[5]:.0%}", flush=True)


if "--shares" in sys.argv:
    shares()
    sys.exit(0)

if "--nh" in sys.argv:
    # the non-hydrostatic C5 domain (768x768x41, 3 km) on the 8-GPU tiling (2x4): each rank's
    # 384x192x41 tile as one single-tile run, its step without any exchange (the floor the
    # 8-GPU C5 run sees per rank), then its per-kernel times
    rc = dataclasses.replace(CONFIGS["C5"], jx=384, iy=192)
    data = icbc.generate_nh(rc)
    e = DynCore(rc, data["split"])
    e.put_state(data["state"])
    e.bdyval()
    e.step(6)
    e.synchronize()
    t0 = time.perf_counter()
    e.step(40)
    e.synchronize()
    dt = (time.perf_counter() - t0) / 40
    print(f"C5 physics on 384x192x{rc.kz} (the 8-GPU rank tile): {dt * 1e3:.3f} ms/step", flush=True)
    kt = e.kernel_times(3)
    for name, (n, us) in sorted(kt.items(), key=lambda kv: -kv[1][1] * kv[1][0]):
        print(f"  {name:32s} {n / 3:4.1f}/step {us * 1e3:9.2f} us")
    sys.exit(0)

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

if "--no-shares" not in sys.argv:
    shares()
