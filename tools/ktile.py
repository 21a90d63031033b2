"""Per-kernel device times (HIP events per launch, eager steps) of the hydrostatic step on the
scaling runs' rank-tile sizes and C3, for timing-only variant builds too (a few steps, results
unchecked).  python tools/ktile.py [--steps 3]"""
import dataclasses
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

from regcm_amd import icbc  # noqa: E402
from regcm_amd.config import CONFIGS  # noqa: E402
from regcm_amd.dycore import DynCore  # noqa: E402

steps = int(sys.argv[sys.argv.index("--steps") + 1]) if "--steps" in sys.argv else 3
for jx, iy in ((96, 48), (192, 192)):
    rc = dataclasses.replace(CONFIGS["C3"], jx=jx, iy=iy)
    data = icbc.generate(rc)
    e = DynCore(rc, data["split"])
    e.put_state(data["state"])
    e.bdyval()
    kt = e.kernel_times(steps)
    tot = sum(n / steps * us for n, us in kt.values())
    print(f"{jx}x{iy}: kernel sum {tot * 1e3:.2f} us/step " +
          " ".join(f"{name.split('(')[0]}={us * 1e3:.2f}" for name, (n, us) in sorted(kt.items(), key=lambda kv: -kv[1][1])),
          flush=True)
