"""Host-side fixed cost of one timed rcmdyn_step call (bench.py's timed region: step(K) then a
synchronize): wall time of K steps for several K after a settle phase, fitted as a + b*K.
    python tools/fixed_overhead.py [--config C3] [--reps 5]"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

import numpy as np  # noqa: E402

from regcm_amd import icbc  # noqa: E402
from regcm_amd.config import CONFIGS  # noqa: E402
from regcm_amd.dycore import DynCore  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C3")
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    rc = CONFIGS[args.config]
    data = icbc.generate(rc)
    eng = DynCore(rc, data["split"])
    eng.put_state(data["state"])
    eng.bdyval()
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.3:
        eng.step(16)
        eng.synchronize()
    ks, ts = [], []
    for _ in range(args.reps):
        for k in (2, 4, 8, 20, 50, 200):
            eng.synchronize()
            a = time.perf_counter()
            eng.step(k)
            eng.synchronize()
            ts.append(time.perf_counter() - a)
            ks.append(k)
    ks, ts = np.array(ks, float), np.array(ts)
    b, a = np.polyfit(ks, ts, 1)
    print(f"{args.config}: fixed {a * 1e6:.1f} us per call, {b * 1e3:.4f} ms per step; K=20 wall/step "
          f"{np.median(ts[ks == 20]) / 20 * 1e3:.4f} ms, K=200 {np.median(ts[ks == 200]) / 200 * 1e3:.4f} ms")
    for k in (2, 20, 200):
        print(f"  K={k}: median {np.median(ts[ks == k]) * 1e3:.3f} ms")


if __name__ == "__main__":
    main()
