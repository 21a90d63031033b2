"""The nqx = 5 step (physicsparam ipptls = 2: qi, qr, qs through qc's chain) against the
nqx = 2 step on the same grid: ms/step of graph-replayed steps after a settle phase, and the
per-kernel times (HIP events, eager steps) of each.  The hydrometeor fields are
icbc.hydrometeor_state's patchy synthetic fields (their negative forecasts exercise the
species' serial fix, k_qx_serial).
    python tools/species_bench.py [--config C3] [--steps 200]"""
import argparse
import dataclasses
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

from regcm_amd import icbc  # noqa: E402
from regcm_amd.config import CONFIGS  # noqa: E402
from regcm_amd.dycore import DynCore  # noqa: E402


def run(rc, data, state, steps):
    eng = DynCore(rc, data["split"])
    eng.put_state(state)
    eng.bdyval()
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.1:          # settle (bench.py's clock ramp)
        eng.step(16)
        eng.synchronize()
    eng.step(10)
    eng.synchronize()
    t0 = time.perf_counter()
    eng.step(steps)
    eng.synchronize()
    ms = (time.perf_counter() - t0) / steps * 1e3
    kt = eng.kernel_times(5)
    return ms, kt


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C3")
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--reps", type=int, default=2)
    args = ap.parse_args()
    rc2 = CONFIGS[args.config]
    rc5 = dataclasses.replace(rc2, ipptls=2)
    data = icbc.generate(rc2)
    st5 = {k: v.copy() for k, v in data["state"].items()}
    st5.update(icbc.hydrometeor_state(rc5, st5, nqx=rc5.nqx))
    for rep in range(args.reps):
        for name, rc, st in (("nqx=2", rc2, data["state"]), ("nqx=5", rc5, st5)):
            ms, kt = run(rc, data, st, args.steps)
            tot = sum(v[0] / 5 * v[1] for v in kt.values()) * 1e3
            print(f"== {args.config} {name} rep {rep}: {ms:.4f} ms/step  (eager kernel sum {tot:.1f} us/step)",
                  flush=True)
            for k, v in sorted(kt.items(), key=lambda kv: -kv[1][0] * kv[1][1])[:14]:
                print(f"  {k:34s} {v[0] / 5:5.1f}/step {v[1] * 1e3:9.2f} us", flush=True)


if __name__ == "__main__":
    main()
