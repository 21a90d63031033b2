"""Per-kernel device times of one configuration (HIP events around every launch, eager
steps) plus the graph-replayed ms/step: the quick loop for kernel work.

    python tools/ktimes.py [--config C3] [--steps 50] [--prof-steps 5]
"""
import argparse
import dataclasses
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

from regcm_amd import icbc  # noqa: E402
from regcm_amd.config import CONFIGS  # noqa: E402
from regcm_amd.dycore import DynCore  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C3")
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--prof-steps", type=int, default=5)
    ap.add_argument("--nproc", default="1x1", help="local tiles jxi (all on this GPU)")
    ap.add_argument("--ipptls", type=int, default=1, help="2: nqx = 5 (qi, qr, qs with icbc.hydrometeor_state)")
    args = ap.parse_args()
    rc = dataclasses.replace(CONFIGS[args.config], ipptls=args.ipptls)
    data = icbc.generate_nh(rc) if rc.idynamic == 2 else icbc.generate(rc)
    st = dict(data["state"])
    if args.ipptls == 2:
        st.update(icbc.hydrometeor_state(rc, st, nqx=rc.nqx))
    pj, pi = (int(x) for x in args.nproc.split("x"))
    e = DynCore(rc, data["split"], nproc_j=pj, nproc_i=pi)
    e.put_state(st)
    e.bdyval()
    e.step(5)
    e.synchronize()
    t0 = time.perf_counter()
    e.step(args.steps)
    e.synchronize()
    ms = (time.perf_counter() - t0) / args.steps * 1e3
    kt = e.kernel_times(args.prof_steps)
    tot = 0.0
    for name, (n, avg) in sorted(kt.items(), key=lambda kv: -kv[1][0] * kv[1][1]):
        per = n / args.prof_steps * avg * 1e3
        tot += per
        print(f"{name:28s} launches/step {n / args.prof_steps:6.2f}  avg {avg * 1e3:9.2f} us  per step {per:9.2f} us")
    print(f"{args.config} ipptls={args.ipptls} tiles {args.nproc}: graph-replayed {ms:.4f} ms/step; eager kernel sum {tot / 1e3:.4f} ms/step")


if __name__ == "__main__":
    main()
