"""Thread-count sweep of the CPU baseline (the oracle as set_nproc tiles on OpenMP threads,
oracle/orc_par.c) on the host the bench runs on: where does the restatement saturate?

    python tools/cpu_sweep.py --config C3 --threads 1,2,4,8,16,32,64,128,256 --budget 4

One JSON line per thread count (ms per step of tend + bdyval, SYPD), then a summary line with the
fastest count.  Thread counts above the CPUs this process may use are skipped.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from regcm_amd.config import CONFIGS, set_nproc  # noqa: E402
from regcm_amd import icbc  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C3")
    ap.add_argument("--threads", default="1,2,4,8,16,32,64,128,256")
    ap.add_argument("--budget", type=float, default=4.0, help="seconds of timed steps per count")
    ap.add_argument("--max-steps", type=int, default=50)
    args = ap.parse_args()
    from oracle.oracle import OracleCore, OracleParallel
    rc = CONFIGS[args.config]
    data = icbc.generate_nh(rc) if rc.idynamic == 2 else icbc.generate(rc)
    aff = len(os.sched_getaffinity(0))
    best = None
    for n in [int(x) for x in args.threads.split(",")]:
        if n > aff:
            continue
        cj, ci = set_nproc(n, rc.jx, rc.iy)
        o = OracleCore(rc, data["split"]) if n == 1 else OracleParallel(rc, data["split"], n)
        o.put_state(data["state"])
        o.bdyval()
        o.step(1)                                   # warm-up (first touch, the dt switch)
        steps, t0 = 0, time.perf_counter()
        while True:
            o.step(1)
            steps += 1
            el = time.perf_counter() - t0
            if el > args.budget or steps >= args.max_steps:
                break
        ms = el / steps * 1e3
        rec = {"config": args.config, "threads": n, "tiles": f"{cj}x{ci}", "steps": steps, "ms_per_step": ms,
               "sypd": rc.dt / (365.0 * ms * 1e-3), "affinity_cpus": aff, "nproc": os.cpu_count()}
        print(json.dumps(rec), flush=True)
        if best is None or ms < best["ms_per_step"]:
            best = rec
        if hasattr(o, "close"):
            o.close()
        del o
    print(json.dumps({"best": best}), flush=True)


if __name__ == "__main__":
    main()
