"""Sustained throughput of the graph-replayed step: ms/step of consecutive chunks of K steps
over several seconds (does the rate hold under a long run?).
    python tools/sustained.py [--config C3] [--seconds 4] [--chunk 200]"""
import argparse
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
    ap.add_argument("--seconds", type=float, default=4.0)
    ap.add_argument("--chunk", type=int, default=200)
    ap.add_argument("--sync-every", type=int, default=1, help="synchronize after every n chunks")
    args = ap.parse_args()
    rc = CONFIGS[args.config]
    data = icbc.generate_nh(rc) if rc.idynamic == 2 else icbc.generate(rc)
    eng = DynCore(rc, data["split"])
    eng.put_state(data["state"])
    eng.bdyval()
    t0 = time.perf_counter()
    n = 0
    while time.perf_counter() - t0 < args.seconds:
        a = time.perf_counter()
        eng.step(args.chunk)
        eng.synchronize()
        b = time.perf_counter()
        n += 1
        print(f"t={b - t0:7.3f} s chunk {n:4d}: {(b - a) / args.chunk * 1e3:.4f} ms/step (device {eng.last_step_ms():.4f})",
              flush=True)


if __name__ == "__main__":
    main()
