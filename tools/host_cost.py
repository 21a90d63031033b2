"""Host cost of the eager step path (the path N>1 RCCL runs take, which are not graph-replayed):
rcmdyn_step wall time eager (RCMDYN_NO_GRAPH) against graph replay, for one tile and for local tilings.

    python tools/host_cost.py [--config C3] [--steps 50]
"""
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
    ap.add_argument("--steps", type=int, default=50)
    args = ap.parse_args()
    rc = CONFIGS[args.config]
    data = icbc.generate_nh(rc) if rc.idynamic == 2 else icbc.generate(rc)
    for nproc in ((1, 1), (2, 1), (2, 2), (2, 4)):
        res = []
        for eager in (False, True):
            if eager:
                os.environ["RCMDYN_NO_GRAPH"] = "1"
            else:
                os.environ.pop("RCMDYN_NO_GRAPH", None)
            e = DynCore(rc, data["split"], nproc_j=nproc[0], nproc_i=nproc[1])
            e.put_state(data["state"])
            e.bdyval()
            e.step(4)
            e.synchronize()
            t0 = time.perf_counter()
            e.step(args.steps)
            e.synchronize()
            res.append((time.perf_counter() - t0) / args.steps * 1e3)
            e.close()
        print(f"{args.config} tiles {nproc[0]}x{nproc[1]}: graph {res[0]:.4f} ms/step, eager step {res[1]:.4f} ms/step",
              flush=True)

if __name__ == "__main__":
    main()
