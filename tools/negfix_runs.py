"""Structure of the serial negative-moisture fix's work on a configuration (oracle, CPU): per
(species, level) plane the rows holding a dependent negative point (a negative point with a
negative sweep-predecessor, Main/mod_tendency.F90:382-393) and the longest run of consecutive
such rows, which bounds a wavefront restricted to the runs (W + 2 (run - 1) steps, against
W + 2 (R - 1) for the whole plane).
    python tools/negfix_runs.py [--config C3] [--ipptls 2] [--steps 2]"""
import argparse
import dataclasses
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

import numpy as np  # noqa: E402

from oracle.oracle import OracleCore  # noqa: E402
from regcm_amd import icbc  # noqa: E402
from regcm_amd.config import CONFIGS  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C3")
    ap.add_argument("--ipptls", type=int, default=2)
    ap.add_argument("--steps", type=int, default=2)
    a = ap.parse_args()
    rc = dataclasses.replace(CONFIGS[a.config], ipptls=a.ipptls)
    data = icbc.generate(CONFIGS[a.config])
    st = {k: v.copy() for k, v in data["state"].items()}
    if rc.nqx > 2:
        st.update(icbc.hydrometeor_state(rc, st, nqx=rc.nqx))
    o = OracleCore(rc, data["split"])
    o.put_state(st)
    o.bdyval()
    o.step(a.steps - 1)
    dt = o.get_time()[1]
    a2 = {n: o.get("ATM2_" + n) for n in ("QI", "QR", "QS")}
    o.step(1)
    # the species' forecasts before the fix (the oracle fixes them in place): atm2 + dt * qten,
    # the same operations as its forecast
    for nm, s in (("cqi", "QI"), ("cqr", "QR"), ("cqs", "QS")):
        q = (a2[s] + dt * o.get_work("qten" + s[1].lower()))[:, 1: rc.iy - 2, 1: rc.jx - 2]
        neg = q < 0
        pn = np.zeros_like(neg)
        pn[:, :, 1:] |= neg[:, :, :-1]                 # (j-1, i)
        pn[:, 1:, 1:] |= neg[:, :-1, :-1]              # (j-1, i-1)
        pn[:, 1:, :] |= neg[:, :-1, :]                 # (j, i-1)
        pn[:, 1:, :-1] |= neg[:, :-1, 1:]              # (j+1, i-1)
        dep = neg & pn
        rows = dep.any(axis=2)                         # [k, i]
        runs = []
        for k in range(rows.shape[0]):
            best = cur = 0
            for r in rows[k]:
                cur = cur + 1 if r else 0
                best = max(best, cur)
            runs.append(best)
        print(f"{nm}: negative {neg.mean():.3f}, dependent {dep.mean():.4f} of the points; marked rows per plane "
              f"max {rows.sum(axis=1).max()} of {rows.shape[1]}; longest run per plane max {max(runs)}, "
              f"median {int(np.median(runs))}; planes with > 16 marked rows {(rows.sum(axis=1) > 16).sum()} of {rows.shape[0]}",
              flush=True)


if __name__ == "__main__":
    main()
