"""Generate tests/golden/c1_oracle.json: fingerprints of the syn-icbc v1 inputs and of the CPU
restatement's state after 1, 10 and 40 steps of tend+bdyval on configuration C1.

Provenance: the reference ships no golden vectors and cannot be executed here (Fortran that
needs netCDF-Fortran, absent from the image), so these fixtures pin the oracle and the engine
against regressions of THIS restatement; they are not reference outputs ("parity unpinned").
Run:  python tests/golden/make_golden.py
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from regcm_amd.config import CONFIGS, STATE_FIELDS  # noqa: E402
from regcm_amd import icbc  # noqa: E402

SAMPLE_SEED = 7


def fingerprint(a: np.ndarray, rng_seed=SAMPLE_SEED, nsample=48):
    a = np.ascontiguousarray(a, dtype=np.float64)
    rng = np.random.Generator(np.random.PCG64(rng_seed))
    idx = rng.integers(0, a.size, nsample)
    flat = a.ravel()
    return {
        "shape": list(a.shape),
        "sum": float(np.sum(flat)),
        "abssum": float(np.sum(np.abs(flat))),
        "max": float(np.max(flat)),
        "min": float(np.min(flat)),
        "samples_idx": [int(x) for x in idx],
        "samples": [float(flat[x]).hex() for x in idx],
    }


def main():
    from oracle.oracle import OracleCore
    rc = CONFIGS["C1"]
    data = icbc.generate(rc)
    out = {"config": "C1", "generator": "syn-icbc v1", "inputs": {}, "split": {}, "steps": {}}
    for name, arr in sorted(data["state"].items()):
        out["inputs"][name] = fingerprint(arr)
    for key in ("hbar", "an", "aam", "dtau"):
        out["split"][key] = [float(x).hex() for x in np.ravel(data["split"][key])]
    o = OracleCore(rc, data["split"])
    o.put_state(data["state"])
    o.bdyval()
    done = 0
    for n in (1, 10, 40):
        o.step(n - done)
        done = n
        out["steps"][str(n)] = {name: fingerprint(o.get(name)) for name in STATE_FIELDS}
        out["steps"][str(n)]["_time"] = list(o.get_time())
        out["steps"][str(n)]["_diag"] = [float(x).hex() for x in o.diagnostics()[:2]]
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "c1_oracle.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=0)
    print("wrote", path)


if __name__ == "__main__":
    main()
