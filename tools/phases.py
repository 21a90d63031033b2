"""Block phase timing of the hydrostatic kernels (library built with -DRCM_PHASE_TIMING, see
devcommon.hpp): per kernel, the span of one launch (first block start to last block end), the
median block lifetime and the median duration of each phase between PT_MARK points.

    make -C regcm_amd/csrc HIPFLAGS="... -DRCM_PHASE_TIMING"   (then rebuild without it)
    python tools/phases.py [--config C3] [--nproc 1x1]
"""
import argparse
import ctypes
import os
import statistics as S
import sys
import tempfile

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

from regcm_amd import icbc  # noqa: E402
from regcm_amd.config import CONFIGS  # noqa: E402
from regcm_amd.dycore import DynCore, lib  # noqa: E402

NAMES = {1: "k_columns", 2: "k_momentum", 3: "k_scalars", 4: "k_qfilter", 5: "k_split_project",
         6: "split_corr bdy", 7: "split_corr cor"}
REC = np.dtype([("kid", "i4"), ("bx", "i4"), ("by", "i4"), ("bz", "i4"), ("n", "i4"), ("pad", "i4"),
                ("t", "i8", (8,))])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C3")
    ap.add_argument("--nproc", default="1x1")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--shape", default="", help="JXxIY: the config on a domain of that size (rank-tile studies)")
    args = ap.parse_args()
    rc = CONFIGS[args.config]
    if args.shape:
        import dataclasses
        jx, iy = (int(x) for x in args.shape.split("x"))
        rc = dataclasses.replace(rc, jx=jx, iy=iy)
    data = icbc.generate(rc)
    pj, pi = (int(x) for x in args.nproc.split("x"))
    e = DynCore(rc, data["split"], nproc_j=pj, nproc_i=pi)
    e.put_state(data["state"])
    e.bdyval()
    e.step(3)
    e.synchronize()
    dump = lib().rcm_phase_dump
    dump.argtypes = [ctypes.c_char_p]
    path = os.path.join(tempfile.gettempdir(), "rcm_phases.bin")
    dump(path.encode())                      # reset
    e.step(args.steps)
    e.synchronize()
    n = dump(path.encode())
    recs = np.fromfile(path, dtype=REC, count=n)
    for kid, name in NAMES.items():
        r = recs[recs["kid"] == kid]
        if not len(r):
            continue
        t0 = r["t"][:, 0]
        order = np.argsort(t0)
        r = r[order]
        # launches: a start gap of more than 20 us separates them
        starts = r["t"][:, 0]
        cut = np.where(np.diff(starts) > 2000)[0] + 1
        groups = np.split(np.arange(len(r)), cut)
        spans, lifes, phases = [], [], []
        for gi in groups:
            rr = r[gi]
            ends = np.array([x["t"][x["n"] - 1] for x in rr])
            spans.append((ends.max() - rr["t"][:, 0].min()) / 100.0)
            lifes.extend(((ends - rr["t"][:, 0]) / 100.0).tolist())
            for x in rr:
                phases.append(np.diff(x["t"][: x["n"]]) / 100.0)
        nph = min(len(p) for p in phases)
        pm = [round(S.median(p[q] for p in phases), 2) for q in range(nph)]
        print(f"{name:16s} launches {len(groups):3d} blocks/launch {len(r) // len(groups):6d} span median "
              f"{S.median(spans):7.2f} us  block life median {S.median(lifes):6.2f} max {max(lifes):6.2f} us  "
              f"phases {pm}")


if __name__ == "__main__":
    main()
