"""Benchmark: simulated-years/wall-day of the RegCM4 hydrostatic dyn step on MI355X.

Contract (see task): `python bench.py --gpus N --steps K --warmup W`; for N>1 launched by
torch.distributed.run, one rank per GPU, RCCL halos between tiles.  Workload: BASELINE.json's
metric grid, 192x192x23 sigma (config C3: 50 km, dt = 150 s, hydrostatic, full
advection + diffusion + split-explicit, physics stubbed), synthetic ICBC (syn-icbc v1).
A step = one `tend` + one `bdyval` (Main/mod_regcm_interface.F90:189,208).
Scaling: strong (the 192x192x23 domain is split into set_nproc tiles across N GPUs).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from regcm_amd.config import CONFIGS, set_nproc  # noqa: E402
from regcm_amd import icbc  # noqa: E402

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E, /opt/skills/guides/MI355X_MICROARCH.md


def algorithmic_bytes_hydro(jx: int, iy: int, kz: int, nspgx: int = 12) -> float:
    """Compulsory HBM bytes of one hydrostatic step, SURVEY.md section 8(d):
    B_h = 8 [N3 (20 + 8 f_b) + N2 (19 + 2 f_b)]."""
    n3, n2 = jx * iy * kz, jx * iy
    fb = 1.0 - ((jx - 1 - 2 * nspgx) * (iy - 1 - 2 * nspgx)) / ((jx - 1) * (iy - 1))
    return 8.0 * (n3 * (20 + 8 * fb) + n2 * (19 + 2 * fb))


def cpu_baseline(rc, data, budget_s: float = 15.0):
    """Time the CPU restatement (oracle, 1 thread) on a bounded sample of the same workload."""
    from oracle.oracle import OracleCore
    o = OracleCore(rc, data["split"])
    o.put_state(data["state"])
    o.bdyval()
    o.step(1)
    n, t0 = 0, time.perf_counter()
    while True:
        o.step(1)
        n += 1
        el = time.perf_counter() - t0
        if el > budget_s or n >= 200:
            break
    t = el / n
    return {"value": rc.dt / (365.0 * t), "unit": "simulated-years/wall-day", "cores": 1,
            "kind": "port", "ms_per_step": t * 1e3,
            "sample": f"{rc.name}: {n} steps of tend+bdyval after 1 warm-up step, 1 host thread "
                      f"(oracle/rcm_oracle.c, gcc -O2)"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", default="C3")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=15.0)
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and world > 1:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    rc = CONFIGS[args.config]
    data = icbc.generate(rc)
    cj, ci = set_nproc(world, rc.jx, rc.iy)

    from regcm_amd.dycore import DynCore, comm_unique_id
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist
        dist.init_process_group(backend="gloo", init_method="env://")
        uid = bytearray(comm_unique_id()) if rank == 0 else bytearray(128)
        t = torch.tensor(list(uid), dtype=torch.uint8)
        dist.broadcast(t, src=0)
        uid = bytes(t.tolist())
        eng = DynCore(rc, data["split"], nproc_j=cj, nproc_i=ci, tile_first=rank, tile_count=1,
                      comm_rank=rank, comm_size=world, device=local_rank, unique_id=uid)
    else:
        eng = DynCore(rc, data["split"], device=local_rank)
    eng.put_state(data["state"])
    eng.bdyval()
    eng.step(args.warmup)

    def barrier():
        eng.synchronize()
        if dist is not None:
            dist.barrier()

    barrier()
    t0 = time.perf_counter()
    eng.step(args.steps)
    barrier()
    t1 = time.perf_counter()
    wall = t1 - t0
    dev_ms = eng.last_step_ms()
    if dist is not None:
        import torch
        tt = torch.tensor([wall], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        wall = float(tt.item())
    t_step = wall / args.steps
    sypd = rc.dt / (365.0 * t_step)
    bstep = algorithmic_bytes_hydro(rc.jx, rc.iy, rc.kz, rc.nspgx)
    achieved = bstep / t_step / 1e9
    if rank != 0:
        if dist is not None:
            dist.destroy_process_group()
        return
    line = {
        "metric": "simulated-years/wall-day, 192x192x23 sigma grid (hydrostatic dyn step)",
        "value": sypd,
        "unit": "simulated-years/wall-day",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": t_step * 1e3,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (syn-icbc v1, PCG64 seed 20261015): no DOMAIN/ICBC files offline",
        "config": {"workload": f"{args.config} {rc.jx}x{rc.iy}x{rc.kz} ds={rc.ds}km dt={rc.dt}s "
                               "hydrostatic, upstream adv + 4th-order diff + split-explicit "
                               "(nsplit=2) + iboudy=5 relaxation, physics stubbed",
                   "tiles": f"{cj}x{ci}", "step": "tend + bdyval"},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": None,
                     "kernel": "whole dyn step (hipGraph of ~30 kernels)",
                     "algorithmic_bytes": bstep},
        "device_ms_per_step": dev_ms,
    }
    if not args.no_cpu_baseline and world == 1:
        line["cpu_baseline"] = cpu_baseline(rc, data, args.cpu_budget)
    print(json.dumps(line))
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
