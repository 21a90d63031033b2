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
from regcm_amd.traffic import kernel_bytes, step_bytes, step_bytes_nh  # noqa: E402

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E, /opt/skills/guides/MI355X_MICROARCH.md
PMC_FILE = os.path.join(ROOT, "profiles", "pmc_traffic.json")


def kernels_digest() -> str:
    import hashlib
    h = hashlib.sha256()
    src = os.path.join(ROOT, "regcm_amd", "csrc")
    for f in sorted(os.listdir(src)):
        if f.endswith((".hip", ".hpp")) or f == "Makefile":     # sources and their compile flags
            with open(os.path.join(src, f), "rb") as fh:
                h.update(fh.read())
    return h.hexdigest()[:16]


def pmc_traffic(kernel: str, config: str):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC summary
    (tools/pmc_summary.py), only if it was measured on this exact kernel source."""
    pmc_file = PMC_FILE if config == "C3" else os.path.join(ROOT, "profiles", f"pmc_traffic_{config}.json")
    try:
        with open(pmc_file) as fh:
            d = json.load(fh)
    except (OSError, ValueError):
        return None, None
    if d.get("digest") != kernels_digest() or d.get("config") != config:
        return None, None
    ks = d.get("kernels", {})
    k = ks.get(kernel) or ks.get("void " + kernel)     # rocprofv3 names templates "void name<...>"
    if not k:
        return None, None
    return k["hbm_bytes_per_launch"], d.get("source")


def _cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _time_steps(o, budget_s):
    o.step(1)                                   # warm-up (the leapfrog dt switch)
    n, t0 = 0, time.perf_counter()
    while True:
        o.step(1)
        n += 1
        el = time.perf_counter() - t0
        if el > budget_s or n >= 200:
            return el / n, n


def cpu_quota() -> int:
    """CPUs' worth of time the cgroup grants this process (cgroup v2 cpu.max, v1 cfs quota);
    0 if unlimited or unknown."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as fh:
            q, per = fh.read().split()[:2]
        return 0 if q == "max" else max(1, int(int(q) // int(per)))
    except (OSError, ValueError):
        pass
    try:
        with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as fh:
            q = int(fh.read())
        with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as fh:
            per = int(fh.read())
        return 0 if q <= 0 else max(1, q // per)
    except (OSError, ValueError):
        return 0


def cpu_baseline(rc, data, budget_s: float = 15.0, threads: int = 0):
    """Time the CPU restatement on a bounded sample of the same workload: on every host CPU this
    process is granted (SURVEY 8(d) / BASELINE.md: set_nproc tiles on OpenMP threads,
    oracle/orc_par.c, bit-identical to one tile, both cores) -- the CPUs it may run on, capped
    by the cgroup's CPU quota: the sweep of profiles/r03/cpu_sweep_c3.jsonl on the GPU box (256
    CPUs visible, a 16-CPU quota) peaks at 16 threads and collapses beyond (28 ms/step at 32,
    1.7 s at 256) -- unless `threads` names a count; the hydrostatic core also on one thread as
    a secondary figure."""
    from oracle.oracle import OracleCore, OracleParallel
    nproc = os.cpu_count() or 1
    try:
        affinity = len(os.sched_getaffinity(0))
    except AttributeError:
        affinity = nproc
    quota = cpu_quota()
    granted = min(affinity, quota) if quota else affinity
    threads = max(1, min(threads or granted, affinity))

    def setup(o):
        o.put_state(data["state"])
        o.bdyval()
        return o

    res = {"unit": "simulated-years/wall-day", "kind": "port", "nproc": nproc, "affinity_cpus": affinity,
           "cgroup_cpu_quota": quota or None, "cpu_model": _cpu_model()}
    if threads > 1:
        o = setup(OracleParallel(rc, data["split"], threads))
        t, n = _time_steps(o, budget_s * (0.65 if rc.idynamic == 1 else 1.0))
        o.close()
        res.update({"value": rc.dt / (365.0 * t), "cores": o.nthreads, "ms_per_step": t * 1e3,
                    "sample": f"{rc.name}: {n} steps of tend+bdyval after 1 warm-up step, "
                              f"{o.nthreads} set_nproc tiles on {o.nthreads} OpenMP threads (oracle/orc_par.c over "
                              f"oracle/rcm_oracle.c, gcc -O2)"})
        if rc.idynamic == 1:
            t1, n1 = _time_steps(setup(OracleCore(rc, data["split"])), budget_s * 0.35)
            res["single_thread"] = {"value": rc.dt / (365.0 * t1), "ms_per_step": t1 * 1e3, "steps": n1}
            res["sample"] += f"; single_thread: {n1} steps on 1 thread"
    else:
        t, n = _time_steps(setup(OracleCore(rc, data["split"])), budget_s)
        res.update({"value": rc.dt / (365.0 * t), "cores": 1, "ms_per_step": t * 1e3,
                    "sample": f"{rc.name}: {n} steps of tend+bdyval after 1 warm-up step, 1 host thread "
                              "(oracle/rcm_oracle.c, gcc -O2)"})
    if (rc.jx, rc.iy, rc.kz, rc.idynamic) == (192, 192, 23, 1):
        # the only timing of the reference itself (the
        # reference's own build, physics stubbed, 1 core of the survey container): the port is
        # the stronger baseline, so the GPU/CPU ratio here understates the gain over the reference
        res["sample"] += ("; note: this port runs the C3 step about 4-5x faster per core than the "
                          "survey-timed reference build (923 ms/step on 1 core, 103 ms/step on 8 MPI ranks)")
        res["reference_build_ms_per_step_1core"] = 923.0
    return res


def settle(eng, seconds: float, bcast=None):
    """Untimed steps until `seconds` of wall time have passed on rank 0 (chunks doubling up to
    64 steps; with more than one rank, bcast(int) -> int returns rank 0's decision, so every
    rank runs the same steps).  Returns (steps, seconds).  From an idle GPU the first tens of
    milliseconds of work run below the steady clock, which a timed window of K = 20 C3 steps
    (4 ms) would otherwise measure."""
    if seconds <= 0:
        return 0, 0.0
    n, chunk, t0 = 0, 1, time.perf_counter()
    while True:
        eng.step(chunk)
        eng.synchronize()
        n += chunk
        done = time.perf_counter() - t0 >= seconds
        if bcast is not None:
            done = bool(bcast(1 if done else 0))
        if done:
            return n, time.perf_counter() - t0
        chunk = min(2 * chunk, 64)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", default="C3")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=15.0)
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="host threads of the CPU baseline (0: every CPU this process is granted)")
    ap.add_argument("--prof-steps", type=int, default=5,
                    help="eager steps timed per kernel with HIP events (dominant-kernel roofline)")
    ap.add_argument("--settle-ms", type=float, default=100.0,
                    help="untimed steps run for this long before the warm-up (GPU clock ramp); 0: none")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and world > 1:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    rc = CONFIGS[args.config]
    nh = rc.idynamic == 2
    data = icbc.generate_nh(rc) if nh else icbc.generate(rc)
    cj, ci = set_nproc(world, rc.jx, rc.iy)

    from regcm_amd.dycore import DynCore, comm_unique_id, runtime_info
    # the engine library (and with it /opt/rocm's librccl.so.1) is loaded before torch, so a
    # multi-rank job binds that RCCL and not the copy torch bundles under the same soname
    # (INTEGRATION.md); every rank reports what it bound
    rt = runtime_info()
    print(f"[bench rank {rank}/{world}] runtime: {rt}", file=sys.stderr, flush=True)
    dist = None
    rts = [rt]
    if world > 1:
        import torch
        import torch.distributed as dist
        dist.init_process_group(backend="gloo", init_method="env://")
        rts = [None] * world
        dist.all_gather_object(rts, rt)
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

    def barrier():
        eng.synchronize()
        if dist is not None:
            dist.barrier()

    bcast = None
    if dist is not None:
        def bcast(v):
            t = torch.tensor([v], dtype=torch.int32)
            dist.broadcast(t, src=0)
            return int(t.item())
    settle_steps, settle_s = settle(eng, args.settle_ms * 1e-3, bcast)
    eng.step(args.warmup)
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
    # the drop-in call sequence of INTEGRATION.md section 4 (RCM_run: rcmdyn_tend then
    # rcmdyn_bdyval per step through the C-ABI, each replaying its own graph), same K steps,
    # after two untimed pairs that capture its graphs (one per ping-pong parity)
    for _ in range(2):
        eng.tend()
        eng.bdyval()
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        eng.tend()
        eng.bdyval()
    barrier()
    wall_d = time.perf_counter() - t0
    if dist is not None:
        import torch
        tt = torch.tensor([wall_d], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        wall_d = float(tt.item())
    # per-kernel device time (HIP events around each launch on the engine's stream), on
    # every rank (the eager steps exchange halos), after the timed region
    kt = eng.kernel_times(args.prof_steps) if args.prof_steps > 0 else {}
    barrier()
    if nh:
        from regcm_amd.nhbase import acoustic_substeps
        istep = acoustic_substeps(rc, data["split"]["nh_dtsmax"], 2.0 * rc.dt, 2)
        bstep = step_bytes_nh(rc.jx, rc.iy, rc.kz, rc.nspgx, istep)
    else:
        istep = None
        bstep = step_bytes(rc.jx, rc.iy, rc.kz, rc.nspgx)
    if rank != 0:
        if dist is not None:
            dist.destroy_process_group()
        return
    # dominant kernel = largest device time per step
    dom = max(kt.items(), key=lambda kv: kv[1][0] * kv[1][1])[0] if kt else None
    roof = {"bound": "hbm", "achieved": None, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": None,
            "traffic": None, "kernel": dom}
    if dom is not None:
        launches, avg_ms = kt[dom]
        tj, ti = rc.jx, rc.iy
        if world > 1:                   # this rank's tile
            from regcm_amd.dycore import tile_extent
            ext, _ = tile_extent(rc.jx, rc.iy, cj, ci, rank)
            tj, ti = ext[1] - ext[0] + 1, ext[3] - ext[2] + 1
        b = kernel_bytes(dom, tj, ti, rc.kz, rc.nspgx)
        traffic, src = pmc_traffic(dom, args.config) if world == 1 else (None, None)
        roof.update({
            "avg_launch_us": avg_ms * 1e3,
            "launches_per_step": launches / args.prof_steps,
            "algorithmic_bytes_per_launch": b,
            "timing": f"HIP events around every launch on the engine stream, {args.prof_steps} eager steps "
                      "(rcmdyn_kernel_times)",
            "traffic_source": src,
        })
        if b is not None:
            achieved = b / (avg_ms * 1e-3) / 1e9
            roof.update({"achieved": achieved, "frac": achieved / HBM_PEAK_GBS, "traffic": traffic})
    step_achieved = bstep / t_step / 1e9
    core = "non-hydrostatic" if nh else "hydrostatic"
    line = {
        "metric": f"simulated-years/wall-day, {rc.jx}x{rc.iy}x{rc.kz} sigma grid ({core} dyn step)",
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
        "data": ("synthetic (syn-icbc v1" + (" NH variant" if nh else "") +
                 ", PCG64 seed 20261015): no DOMAIN/ICBC files offline"),
        "config": {"workload": (f"{args.config} {rc.jx}x{rc.iy}x{rc.kz} ds={rc.ds}km dt={rc.dt}s " +
                                ("non-hydrostatic (MM5 core), upstream adv + 4th-order diff + sound "
                                 f"({istep} acoustic sub-steps, upper radiative BC, Rayleigh damping) "
                                 "+ iboudy=5 relaxation, physics stubbed" if nh else
                                 "hydrostatic, upstream adv + 4th-order diff + split-explicit "
                                 "(nsplit=2) + iboudy=5 relaxation, physics stubbed")),
                   "tiles": f"{cj}x{ci}", "step": "tend + bdyval"},
        "roofline": roof,
        "step_roofline": {"achieved": step_achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                          "frac": step_achieved / HBM_PEAK_GBS, "algorithmic_bytes": bstep,
                          "note": "SURVEY 8(d) " + ("B_nh" if nh else "B_h") + " per step / wall time per step"},
        "kernel_us": {k: round(v[1] * 1e3, 2) for k, v in sorted(kt.items(), key=lambda kv: -kv[1][0] * kv[1][1])},
        "device_ms_per_step": dev_ms,
        "dropin_ms_per_step": wall_d / args.steps * 1e3,
        "dropin_note": "rcmdyn_tend + rcmdyn_bdyval per step (INTEGRATION.md section 4), timed like value",
        "runtime": rt,
        "settle": {"steps": settle_steps, "s": round(settle_s, 3),
                   "note": "untimed steps before the W warm-up steps, until --settle-ms of wall time has "
                           "passed: from an idle GPU the first ~40 ms of steps run at a lower clock "
                           "(C3, one box: 0.218-0.221 ms/step timed over 20 steps after 5 warm-up, "
                           "0.2025 over 200 or 1000; 100 ms of settle measured as good as 300; profiles/r04/c3_settle.log)"},
    }
    if world > 1:
        line["runtime_per_rank"] = rts
    if not args.no_cpu_baseline and world == 1:
        line["cpu_baseline"] = cpu_baseline(rc, data, args.cpu_budget, args.cpu_threads)
    print(json.dumps(line))
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
