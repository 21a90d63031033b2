"""Decomposed run over RCCL, one tile per process, against one tile: the gathered state
after N steps must be bit-identical (the decomposition invariance of the hydrostatic core,
SURVEY.md section 8(e), and of the NH core).

    python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
        --master-port 29511 tools/rccl_check.py --config C1 --steps 6

Each rank needs a device of its own: RCCL refuses two ranks of one communicator on the same
GPU (ncclCommInitRank: invalid usage), so the check exits early, with a message, when fewer
devices than ranks are visible.  On a one-GPU box the RCCL transport is exercised instead by
the one-rank self communicator (RCMDYN_FORCE_RCCL, tests/test_rccl_gpu.py).
Rank 0 prints one JSON line and exits non-zero on a mismatch.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C1")
    ap.add_argument("--steps", type=int, default=6)
    ap.add_argument("--timed-steps", type=int, default=0)
    args = ap.parse_args()
    import torch
    import torch.distributed as dist
    from regcm_amd import icbc
    from regcm_amd.config import CONFIGS, NH_STATE_FIELDS, STATE_FIELDS
    from regcm_amd.dycore import DynCore, comm_unique_id, set_nproc

    world = int(os.environ["WORLD_SIZE"])
    rank = int(os.environ["RANK"])
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    ndev = torch.cuda.device_count()
    if ndev < world:
        print(f"rccl_check: {world} ranks need {world} GPUs, {ndev} visible (RCCL allows one rank per "
              "device); use tests/test_rccl_gpu.py on a one-GPU box", file=sys.stderr, flush=True)
        sys.exit(2)
    dev = local_rank
    dist.init_process_group(backend="gloo", init_method="env://")
    rc = CONFIGS[args.config]
    nh = rc.idynamic == 2
    data = icbc.generate_nh(rc) if nh else icbc.generate(rc)
    cj, ci = set_nproc(world, rc.jx, rc.iy)
    uid = bytearray(comm_unique_id()) if rank == 0 else bytearray(128)
    t = torch.tensor(list(uid), dtype=torch.uint8)
    dist.broadcast(t, src=0)
    uid = bytes(t.tolist())
    eng = DynCore(rc, data["split"], nproc_j=cj, nproc_i=ci, tile_first=rank, tile_count=1,
                  comm_rank=rank, comm_size=world, device=dev, unique_id=uid)
    eng.put_state(data["state"])
    eng.bdyval()
    eng.step(args.steps)
    eng.synchronize()
    names = STATE_FIELDS + (NH_STATE_FIELDS if nh else [])
    got = {}
    for n in names:
        a = torch.from_numpy(eng.get(n))
        dist.all_reduce(a, op=dist.ReduceOp.SUM)   # owned regions are disjoint: exact
        got[n] = a.numpy()
    ms = None
    if args.timed_steps > 0:
        eng.synchronize()
        dist.barrier()
        t0 = time.perf_counter()
        eng.step(args.timed_steps)
        eng.synchronize()
        dist.barrier()
        ms = (time.perf_counter() - t0) / args.timed_steps * 1e3
    bad = []
    if rank == 0:
        ref = DynCore(rc, data["split"], device=dev)
        ref.put_state(data["state"])
        ref.bdyval()
        ref.step(args.steps)
        for n in names:
            if not np.array_equal(ref.get(n), got[n]):
                bad.append(n)
        print(json.dumps({"config": args.config, "world": world, "tiles": [cj, ci], "steps": args.steps,
                          "mismatch": bad, "ms_per_step": ms}), flush=True)
    flag = torch.tensor([len(bad)])
    dist.broadcast(flag, src=0)
    eng.close()
    dist.destroy_process_group()
    sys.exit(1 if int(flag.item()) else 0)


if __name__ == "__main__":
    main()
