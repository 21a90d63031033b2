"""bench.py's settle phase (untimed steps before the warm-up, until --settle-ms of wall time has
passed on rank 0): every rank must run the same number of steps, since each step exchanges
halos with the neighbours.  Checked on CPU with gloo, world size 2, the ranks' steps taking
different host times (a stand-in engine that only counts and sleeps)."""
import os
import socket
import sys
import time

import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


class _CountingEngine:
    def __init__(self, step_s):
        self.steps = 0
        self.step_s = step_s

    def step(self, n):
        self.steps += n
        time.sleep(self.step_s * n)

    def synchronize(self):
        pass


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch.distributed as dist
    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    eng = _CountingEngine(0.002 if rank == 0 else 0.0005)    # rank 1 three times faster
    import torch

    def bcast(v):
        t = torch.tensor([v], dtype=torch.int32)
        dist.broadcast(t, src=0)
        return int(t.item())
    n, s = bench.settle(eng, 0.05, bcast)
    q.put((rank, n, eng.steps, s))
    dist.destroy_process_group()


def test_settle_same_steps_on_every_rank():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    out = sorted(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    (r0, n0, c0, s0), (r1, n1, c1, _) = out
    assert n0 == c0 and n1 == c1 and n0 == n1 and n0 > 1
    assert s0 >= 0.05


def test_settle_off():
    sys.path.insert(0, ROOT)
    import bench
    eng = _CountingEngine(0.0)
    assert bench.settle(eng, 0.0, None) == (0, 0.0)
    assert eng.steps == 0
