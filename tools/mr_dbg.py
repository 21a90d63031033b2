import os, sys, threading, faulthandler
sys.path.insert(0, os.getcwd())
faulthandler.enable()
os.environ["RCMDYN_SEGV_TRACE"] = "1"
os.environ["RCMDYN_LOCAL_TRACE"] = "1"
from regcm_amd.config import CONFIGS
from regcm_amd import icbc
from regcm_amd.dycore import DynCore
rc = CONFIGS["C1"]; data = icbc.generate(rc)
os.environ["RCMDYN_LOCAL_COMM"] = "dbg"
engs = [DynCore(rc, data["split"], nproc_j=2, nproc_i=2, tile_first=r, tile_count=1, comm_rank=r, comm_size=4, device=0) for r in range(4)]
print("created", flush=True)
def work(e, r):
    e.put_state(data["state"]); print("put", r, flush=True)
    e.bdyval(); print("bdyval", r, flush=True)
    e.step(10); print("step", r, flush=True)
    e.synchronize(); print("sync", r, flush=True)
th = [threading.Thread(target=work, args=(e, r)) for r, e in enumerate(engs)]
[t.start() for t in th]; [t.join() for t in th]
print("done")
