"""One FORCE_RCCL decomposed C1 run in this process (mode: graph | eager | dropin), for
locating a crash of the one-rank RCCL transport outside pytest.  Prints one line per phase."""
import faulthandler
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
faulthandler.enable()
os.environ["RCMDYN_SEGV_TRACE"] = "1"
mode = sys.argv[1] if len(sys.argv) > 1 else "graph"
if "--torch-first" in sys.argv:        # as in a pytest session or bench.py: torch's own librccl.so.1
    import torch  # noqa: F401
import numpy as np  # noqa: E402
from regcm_amd import icbc  # noqa: E402
from regcm_amd.config import CONFIGS, STATE_FIELDS  # noqa: E402
from regcm_amd.dycore import DynCore  # noqa: E402

rc = CONFIGS["C1"]
data = icbc.generate(rc)


def eng(nj, ni):
    e = DynCore(rc, data["split"], nproc_j=nj, nproc_i=ni)
    e.put_state(data["state"])
    e.bdyval()
    return e


one = eng(1, 1)
os.environ["RCMDYN_FORCE_RCCL"] = "1"
if mode == "eager":
    os.environ["RCMDYN_NO_GRAPH"] = "1"
dec = eng(2, 2)
from regcm_amd.dycore import runtime_info  # noqa: E402
print("created", runtime_info(), flush=True)
one.step(6)
print("one stepped", flush=True)
if mode == "dropin":
    for _ in range(6):
        dec.tend()
        dec.bdyval()
else:
    for s in range(6):
        dec.step(1)
        print("dec step", s, flush=True)
bad = [n for n in STATE_FIELDS if not np.array_equal(one.get(n), dec.get(n))]
print("mode", mode, "mismatch", bad, flush=True)
sys.exit(1 if bad else 0)
