"""Per-kernel device time (HIP events per launch, rcmdyn_kernel_times) of a config after a few
warm-up steps, for A/B of engine variants (RCMDYN_LIB=varlib/var_<name>.so):
    python tools/kt_run.py [CONFIG] [warmup] [profiled steps]"""
import os
import sys

sys.path.insert(0, os.getcwd())
from regcm_amd.config import CONFIGS  # noqa: E402
from regcm_amd import icbc  # noqa: E402
from regcm_amd.dycore import DynCore  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "C3"
warm = int(sys.argv[2]) if len(sys.argv) > 2 else 2
nprof = int(sys.argv[3]) if len(sys.argv) > 3 else 5
rc = CONFIGS[name]
data = icbc.generate_nh(rc) if rc.idynamic == 2 else icbc.generate(rc)
e = DynCore(rc, data["split"])
e.put_state(data["state"])
e.bdyval()
e.step(warm)
kt = e.kernel_times(nprof)
tot = sum(v[0] * v[1] for v in kt.values()) / nprof
print(os.environ.get("RCMDYN_LIB"), f"sum {tot:.4f} ms/step",
      {k: round(v[1] * 1e3, 2) for k, v in sorted(kt.items(), key=lambda kv: -kv[1][0] * kv[1][1])}, flush=True)
