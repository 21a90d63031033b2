"""Graph-replayed steps of the hydrostatic step on one small tile (a rank tile of the scaling
runs), for a rocprofv3 kernel trace: per-kernel device durations and the gaps between
consecutive kernels inside the replayed graphs.
    rocprofv3 --kernel-trace --output-format csv -d DIR -o run -- python3 tools/tile_trace.py 96x48
    python3 tools/tile_trace.py --summary DIR"""
import csv
import dataclasses
import glob
import os
import statistics as S
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def summary(d):
    rows = []
    for fn in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        with open(fn) as fh:
            rows += list(csv.DictReader(fh))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    rows = rows[len(rows) // 3:]                      # steady state: drop set-up and warm-up
    by, gaps = {}, {}
    for a, b in zip(rows, rows[1:]):
        na = a["Kernel_Name"].split("(")[0].replace("rcm::", "").replace("void ", "")
        nb = b["Kernel_Name"].split("(")[0].replace("rcm::", "").replace("void ", "")
        by.setdefault(na, []).append((int(a["End_Timestamp"]) - int(a["Start_Timestamp"])) / 1e3)
        g = (int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3
        if 0 <= g < 50:
            gaps.setdefault(f"{na} -> {nb}", []).append(g)
    for n, v in sorted(by.items(), key=lambda kv: -S.median(kv[1])):
        print(f"{n:32s} n {len(v):5d} median {S.median(v):8.2f} us")
    for n, v in sorted(gaps.items(), key=lambda kv: -S.median(kv[1])):
        print(f"gap {n:60s} median {S.median(v):6.2f} us")


if sys.argv[1] == "--summary":
    summary(sys.argv[2])
    sys.exit(0)
from regcm_amd import icbc  # noqa: E402
from regcm_amd.config import CONFIGS  # noqa: E402
from regcm_amd.dycore import DynCore  # noqa: E402

jx, iy = (int(x) for x in sys.argv[1].split("x"))
rc = dataclasses.replace(CONFIGS["C3"], jx=jx, iy=iy)
data = icbc.generate(rc)
e = DynCore(rc, data["split"])
e.put_state(data["state"])
e.bdyval()
e.step(100)
e.synchronize()
