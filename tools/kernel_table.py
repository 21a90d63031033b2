"""Per-kernel table of DESIGN.md section 4: device time (rocprofv3 kernel-trace stats or the
bench line's HIP-event times), algorithmic bytes (regcm_amd/traffic.py), the PMC bytes beyond
L2 (profiles/pmc_traffic*.json: FETCH_SIZE calibrated + WRITE_SIZE), and the VALU share:
SQ_ACTIVE_INST_VALU (quad-cycles) x 4 over the SIMD-cycles of the launch (1024 SIMDs at
2.4 GHz), and VALU instructions per wave.

    python tools/kernel_table.py C3 profiles/r03/c3_kernel_stats.csv
    python tools/kernel_table.py C5 profiles/r03/c5_bench.json
"""
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from regcm_amd.config import CONFIGS  # noqa: E402
from regcm_amd.traffic import kernel_bytes  # noqa: E402


def times(path):
    if path.endswith(".csv"):
        out = {}
        for r in csv.DictReader(open(path)):
            n = r["Name"].split("(")[0].replace("rcm::", "").replace("void ", "")
            out[n] = float(r["AverageNs"]) / 1000.0
        return out
    d = json.loads(open(path).read().strip().splitlines()[-1])
    return dict(d["kernel_us"])


def main():
    cfg, tpath = sys.argv[1], sys.argv[2]
    rc = CONFIGS[cfg]
    pm = json.load(open(os.path.join(ROOT, "profiles", "pmc_traffic.json" if cfg == "C3" else f"pmc_traffic_{cfg}.json")))
    t = times(tpath)
    print("| kernel | µs | algorithmic MB | PMC MB (R + W) | VALU busy % | VALU instr / wave |")
    print("|---|---|---|---|---|---|")
    for name, us in sorted(t.items(), key=lambda kv: -kv[1]):
        k = pm["kernels"].get(name) or pm["kernels"].get("void " + name)
        if k is None or us < 1.0:
            continue
        c = k["counters"]
        alg = kernel_bytes(name, rc.jx, rc.iy, rc.kz, rc.nspgx)
        valu = c.get("SQ_ACTIVE_INST_VALU", 0.0) * 4.0 / (us * 1e-6 * 2.4e9 * 1024) * 100.0
        ipw = c.get("SQ_INSTS_VALU", 0.0) / max(c.get("SQ_WAVES", 1.0), 1.0)
        mb = k["hbm_bytes_per_launch"] / 1e6
        print(f"| `{name}` | {us:.1f} | {alg / 1e6:.0f} | {mb:.0f} ({k['read_bytes_per_launch'] / 1e6:.0f} + "
              f"{k['write_bytes_per_launch'] / 1e6:.0f}) | {valu:.0f} | {ipw:.0f} |"
              if alg else
              f"| `{name}` | {us:.1f} | — | {mb:.0f} ({k['read_bytes_per_launch'] / 1e6:.0f} + "
              f"{k['write_bytes_per_launch'] / 1e6:.0f}) | {valu:.0f} | {ipw:.0f} |")


if __name__ == "__main__":
    main()
