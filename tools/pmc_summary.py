"""Summarise rocprofv3 --pmc CSV passes (tools/pmc.sh) per kernel and write
profiles/pmc_traffic.json (HBM bytes per launch, consumed by bench.py's roofline.traffic).

FETCH_SIZE / WRITE_SIZE are rocprofv3 derived counters in KiB (memory side of the L2,
Infinity-Cache hits included).  The read correction comes from the calibration pass
(tools/calib/calib_fetch.hip: 512 MiB read + 512 MiB written per launch with the engine's
8-byte-per-lane access width), as /opt/skills/guides/MI355X_MICROARCH.md prescribes for
uncalibrated access widths.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def load(pass_dir):
    """{kernel: {counter: mean value per dispatch}}"""
    files = glob.glob(os.path.join(pass_dir, "**", "*counter_collection.csv"), recursive=True)
    acc = defaultdict(lambda: defaultdict(list))
    for fn in files:
        with open(fn) as fh:
            for r in csv.DictReader(fh):
                name = r["Kernel_Name"].split("(")[0].replace("rcm::", "")
                acc[name][(r["Counter_Name"], r.get("Dispatch_Id", ""))].append(float(r["Counter_Value"]))
    out = {}
    for k, d in acc.items():
        per = defaultdict(list)
        for (cn, _disp), vals in d.items():
            per[cn].append(sum(vals))          # sum over instances of one dispatch
        out[k] = {cn: sum(v) / len(v) for cn, v in per.items()}
    return out


def main():
    cfg = sys.argv[2] if len(sys.argv) > 2 else "C3"
    base = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out", "pmc_" + cfg)
    known = 64 * 2**20 * 8
    cf = load(os.path.join(base, "cal_fetch")).get("k_calib_copy", {}).get("FETCH_SIZE")
    cw = load(os.path.join(base, "cal_write")).get("k_calib_copy", {}).get("WRITE_SIZE")
    rf = known / (cf * 1024.0) if cf else None      # bytes per reported KiB unit
    rw = known / (cw * 1024.0) if cw else None
    fetch = load(os.path.join(base, "fetch"))
    write = load(os.path.join(base, "write"))
    extra = {}
    for p in ("sq1", "sq2", "tcc"):
        if os.path.isdir(os.path.join(base, p)):
            for k, d in load(os.path.join(base, p)).items():
                extra.setdefault(k, {}).update(d)
    from bench import kernels_digest
    res = {"digest": kernels_digest(), "config": cfg,
           "source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes), bench.py {cfg} graph replay; "
                     "read scale from tools/calib/calib_fetch.hip",
           "calibration": {"fetch_kib_reported": cf, "write_kib_reported": cw, "bytes_known": known,
                           "read_scale": rf, "write_scale": rw},
           "kernels": {}}
    for k in sorted(set(fetch) | set(write)):
        f = fetch.get(k, {}).get("FETCH_SIZE")
        w = write.get(k, {}).get("WRITE_SIZE")
        if f is None or w is None:
            continue
        rb = f * 1024.0 * (rf or 1.0)
        wb = w * 1024.0 * (rw or 1.0)
        res["kernels"][k] = {"read_bytes_per_launch": rb, "write_bytes_per_launch": wb,
                             "hbm_bytes_per_launch": rb + wb, "counters": extra.get(k, {})}
    if not res["kernels"] or rf is None or rw is None:
        sys.exit(f"pmc_summary: no counter data under {base}; nothing written")
    out = os.path.join(ROOT, "profiles", "pmc_traffic.json" if cfg == "C3" else f"pmc_traffic_{cfg}.json")
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1, sort_keys=True)
    print(json.dumps(res["calibration"]))
    for k, v in sorted(res["kernels"].items(), key=lambda kv: -kv[1]["hbm_bytes_per_launch"]):
        c = v["counters"]
        print(f"{k:22s} R {v['read_bytes_per_launch']/1e6:8.2f} MB  W {v['write_bytes_per_launch']/1e6:8.2f} MB  "
              + " ".join(f"{n}={c[n]:.3g}" for n in sorted(c)))


if __name__ == "__main__":
    main()
