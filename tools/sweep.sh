#!/bin/bash
# Tuning sweep of the C3 step: one bench run per env setting given as arguments
# ("RCMDYN_KS_TJ=64 RCMDYN_KS_KC=4" ...), each under its own time limit; prints ms/step and
# the per-launch time of the kernels named in KERN.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
CFG=${CFG:-C3}
KERN=${KERN:-k_scalars k_momentum}
i=0
for sw in "" "$@"; do
  i=$((i+1))
  timeout -k 10 200 env $sw python bench.py --config $CFG --steps ${STEPS:-200} --warmup 20 --no-cpu-baseline \
    > gpurun_out/sw_$i.json 2> gpurun_out/sw_$i.err || { echo "run [$sw] failed rc=$?"; tail -5 gpurun_out/sw_$i.err; exit 3; }
  python3 - "$i" "$sw" "$KERN" <<'PY'
import json, sys
d = json.loads([l for l in open(f"gpurun_out/sw_{sys.argv[1]}.json") if l.startswith("{")][-1])
ku = d.get("kernel_us", {})
print(f"[{sys.argv[2] or 'default'}] {d['ms_per_step']*1e3:.1f} us/step", " ".join(f"{k}={ku.get(k)}" for k in sys.argv[3].split()))
PY
done
