#!/bin/bash
# A/B of an on/off engine switch (an env var whose presence turns a path off) with bench.py on C3:
#   EV=RCMDYN_NO_FUSE_UPDATE N=4 bash tools/fuse_ab.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in $(seq 1 ${N:-3}); do
  for m in on off; do
    if [ $m = off ]; then X="env $EV=1"; else X="env"; fi
    timeout -k 10 200 $X python bench.py --steps ${STEPS:-200} --warmup 10 --no-cpu-baseline --prof-steps 5 \
      --config ${CFG:-C3} > gpurun_out/fab_$m.json 2> gpurun_out/fab_$m.err || { echo "run $m failed"; tail -3 gpurun_out/fab_$m.err; exit 3; }
    python3 -c "import json; d=json.loads(open('gpurun_out/fab_$m.json').read().strip().splitlines()[-1]); print('$m', round(d['ms_per_step']*1e3,2), 'dropin', round(d['dropin_ms_per_step']*1e3,2), d['kernel_us'])"
  done
done
