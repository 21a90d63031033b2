#!/bin/bash
# A/B of one engine environment switch on the C3 bench, alternating runs on one box:
#   VAR=RCMDYN_GRAPH_STEPS A=1 B=2 N=3 tools/ab_env.sh
# Each run under its own time limit; a failing run ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
CFG=${CFG:-C3}
for r in $(seq 1 ${N:-3}); do
  for v in "$A" "$B"; do
    env "$VAR=$v" timeout -k 10 300 python bench.py --config $CFG --steps ${STEPS:-200} --warmup 20 --no-cpu-baseline \
      --prof-steps 0 > gpurun_out/ab_tmp.log 2>&1 || { echo "run failed"; tail -5 gpurun_out/ab_tmp.log; exit 3; }
    python -c "import json,sys; d=json.loads([l for l in open('gpurun_out/ab_tmp.log') if l.startswith('{')][-1]); print('$VAR=$v', round(d['ms_per_step'],5), round(d['dropin_ms_per_step'],5))" | tee -a gpurun_out/ab.log
  done
done
