#!/bin/bash
# A/B of an engine environment switch on one configuration (per-kernel times), GPU box:
#   EV=RCMDYN_ARENA SV="0 1 0 1" CFG=C5 bash tools/env_ab.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
n=0
for v in ${SV:-0 1}; do
  n=$((n + 1))
  log=gpurun_out/envab_${CFG:-C5}_${n}_$v.log
  timeout -k 10 300 env ${EV:-RCMDYN_ARENA}=$v python tools/ktimes.py --config ${CFG:-C5} --steps ${STEPS:-6} --prof-steps 3 > $log 2>&1 || { echo "run $v failed"; tail -3 $log; exit 3; }
  echo "== ${EV:-RCMDYN_ARENA}=$v"; head -${TOP:-6} $log; tail -1 $log
done
