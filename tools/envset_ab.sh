#!/bin/bash
# A/B of an engine switch that acts when its variable is SET (any value) against the default
# (unset), alternating on one box, per-kernel times of one configuration:
#   EV=RCMDYN_NH_NO_A1R SV="off on off on" CFG=C5 bash tools/envset_ab.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
n=0
for v in ${SV:-off on off on}; do
  n=$((n + 1))
  log=gpurun_out/esab_${CFG:-C5}_${n}_$v.log
  if [ "$v" = on ]; then
    timeout -k 10 300 env ${EV}=1 python tools/ktimes.py --config ${CFG:-C5} --steps ${STEPS:-6} --prof-steps 3 > $log 2>&1
  else
    timeout -k 10 300 python tools/ktimes.py --config ${CFG:-C5} --steps ${STEPS:-6} --prof-steps 3 > $log 2>&1
  fi
  rc=$?
  [ $rc -eq 0 ] || { echo "run $v failed rc=$rc"; tail -3 $log; exit 3; }
  echo "== ${EV} $v"; head -${TOP:-8} $log; tail -1 $log
done
