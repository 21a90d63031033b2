#!/bin/bash
# A/B of engine environment combinations on one configuration (per-kernel times and the
# graph-replayed step), alternating on one box.  COMBOS: space-separated name=VAR:val,VAR:val
# items ("base=" for no variables):
#   COMBOS="base= side=RCMDYN_MOIST_LDS:40000 base=" CFG=C3 STEPS=200 bash tools/envcombo_ab.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
n=0
for item in ${COMBOS:-base=}; do
  n=$((n + 1))
  name=${item%%=*}
  vars=${item#*=}
  envs=()
  IFS=',' read -ra kv <<< "$vars"
  for p in "${kv[@]}"; do [ -n "$p" ] && envs+=("${p%%:*}=${p#*:}"); done
  log=gpurun_out/ecab_${CFG:-C3}_${n}_$name.log
  timeout -k 10 300 env "${envs[@]}" python tools/ktimes.py --config ${CFG:-C3} --steps ${STEPS:-200} --prof-steps ${PSTEPS:-5} > $log 2>&1
  rc=$?
  [ $rc -eq 0 ] || { echo "run $name failed rc=$rc"; tail -3 $log; exit 3; }
  echo "== $name ${envs[*]}"; head -${TOP:-8} $log; tail -1 $log
done
