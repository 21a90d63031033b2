#!/bin/bash
# A/B of engine variant libraries on the C5 step (per-kernel times), on the GPU box:
#   VARS="head tc11 tc10" bash tools/nh_ab.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in ${VARS:-}; do
  timeout -k 10 300 env RCMDYN_TIMING_BUILD=1 RCMDYN_LIB=varlib/var_$v.so python tools/ktimes.py --config ${CFG:-C5} --steps ${STEPS:-6} --prof-steps ${PSTEPS:-3} > gpurun_out/nhab_$v.log 2>&1 || { echo "run $v failed"; tail -3 gpurun_out/nhab_$v.log; exit 3; }
  echo "== $v"; head -${TOP:-6} gpurun_out/nhab_$v.log; tail -1 gpurun_out/nhab_$v.log
done
