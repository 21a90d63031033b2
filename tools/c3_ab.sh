#!/bin/bash
# A/B of engine variant libraries on the C3 step (graph-replayed ms/step and per-kernel times),
# alternating, after a hydrostatic parity run of each (varlib/var_<name>.so):
#   VARS="head skip head skip" CHECK="skip" bash tools/c3_ab.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in ${CHECK:-}; do
  timeout -k 10 300 env RCMDYN_TIMING_BUILD=1 RCMDYN_LIB=varlib/var_$v.so python -m pytest tests/test_parity_gpu.py tests/test_configs_gpu.py -m gpu -q -x -p no:cacheprovider > gpurun_out/c3ab_check_$v.log 2>&1 || { echo "parity failed $v"; tail -20 gpurun_out/c3ab_check_$v.log; exit 3; }
  echo "parity $v: $(tail -1 gpurun_out/c3ab_check_$v.log)"
done
i=0
for v in ${VARS:-}; do
  i=$((i+1))
  timeout -k 10 200 env RCMDYN_TIMING_BUILD=1 RCMDYN_LIB=varlib/var_$v.so python tools/ktimes.py --config C3 --steps 200 --prof-steps 10 > gpurun_out/c3ab_${i}_$v.log 2>&1 || { echo "run $v failed"; tail -3 gpurun_out/c3ab_${i}_$v.log; exit 3; }
  echo "== $v"; head -${TOP:-4} gpurun_out/c3ab_${i}_$v.log; tail -1 gpurun_out/c3ab_${i}_$v.log
done
