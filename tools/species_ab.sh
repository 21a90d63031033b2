#!/bin/bash
# A/B of engine variants (tools/variant_build.sh) on the nqx = 5 step (tools/species_bench.py),
# alternating on one box, after the species/hydrostatic moisture tests on each CHECK variant:
#   CHECK="dpp" VARS="head dpp head dpp" bash tools/species_ab.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for c in ${CHECK:-}; do
  timeout -k 10 400 env RCMDYN_LIB=varlib/var_$c.so python -u -m pytest tests/test_species_gpu.py tests/test_parity_gpu.py -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/sab_check_$c.log 2>&1 || { echo "tests failed on $c"; tail -20 gpurun_out/sab_check_$c.log; exit 3; }
  echo "$c: $(tail -1 gpurun_out/sab_check_$c.log)"
done
n=0
for v in ${VARS:-head}; do
  n=$((n + 1))
  timeout -k 10 300 env RCMDYN_LIB=varlib/var_$v.so python tools/species_bench.py --reps 1 > gpurun_out/sab_${n}_$v.log 2>&1 || { echo "species_bench $v failed"; tail -3 gpurun_out/sab_${n}_$v.log; exit 3; }
  echo "== $n $v"; grep -E "^== |negfix_serial|k_qx_serial" gpurun_out/sab_${n}_$v.log
done
