#!/bin/bash
# A/B of engine variants (tools/variant_build.sh) on the small single-tile domains of the
# scaling runs' rank tiles (tools/small_tile.py) and on C3, alternating on one GPU box:
#   CHECK=<variant> VARS="head v head v" bash tools/tile_ab.sh
# CHECK: the hydrostatic parity tests run first on that variant (skipped when empty).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
if [ -n "${CHECK:-}" ]; then
  for c in $CHECK; do
    timeout -k 10 400 env RCMDYN_LIB=varlib/var_$c.so python -m pytest tests/test_parity_gpu.py tests/test_species_gpu.py -m gpu -q -x -p no:cacheprovider > gpurun_out/t_check_$c.log 2>&1 || { echo "parity failed on $c"; tail -20 gpurun_out/t_check_$c.log; exit 3; }
    echo "$c: $(tail -1 gpurun_out/t_check_$c.log)"
  done
fi
n=0
for v in ${VARS:-head}; do
  n=$((n+1))
  timeout -k 10 200 env RCMDYN_TIMING_BUILD=1 RCMDYN_LIB=varlib/var_$v.so python tools/small_tile.py --no-shares > gpurun_out/t_${n}_$v.log 2>&1 || { echo "small_tile $v failed"; tail -3 gpurun_out/t_${n}_$v.log; exit 3; }
  timeout -k 10 200 env RCMDYN_TIMING_BUILD=1 RCMDYN_LIB=varlib/var_$v.so python bench.py --steps 200 --warmup 20 --no-cpu-baseline --prof-steps 5 > gpurun_out/t_${n}_$v.json 2> gpurun_out/t_${n}_$v.err || { echo "bench $v failed"; tail -3 gpurun_out/t_${n}_$v.err; exit 3; }
  echo "== $n $v"; cat gpurun_out/t_${n}_$v.log
  python3 -c "import json; d=json.loads(open('gpurun_out/t_${n}_$v.json').read().strip().splitlines()[-1]); k=d.get('kernel_us',{}); print('C3', round(d['ms_per_step']*1e3,1), 'us/step', k)"
done
