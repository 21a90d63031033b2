#!/bin/bash
# A/B of engine variant libraries (varlib/var_<name>.so, tools/variant_build.sh output moved
# there so it travels with gpurun) on the GPU box: hydrostatic parity tests on each variant,
# then the C3 step with per-kernel times, the default engine first.
#   VARS="pf1w4 pf0w4" bash tools/km_ab.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
summ() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); k=d['kernel_us']; print(sys.argv[2], round(d['ms_per_step']*1e3,1), 'us/step', dict(list(k.items())[:5]))" "$@"; }
for v in ${CHECK:-}; do
  timeout -k 10 300 env RCMDYN_LIB=varlib/var_$v.so python -m pytest tests/test_parity_gpu.py -m gpu -q -x -p no:cacheprovider > gpurun_out/km_check_$v.log 2>&1 || { echo "parity failed $v"; tail -30 gpurun_out/km_check_$v.log; exit 3; }
  echo "parity $v: $(tail -1 gpurun_out/km_check_$v.log)"
done
timeout -k 10 200 env RCMDYN_SCALARS_LEVEL=1 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --prof-steps 5 > gpurun_out/km_level.json 2> gpurun_out/km_level.err || { echo "level run failed"; tail -3 gpurun_out/km_level.err; exit 3; }
summ gpurun_out/km_level.json level
for v in ${VARS:-}; do
  timeout -k 10 200 env RCMDYN_LIB=varlib/var_$v.so ${VENV:-} python bench.py --steps 100 --warmup 10 --no-cpu-baseline --prof-steps 5 > gpurun_out/km_$v.json 2> gpurun_out/km_$v.err || { echo "run $v failed"; tail -3 gpurun_out/km_$v.err; exit 3; }
  summ gpurun_out/km_$v.json $v
done
