#!/bin/bash
# A/B of engine variants built by tools/variant_build.sh, on the GPU box:
#   CHECK=<variant> VARS="base v base v" bash tools/variant_ab.sh
# runs the hydrostatic parity tests on varlib/var_$CHECK.so, then the C3 bench (with per-kernel
# times) for each variant in turn.
set -u
cd $GRAFT_REPO_ROOT
timeout -k 10 300 env RCMDYN_LIB=varlib/var_${CHECK:-xcd}.so python -m pytest tests/test_parity_gpu.py -m gpu -q -x -p no:cacheprovider > gpurun_out/v_check.log 2>&1 || { echo "parity failed"; tail -20 gpurun_out/v_check.log; exit 3; }
tail -1 gpurun_out/v_check.log
for v in ${VARS:-base xcd base xcd}; do
  timeout -k 10 200 env RCMDYN_LIB=varlib/var_$v.so python bench.py --steps 100 --warmup 10 --no-cpu-baseline --prof-steps 5 > gpurun_out/v_$v.json 2> gpurun_out/v_$v.err || { echo "run $v failed"; tail -3 gpurun_out/v_$v.err; exit 3; }
  python3 -c "import json; d=json.loads(open('gpurun_out/v_$v.json').read().strip().splitlines()[-1]); k=d['kernel_us']; print('$v', round(d['ms_per_step']*1e3,1), {n:k[n] for n in ('k_scalars','k_momentum','k_columns','k_split_project')})"
done
