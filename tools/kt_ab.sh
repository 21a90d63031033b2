#!/bin/bash
# per-kernel times of engine variants (timing only, results may be wrong): VARS="a b" tools/kt_ab.sh
cd $GRAFT_REPO_ROOT
for r in 1 2; do
for v in ${VARS}; do
  RCMDYN_LIB=varlib/var_$v.so timeout -k 10 200 python bench.py --steps ${STEPS:-8} --warmup 2 --no-cpu-baseline --prof-steps 3 > gpurun_out/kt.json 2>gpurun_out/kt.err || { tail -3 gpurun_out/kt.err; exit 3; }
  python3 -c "import json; d=json.loads(open('gpurun_out/kt.json').read().strip().splitlines()[-1]); k=d['kernel_us']; print('$v', round(d['ms_per_step']*1e3,1), k)"
done; done
