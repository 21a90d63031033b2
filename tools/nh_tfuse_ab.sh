set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for r in 1 2 3; do
  for v in fused inplace; do
    if [ $v = inplace ]; then export RCMDYN_NH_NO_TFUSE=1; else unset RCMDYN_NH_NO_TFUSE; fi
    timeout -k 10 200 python bench.py --config C5 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/nhab_${v}_$r.json 2>gpurun_out/nhab_${v}_$r.err || exit 3
    python -c "import json,sys; d=json.loads(open('gpurun_out/nhab_${v}_$r.json').read().strip().splitlines()[-1]); print('$v', d['ms_per_step'])"
  done
done
unset RCMDYN_NH_NO_TFUSE
timeout -k 10 200 python tools/kt_run.py C5 3 3 > gpurun_out/nhab_kt_fused.log 2>&1 || exit 3
head -c 600 gpurun_out/nhab_kt_fused.log
