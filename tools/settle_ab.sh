set -u
cd "${GRAFT_REPO_ROOT}"
for r in 1 2; do
  for s in 100 300 1000; do
    timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --prof-steps 0 --settle-ms $s > gpurun_out/st_${s}_$r.log 2>&1 || exit 3
    python3 -c "import json; d=json.loads(open('gpurun_out/st_${s}_$r.log').read().strip().splitlines()[-1]); print('settle', $s, 'rep', $r, round(d['ms_per_step'],5), d['settle'])"
  done
done
timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --prof-steps 0 > gpurun_out/st_k200.log 2>&1 && python3 -c "import json; d=json.loads(open('gpurun_out/st_k200.log').read().strip().splitlines()[-1]); print('K=200', round(d['ms_per_step'],5))"
