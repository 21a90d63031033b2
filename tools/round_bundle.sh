#!/bin/bash
# The round's measurement bundle on the GPU box (each step under its own limit; a crash or a
# timeout ends the script): GPU tests, smoke, the C3 bench line (with the PMC traffic of
# profiles/pmc_traffic.json when it matches the kernel sources), rocprofv3 kernel stats of C3,
# the C5 bench line and its rocprofv3 kernel stats.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {  # run <name> <timeout> <cmd...>
  local name=$1 tmo=$2; shift 2
  timeout -k 10 "$tmo" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "[$name] rc=$rc"; tail -n 3 "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
STAGES=${STAGES:-"pytest smoke bench prof c5bench c5prof"}
for s in $STAGES; do
  case $s in
    pytest) run pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --durations=0 --timeout 300 --timeout-method thread -p no:cacheprovider ;;
    smoke)  run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench)  run bench 600 python bench.py --steps 200 --warmup 20 ;;
    prof)   run prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 2 --no-cpu-baseline ;;
    c5bench) run c5bench 600 python bench.py --config C5 --steps 10 --warmup 3 --no-cpu-baseline ;;
    c5prof) run c5prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/c5prof -o run --output-format csv -- python3 bench.py --config C5 --steps 4 --warmup 2 --no-cpu-baseline --prof-steps 0 ;;
  esac
done
