#!/bin/bash
# One GPU session: parity tests, smoke, short bench, rocprof kernel-trace summary.
# Every GPU step has its own time limit; a crash/timeout (status other than 0/1) ends the call.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {  # run <name> <timeout> <cmd...>
  local name=$1 tmo=$2; shift 2
  timeout -k 10 "$tmo" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "[$name] rc=$rc"; tail -n 5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
STAGES=${STAGES:-"pytest smoke bench prof"}
for s in $STAGES; do
  case $s in
    pytest) run pytest_gpu 900 python -m pytest tests -m gpu -q -p no:cacheprovider ;;
    smoke)  run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench)  run bench 600 python bench.py --steps ${STEPS:-100} --warmup ${WARMUP:-10} ;;
    prof)   run prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 2 --no-cpu-baseline ;;
  esac
done
