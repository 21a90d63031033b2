#!/bin/bash
# A/B timing of the C3 step: default engine vs env switches given as arguments
# (e.g. tools/ab_bench.sh RCMDYN_SERIAL=1).  Each run has its own time limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
CFG=${CFG:-C3}
one() {  # one <tag> [VAR=val ...]
  local tag=$1; shift
  timeout -k 10 200 env "$@" python bench.py --config $CFG --steps ${STEPS:-200} --warmup 20 --no-cpu-baseline --prof-steps 0 \
    > gpurun_out/ab_$tag.json 2> gpurun_out/ab_$tag.err || { echo "run $tag failed rc=$?"; tail -5 gpurun_out/ab_$tag.err; exit 3; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/ab_$tag.json')); print('$tag', '$*', round(d['ms_per_step']*1e3,1), 'us/step')"
}
one base
i=0
for sw in "$@"; do i=$((i+1)); one v$i $sw; done
one base2
