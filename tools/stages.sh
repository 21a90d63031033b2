#!/bin/bash
# Run "name|timeout|command" stages from the arguments in order on the GPU box; each under its
# own time limit, output in gpurun_out/<name>.log.  rc 0/1 goes on (1 = test failure), any
# other status (crash, abort, time limit) ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for st in "$@"; do
  name=${st%%|*}; rest=${st#*|}; tmo=${rest%%|*}; cmd=${rest#*|}
  timeout -k 10 "$tmo" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "[$name] rc=$rc"; tail -n 4 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
done
