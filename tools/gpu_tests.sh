#!/bin/bash
# GPU session: the given test files (default: the whole -m gpu suite), each step under its own
# time limit (KEXPR: a pytest -k expression); a crash or timeout (status other than 0/1) ends the call.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
FILES=${FILES:-tests}
timeout -k 10 ${TMO:-900} python -u -m pytest $FILES -m gpu -v --timeout 120 --timeout-method thread \
  -p no:cacheprovider ${PYARGS:-} ${KEXPR:+-k "$KEXPR"} > gpurun_out/${LOG:-gpu_tests}.log 2>&1
rc=$?
grep -E "passed|failed|error" gpurun_out/${LOG:-gpu_tests}.log | tail -3
grep -E "^(FAILED|ERROR)" gpurun_out/${LOG:-gpu_tests}.log | head -20
exit $rc
