#!/bin/bash
# Selected GPU tests on the box (prebuilt in-tree .so): gpu_pytest.sh <pytest args...>
# Output in gpurun_out/pytest_sel.log; stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 ${T:-900} python -u -m pytest -m gpu -x -v --timeout ${TT:-300} --timeout-method thread "$@" \
  > gpurun_out/pytest_sel.log 2>&1; rc=$?
grep -E "passed|failed|error" gpurun_out/pytest_sel.log | tail -3
exit $rc
