#!/bin/bash
# GPU test suite on the box (prebuilt in-tree .so); stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 ${T:-1000} python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_ARGS} \
  > gpurun_out/pytest_gpu.log 2>&1; rc=$?
grep -E "passed|failed|error" gpurun_out/pytest_gpu.log | tail -3
exit $rc
