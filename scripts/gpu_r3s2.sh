#!/bin/bash
# Round-3 session-2 check: GPU tests (prebuilt in-tree libraries), then the ingest legs under kernel stats.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || { echo "pytest rc=$rc"; exit $rc; }
JOBS="C3 --no-frag;T --no-frag" bash scripts/gpu_legs.sh
