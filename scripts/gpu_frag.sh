#!/bin/bash
# DataFrag reassembly on the GPU box: parity tests first, then timing.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests/test_frag_gpu.py -m gpu -x -q > gpurun_out/pytest_frag.log 2>&1; rc=$?
tail -30 gpurun_out/pytest_frag.log
exit $rc
