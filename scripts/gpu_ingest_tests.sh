#!/bin/bash
# ingest / topic / shard GPU tests only (quick iteration on the history-cache kernels)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_ingest_gpu.py tests/test_topic_gpu.py tests/test_frag_gpu.py -m gpu -x -q \
  --timeout 300 --timeout-method thread > gpurun_out/pytest_ingest.log 2>&1; rc=$?
tail -15 gpurun_out/pytest_ingest.log; exit $rc
