#!/bin/bash
# gpu_final_r3.sh plus the C3 ingest kernel stats / leg time first.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_ingest_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pt_ingest.log 2>&1; rc=$?
tail -2 gpurun_out/pt_ingest.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_kstat_libs.sh C3 "--no-c1 --no-cpu-baseline --no-e2e --no-cdr --no-frag" "k_proxy|k_classify" || exit 7
WLS="C3" timeout -k 10 300 bash scripts/gpu_ingest_ab.sh || exit 8
bash scripts/gpu_final_r3.sh
