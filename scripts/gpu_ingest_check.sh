#!/bin/bash
# Ingest + bench GPU tests (prebuilt in-tree libraries), then the C3 / T ingest legs' per-kernel stats.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest ${TESTS:-tests/test_ingest_gpu.py tests/test_frag_gpu.py tests/test_bench_gpu.py} -x -q \
  --timeout 300 --timeout-method thread > gpurun_out/pt_ingest.log 2>&1; rc=$?
tail -8 gpurun_out/pt_ingest.log
[ $rc -eq 0 ] || { echo "pytest rc=$rc"; exit $rc; }
bash scripts/gpu_kstat_libs.sh C3 "--no-c1 --no-cpu-baseline --no-e2e --no-cdr --no-frag" "k_|sort|trampoline" || exit $?
bash scripts/gpu_kstat_libs.sh T "--no-c1 --no-cpu-baseline --no-e2e --no-cdr --no-frag" "k_|sort|trampoline"
