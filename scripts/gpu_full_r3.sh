#!/bin/bash
# Full GPU suite + smoke on the prebuilt in-tree libraries, then ablation / ingest timings (round 3).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -4 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || { echo "pytest rc=$rc"; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?
tail -2 gpurun_out/smoke.log
[ $rc -eq 0 ] || { echo "smoke rc=$rc"; exit $rc; }
[ -d rustdds-io_uring_amd/variants ] || exit 0
bash scripts/gpu_kstat_libs.sh C3 "--no-c1 --no-cpu-baseline --no-e2e --no-cdr --no-frag" "k_proxy" || exit $?
bash scripts/gpu_kstat_libs.sh C4 "--no-c1 --no-cpu-baseline --no-e2e --no-cdr --no-ingest" "k_keys|k_walk" || exit $?
WLS="C3" timeout -k 10 300 bash scripts/gpu_ingest_ab.sh
