#!/bin/bash
# Parity tests + bench (all workloads) + rocprof kernel trace + PMC passes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
ok_or_stop() { if [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; then echo "STOP after $2 (exit $1)"; exit "$1"; fi; }
echo "== build"; timeout -k 10 300 python -c "import __graft_entry__ as g; g.build()" || exit 2
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  echo "== pytest -m gpu"
  timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?
  tail -15 gpurun_out/pytest_gpu.log; ok_or_stop $rc pytest
fi
echo "== bench"
for wl in ${WORKLOADS:-T C2 C3 C4}; do
  extra="--no-cpu-baseline"; [ "$wl" = T ] && extra=""
  timeout -k 10 300 python bench.py --workload $wl $extra > gpurun_out/bench_$wl.log 2>&1; rc=$?
  tail -1 gpurun_out/bench_$wl.log | cut -c1-400; ok_or_stop $rc bench_$wl
done
echo "== rocprof kernel trace"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" -o run --output-format csv \
  -- python3 "$R/bench.py" --steps 20 --warmup 5 --no-cpu-baseline > "$R/gpurun_out/rocprof.log" 2>&1; rc=$?
ok_or_stop $rc rocprof
grep -h parse "$R/gpurun_out/prof/"*kernel_stats.csv
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c -d "$R/gpurun_out/pmc_$c" -o run --output-format csv \
    -- python3 "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline > "$R/gpurun_out/pmc_$c.log" 2>&1; rc=$?
  ok_or_stop $rc pmc_$c
done
echo "== done"
