#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, rocprof kernel trace.
# Stops at the first GPU fault / abort / timeout (exit codes >= 124 or signals).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
ok_or_stop() {  # $1 = exit code, $2 = step name
  if [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; then echo "STOP after $2 (exit $1)"; exit "$1"; fi
}
echo "== build"; timeout -k 10 300 python -c "import __graft_entry__ as g; g.build()" || exit 2
echo "== pytest -m gpu"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -30 gpurun_out/pytest_gpu.log; ok_or_stop $rc pytest
echo "== smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?
tail -5 gpurun_out/smoke.log; ok_or_stop $rc smoke
echo "== bench"
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1; rc=$?
tail -5 gpurun_out/bench.log; ok_or_stop $rc bench
for wl in C2 C3 C4; do
  timeout -k 10 200 python bench.py --workload $wl --no-cpu-baseline --no-c1 > gpurun_out/bench_$wl.log 2>&1; rc=$?
  tail -2 gpurun_out/bench_$wl.log; ok_or_stop $rc bench_$wl
done
echo "== rocprof"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o run \
  --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 20 --warmup 5 --no-cpu-baseline --no-e2e --no-c1 --no-ingest --no-cdr \
  > "$GRAFT_REPO_ROOT/gpurun_out/rocprof.log" 2>&1; rc=$?
tail -5 "$GRAFT_REPO_ROOT/gpurun_out/rocprof.log"; ok_or_stop $rc rocprof
find "$GRAFT_REPO_ROOT/gpurun_out/prof" -name "*stats*" | head
echo "== done"
