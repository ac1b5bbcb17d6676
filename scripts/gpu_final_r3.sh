#!/bin/bash
# Round-3 final check: full GPU suite + smoke, the default bench line (T) and its kernel-trace stats.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || { echo "pytest rc=$rc"; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -5 gpurun_out/smoke.log; exit 3; }
tail -1 gpurun_out/smoke.log
timeout -k 10 400 python bench.py > gpurun_out/r3_bench_T.json 2> gpurun_out/r3_bench_T.err || { tail -5 gpurun_out/r3_bench_T.err; exit 4; }
for w in C2 C4; do
  timeout -k 10 300 python bench.py --workload $w --steps 20 --warmup 5 --no-c1 --no-e2e --no-cpu-baseline > gpurun_out/r3_bench_$w.json 2> gpurun_out/r3_bench_$w.err || exit 5
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_T -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-e2e --no-c1 > $R/gpurun_out/prof_T.log 2>&1 || exit 6
echo done
