#!/bin/bash
# One measurement session on the box (prebuilt in-tree libraries):
#   PMC passes (T, C3) -> profiles/r${ROUND}_pmc_*.json on the box, so the bench lines below use them;
#   bench.py T (default line), C3, C5 at N=1; rocprofv3 kernel-trace stats of the T and C3 parse.
# Every GPU step has its own time limit; the script stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
ROUND=${ROUND:-2}
step() { echo "== $1 ($(date +%T))"; }
step pmc; ROUND=$ROUND bash scripts/gpu_pmc.sh > gpurun_out/pmc.log 2>&1 || { tail -5 gpurun_out/pmc.log; exit 3; }
cp gpurun_out/r${ROUND}_pmc_T.json gpurun_out/r${ROUND}_pmc_C3.json profiles/
step "bench T"; timeout -k 10 400 python bench.py > gpurun_out/bench_T.json 2> gpurun_out/bench_T.err || exit 4
tail -c 600 gpurun_out/bench_T.json; echo
step "bench C3"; timeout -k 10 300 python bench.py --workload C3 --no-c1 > gpurun_out/bench_C3.json 2> gpurun_out/bench_C3.err || exit 5
step "bench C2"; timeout -k 10 300 python bench.py --workload C2 --no-c1 --no-cpu-baseline > gpurun_out/bench_C2.json 2> gpurun_out/bench_C2.err || exit 5
step "bench C4"; timeout -k 10 300 python bench.py --workload C4 --no-c1 --no-cpu-baseline > gpurun_out/bench_C4.json 2> gpurun_out/bench_C4.err || exit 5
step "bench C5 N=1"; timeout -k 10 400 python bench.py --workload C5 --steps 10 --warmup 3 > gpurun_out/bench_C5_n1.json 2> gpurun_out/bench_C5_n1.err || exit 6
tail -c 400 gpurun_out/bench_C5_n1.json; echo
cd /tmp
for wl in T C3; do
  step "rocprof $wl"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_$wl" -o run --output-format csv \
    -- python3 "$R/bench.py" --workload $wl --steps 20 --warmup 5 --no-cpu-baseline --no-e2e --no-c1 \
    > "$R/gpurun_out/prof_$wl.log" 2>&1 || { echo "STOP rocprof $wl"; exit 7; }
done
step done
