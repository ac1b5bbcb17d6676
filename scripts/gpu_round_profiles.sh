#!/bin/bash
# Round profile set: PMC passes (scripts/gpu_pmc.sh, ROUND=$ROUND) then rocprofv3 --kernel-trace --stats of
# the default bench.py command (T) and of the C3 / C4 lines; kernel-stats CSVs + bench JSONs into gpurun_out/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
ROUND=${ROUND:-3}
[ "${PMC:-1}" = 1 ] && { ROUND=$ROUND bash scripts/gpu_pmc.sh > gpurun_out/pmc_run.log 2>&1 || { tail -5 gpurun_out/pmc_run.log; exit 3; }; }
cp gpurun_out/r${ROUND}_pmc_T.json gpurun_out/r${ROUND}_pmc_C3.json /tmp/ 2>/dev/null
rm -rf gpurun_out/pmc_T_* gpurun_out/pmc_C3_*
for wl in T C3 C4; do
  args="--no-c1 --no-e2e --no-cpu-baseline"; [ $wl = T ] || args="$args --workload $wl"
  (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/kt_$wl -o run --output-format csv \
     -- python3 $R/bench.py $args > $R/gpurun_out/r${ROUND}_prof_bench_$wl.json 2> $R/gpurun_out/kt_$wl.err) \
     || { echo "STOP $wl"; tail -5 gpurun_out/kt_$wl.err; exit 4; }
  f=$(find gpurun_out/kt_$wl -name "*kernel_stats.csv" | head -1)
  cp "$f" gpurun_out/r${ROUND}_bench_${wl}_kernel_stats.csv
  rm -rf gpurun_out/kt_$wl
  echo "$wl done"
done
