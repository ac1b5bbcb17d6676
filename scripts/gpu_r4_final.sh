#!/bin/bash
# Round 4 record: PMC passes (FETCH / WRITE) for T and C3, the full bench line of every
# workload (T with its CPU baseline, C1 loopback and end to end; C2, C3 with its CPU baseline,
# C4, C5 at N = 1), and kernel-trace stats of T, C3, C4.  Outputs under gpurun_out/final/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$(pwd); mkdir -p gpurun_out/final; export TMPDIR=/tmp
F=$R/gpurun_out/final
ROUND=4 timeout -k 10 700 bash scripts/gpu_pmc.sh > $F/pmc.log 2>&1 || { tail -5 $F/pmc.log; exit 3; }
cp gpurun_out/r4_pmc_T.json gpurun_out/r4_pmc_C3.json $F/ && cp $F/r4_pmc_T.json $F/r4_pmc_C3.json profiles/ || exit 3
for wl in T C2 C3 C4; do
  extra=""; [ $wl = T ] || extra="--no-c1 --no-e2e"; [ $wl = C2 -o $wl = C4 ] && extra="$extra --no-cpu-baseline"
  timeout -k 10 600 python3 bench.py --workload $wl --steps 20 --warmup 5 $extra > $F/bench_$wl.json 2> $F/bench_$wl.err || { tail -5 $F/bench_$wl.err; exit 4; }
done
timeout -k 10 600 python3 bench.py --workload C5 --steps 10 --warmup 3 > $F/bench_C5_n1.json 2> $F/bench_C5_n1.err || { tail -5 $F/bench_C5_n1.err; exit 5; }
for wl in T C3 C4; do
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $F/kstats_$wl -o run --output-format csv -- python3 $R/bench.py --workload $wl --steps 20 --warmup 5 --no-cpu-baseline --no-e2e --no-c1 > $F/kstats_$wl.log 2>&1 || { tail -5 $F/kstats_$wl.log; exit 6; }
  cd $R
done
echo done
