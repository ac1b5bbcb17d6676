#!/bin/bash
# Round-6 record set on one box, each step under its own limit, stopping at the first failure:
#   pmc    FETCH_SIZE / WRITE_SIZE passes (one rocprofv3 run per counter): T (ceiling + parse,
#          scripts/diag_ceiling.py), C3, C2, C4 (bench.py parse only) -> gpurun_out/r6_pmc_{T,C3,C2,C4}.json
#   kstats rocprofv3 --kernel-trace --stats of the T (default command), C3 and C4 bench lines
#   bench  the bench lines: T (default command: CPU baseline, e2e, pipelined chain), C2, C3, C4, C5 at N = 1
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$(pwd); O=$R/gpurun_out; mkdir -p $O; export TMPDIR=/tmp
for step in "$@"; do
  echo "== $step $(date +%T)"
  case $step in
    pmc)
      cd /tmp
      for c in FETCH_SIZE WRITE_SIZE; do
        timeout -s KILL 120 rocprofv3 --pmc $c -d "$O/pmc_T_$c" -o run --output-format csv \
          -- python3 "$R/scripts/diag_ceiling.py" T > "$O/pmc_T_$c.log" 2>&1 || { echo "STOP pmc T $c"; exit 3; }
        for wl in C3 C2 C4; do
          timeout -s KILL 180 rocprofv3 --pmc $c -d "$O/pmc_${wl}_$c" -o run --output-format csv \
            -- python3 "$R/bench.py" --workload $wl --steps 5 --warmup 2 --no-cpu-baseline --no-c1 --no-e2e --no-cdr \
               --no-ingest --no-frag > "$O/pmc_${wl}_$c.log" 2>&1 || { echo "STOP pmc $wl $c"; exit 3; }
        done
      done
      cd $R
      python3 scripts/pmc_summary.py $O/pmc_T T > $O/r6_pmc_T.json || exit 3
      for wl in C3 C2 C4; do python3 scripts/pmc_summary.py $O/pmc_$wl $wl $O/r6_pmc_T.json > $O/r6_pmc_$wl.json || exit 3; done
      rm -rf $O/pmc_T_* $O/pmc_C3_* $O/pmc_C2_* $O/pmc_C4_*
      python3 -c "
import json
for w in ('T','C3','C2','C4'):
    d=json.load(open('$O/r6_pmc_%s.json' % w)); print(w, {k: {c: round(v/1e6, 1) for c, v in x.items() if c != 'grid'} for k, x in d.items() if isinstance(x, dict)}, d.get('fetch_scale'))" ;;
    kstats)
      for wl in T C3 C4; do
        args="--no-c1 --no-e2e --no-cpu-baseline"; [ $wl = T ] || args="$args --workload $wl"
        (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/kt_$wl -o run --output-format csv \
           -- python3 $R/bench.py $args > $O/r6_prof_bench_$wl.json 2> $O/kt_$wl.err) \
           || { echo "STOP $wl"; tail -5 $O/kt_$wl.err; exit 4; }
        f=$(find $O/kt_$wl -name "*kernel_stats.csv" | head -1)
        cp "$f" $O/r6_bench_${wl}_kernel_stats.csv
        rm -rf $O/kt_$wl
        echo "$wl kernel stats done"
      done ;;
    bench)
      timeout -k 10 600 python bench.py > $O/r6_bench_T.json 2> $O/r6_bench_T.err || { tail -20 $O/r6_bench_T.err; exit 5; }
      for wl in C2 C3 C4; do
        timeout -k 10 600 python bench.py --workload $wl --no-c1 > $O/r6_bench_$wl.json 2> $O/r6_bench_$wl.err || { tail -20 $O/r6_bench_$wl.err; exit 5; }
      done
      timeout -k 10 900 python bench.py --workload C5 --steps 10 --warmup 3 > $O/r6_bench_C5_n1.json 2> $O/r6_bench_C5_n1.err || { tail -20 $O/r6_bench_C5_n1.err; exit 5; }
      for f in T C2 C3 C4 C5_n1; do python3 scripts/bench_summary.py $O/r6_bench_$f.json || true; done ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
