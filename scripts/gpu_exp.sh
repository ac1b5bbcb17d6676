#!/bin/bash
# Parametrised GPU steps (round 5): scripts/gpu_exp.sh STEP [STEP ...], each step under its own
# time limit, stopping at the first failure.  Outputs under gpurun_out/exp/.
#   parity_mixed   the mixed-pass parity subset of tests/test_gpu_parity.py
#   c3_emit        C3 bench lines for each record pass (RTPS_RX_EMIT=1/2/3)
#   kstats_C3      rocprofv3 kernel-trace stats of the C3 bench
#   gpu_tests      the whole -m gpu suite
shopt -s nullglob  # (no variants: the loops run the in-tree library only)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$(pwd); O=$R/gpurun_out/exp; mkdir -p $O; export TMPDIR=/tmp
PYT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
for step in "$@"; do
  echo "== $step $(date +%T)"
  case $step in
    parity_mixed)
      timeout -k 10 600 $PYT tests/test_gpu_parity.py -k "mixed or chained_launch or lds_tile or soup or edge or reader_sets or full_size or launch_choice or spec_hint or golden or record_passes" > $O/parity_mixed.log 2>&1 \
        || { tail -30 $O/parity_mixed.log; exit 3; }
      tail -2 $O/parity_mixed.log ;;
    c3_emit)
      for e in ${EMITS:-1 2 3 4 5}; do
        RTPS_RX_EMIT=$e timeout -k 10 300 python bench.py --workload C3 --steps 20 --warmup 5 --no-c1 --no-e2e --no-cpu-baseline --no-ingest --no-cdr > $O/c3_emit$e.json 2> $O/c3_emit$e.err || { tail -5 $O/c3_emit$e.err; exit 4; }
        python - $O/c3_emit$e.json $e <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("emit", sys.argv[2], "ms_per_step", d["ms_per_step"], {k: v for k, v in d.get("roofline", {}).items() if k in ("kernel", "achieved", "frac")},
      {k: d.get(k) for k in ("item_kernel_ms", "scan_plus_emit_ms")}, d.get("parse_kernels", ""))
PY
      done ;;
    c3_var)  # the in-tree library, then every tuning variant under rustdds-io_uring_amd/variants/, RTPS_RX_EMIT as set
      for lib in $R/rustdds-io_uring_amd/librtps_rx.so $R/rustdds-io_uring_amd/variants/librtps_rx_*.so $R/rustdds-io_uring_amd/librtps_rx.so; do
        v=$(basename $lib .so)  # the in-tree library twice: the first run of a fresh box reads ~15 us slow
        RTPS_RX_LIB=$lib timeout -k 10 300 python bench.py --workload C3 --steps 20 --warmup 5 --no-c1 --no-e2e --no-cpu-baseline --no-ingest --no-cdr > $O/c3_$v.json 2> $O/c3_$v.err || { tail -5 $O/c3_$v.err; exit 4; }
        python - $O/c3_$v.json $v <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r = d["roofline"]
print(sys.argv[2], "step", round(d["ms_per_step"] * 1e3, 1), "us", {k: round(r[k] * 1e3, 1) for k in ("item_kernel_ms", "emit_kernel_ms", "scan_ms") if k in r})
PY
      done ;;
    t_var)  # as c3_var on the T workload (spec A+B pass)
      for lib in $R/rustdds-io_uring_amd/librtps_rx.so $R/rustdds-io_uring_amd/variants/librtps_rx_*.so $R/rustdds-io_uring_amd/librtps_rx.so; do
        v=$(basename $lib .so)
        RTPS_RX_LIB=$lib timeout -k 10 300 python bench.py --workload T --steps 20 --warmup 5 --no-c1 --no-e2e --no-cpu-baseline --no-ingest --no-cdr > $O/t_$v.json 2> $O/t_$v.err || { tail -5 $O/t_$v.err; exit 4; }
        python - $O/t_$v.json $v <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r = d["roofline"]
print(sys.argv[2], "step", round(d["ms_per_step"] * 1e3, 1), "us", "frac", round(r["frac"], 3), "kernel_us", round(r.get("kernel_ms", 0) * 1e3, 1))
PY
      done ;;
    ing_var)  # C3 and T parse + ingest for the in-tree library and every variant (RTPS_RX_LIB)
      for wl in C3 T; do
      for lib in $R/rustdds-io_uring_amd/librtps_rx.so $R/rustdds-io_uring_amd/variants/librtps_rx_*.so $R/rustdds-io_uring_amd/librtps_rx.so; do
        v=$(basename $lib .so)
        RTPS_RX_LIB=$lib timeout -k 10 300 python bench.py --workload $wl --steps 20 --warmup 5 --no-c1 --no-e2e --no-cpu-baseline --no-cdr > $O/ing_${wl}_$v.json 2> $O/ing_${wl}_$v.err || { tail -5 $O/ing_${wl}_$v.err; exit 4; }
        python - $O/ing_${wl}_$v.json $v $wl <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); g = d["ingest"]
print(sys.argv[3], sys.argv[2], "step", round(d["ms_per_step"] * 1e3, 1), "us ingest", round(g["ms"] * 1e3, 1), "tc", round(g["topic_cache_ms"] * 1e3, 1))
PY
      done; done ;;
    pmc)  # FETCH / WRITE passes of T (ceiling + parse) and C3 -> gpurun_out/r${ROUND}_pmc_{T,C3}.json
      ROUND=${ROUND:-5} timeout -k 10 700 bash scripts/gpu_pmc.sh > $O/pmc.log 2>&1 || { tail -5 $O/pmc.log; exit 12; }
      cp gpurun_out/r${ROUND:-5}_pmc_T.json gpurun_out/r${ROUND:-5}_pmc_C3.json $O/ ;;
    bench_C5)
      timeout -k 10 600 python bench.py --workload C5 --steps 10 --warmup 3 > $O/bench_C5.json 2> $O/bench_C5.err || { tail -20 $O/bench_C5.err; exit 10; }
      tail -c 600 $O/bench_C5.json ;;
    kstats_T|kstats_C4)
      wl=${step#kstats_}
      cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kstats_$wl -o run --output-format csv -- python3 $R/bench.py --workload $wl --steps 20 --warmup 5 --no-cpu-baseline --no-e2e --no-c1 > $O/kstats_$wl.log 2>&1 || { tail -5 $O/kstats_$wl.log; exit 6; }
      cd $R; python scripts/prof_table.py $(find $O/kstats_$wl -name "*kernel_stats.csv") | head -30 ;;
    kstats_C3)
      cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kstats_C3 -o run --output-format csv -- python3 $R/bench.py --workload C3 --steps 20 --warmup 5 --no-cpu-baseline --no-e2e --no-c1 > $O/kstats_C3.log 2>&1 || { tail -5 $O/kstats_C3.log; exit 6; }
      cd $R; python scripts/prof_table.py $(find $O/kstats_C3 -name "*kernel_stats.csv") | head -40 ;;
    shard)
      timeout -k 10 900 $PYT tests/test_shard_gpu.py > $O/shard.log 2>&1 || { grep -E "FAILED|Error" $O/shard.log | head; tail -30 $O/shard.log; exit 7; }
      tail -2 $O/shard.log ;;
    topic)
      timeout -k 10 900 $PYT tests/test_topic_gpu.py tests/test_cdr_gpu.py > $O/topic.log 2>&1 || { grep -E "FAILED|Error" $O/topic.log | head; tail -30 $O/topic.log; exit 8; }
      tail -2 $O/topic.log ;;
    rccl_probe)
      timeout -k 10 300 python -m torch.distributed.run --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 scripts/rccl_size_probe.py > $O/rccl_probe.log 2>&1 || { tail -20 $O/rccl_probe.log; exit 9; }
      grep rccl_p2p_size_probe $O/rccl_probe.log ;;
    bench_T|bench_C3|bench_C2|bench_C4)
      wl=${step#bench_}; extra=""
      [ $wl = T ] || extra="--no-c1"
      timeout -k 10 600 python bench.py --workload $wl --steps 20 --warmup 5 $extra > $O/bench_$wl.json 2> $O/bench_$wl.err || { tail -20 $O/bench_$wl.err; exit 10; }
      python scripts/bench_summary.py $O/bench_$wl.json ;;
    diag_tests)  # the rejected mixed passes, in their diagnostic build (make variant NAME=passes VDEFS=-DRTPS_DIAG_PASSES)
      RTPS_RX_LIB=$R/rustdds-io_uring_amd/variants/librtps_rx_passes.so RTPS_RX_DIAG_PASSES=1 timeout -k 10 900 $PYT tests/diag_mixed_passes.py tests/test_gpu_parity.py -k "mixed or record_passes or lds_tile or chained" > $O/diag_tests.log 2>&1 || { grep -E "FAILED|Error" $O/diag_tests.log | head; tail -20 $O/diag_tests.log; exit 11; }
      tail -2 $O/diag_tests.log ;;
    gpu_tests)
      timeout -k 10 1000 $PYT tests -m gpu > $O/gpu_tests.log 2>&1 || { grep -E "FAILED|Error" $O/gpu_tests.log | head; tail -5 $O/gpu_tests.log; exit 5; }
      tail -2 $O/gpu_tests.log ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo done
