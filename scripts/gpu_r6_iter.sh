#!/bin/bash
# Round-6 iteration steps on the box: gpu_r6_iter.sh STEP [STEP ...], each under its own limit,
# stopping at the first failure.  Logs under gpurun_out/r6/.
#   topic      topic-cache + ingest GPU tests
#   wab        W2 variant A/B (scripts/gpu_variant_ab.sh, C3)
#   ing        T and C3 bench lines with the ingest + topic-cache legs (no CPU baseline / C1 / e2e)
#   spdp       C3 bench line's SPDP repeats leg only numbers (part of ing)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$(pwd); O=$R/gpurun_out/r6; mkdir -p $O; export TMPDIR=/tmp
PYT="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
shopt -s nullglob  # (no variants: the variant loops run the in-tree library only)
for step in "$@"; do
  echo "== $step $(date +%T)"
  case $step in
    topic)
      timeout -k 10 900 $PYT tests/test_topic_gpu.py tests/test_ingest_gpu.py tests/test_shard_gpu.py -m gpu > $O/topic.log 2>&1 \
        || { grep -E "FAILED|Error|error" $O/topic.log | head -20; tail -30 $O/topic.log; exit 3; }
      tail -2 $O/topic.log ;;
    wab)
      WLS=C3 timeout -k 10 900 bash scripts/gpu_variant_ab.sh > $O/wab.log 2>&1 || { tail -20 $O/wab.log; exit 4; }
      cat $O/wab.log ;;
    ing)
      for wl in T C3; do
        timeout -k 10 300 python bench.py --workload $wl --steps 20 --warmup 5 --no-c1 --no-e2e --no-cpu-baseline --no-cdr > $O/ing_$wl.json 2> $O/ing_$wl.err || { tail -20 $O/ing_$wl.err; exit 5; }
        python3 - $O/ing_$wl.json $wl <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); g = d["ingest"]
print(sys.argv[2], "step %.1f us" % (d["ms_per_step"] * 1e3), "ingest %.1f us" % (g["ms"] * 1e3),
      "tc_extra %.1f us" % (g["topic_cache_extra_ms"] * 1e3), "stored", g.get("topic_cache_stored"))
s = d.get("topic_cache_spdp_repeats")
if s:
    for k in ("pairs", "halves"):
        v = s[k]; print("  spdp", k, "parity", v["parity_ok"], "ingest %.1f us" % (v["ingest_ms"] * 1e3), "tc_extra %.1f us" % (v["topic_cache_extra_ms"] * 1e3))
PY
      done ;;
    kt_T|kt_C3|kt_C4)  # rocprofv3 kernel stats of one bench line (no CPU baseline / C1 / e2e)
      wl=${step#kt_}
      (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt_$wl -o run --output-format csv \
        -- python3 $R/bench.py --workload $wl --steps 20 --warmup 5 --no-cpu-baseline --no-e2e --no-c1 ${KT_ARGS} > $O/kt_$wl.json 2> $O/kt_$wl.err) \
        || { tail -5 $O/kt_$wl.err; exit 6; }
      f=$(find $O/kt_$wl -name "*kernel_stats.csv" | head -1); cp "$f" $O/kt_${wl}_kernel_stats.csv; rm -rf $O/kt_$wl
      python3 scripts/prof_table.py $O/kt_${wl}_kernel_stats.csv | head -45 ;;
    tl_T|tl_C3)  # rocprofv3 kernel trace (per dispatch) of one bench line, for gap analysis
      wl=${step#tl_}
      (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tl_$wl -o run --output-format csv \
        -- python3 $R/bench.py --workload $wl --steps 6 --warmup 2 --no-cpu-baseline --no-e2e --no-c1 --no-cdr --no-frag > $O/tl_$wl.json 2> $O/tl_$wl.err) \
        || { tail -5 $O/tl_$wl.err; exit 7; }
      f=$(find $O/tl_$wl -name "*kernel_trace.csv" | head -1); cp "$f" $O/tl_${wl}_kernel_trace.csv; rm -rf $O/tl_$wl
      wc -l $O/tl_${wl}_kernel_trace.csv ;;
    probe)  # T ingest legs with the topic step queued normally / not at all / gated off (RTPS_TC_PROBE)
      for pr in ${PROBES:-0 1 2}; do
        RTPS_TC_PROBE=$pr timeout -k 10 300 python bench.py --workload T --steps 20 --warmup 5 --no-c1 --no-e2e --no-cpu-baseline --no-cdr > $O/probe_$pr.json 2> $O/probe_$pr.err || { tail -20 $O/probe_$pr.err; exit 8; }
        python3 -c "import json; d=json.loads(open('$O/probe_$pr.json').read().strip().splitlines()[-1]); g=d['ingest']; print('probe $pr ingest %.1f us tc_extra %.1f us' % (g['ms']*1e3, g['topic_cache_extra_ms']*1e3))"
      done ;;
    cdr)  # C3 CDR decode legs (list / per record), flat kernel vs RTPS_CDR_NESTED=1 (+ CDR_ENV)
      for nest in 0 1; do
        RTPS_CDR_NESTED=$nest timeout -k 10 300 python bench.py --workload C3 --steps 20 --warmup 5 --no-c1 --no-e2e --no-cpu-baseline --no-frag > $O/cdr_$nest.json 2> $O/cdr_$nest.err || { tail -20 $O/cdr_$nest.err; exit 9; }
        python3 -c "import json; d=json.loads(open('$O/cdr_$nest.json').read().strip().splitlines()[-1]); c=d['cdr_decode']; print('nested $nest list %.1f us (%d rows, ok %d) per-record %.1f us' % (c['kernel_ms']*1e3, c['rows'], c['rows_ok'], c['per_record_layout']['kernel_ms']*1e3))"
      done ;;
    cdr_var)  # C3 CDR legs for the product library and each variant (twice, interleaved)
      for wl in ${WLS:-C3}; do
      for round in 1 2; do
      for lib in $R/rustdds-io_uring_amd/librtps_rx.so $R/rustdds-io_uring_amd/variants/librtps_rx_*.so; do
        v=$(basename $lib .so)
        RTPS_RX_LIB=$lib timeout -k 10 300 python bench.py --workload $wl --steps 20 --warmup 5 --no-c1 --no-e2e --no-cpu-baseline --no-frag > $O/cdrv_$v.json 2> $O/cdrv_$v.err || { tail -20 $O/cdrv_$v.err; exit 9; }
        python3 -c "import json; d=json.loads(open('$O/cdrv_$v.json').read().strip().splitlines()[-1]); c=d['cdr_decode']; p=c.get('per_record_layout') or {}; print('$wl $v list %.1f us per-record %.1f us' % (c['kernel_ms']*1e3, (p.get('kernel_ms') or 0)*1e3))"
      done; done; done ;;
    shard)  # owner-side exchange GPU tests
      timeout -k 10 900 $PYT tests/test_shard_gpu.py -m gpu > $O/shard.log 2>&1 || { grep -E "FAILED|Error|error" $O/shard.log | head -20; tail -30 $O/shard.log; exit 10; }
      tail -2 $O/shard.log ;;
    xpred)  # C3 line's exchange prediction (N = 2/4/8) and step
      timeout -k 10 300 python bench.py --workload C3 --steps 20 --warmup 5 --no-c1 --no-e2e --no-cpu-baseline --no-cdr > $O/xpred.json 2> $O/xpred.err || { tail -20 $O/xpred.err; exit 11; }
      python3 -c "import json; d=json.loads(open('$O/xpred.json').read().strip().splitlines()[-1]); x=d['exchange_prediction']; print('C3 step %.1f us' % (d['ms_per_step']*1e3), {k: (round(v['predicted_xgmi_ms'], 3), v['max_bytes_per_peer']) for k, v in x.items() if isinstance(v, dict)})" ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
