#!/bin/bash
# Ingest experiments: parity of the product build, then per-kernel times of T ingest
# for the product build and tuning variants (RTPS_RX_LIB).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_ingest_gpu.py tests/test_topic_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/exp_ing_pytest.log 2>&1; rc=$?
tail -2 gpurun_out/exp_ing_pytest.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/exp_ing_pytest.log | head -20; exit $rc; }
for v in product ${VARIANTS:-nomark nomerge}; do
  if [ $v = product ]; then unset RTPS_RX_LIB; else export RTPS_RX_LIB=$R/rustdds-io_uring_amd/variants/librtps_rx_$v.so; fi
  for wl in ${WLS:-T}; do
    cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/exp_prof_${v}_$wl -o run --output-format csv -- python3 $R/bench.py --workload $wl --steps 20 --warmup 5 --no-cpu-baseline --no-e2e --no-c1 --no-cdr > $R/gpurun_out/exp_${v}_$wl.json 2> $R/gpurun_out/exp_${v}_$wl.err || { tail -5 $R/gpurun_out/exp_${v}_$wl.err; exit 6; }
  done
done
echo done
