#!/bin/bash
# Round 4 experiments: ingest parity (far sets), the kind-sorted record pass variant's parity,
# then per-kernel times (rocprofv3 kernel trace) of the product build and the tuning variants.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
V=$R/rustdds-io_uring_amd/variants
timeout -k 10 600 python -u -m pytest tests/test_ingest_gpu.py tests/test_topic_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/b_ing_pytest.log 2>&1; rc=$?
tail -2 gpurun_out/b_ing_pytest.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/b_ing_pytest.log | head -30; exit $rc; }
RTPS_RX_LIB=$V/librtps_rx_emsort.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "mixed or soup or full_size or edge" > gpurun_out/b_emsort_pytest.log 2>&1; rc=$?
tail -2 gpurun_out/b_emsort_pytest.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/b_emsort_pytest.log | head -20; exit $rc; }
prof() {  # name lib workload
  if [ "$2" = product ]; then unset RTPS_RX_LIB; else export RTPS_RX_LIB=$V/librtps_rx_$2.so; fi
  cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/bprof_$1 -o run --output-format csv -- python3 $R/bench.py --workload $3 --steps 20 --warmup 5 --no-cpu-baseline --no-e2e --no-c1 --no-cdr > $R/gpurun_out/bprof_$1.json 2> $R/gpurun_out/bprof_$1.err || { tail -5 $R/gpurun_out/bprof_$1.err; exit 6; }
  cd $R
}
prof prod_T product T && prof prod_C3 product C3 && prof nomark_T nomark T && prof nomerge_T nomerge T && prof emsort_C3 emsort C3
unset RTPS_RX_LIB
echo done
