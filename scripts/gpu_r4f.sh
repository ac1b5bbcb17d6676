#!/bin/bash
# Parity (mixed passes with wide items; ingest / topic / frag), then kernel-trace profiles of
# T, C3 (wide items) and C3 with 16-B items (variant build).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
V=$R/rustdds-io_uring_amd/variants
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "mixed or chained or lds or soup or edge or reader_sets or full_size or launch_choice or spec_hint" > gpurun_out/f_parity.log 2>&1; rc=$?
tail -2 gpurun_out/f_parity.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/f_parity.log | head -30; exit $rc; }
timeout -k 10 900 python -u -m pytest tests/test_ingest_gpu.py tests/test_topic_gpu.py tests/test_frag_gpu.py -x -q --timeout 400 --timeout-method thread > gpurun_out/f_pytest.log 2>&1; rc=$?
tail -2 gpurun_out/f_pytest.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/f_pytest.log | head -30; exit $rc; }
prof() {  # name lib workload
  if [ "$2" = product ]; then unset RTPS_RX_LIB; else export RTPS_RX_LIB=$V/librtps_rx_$2.so; fi
  cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/fprof_$1 -o run --output-format csv -- python3 $R/bench.py --workload $3 --steps 20 --warmup 5 --no-cpu-baseline --no-e2e --no-c1 > $R/gpurun_out/fprof_$1.json 2> $R/gpurun_out/fprof_$1.err || { tail -5 $R/gpurun_out/fprof_$1.err; exit 6; }
  cd $R
}
prof T product T && prof C3 product C3 && prof nar_C3 narrow C3
unset RTPS_RX_LIB
echo done
