#!/bin/bash
# Round 4: parity (ingest/topic/frag/shard; the mixed passes incl. the record-slab pass), T / C3
# profiles of the product build, then the record-slab pass (mixed pass 3) at 6 / 5 / 4 waves per SIMD.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
V=$R/rustdds-io_uring_amd/variants
timeout -k 10 900 python -u -m pytest tests/test_ingest_gpu.py tests/test_topic_gpu.py tests/test_frag_gpu.py tests/test_shard_gpu.py -x -q --timeout 400 -k "not past_64" --timeout-method thread > gpurun_out/d_pytest.log 2>&1; rc=$?
tail -2 gpurun_out/d_pytest.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/d_pytest.log | head -30; exit $rc; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "mixed or chained or lds or soup or edge or reader_sets or full_size or launch_choice or spec_hint" > gpurun_out/d_parity.log 2>&1; rc=$?
tail -2 gpurun_out/d_parity.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/d_parity.log | head -30; exit $rc; }
prof() {  # name lib workload mixed_pass
  if [ "$2" = product ]; then unset RTPS_RX_LIB; else export RTPS_RX_LIB=$V/librtps_rx_$2.so; fi
  cd /tmp && RTPS_RX_MIXED_PASS=$4 timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/dprof_$1 -o run --output-format csv -- python3 $R/bench.py --workload $3 --steps 20 --warmup 5 --no-cpu-baseline --no-e2e --no-c1 > $R/gpurun_out/dprof_$1.json 2> $R/gpurun_out/dprof_$1.err || { tail -5 $R/gpurun_out/dprof_$1.err; exit 6; }
  cd $R
}
prof T product T 2 && prof C3 product C3 2 && prof rs6_C3 product C3 3 && prof rs5_C3 rs5 C3 3 && prof rs4_C3 rs4 C3 3
unset RTPS_RX_LIB
timeout -k 10 300 python -u -m pytest tests/test_frag_gpu.py -x -q --timeout 200 --timeout-method thread -k past_64 > gpurun_out/d_past64.log 2>&1; tail -3 gpurun_out/d_past64.log
echo done
