#!/bin/bash
# Round 4: the item pass (E/S/W) for mixed traffic, topic caches, compact CDR rows, the fused
# ingest path: parity tests, then C3 timings of both mixed passes, T, and a kernel-trace profile.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread \
  -k "mixed or chained or lds or soup or edge or reader_sets or full_size or launch_choice or spec_hint" > gpurun_out/r4_item_pytest.log 2>&1; rc=$?
tail -3 gpurun_out/r4_item_pytest.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/r4_item_pytest.log | head -20; exit $rc; }
timeout -k 10 900 python -u -m pytest tests/test_shard_gpu.py tests/test_topic_gpu.py tests/test_cdr_gpu.py tests/test_ingest_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r4_ing_pytest.log 2>&1; rc=$?
tail -3 gpurun_out/r4_ing_pytest.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/r4_ing_pytest.log | head -20; exit $rc; }
for mp in 2 0; do
  RTPS_RX_MIXED_PASS=$mp timeout -k 10 300 python bench.py --workload C3 --steps 20 --warmup 5 --no-c1 --no-e2e --no-cpu-baseline > gpurun_out/r4_c3_mp$mp.json 2> gpurun_out/r4_c3_mp$mp.err || { tail -5 gpurun_out/r4_c3_mp$mp.err; exit 4; }
done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-c1 --no-e2e --no-cpu-baseline > gpurun_out/r4_T.json 2> gpurun_out/r4_T.err || { tail -5 gpurun_out/r4_T.err; exit 5; }
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_C3 -o run --output-format csv -- python3 $R/bench.py --workload C3 --steps 20 --warmup 5 --no-cpu-baseline --no-e2e --no-c1 > $R/gpurun_out/prof_C3.log 2>&1 || exit 6
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_T -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-e2e --no-c1 > $R/gpurun_out/prof_T.log 2>&1 || exit 7
echo done
