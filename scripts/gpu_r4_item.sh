#!/bin/bash
# Round 4: the item pass (E/S/W) for mixed traffic: parity tests, then C3 timings of every pass.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread \
  -k "mixed or chained or lds or soup or edge or reader_sets or full_size or launch_choice or spec_hint" > gpurun_out/r4_item_pytest.log 2>&1; rc=$?
tail -5 gpurun_out/r4_item_pytest.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/r4_item_pytest.log | head -20; exit $rc; }
for mp in 2 0; do
  RTPS_RX_MIXED_PASS=$mp timeout -k 10 300 python bench.py --workload C3 --steps 20 --warmup 5 --no-c1 --no-e2e --no-cpu-baseline --no-cdr --no-ingest > gpurun_out/r4_c3_mp$mp.json 2> gpurun_out/r4_c3_mp$mp.err || { tail -5 gpurun_out/r4_c3_mp$mp.err; exit 4; }
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_C3 -o run --output-format csv -- python3 $R/bench.py --workload C3 --steps 20 --warmup 5 --no-cpu-baseline --no-e2e --no-c1 --no-cdr --no-ingest > $R/gpurun_out/prof_C3.log 2>&1 || exit 6
echo done
