#!/bin/bash
# Ingest / topic / frag parity, then T and C3 kernel-trace profiles (product build).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_ingest_gpu.py tests/test_topic_gpu.py tests/test_frag_gpu.py -x -q --timeout 400 --timeout-method thread > gpurun_out/e_pytest.log 2>&1; rc=$?
tail -2 gpurun_out/e_pytest.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/e_pytest.log | head -30; exit $rc; }
for wl in T C3; do
  cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/eprof_$wl -o run --output-format csv -- python3 $R/bench.py --workload $wl --steps 20 --warmup 5 --no-cpu-baseline --no-e2e --no-c1 > $R/gpurun_out/eprof_$wl.json 2> $R/gpurun_out/eprof_$wl.err || { tail -5 $R/gpurun_out/eprof_$wl.err; exit 6; }
  cd $R
done
echo done
