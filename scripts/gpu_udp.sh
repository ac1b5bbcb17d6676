#!/bin/bash
# UDP receive -> zero-copy GPU parse: parity tests, then the C1 loopback bench leg.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_udp_gpu.py tests/test_pump_gpu.py tests/test_udp.py -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_udp.log 2>&1; rc=$?
tail -12 gpurun_out/pytest_udp.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --workload C2 --steps 10 --no-cpu-baseline --no-e2e --no-cdr --no-frag --no-ingest \
  > gpurun_out/bench_c1.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_c1.log; exit 4; }
python -c "import json; d=json.loads(open('gpurun_out/bench_c1.log').read().strip().splitlines()[-1]); print(json.dumps(d.get('c1_loopback'), indent=1))"
