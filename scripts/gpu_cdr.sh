#!/bin/bash
# CDR decode (a18) on the GPU box: parity tests + decode timing on T / C2 / C3.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_cdr_gpu.py -m gpu -x -q > gpurun_out/pytest_cdr.log 2>&1; rc=$?
tail -30 gpurun_out/pytest_cdr.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP pytest (exit $rc)"; exit $rc; fi
for wl in T C2 C3; do
  timeout -k 10 200 python bench.py --workload $wl --no-cpu-baseline --no-e2e --steps 20 > gpurun_out/bench_cdr_$wl.log 2>&1 || { echo "STOP bench $wl"; tail -20 gpurun_out/bench_cdr_$wl.log; exit 3; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/bench_cdr_$wl.log').read().strip().splitlines()[-1]); print('$wl', d['value'], json.dumps(d.get('cdr_decode')))"
done
