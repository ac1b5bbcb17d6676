#!/bin/bash
# Quick GPU check: parse parity subset + match/no-match bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -m gpu -x -q > gpurun_out/pytest_quick.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_quick.log
[ $rc -ne 0 ] && exit $rc
for m in none writers; do
  timeout -k 10 300 python bench.py --steps 30 --no-cpu-baseline --no-e2e --no-cdr --match $m > gpurun_out/bench_m_$m.log 2>&1 || exit 4
  python -c "import json; d=json.loads(open('gpurun_out/bench_m_$m.log').read().strip().splitlines()[-1]); print('$m', d['value'], d['roofline']['kernel_ms'])"
done
