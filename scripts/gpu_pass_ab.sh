#!/bin/bash
# Same-box A/B of the chained passes for mixed traffic (RTPS_RX_MIXED_PASS: 0 lane walk C,
# 2 pipelined lane walk E): parity of the passes first, then bench.py C3 alternating.
# Usage: gpu_pass_ab.sh [passes] (default "0 2")
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
PASSES=${1:-"0 2"}
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread \
  -k "mixed_passes or fallback_to_fix or chained" > gpurun_out/pass_parity.log 2>&1 \
  || { echo "parity FAILED"; grep -E "^E |FAILED|passed|failed" gpurun_out/pass_parity.log | head -20; exit 5; }
grep -E "passed|failed" gpurun_out/pass_parity.log | tail -1
for round in 1 2; do
  for m in $PASSES; do
    RTPS_RX_MIXED_PASS=$m timeout -k 10 200 python bench.py --workload ${WL:-C3} --no-c1 --no-cpu-baseline --no-e2e \
      --no-cdr --no-ingest --no-frag > gpurun_out/pass_${m}.json 2> gpurun_out/pass_${m}.err || { tail -5 gpurun_out/pass_${m}.err; exit 4; }
    python3 -c "import json; d=json.loads([l for l in open('gpurun_out/pass_${m}.json') if l.startswith('{')][-1]); r=d['roofline']; print('pass $m', r['kernel'], 'kernel %.1f us' % (r['kernel_ms']*1e3), 'step %.1f us' % (d['ms_per_step']*1e3), 'att2 %.3f' % r.get('attainable_frac_two_walk', 0))"
  done
done
