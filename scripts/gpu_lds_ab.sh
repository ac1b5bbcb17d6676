#!/bin/bash
# LDS-tile mixed pass: GPU parity (test_gpu_parity.py), then the C3 bench with the LDS
# tiles (D) and the lane walk (C) on the same box, plus the tile-size variants built by
# `make variant` (rustdds-io_uring_amd/variants/*.so; parity of D checked for each first).
# Prebuilt in-tree libraries.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_parity.log 2>&1; rc=$?
grep -E "passed|failed" gpurun_out/pytest_parity.log | tail -2
[ $rc -ne 0 ] && { grep -E "^E |FAILED" gpurun_out/pytest_parity.log | head -20; exit $rc; }
bench() {  # label, env...
  local label=$1; shift
  env "$@" timeout -k 10 200 python bench.py --workload C3 --no-c1 --no-cpu-baseline --no-e2e --no-cdr \
    --no-ingest > gpurun_out/bench_C3_$label.json 2>&1 || return 4
  python3 -c "import json; d=json.loads(open('gpurun_out/bench_C3_$label.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$label', r['kernel'], 'kernel %.1f us' % (r['kernel_ms']*1e3), 'step %.1f us' % (d['ms_per_step']*1e3), '%.2f Gdgram/s' % (d['value']/1e9))"
}
bench mp1 RTPS_RX_MIXED_PASS=1 && bench mp0 RTPS_RX_MIXED_PASS=0 || exit 4
for v in rustdds-io_uring_amd/variants/*.so; do
  [ -e "$v" ] || continue
  n=$(basename "$v" .so); n=${n#librtps_rx_}
  if [[ $n == *stamps* ]]; then  # phase timing of D (tuning builds with RTPS_LDS_STAMPS)
    lt=32; [[ $n == lt16* ]] && lt=16
    LT=$lt RTPS_RX_LIB=$PWD/$v timeout -k 10 120 python scripts/lds_stamps.py > gpurun_out/stamps_$n.txt 2>&1 \
      || { echo "$n stamps FAILED"; tail -5 gpurun_out/stamps_$n.txt; exit 6; }
    cat gpurun_out/stamps_$n.txt; continue
  fi
  RTPS_RX_LIB=$PWD/$v timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 \
    --timeout-method thread -k "mixed_passes or lds_tile or full_size_parity or chained_fallback" \
    > gpurun_out/pytest_$n.log 2>&1 || { echo "$n parity FAILED"; grep -E "^E |FAILED" gpurun_out/pytest_$n.log | head; exit 5; }
  bench "$n" RTPS_RX_LIB=$PWD/$v || exit 4
done
