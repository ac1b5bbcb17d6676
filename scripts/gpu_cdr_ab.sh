#!/bin/bash
# CDR decode A/B on the box: the product library and each rustdds-io_uring_amd/variants/*.so
# (decode parity tests first, then the bench decode leg on $WLS, twice, interleaved).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
WLS=${WLS:-"T C2"}
libs="$PWD/rustdds-io_uring_amd/librtps_rx.so $(ls $PWD/rustdds-io_uring_amd/variants/*.so 2>/dev/null)"
for v in $libs; do
  n=$(basename "$v" .so); [ "$n" = librtps_rx ] && continue
  RTPS_RX_LIB=$v timeout -k 10 300 python -u -m pytest tests/test_cdr_gpu.py -m gpu -x -q --timeout 200 \
    --timeout-method thread > gpurun_out/pytest_cdr_$n.log 2>&1 || { echo "$n parity FAILED"; tail -5 gpurun_out/pytest_cdr_$n.log; exit 5; }
done
for round in 1 2; do
  for v in $libs; do
    n=$(basename "$v" .so)
    for wl in $WLS; do
      RTPS_RX_LIB=$v timeout -k 10 200 python bench.py --workload $wl --no-c1 --no-cpu-baseline --no-e2e --no-ingest \
        --no-frag --steps 10 --warmup 3 > gpurun_out/cdrab_${n}_$wl.json 2>&1 || exit 4
      python3 -c "import json; d=json.loads([l for l in open('gpurun_out/cdrab_${n}_$wl.json') if l.startswith('{')][-1]); c=d['cdr_decode']; print('$n $wl cdr %.1f us %.0f GB/s' % (c['kernel_ms']*1e3, c['achieved_gbs']))"
    done
  done
done
