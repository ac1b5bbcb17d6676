#!/bin/bash
# Parse A/B on the box: the product library and each `make variant` build
# (rustdds-io_uring_amd/variants/*.so): parity subset first, then bench.py on the
# workloads in $WLS (default "T C3"), twice, interleaved.  Prebuilt in-tree libraries.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
WLS=${WLS:-"T C3"}
libs="$PWD/rustdds-io_uring_amd/librtps_rx.so $(ls $PWD/rustdds-io_uring_amd/variants/*.so 2>/dev/null)"
for v in $libs; do
  n=$(basename "$v" .so)
  [ "$n" = librtps_rx ] && continue
  RTPS_RX_LIB=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 \
    --timeout-method thread -k "full_size_parity or chained or mixed_passes or golden" > gpurun_out/pytest_$n.log 2>&1 \
    || { echo "$n parity FAILED"; grep -E "^E |FAILED" gpurun_out/pytest_$n.log | head; exit 5; }
done
for round in 1 2; do
  for v in $libs; do
    n=$(basename "$v" .so)
    for wl in $WLS; do
      RTPS_RX_LIB=$v timeout -k 10 200 python bench.py --workload $wl --no-c1 --no-cpu-baseline --no-e2e --no-cdr \
        --no-ingest --no-frag > gpurun_out/ab_${n}_$wl.json 2>&1 || exit 4
      python3 -c "import json; d=json.loads([l for l in open('gpurun_out/ab_${n}_$wl.json') if l.startswith('{')][-1]); r=d['roofline']; print('$n $wl', r['kernel'], 'kernel %.1f us' % (r['kernel_ms']*1e3), 'step %.1f us' % (d['ms_per_step']*1e3))"
    done
  done
done
