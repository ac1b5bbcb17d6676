#!/bin/bash
# DataFrag reassembly A/B on the box: the product library and each tuning variant
# (rustdds-io_uring_amd/variants/*.so, `make variant`): frag parity tests, then the
# C4 bench's frag_assemble leg, twice, interleaved.  Prebuilt in-tree libraries.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
libs="$PWD/rustdds-io_uring_amd/librtps_rx.so $(ls $PWD/rustdds-io_uring_amd/variants/*.so 2>/dev/null)"
for v in $libs; do
  n=$(basename "$v" .so)
  RTPS_RX_LIB=$v timeout -k 10 300 python -u -m pytest tests/test_frag_gpu.py -m gpu -x -q --timeout 200 \
    --timeout-method thread > gpurun_out/pytest_frag_$n.log 2>&1 || { echo "$n parity FAILED"; grep -E "^E " gpurun_out/pytest_frag_$n.log | head; exit 5; }
done
for round in $(seq ${ROUNDS:-2}); do
  for v in $libs; do
    n=$(basename "$v" .so)
    RTPS_RX_LIB=$v timeout -k 10 200 python bench.py --workload C4 --no-c1 --no-cpu-baseline --no-e2e --no-cdr \
      --no-ingest > gpurun_out/frag_$n.json 2>&1 || exit 4
    python3 -c "import json; d=json.loads([l for l in open('gpurun_out/frag_$n.json') if l.startswith('{')][-1]); f=d['frag_assemble']; print('$n', 'frag %.3f ms' % f['ms'], '%.2f TB/s alg' % (f['achieved_gbs']/1e3))"
  done
done
