#!/bin/bash
# Chained launch on C3 with the look-back skipped (ABL_NO_LOOKBACK, wrong output,
# timing only) vs the product build: what waiting for predecessors costs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$PWD; mkdir -p gpurun_out build; export TMPDIR=/tmp
C=rustdds-io_uring_amd/csrc
(cd $C && /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -Wno-unused-function -DABL_NO_LOOKBACK -shared \
   -o $R/build/librtps_nolb.so rtps_rx.hip rtps_cdr.hip rtps_frag.hip rtps_ingest.hip rtps_udp.cpp rtps_pump.cpp) || exit 2
for lib in $C/../librtps_rx.so build/librtps_nolb.so; do
  RTPS_RX_LIB=$R/$lib timeout -k 10 200 python bench.py --workload C3 --spec-hint 0 --steps 30 --no-cpu-baseline --no-e2e \
    --no-cdr --no-frag --no-ingest --no-c1 > gpurun_out/chain_abl.log 2>&1 || { tail -5 gpurun_out/chain_abl.log; exit 4; }
  python -c "import json; d=json.loads(open('gpurun_out/chain_abl.log').read().strip().splitlines()[-1]); print('$lib', 'kernel %.1f us' % (d['roofline']['kernel_ms']*1e3))"
done
