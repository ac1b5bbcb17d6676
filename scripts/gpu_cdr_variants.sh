#!/bin/bash
# Decode-kernel tuning: every build/cdrvar/*.so on T, C2, C3 (decode leg only).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for lib in build/cdrvar/*.so; do
  for wl in T C2 C3; do
    RTPS_RX_LIB=$PWD/$lib timeout -k 10 120 python bench.py --workload $wl --no-cpu-baseline --no-e2e --steps 10 --warmup 3 > gpurun_out/var.log 2>&1 || { echo "STOP $lib $wl"; tail -5 gpurun_out/var.log; exit 3; }
    python -c "import json; d=json.loads(open('gpurun_out/var.log').read().strip().splitlines()[-1]); c=d['cdr_decode']; print('$(basename $lib)', '$wl', round(c['kernel_ms']*1000,1), 'us', round(c['achieved_gbs']), 'GB/s')"
  done
done
