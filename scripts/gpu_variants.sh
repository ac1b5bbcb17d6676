#!/bin/bash
# A/B of prebuilt kernel variants (build/var/lib_*.so): bench T and C3 for each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "${RUN_TESTS:-1}" = 1 ]; then
  timeout -k 10 300 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?
  tail -3 gpurun_out/pytest_gpu.log; [ $rc -le 1 ] || exit $rc
fi
for rep in 1 2; do
for lib in build/var/lib_*.so; do
  for wl in ${WORKLOADS:-T C3}; do
    RTPS_RX_LIB=$R$lib timeout -k 10 120 python bench.py --workload $wl --no-cpu-baseline --steps 30 > gpurun_out/v.log 2>&1; rc=$?
    [ $rc -le 1 ] || { echo "STOP $lib $wl rc=$rc"; tail -5 gpurun_out/v.log; exit $rc; }
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/v.log').read().strip().splitlines()[-1]); print('$lib', '$wl', 'kernel_us=%.1f'%(d['roofline']['kernel_ms']*1e3), 'Gdgram/s=%.2f'%(d['value']/1e9))"
  done
done
done
