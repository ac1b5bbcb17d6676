#!/bin/bash
# Same-box A/B of two builds of the library on the back-to-back step time (scripts/diag_step_gap.py):
# build/librtps_base.so (the previous source) against the in-tree library.  Usage: gpu_ab_step.sh WL [match]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$PWD; mkdir -p gpurun_out
for rep in 1 2; do
  for lib in build/librtps_base.so rustdds-io_uring_amd/librtps_rx.so; do
    echo "== $lib"
    RTPS_RX_LIB=$R/$lib timeout -k 10 100 python scripts/diag_step_gap.py "$@" > gpurun_out/ab_step.log 2>&1 \
      || { tail -5 gpurun_out/ab_step.log; exit 4; }
    grep "^ev2" gpurun_out/ab_step.log
  done
done
