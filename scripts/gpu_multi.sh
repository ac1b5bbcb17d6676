#!/bin/bash
# Multi-rank rehearsal on a 1-GPU box: sharded parity (gloo, contiguous + padded),
# padded bucket test, and bench.py --gpus 2 over gloo (2 ranks on one GPU).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
true; rc=0

[ $rc -ne 0 ] && { echo "STOP pytest ($rc)"; exit $rc; }
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 2 --steps 10 --warmup 3 --backend gloo --datagrams 262144 > gpurun_out/bench_n2_gloo.log 2>&1 || { echo "STOP bench n2"; tail -30 gpurun_out/bench_n2_gloo.log; exit 3; }
tail -1 gpurun_out/bench_n2_gloo.log
