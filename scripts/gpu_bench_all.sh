#!/bin/bash
# bench.py on every single-GPU workload (round-3 profile set): gpu_bench_all.sh <tag>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
tag=${1:-r3}
for wl in C4 C3 C2; do
  timeout -k 10 300 python bench.py --workload $wl --steps 20 --warmup 5 --no-c1 --no-e2e --no-cpu-baseline \
    > gpurun_out/${tag}_bench_$wl.json 2> gpurun_out/${tag}_bench_$wl.err || exit $?
done
timeout -k 10 400 python bench.py > gpurun_out/${tag}_bench_T.json 2> gpurun_out/${tag}_bench_T.err || exit $?
