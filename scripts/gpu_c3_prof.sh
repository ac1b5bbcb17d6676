#!/bin/bash
# C3 line under rocprofv3 --kernel-trace --stats (ingest, topic caches, SPDP leg): gpu_c3_prof.sh <tag>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
tag=${1:-r6}
(cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/kt_c3 -o run --output-format csv \
   -- python3 $R/bench.py --workload C3 --steps 20 --warmup 5 --no-cpu-baseline --no-c1 --no-e2e \
   > $R/gpurun_out/${tag}_prof_bench_C3.json 2> $R/gpurun_out/kt_c3.err) || { tail -5 gpurun_out/kt_c3.err; exit 4; }
f=$(find gpurun_out/kt_c3 -name "*kernel_stats.csv" | head -1)
cp "$f" gpurun_out/${tag}_bench_C3_kernel_stats.csv
rm -rf gpurun_out/kt_c3
