#!/bin/bash
# CDR decode: ablation timings + PMC traffic (separate kernel-trace-only passes per counter).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
mkdir -p gpurun_out/cdr_pmc
export TMPDIR=/tmp
bash scripts/gpu_cdr_variants.sh || exit 3
cd /tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 200 rocprofv3 --kernel-trace --pmc $c -d "$R/gpurun_out/cdr_pmc/$c" -o run --output-format csv \
    -- python3 "$R/bench.py" --workload T --no-cpu-baseline --no-e2e --steps 5 --warmup 2 > "$R/gpurun_out/cdr_pmc/$c.log" 2>&1 || { echo "STOP pmc $c"; exit 4; }
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/cdr_pmc/stats" -o run --output-format csv \
  -- python3 "$R/bench.py" --workload T --no-cpu-baseline --no-e2e --steps 20 --warmup 3 > "$R/gpurun_out/cdr_pmc/stats.log" 2>&1 || exit 5
find "$R/gpurun_out/cdr_pmc" -name "*.csv" | head -20
