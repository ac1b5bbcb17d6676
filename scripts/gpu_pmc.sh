#!/bin/bash
# PMC passes (one rocprofv3 run per counter, --pmc only) over
#   T : scripts/diag_ceiling.py T  (ceiling kernels + the T parse, 1M datagrams)
#   C3: bench.py --workload C3     (the chained parse, 1M datagrams)
# then profiles/r${ROUND}_pmc_{T,C3}.json via scripts/pmc_summary.py.  Prebuilt in-tree libraries.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
ROUND=${ROUND:-2}
cd /tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c -d "$R/gpurun_out/pmc_T_$c" -o run --output-format csv \
    -- python3 "$R/scripts/diag_ceiling.py" T > "$R/gpurun_out/pmc_T_$c.log" 2>&1 || { echo "STOP pmc T $c"; exit 3; }
  timeout -s KILL 180 rocprofv3 --pmc $c -d "$R/gpurun_out/pmc_C3_$c" -o run --output-format csv \
    -- python3 "$R/bench.py" --workload C3 --steps 5 --warmup 2 --no-cpu-baseline --no-c1 --no-e2e --no-cdr \
       --no-ingest > "$R/gpurun_out/pmc_C3_$c.log" 2>&1 || { echo "STOP pmc C3 $c"; exit 3; }
done
python3 "$R/scripts/pmc_summary.py" "$R/gpurun_out/pmc_T" T > "$R/gpurun_out/r${ROUND}_pmc_T.json" &&
python3 "$R/scripts/pmc_summary.py" "$R/gpurun_out/pmc_C3" C3 "$R/gpurun_out/r${ROUND}_pmc_T.json" \
  > "$R/gpurun_out/r${ROUND}_pmc_C3.json" && cat "$R/gpurun_out/r${ROUND}_pmc_T.json" "$R/gpurun_out/r${ROUND}_pmc_C3.json"
