#!/bin/bash
# DataFrag reassembly timing (bench C4 leg) + rocprof kernel breakdown.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --workload C4 --no-cpu-baseline --no-e2e --no-cdr --no-ingest --no-c1 --steps 10 --warmup 3 > gpurun_out/bench_frag.log 2>&1 || { tail -20 gpurun_out/bench_frag.log; exit 3; }
python -c "import json; d=json.loads(open('gpurun_out/bench_frag.log').read().strip().splitlines()[-1]); print(json.dumps(d['frag_assemble']))"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_frag" -o run --output-format csv \
  -- python3 "$R/bench.py" --workload C4 --no-cpu-baseline --no-e2e --no-cdr --no-ingest --no-c1 --steps 10 --warmup 3 > "$R/gpurun_out/prof_frag.log" 2>&1 || exit 4
python3 - "$R/gpurun_out/prof_frag/run_kernel_stats.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"]
    n = n.split("::")[1].split("(")[0] if n.startswith("(anonymous") else n[:90]
    print("%-90s calls %6s avg %9.1f us total %9.1f us" % (n, r["Calls"], float(r["AverageNs"]) / 1e3, float(r["TotalDurationNs"]) / 1e3))
PY
