#!/bin/bash
# C3 parse time vs batch size (does the second pass re-read from the Infinity Cache?)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
cd /tmp
for n in 131072 262144 524288 1048576; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_sz_$n" -o run --output-format csv \
    -- python3 "$R/bench.py" --workload C3 --datagrams $n --steps 20 --warmup 5 --no-cpu-baseline --no-e2e --no-cdr --no-frag > "$R/gpurun_out/prof_sz_$n.log" 2>&1 || { echo "STOP $n"; exit 3; }
  python3 - "$R/gpurun_out/prof_sz_$n" $n <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Name"]
        if "rtps_parse" in n:
            us = float(r["AverageNs"]) / 1e3
            print("  n=%8s %-24s avg %7.1f us  (%.1f ns/1k dgram)" % (sys.argv[2], n.split("::")[1].split("(")[0], us, us * 1e3 / int(sys.argv[2]) * 1e3 / 1e3))
PY
done
