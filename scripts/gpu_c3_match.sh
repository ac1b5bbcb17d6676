#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
cd /tmp
for m in none writers; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_m_$m" -o run --output-format csv \
    -- python3 "$R/bench.py" --workload ${WL:-C3} --match $m --steps 20 --warmup 5 --no-cpu-baseline --no-e2e --no-cdr --no-frag > "$R/gpurun_out/prof_m_$m.log" 2>&1 || { echo "STOP $m"; exit 3; }
  python3 - "$R/gpurun_out/prof_m_$m" $m <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Name"]
        if "rtps_parse" in n:
            print("  match=%-8s %-24s avg %7.1f us" % (sys.argv[2], n.split("::")[1].split("(")[0], float(r["AverageNs"]) / 1e3))
PY
done
