#!/bin/bash
# Parse-kernel time per library variant (build/abl/lib_*.so; "base" = the product library).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
cd /tmp
for v in base $(cd "$R/build/abl" 2>/dev/null && ls lib_*.so | sed 's/^lib_//; s/\.so$//'); do
  if [ "$v" = base ]; then unset RTPS_RX_LIB; else export RTPS_RX_LIB="$R/build/abl/lib_$v.so"; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/abl_$v" -o run --output-format csv \
    -- python3 "$R/bench.py" --workload ${WL:-C3} --steps 20 --warmup 5 --no-cpu-baseline --no-e2e --no-cdr --no-frag $BENCH_ARGS > "$R/gpurun_out/abl_$v.log" 2>&1 || { echo "STOP $v"; tail -3 "$R/gpurun_out/abl_$v.log"; exit 3; }
  python3 - "$R/gpurun_out/abl_$v" $v <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Name"]
        if "rtps_parse" in n:
            print("  %-20s %-24s avg %7.1f us" % (sys.argv[2], n.split("::")[1].split("(")[0], float(r["AverageNs"]) / 1e3))
PY
done
