#!/bin/bash
# rocprofv3 kernel trace of bench.py for each workload in $WORKLOADS; prints per-kernel avg us.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
python -c "import __graft_entry__ as g; g.build()" || exit 2
if [ "${RUN_TESTS:-0}" = 1 ]; then
  timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?
  tail -3 gpurun_out/pytest_gpu.log; [ $rc -le 1 ] || exit $rc
fi
cd /tmp
for wl in ${WORKLOADS:-T C3}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_$wl" -o run --output-format csv \
    -- python3 "$R/bench.py" --workload $wl --steps 20 --warmup 5 --no-cpu-baseline --no-e2e $BENCH_ARGS > "$R/gpurun_out/prof_$wl.log" 2>&1 || { echo "STOP $wl"; exit 3; }
  echo "== $wl: $(tail -1 $R/gpurun_out/prof_$wl.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("%.2f Gdgram/s, step %.1f us" % (d["value"]/1e9, d["ms_per_step"]*1e3))')"
  python3 - "$R/gpurun_out/prof_$wl" <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Name"]
        if "rtps_" in n or "bucket" in n:
            print("   %-40s calls %4s avg %8.1f us" % (n.split("::")[1].split("(")[0] if "::" in n else n[:40], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
done
