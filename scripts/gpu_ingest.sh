#!/bin/bash
# History-cache ingest: GPU parity tests, then the bench ingest leg on T and C3.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_ingest_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_ingest.log 2>&1; rc=$?
tail -15 gpurun_out/pytest_ingest.log; [ $rc -eq 0 ] || exit $rc
for wl in T C3; do
  timeout -k 10 300 python bench.py --workload $wl --steps 20 --no-cpu-baseline --no-e2e --no-cdr --no-frag --no-c1 \
    > gpurun_out/bench_ingest_$wl.log 2>&1 || { echo "bench $wl failed"; tail -5 gpurun_out/bench_ingest_$wl.log; exit 4; }
  python -c "import json; d=json.loads(open('gpurun_out/bench_ingest_$wl.log').read().strip().splitlines()[-1]); print('$wl', json.dumps(d.get('ingest')))"
done
cd /tmp
for wl in ${PROF_WL:-T C3}; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_ingest_$wl" -o run --output-format csv \
  -- python3 "$R/bench.py" --workload $wl --steps 10 --warmup 2 --no-cpu-baseline --no-e2e --no-cdr --no-frag --no-c1 > "$R/gpurun_out/prof_ingest_$wl.log" 2>&1 || exit 3
echo "== $wl"
python3 - "$R/gpurun_out/prof_ingest_$wl" <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in sorted(csv.DictReader(open(f)), key=lambda r: -float(r["TotalDurationNs"]))[:18]:
        n = r["Name"]
        n = n.split("::")[1].split("(")[0] if n.startswith("(anon") else n[:60]
        print("   %-60s calls %4s avg %8.1f us" % (n, r["Calls"], float(r["AverageNs"]) / 1e3))
PY
done
