#!/bin/bash
# Parse-kernel iteration loop: parity tests, then per-workload parse time and a
# rocprof A/B split.  Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_parity.log 2>&1; rc=$?
tail -4 gpurun_out/pytest_parity.log; [ $rc -eq 0 ] || exit $rc
for wl in ${WORKLOADS:-T C2 C3 C4}; do
  timeout -k 10 200 python bench.py --workload $wl --steps 30 --no-cpu-baseline --no-e2e --no-cdr --no-frag --no-ingest --no-c1 \
    > gpurun_out/it_$wl.log 2>&1 || { echo "bench $wl failed"; tail -5 gpurun_out/it_$wl.log; exit 4; }
  python -c "import json; d=json.loads(open('gpurun_out/it_$wl.log').read().strip().splitlines()[-1]); print('$wl', '%.2f Gdgram/s' % (d['value']/1e9), 'kernel %.1f us' % (d['roofline']['kernel_ms']*1e3), 'frac %.3f' % d['roofline']['frac'])"
done
cd /tmp
for wl in ${PROF_WL:-C3}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_it_$wl" -o run --output-format csv \
    -- python3 "$R/bench.py" --workload $wl --steps 20 --warmup 5 --no-cpu-baseline --no-e2e --no-cdr --no-frag --no-ingest --no-c1 > "$R/gpurun_out/prof_it_$wl.log" 2>&1 || { echo "STOP prof $wl"; exit 3; }
  python3 - "$R/gpurun_out/prof_it_$wl" $wl <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Name"]
        if "rtps_parse" in n:
            print("  ", sys.argv[2], n.split("::")[1].split("(")[0], "calls", r["Calls"], "avg %.1f us" % (float(r["AverageNs"]) / 1e3))
PY
done
