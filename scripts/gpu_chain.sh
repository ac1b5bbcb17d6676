#!/bin/bash
# Chained look-back launch (spec hint 0) vs the two-launch parse: parity, then timings.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread \
  -k "spec_hint or chained or workload_parity or golden or launch_choice or fallback" > gpurun_out/pytest_chain.log 2>&1; rc=$?
tail -4 gpurun_out/pytest_chain.log; [ $rc -eq 0 ] || exit $rc
for wl in C3 T C2 C4; do for h in 1 0; do
  timeout -k 10 200 python bench.py --workload $wl --spec-hint $h --steps 30 --no-cpu-baseline --no-e2e --no-cdr --no-frag \
    --no-ingest --no-c1 > gpurun_out/chain_${wl}_$h.log 2>&1 || { echo "bench $wl $h failed"; tail -5 gpurun_out/chain_${wl}_$h.log; exit 4; }
  python -c "import json; d=json.loads(open('gpurun_out/chain_${wl}_$h.log').read().strip().splitlines()[-1]); print('$wl hint $h', '%.2f Gdgram/s' % (d['value']/1e9), 'kernel %.1f us' % (d['roofline']['kernel_ms']*1e3))"
done; done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_chain" -o run --output-format csv \
  -- python3 "$R/bench.py" --workload C3 --spec-hint 0 --steps 20 --warmup 5 --no-cpu-baseline --no-e2e --no-cdr --no-frag --no-ingest --no-c1 > "$R/gpurun_out/prof_chain.log" 2>&1 || exit 3
python3 - "$R/gpurun_out/prof_chain/run_kernel_stats.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"]
    if "rtps_parse" in n or "fillBuffer" in n:
        print("  C3 hint0", n.split("::")[-1].split("(")[0][:40], "calls", r["Calls"], "avg %.1f us" % (float(r["AverageNs"]) / 1e3))
PY
