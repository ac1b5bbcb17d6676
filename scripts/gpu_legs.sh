#!/bin/bash
# The §8f legs on the box: ingest (C3, T) and DataFrag reassembly (C4) bench lines,
# each under rocprofv3 kernel-trace stats (per-kernel times of the leg's launches).
# Prebuilt in-tree libraries; every GPU step has its own time limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
SKIP="--no-c1 --no-cpu-baseline --no-e2e --no-cdr --steps 20 --warmup 5"
cd /tmp
IFS=";" read -ra JL <<< "${JOBS:-C3 --no-frag;T --no-frag;C4 --no-ingest}"
for job in "${JL[@]}"; do
  set -- $job; wl=$1; shift
  echo "== $wl ($(date +%T))"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/legs_$wl" -o run --output-format csv \
    -- python3 "$R/bench.py" --workload $wl $SKIP "$@" > "$R/gpurun_out/legs_$wl.json" 2> "$R/gpurun_out/legs_$wl.err" \
    || { echo "STOP $wl"; tail -5 "$R/gpurun_out/legs_$wl.err"; exit 3; }
  python3 - "$R/gpurun_out/legs_$wl.json" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
for k in ("ingest", "frag_assemble"):
    if k in d:
        print(k, {kk: d[k][kk] for kk in ("ms", "events", "accepted", "samples", "fragments", "achieved_gbs") if kk in d[k]})
PY
done
