#!/bin/bash
# PMC passes (one rocprofv3 run per counter, --pmc only) over the C3 ingest leg (bench.py, 1M datagrams):
# per-launch FETCH_SIZE / WRITE_SIZE of the ingest kernels -> gpurun_out/r3_pmc_ingest_C3.json.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
cd /tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 180 rocprofv3 --pmc $c -d "$R/gpurun_out/pmci_C3_$c" -o run --output-format csv \
    -- python3 "$R/bench.py" --workload C3 --steps 5 --warmup 2 --no-cpu-baseline --no-c1 --no-e2e --no-cdr \
       --no-frag > "$R/gpurun_out/pmci_C3_$c.log" 2>&1 || { echo "STOP pmc C3 $c"; exit 3; }
done
python3 - "$R/gpurun_out/pmci_C3" > "$R/gpurun_out/r3_pmc_ingest_C3.json" <<'PY'
import collections, csv, glob, json, sys
root = sys.argv[1]
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    for f in glob.glob(f"{root}_{c}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            n = r["Kernel_Name"]
            for k in ("k_classify", "k_proxy", "k_dwrite", "k_dcount"):
                if k in n:
                    vals[k][c].append(float(r["Counter_Value"]) * 1024.0)
out = {"source": f"{root}_{{FETCH_SIZE,WRITE_SIZE}} (scripts/gpu_pmc_ingest.sh), bytes per launch (counter KiB x 1024, "
       "uncalibrated)", "workload": "C3 ingest, 1M datagrams (3.98M records, 2.3M events)"}
for k, d in vals.items():
    out[k] = {c: sum(v) / len(v) for c, v in d.items() if v}
    out[k]["launches"] = max(len(v) for v in d.values())
print(json.dumps(out, indent=1))
PY
cat "$R/gpurun_out/r3_pmc_ingest_C3.json"
