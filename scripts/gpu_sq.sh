#!/bin/bash
# SQ / TA / TD counter passes (one rocprofv3 --pmc run each) over the C3 parse (bench.py, parse only),
# summed per kernel name for the item pass E and the record pass W2: gpurun_out/sq_C3.json.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
cd /tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS"
P2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT TA_TA_BUSY_sum TD_TD_BUSY_sum"
i=0
for P in "$P1" "$P2"; do
  i=$((i + 1))
  timeout -s KILL 120 rocprofv3 --pmc $P -d "$R/gpurun_out/sq_C3_$i" -o run --output-format csv \
    -- python3 "$R/bench.py" --workload C3 --steps 3 --warmup 1 --no-cpu-baseline --no-c1 --no-e2e --no-cdr \
       --no-ingest > "$R/gpurun_out/sq_C3_$i.log" 2>&1 || { echo "STOP sq pass $i"; tail -3 "$R/gpurun_out/sq_C3_$i.log"; exit 3; }
done
python3 - "$R/gpurun_out" <<'PY' > "$R/gpurun_out/sq_C3.json"
import csv, glob, json, os, sys
out = {}
for f in glob.glob(os.path.join(sys.argv[1], "sq_C3_*", "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        k = r.get("Kernel_Name", "")
        name = "E" if "parse_item_kernel" in k else "W2" if "parse_emit2_kernel" in k else None
        if not name:
            continue
        d = out.setdefault(name, {})
        c = r["Counter_Name"]
        d.setdefault(c, []).append(float(r["Counter_Value"]))
res = {k: {c: sum(v) / len(v) for c, v in d.items()} for k, d in out.items()}
print(json.dumps(res, indent=1))
PY
cat "$R/gpurun_out/sq_C3.json"
