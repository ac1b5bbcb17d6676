#!/bin/bash
# PMC passes (one counter group per run) on the C3 item-pass kernels (E, W) and the chain kernel (RTPS_RX_MIXED_PASS).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
cd /tmp
timeout -s KILL 60 rocprofv3 -L > "$R/gpurun_out/pmc_list.txt" 2>&1 || true
i=0
while IFS= read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp -d "$R/gpurun_out/pmc_it_$i" -o run --output-format csv \
    -- python3 "$R/bench.py" --workload ${WL:-C3} --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --no-cdr --no-frag --no-ingest --no-c1 \
    > "$R/gpurun_out/pmc_it_$i.log" 2>&1 || { echo "STOP pmc group $i ($grp)"; tail -3 "$R/gpurun_out/pmc_it_$i.log"; exit 3; }
done <<'GROUPS'
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU
SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_WAIT_INST_LDS
FETCH_SIZE
WRITE_SIZE
TA_BUSY_avr TA_TA_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum
GROUPS
python3 - "$R/gpurun_out" <<'PY'
import csv, glob, sys, collections
root = sys.argv[1]
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(root + "/pmc_it_*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"]
        k = "item" if "parse_item" in n else "emit" if "parse_emit" in n else "chain" if "parse_chain" in n else None
        if k: vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in vals.items():
    print(k)
    for c, v in sorted(d.items()):
        print("   %-28s %16.0f" % (c, sum(v) / len(v)))
PY
