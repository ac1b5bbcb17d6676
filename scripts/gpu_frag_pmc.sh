#!/bin/bash
# PMC passes (one counter group per run, kernel-trace only) on the reassembly's kernels (C4).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
cd /tmp
i=0
while IFS= read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp -d "$R/gpurun_out/pmc_frag_$i" -o run --output-format csv \
    -- python3 "$R/bench.py" --workload C4 --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --no-cdr --no-ingest --no-c1 \
    > "$R/gpurun_out/pmc_frag_$i.log" 2>&1 || { echo "STOP pmc group $i ($grp)"; tail -3 "$R/gpurun_out/pmc_frag_$i.log"; exit 3; }
done <<'GROUPS'
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU
SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_WAIT_INST_LDS
FETCH_SIZE
WRITE_SIZE
GROUPS
python3 - "$R/gpurun_out" <<'PY'
import csv, glob, sys, collections, re
root = sys.argv[1]
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(root + "/pmc_frag_*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        m = re.search(r"(k_keys|k_walk|k_span|k_place\b|k_fill|k_hist|k_scatter|k_sub|k_colscan|k_place_tiles)", r["Kernel_Name"])
        if m: vals[m.group(1)][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in sorted(vals.items()):
    print(k)
    for c, v in sorted(d.items()):
        print("   %-28s %16.0f" % (c, sum(v) / len(v)))
PY
