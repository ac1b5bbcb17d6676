#!/bin/bash
# Kernel-level A/B: rocprofv3 kernel stats of one bench.py leg for the product library and each
# rustdds-io_uring_amd/variants/*.so; prints the kernels matching $KRE.  Prebuilt in-tree libraries.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$PWD; mkdir -p gpurun_out; export TMPDIR=/tmp
ARGS=${ARGS:-"--workload C3 --no-cpu-baseline --no-e2e --no-c1 --no-cdr --steps 5 --warmup 2"}
KRE=${KRE:-"k_classify"}
libs="$R/rustdds-io_uring_amd/librtps_rx.so $(ls $R/rustdds-io_uring_amd/variants/*.so 2>/dev/null)"
for round in 1 2; do
  for v in $libs; do
    n=$(basename "$v" .so)
    (cd /tmp && RTPS_RX_LIB=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/ks_$n" -o run \
      --output-format csv -- python3 "$R/bench.py" $ARGS > "$R/gpurun_out/ks_$n.log" 2>&1) || { echo "STOP $n"; exit 3; }
    python3 - "$R/gpurun_out/ks_$n/run_kernel_stats.csv" "$n" "$KRE" <<'PY'
import csv, re, sys
for r in csv.DictReader(open(sys.argv[1])):
    if re.search(sys.argv[3], r["Name"]):
        print("%-22s %-40s %9.1f us" % (sys.argv[2], r["Name"][:40], float(r["AverageNs"]) / 1e3))
PY
  done
done
