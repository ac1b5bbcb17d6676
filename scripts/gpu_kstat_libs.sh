#!/bin/bash
# Per-kernel average durations (rocprofv3 --kernel-trace --stats) of bench.py's legs for the product
# library and each variants/*.so: gpu_kstat_libs.sh WL "<bench flags>" "<kernel name regex>"
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp; R=$PWD
WL=${1:-C3}; FLAGS=${2:-"--no-c1 --no-cpu-baseline --no-e2e --no-cdr --no-frag"}; RX=${3:-"k_|parse|sort"}
for lib in $R/rustdds-io_uring_amd/librtps_rx.so $(ls $R/rustdds-io_uring_amd/variants/*.so 2>/dev/null); do
  n=$(basename $lib .so)
  rm -rf gpurun_out/ks_$n
  (cd /tmp && RTPS_RX_LIB=$lib timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/ks_$n -o run \
    --output-format csv -- python3 $R/bench.py --workload $WL --steps 10 --warmup 3 $FLAGS > $R/gpurun_out/ks_$n.log 2>&1) \
    || { echo "FAIL $n"; tail -5 gpurun_out/ks_$n.log; exit 4; }
  f=$(find gpurun_out/ks_$n -name "*kernel_stats.csv" | head -1)
  [ -n "$f" ] && cp "$f" gpurun_out/ks_${n}_kernel_stats.csv
  echo "== $n"
  python3 - "$f" "$RX" <<'PY'
import csv, re, sys
for r in csv.DictReader(open(sys.argv[1])):
    if re.search(sys.argv[2], r["Name"]):
        print(f"  {r['Name'][:80]:82s} {int(r['Calls']):5d} {float(r['AverageNs'])/1e3:8.1f} us")
PY
  rm -rf gpurun_out/ks_$n
done
