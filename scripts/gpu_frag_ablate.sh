#!/bin/bash
# k_walk ablations (results of the ablated builds are wrong; timing only):
#   ABL_WALK=1 no per-record step loop, ABL_WALK=2 run detection only.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$PWD; mkdir -p gpurun_out build; export TMPDIR=/tmp
C=rustdds-io_uring_amd/csrc
for v in 0 1 2; do
  (cd $C && /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -Wno-unused-function -DABL_WALK=$v -shared \
     -o $R/build/librtps_abl$v.so rtps_rx.hip rtps_cdr.hip rtps_frag.hip rtps_ingest.hip rtps_udp.cpp rtps_pump.cpp) || exit 2
done
cd /tmp
for v in 0 1 2; do
  RTPS_RX_LIB=$R/build/librtps_abl$v.so timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_abl$v" -o run \
    --output-format csv -- python3 "$R/bench.py" --workload C4 --no-cpu-baseline --no-e2e --no-cdr --no-ingest --no-c1 \
    --steps 10 --warmup 3 > "$R/gpurun_out/prof_abl$v.log" 2>&1 || { echo "STOP $v"; exit 3; }
  python3 - "$R/gpurun_out/prof_abl$v/run_kernel_stats.csv" $v <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"]
    if "k_walk" in n or "k_span" in n:
        print("ABL_WALK=%s" % sys.argv[2], n.split("::")[1].split("(")[0], "avg %.1f us" % (float(r["AverageNs"]) / 1e3))
PY
done
