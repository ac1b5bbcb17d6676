#!/bin/bash
# DataFrag span copy (k_span) on C4: the product against prebuilt variants in build/
# (ABL_SPAN_NOCOPY: resolve only, copy nothing - timing only; SPAN_GRID=2048/1024: fewer
# workgroups, each wave loops over several 64-position chunks; ABL_SPAN_ALIGN: 16-B-aligned source
# reads, timing only).  rocprof kernel stats per library; SPAN_LIBS overrides the list.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$PWD; mkdir -p gpurun_out; export TMPDIR=/tmp
cd /tmp
for lib in ${SPAN_LIBS:-rustdds-io_uring_amd/librtps_rx.so build/libspan_nocopy.so build/libspan_g2048.so build/libspan_g1024.so}; do
  tag=$(basename $lib .so)
  RTPS_RX_LIB=$R/$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_span_$tag" -o run \
    --output-format csv -- python3 "$R/bench.py" --workload C4 --no-cpu-baseline --no-e2e --no-cdr --no-ingest --no-c1 \
    --steps 10 --warmup 3 > "$R/gpurun_out/prof_span_$tag.log" 2>&1 || { echo "STOP $tag"; tail -5 "$R/gpurun_out/prof_span_$tag.log"; exit 3; }
  python3 - "$R/gpurun_out/prof_span_$tag/run_kernel_stats.csv" $tag <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"]
    if "k_span" in n:
        print(sys.argv[2], "k_span avg %.1f us (%s calls)" % (float(r["AverageNs"]) / 1e3, r["Calls"]))
PY
done
