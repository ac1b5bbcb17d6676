#!/bin/bash
# One C4 reassembly step's kernel sequence per library (product + variants/*.so):
# rocprofv3 kernel trace of the bench's frag leg, then scripts/trace_step.py on it.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; R=$PWD
libs="$R/rustdds-io_uring_amd/librtps_rx.so $(ls $R/rustdds-io_uring_amd/variants/*.so 2>/dev/null)"
cd /tmp; export TMPDIR=/tmp
for v in $libs; do
  n=$(basename "$v" .so)
  RTPS_RX_LIB=$v timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/trace_$n" -o c4 -- python3 "$R/bench.py" \
    --workload C4 --no-c1 --no-cpu-baseline --no-e2e --no-cdr --no-ingest > "$R/gpurun_out/trace_$n.log" 2>&1 || exit 4
  echo "== $n"; python3 "$R/scripts/trace_step.py" "$R/gpurun_out/trace_$n/c4_results.db" k_keys k_span || exit 5
done
