#!/bin/bash
# PMC passes (separate runs per counter, kernel-trace only) on the T ceiling + parse kernels.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
python -c "import __graft_entry__ as g; g.build()" || exit 2
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -shared -o build/libdiag_ceiling.so rustdds-io_uring_amd/csrc/diag/ceiling.hip || exit 2
cd /tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c -d "$R/gpurun_out/pmc_ceil_$c" -o run --output-format csv \
    -- python3 "$R/scripts/diag_ceiling.py" T > "$R/gpurun_out/pmc_ceil_$c.log" 2>&1 || { echo "STOP pmc $c"; exit 3; }
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_ceil" -o run --output-format csv \
  -- python3 "$R/scripts/diag_ceiling.py" T > "$R/gpurun_out/prof_ceil.log" 2>&1 || exit 4
python3 "$R/scripts/pmc_summary.py" "$R/gpurun_out/pmc_ceil"
