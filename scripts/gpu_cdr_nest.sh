# Composite-program CDR decode on the box: the CDR GPU parity tests, then the timing
# of scripts/diag_cdr_composite.py (POLYGON / NESTED, 512K rows) for the in-tree
# library and each rustdds-io_uring_amd/variants/*.so (RTPS_RX_LIB).
shopt -s nullglob
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_cdr_gpu.py > gpurun_out/cdr_tests.log 2>&1; rc=$?; tail -3 gpurun_out/cdr_tests.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -u scripts/diag_cdr_composite.py && timeout -k 10 300 python -u scripts/diag_cdr_composite.py --ascii || exit 1
for v in rustdds-io_uring_amd/variants/*.so; do echo "== $v"; RTPS_RX_LIB=$PWD/$v timeout -k 10 300 python -u scripts/diag_cdr_composite.py || exit 1; done
