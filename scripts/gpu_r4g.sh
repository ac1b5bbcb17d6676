#!/bin/bash
# Hash-probe change (rt_writer_set loads set and key together): parse parity, then the ingest
# experiment (tests + product vs c2kfni on C3 / T), then the classify stamps.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest tests/test_gpu_parity.py tests/test_frag_gpu.py tests/test_shard_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/g_parity.log 2>&1; rc=$?
tail -2 gpurun_out/g_parity.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/g_parity.log | head -30; exit $rc; }
VARIANTS="${VARIANTS:-c2kfni}" WLS="${WLS:-C3 T}" bash scripts/gpu_exp_ingest.sh || exit 5
RTPS_RX_LIB=$R/rustdds-io_uring_amd/variants/librtps_rx_cstp.so CHR=2048 timeout -k 10 150 python3 scripts/cls_stamps.py > gpurun_out/cstp.txt 2>&1 || exit 6
echo done
