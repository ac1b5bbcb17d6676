#!/bin/bash
# Multi-rank rehearsal on a 1-GPU box: bucket/sharding tests (gloo, records,
# padded, descriptors) and bench.py --gpus 2 over gloo (2 ranks on one GPU).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "bucket or sharded" > gpurun_out/pytest_multi.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_multi.log
[ $rc -ne 0 ] && { echo "STOP pytest ($rc)"; exit $rc; }
for ex in descriptors records; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
    bench.py --gpus 2 --steps 10 --warmup 3 --backend gloo --datagrams 262144 --exchange $ex > gpurun_out/bench_n2_$ex.log 2>&1 || { echo "STOP bench n2 $ex"; tail -30 gpurun_out/bench_n2_$ex.log; exit 3; }
  python -c "import json; d=json.loads(open('gpurun_out/bench_n2_$ex.log').read().strip().splitlines()[-1]); print('$ex', d['value'], json.dumps(d['config']['exchange']), d['config']['received_records_rank0'])"
done
timeout -k 10 300 python bench.py --steps 20 --no-cpu-baseline --no-e2e --no-cdr --no-c1 --no-ingest --match none > gpurun_out/bench_nomatch.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 20 --no-cpu-baseline --no-e2e --no-cdr --no-c1 --no-ingest --match writers > gpurun_out/bench_match.log 2>&1 || exit 4
python -c "
import json
for f in ('nomatch','match'):
    d=json.loads(open('gpurun_out/bench_%s.log'%f).read().strip().splitlines()[-1]); print(f, d['value'], d['roofline']['kernel_ms'], d['config']['matched_writers'])"
