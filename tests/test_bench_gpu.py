"""bench.py itself on the GPU at a small size: the one-rank JSON line keeps the
driver's contract, and the N>1 path (writer-GUID descriptor exchange, pipelined
with the next parse) runs end to end with two ranks on one GPU over gloo, the
rehearsal DESIGN.md §3.7 describes.  The 8-GPU RCCL run is the driver's."""
import json
import os
import socket
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SMALL = ["--steps", "3", "--warmup", "1", "--datagrams", "20000", "--no-cpu-baseline", "--no-c1", "--no-e2e",
         "--no-cdr", "--no-frag", "--no-ingest"]


def _json_line(out):
    lines = [l for l in out.splitlines() if l.startswith("{")]
    assert lines, out[-2000:]
    return json.loads(lines[-1])


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.gpu
@pytest.mark.parametrize("workload", ["T", "C3"])
def test_bench_one_rank_line(workload):
    r = subprocess.run([sys.executable, "bench.py", "--workload", workload] + SMALL, cwd=REPO,
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    d = _json_line(r.stdout)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config", "roofline"):
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == 3 and d["value"] > 0
    assert d["config"]["ok_datagrams"] > 0.9 * 20000
    rf = d["roofline"]
    assert rf["bound"] == "hbm" and 0 < rf["frac"] < 1 and rf["kernel_ms"] > 0


@pytest.mark.gpu
def test_bench_two_ranks_gloo_exchange():
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", "2",
           "--backend", "gloo"] + SMALL
    r = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _json_line(r.stdout)
    assert d["n_gpus"] == 2 and d["value"] > 0
    ex = d["config"]["exchange"]
    assert ex["overflow"] is False
    # 16 writers, owner = match-table entry % 2: rank 0 owns about half of both ranks' records
    got, per = d["config"]["received_records_rank0"], d["config"]["records_per_gpu"]
    assert abs(got - per) <= 0.1 * per, (got, per)
