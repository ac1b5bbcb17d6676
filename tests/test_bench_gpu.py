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
    # achieved = bytes the dominant kernel reads per launch (FETCH basis: the parse is
    # zero-copy, so fewer than the datagrams' bytes) / its launch time; writes reported beside it
    assert rf["read_bytes"] < rf["sum_datagram_bytes"]
    assert abs(rf["achieved"] - rf["read_bytes"] / (rf["kernel_ms"] * 1e-3) / 1e9) < 1e-6 * rf["achieved"]
    assert abs(rf["frac"] - rf["achieved"] / rf["peak"]) < 1e-9 and rf["peak"] == 8000.0
    # T: the speculative kernel; C3: the slower of the item pass's walk E and its record pass W
    # (the line names the dominant kernel, with its own time)
    if workload == "T":
        assert rf["kernel"] == "rtps_parse_spec_kernel"
    else:
        e, w = rf["item_kernel_ms"], rf["emit_kernel_ms"]
        assert rf["emit_kernel"] == "rtps_parse_emit2_kernel"
        assert rf["kernel"] == ("rtps_parse_item_kernel" if e >= w else "rtps_parse_emit2_kernel")
        assert rf["kernel_ms"] == max(e, w) and rf["scan_ms"] >= 0
    assert "gib_per_s_parsed" not in d and d["gib_per_s_covered"] > 0


@pytest.mark.gpu
@pytest.mark.parametrize("exchange", ["owner", "records", "descriptors"])
def test_bench_two_ranks_gloo_exchange(exchange):
    """N=2 as the driver runs it (owner: no --workload): the T line (the headline config, weak
    scaling) with the owner-side exchange and its ingest pipeline, then the C5 config (C3 mix,
    64M / N per rank, here reduced) as `c5`; the record and descriptor exchanges (options) on C5."""
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", "2",
           "--backend", "gloo", "--exchange", exchange] + SMALL + ([] if exchange == "owner" else ["--workload", "C5"])
    r = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _json_line(r.stdout)
    assert d["n_gpus"] == 2 and d["value"] > 0
    if exchange == "owner":
        assert d["config"]["workload"].startswith("T") and d["scaling"] == "weak"
        ex = d["config"]["exchange"]
        assert ex["overflow"] is False and "owner-side" in ex["mode"] and ex["spilled_records_rank0"] == 0
        # T: one DATA per datagram from 16 writers; rank 0 owns the writers whose GUID hashes to it
        got, per = d["config"]["received_records_rank0"], d["config"]["records_per_gpu"]
        assert 0.1 * per < got < 1.9 * per, (got, per)
        p = d["pipeline_with_ingest"]
        assert p["value"] > 0 and p["deliveries_per_step_all_ranks"] == 2 * per
        d = d["c5"]
        assert d["value"] > 0 and d["scaling"] == "strong"
    assert d["config"]["workload"].startswith("C5") and d["scaling"] == "strong"
    ex = d["config"]["exchange"]
    assert ex["overflow"] is False
    got, per = d["config"]["received_records_rank0"], d["config"]["records_per_gpu"]
    if exchange == "owner":
        # rank 0 owns about half of both ranks' writer records that pass (about 2.3 of the 3.8
        # records per C3 datagram); the second timed loop adds every owner's ingest
        assert "owner-side" in ex["mode"] and ex["spilled_records_rank0"] == 0
        assert 0.35 * per < got < 0.8 * per, (got, per)
        p = d["pipeline_with_ingest"]
        assert p["value"] > 0 and p["deliveries_per_step_all_ranks"] > 0.5 * per
    elif exchange == "records":
        # owner = writer-GUID hash % 2 over 256 writers: rank 0 receives about half of both ranks'
        # writer / reader records (about 2.8 of the 3.8 records per C3 datagram)
        assert "writer-GUID hash" in ex["item"]
        assert 0.5 * per < got < 0.85 * per, (got, per)
    else:
        assert "rtps_xdesc" in ex["item"] and got > 0
