"""N>1 path on CPU: world_size-2 gloo run of the record exchange (rtps_rx.shard)
with oracle-parsed records bucketed by the numpy reference of the device hash."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle
from rtps_rx.records import RECORD_DTYPE
from rtps_rx.shard import Exchange, owner_hash_words
from shard_ref import bucket_np, owner_np


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _rank_records(rank, n):
    arena, off, ln = oracle.gen(oracle.WL_C3, n, first_idx=rank * n)
    st, recs, _, _ = oracle.parse(arena, off, ln)
    return recs


def _worker(rank, world, port, n, q, padded):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        recs = _rank_records(rank, n)
        bucketed, counts = bucket_np(recs, world)
        raw = bucketed.view(np.uint8).reshape(-1, 64)
        if padded:  # fixed slots of cap records (what rtps_rx_bucket_by_writer_padded writes)
            cap = int(padded)
            ex = Exchange(rx=None, max_records=len(bucketed), world=world, dist=dist, device=torch.device("cpu"),
                          cap=cap)
            ex.bucketed.zero_()
            start = np.concatenate([[0], np.cumsum(counts)[:-1]])
            for d in range(world):
                k = min(int(counts[d]), cap)
                ex.bucketed[d * cap:d * cap + k] = torch.from_numpy(raw[start[d]:start[d] + k])
            ex.counts.copy_(torch.from_numpy(counts))
            assert ex.overflowed() == (counts.max() > cap)
        else:
            ex = Exchange(rx=None, max_records=len(bucketed), world=world, dist=dist, device=torch.device("cpu"))
            ex.bucketed[:len(bucketed)] = torch.from_numpy(raw)
            ex.counts.copy_(torch.from_numpy(counts))
        got, split = ex.exchange()
        q.put((rank, got.numpy().tobytes(), split))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,padded", [(2, 0), (3, 0), (2, 8000), (3, 6000)])
def test_exchange_gloo(world, padded):
    """padded = fixed bucket capacity (equal-split all-to-all, counts sent alongside)."""
    n = 3000
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, q, padded)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        rank, buf, split = q.get(timeout=300)
        res[rank] = (np.frombuffer(buf, dtype=RECORD_DTYPE), split)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    all_recs = [_rank_records(r, n) for r in range(world)]
    for owner in range(world):
        got, split = res[owner]
        # the owner receives, from every source rank in rank order, that rank's records it owns
        exp = np.concatenate([r[owner_np(r, world) == owner] for r in all_recs])
        assert got.tobytes() == exp.tobytes()
        assert sum(split) == len(got)


def test_owner_hash_scalar_matches_vectorized():
    recs = _rank_records(0, 500)
    o = owner_np(recs, 5)
    w = recs.view(np.uint32).reshape(-1, 16)[:, 2:6]
    for i in range(0, len(recs), 37):
        if o[i] >= 0:
            assert owner_hash_words(w[i]) % 5 == o[i]


def _desc_worker(rank, world, port, n, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from shard_ref import desc_bucket_np
        recs = _rank_records(rank, n)
        guids = sorted({bytes(r["prefix"]) + bytes(r["writer_id"]) for r in recs})
        # MATCHED needs a match table in the parse: mark every writer record as matched here
        recs = recs.copy()
        wk = np.isin(recs["kind"], [0x15, 0x16, 0x07, 0x08, 0x13])
        recs["route"][wk] |= 0x20
        buckets = desc_bucket_np(recs, guids, world)
        cap = 4 * n  # the same on every rank (equal-split all-to-all)
        ex = Exchange(rx=None, max_records=len(recs), world=world, dist=dist, device=torch.device("cpu"), cap=cap,
                      item="descriptors")
        ex.bucketed.zero_()
        for d in range(world):
            raw = buckets[d].view(np.uint8).reshape(-1, 16)
            ex.bucketed[d * cap:d * cap + len(raw)] = torch.from_numpy(raw)
        ex.counts.copy_(torch.tensor([len(b) for b in buckets]))
        got, split = ex.exchange()
        q.put((rank, got.numpy().tobytes(), split, [b.tobytes() for b in buckets]))
    finally:
        dist.destroy_process_group()


def test_descriptor_exchange_gloo():
    world, n = 3, 2000
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_desc_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        rank, buf, split, sent = q.get(timeout=300)
        res[rank] = (buf, split, sent)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for owner in range(world):
        exp = b"".join(res[src][2][owner] for src in range(world))
        assert res[owner][0] == exp and sum(res[owner][1]) * 16 == len(exp)
