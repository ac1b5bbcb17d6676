"""Owner-side exchange on CPU: world_size 2 / 3 gloo runs of
the rtps_rx_shard protocol, with the numpy model of the device pack / unpack
(tests/shard_ref.py) around the transport's real round-1 plan
(rtps_rx.shard.spill_plan), and the CPU oracle's fragment assembly + history
ingest on every owner's batch.

The check is the one the multi-GPU path must pass: the union of the owners'
deliveries (mapped back through `origin` to the records of the whole stream)
and every writer proxy's all_ackable_before equal what ONE rank's oracle ingest
of the whole stream gives (reader.rs:563-758, rtps_writer_proxy.rs:202-355),
including with slots so small that most items travel in the spill."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle
from rtps_rx.records import RECORD_DTYPE, DELIVERY_DTYPE, FRAG_SAMPLE_DTYPE, pack_match_table, WRITER_KINDS
from rtps_rx.shard import spill_plan
from shard_ref import COUNTS_DTYPE, ITEM_DTYPE, shard_pack_np, shard_unpack_np

C5_STRIDE = 8 << 20  # rank r's chunk starts at generator index r * 8M (BASELINE C5: 64M over 8 GPUs)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _chunk(wl, rank, n, stride):
    return oracle.gen(wl, n, first_idx=rank * stride)


def _whole(wl, world, n, stride):
    """The whole stream as one batch: the ranks' chunks back to back."""
    arenas, offs, lens, base = [], [], [], 0
    for r in range(world):
        a, o, l = _chunk(wl, r, n, stride)
        arenas.append(a[:int(o[-1]) + int(l[-1])] if len(o) else a[:0])
        offs.append(o + np.uint64(base))
        lens.append(l)
        base += len(arenas[-1])
        pad = (-base) % 16
        arenas.append(np.zeros(pad, np.uint8))
        base += pad
    return np.concatenate(arenas), np.concatenate(offs), np.concatenate(lens)


def _table(wl, world, n, stride):
    a, o, l = _whole(wl, world, n, stride)
    _, recs, _, _ = oracle.parse(a, o, l)
    wk = np.isin(recs["kind"], WRITER_KINDS)
    guids = sorted({bytes(r["prefix"]) + bytes(r["writer_id"]) for r in recs[wk]})
    # a15: every writer to reader 100, every other one also to reader 101 (two-reader target sets)
    return pack_match_table([(g, 100) for g in guids] + [(g, 101) for g in guids[::2]])


def _layout(packed, world, cap, bcap):
    """The library's send buffers: slots [world * cap] items, blob slots [world * bcap],
    exact-layout spills, counts."""
    slots = np.zeros(world * cap, dtype=ITEM_DTYPE)
    blob = np.zeros(world * bcap, dtype=np.uint8)
    counts = np.zeros(world, dtype=COUNTS_DTYPE)
    spill_r, spill_b = [], []
    for d, x in enumerate(packed):
        c = x["counts"][0]
        counts[d] = c
        slots[d * cap:d * cap + int(c["cut"])] = x["slot_items"]
        blob[d * bcap:d * bcap + int(c["cut_bytes"])] = x["slot_blob"]
        spill_r.append(np.concatenate([np.zeros(int(c["cut"]), ITEM_DTYPE), x["spill_items"]]))
        spill_b.append(np.concatenate([np.zeros(int(c["cut_bytes"]), np.uint8), x["spill_blob"]]))
    return slots, blob, counts, np.concatenate(spill_r), np.concatenate(spill_b)


def _a2a(send, recv, ss=None, rs=None):
    out = torch.from_numpy(recv)
    dist.all_to_all_single(out, torch.from_numpy(np.ascontiguousarray(send)), rs, ss)


def _worker(rank, world, port, wl, n, stride, cap, bcap, tbl, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        arena, off, ln = _chunk(wl, rank, n, stride)
        _, recs, _, _ = oracle.parse(arena, off, ln, match_table=tbl)
        packed = shard_pack_np(arena, off, recs, world, cap, bcap)
        slots, blob, sc, sspill, sbspill = _layout(packed, world, cap, bcap)
        # round 0: counts, slots, blob slots (equal splits)
        rc = np.zeros(world, dtype=COUNTS_DTYPE)
        _a2a(sc.view(np.uint8), rc.view(np.uint8))
        rslots = np.zeros_like(slots)
        _a2a(slots.view(np.uint8), rslots.view(np.uint8))
        rblob = np.zeros_like(blob)
        _a2a(blob, rblob)
        # round 1: the exact spill, from the counts alone
        plan = spill_plan(sc, rc)
        sr = sspill.view(np.uint8)
        sends = [sr[p["send_rec"][0] * 32:(p["send_rec"][0] + p["send_rec"][1]) * 32] for p in plan]
        rspill = np.zeros(sum(p["recv_rec"][1] for p in plan) * 32, np.uint8)
        _a2a(np.concatenate(sends), rspill, [len(x) for x in sends], [p["recv_rec"][1] * 32 for p in plan])
        sends = [sbspill[p["send_bytes"][0]:p["send_bytes"][0] + p["send_bytes"][1]] for p in plan]
        rbspill = np.zeros(sum(p["recv_bytes"][1] for p in plan), np.uint8)
        _a2a(np.concatenate(sends), rbspill, [len(x) for x in sends], [p["recv_bytes"][1] for p in plan])
        rspill = rspill.view(ITEM_DTYPE)
        # what each source sent this owner, rebuilt from the receive buffers as the device unpack reads them
        received, rs, rbs = [], 0, 0
        for s in range(world):
            c = rc[s]
            cut, cb, nn, nb = int(c["cut"]), int(c["cut_bytes"]), int(c["n"]), int(c["bytes"])
            received.append({"slot_items": rslots[s * cap:s * cap + cut], "slot_blob": rblob[s * bcap:s * bcap + cb],
                             "spill_items": rspill[rs:rs + nn - cut], "spill_blob": rbspill[rbs:rbs + nb - cb]})
            rs += nn - cut
            rbs += nb - cb
        orecs, ooff, oarena, (orank, osrc) = shard_unpack_np(received)
        fa = oracle.FragAssembler()
        samples = fa.batch_readers(oarena, ooff, orecs, tbl)[0]
        ing = oracle.HistoryIngest(tbl)
        acc, dels, ack = ing.batch(oarena, ooff, orecs, samples)
        q.put((rank, dels.tobytes(), ack.tobytes(), orank.tobytes(), osrc.tobytes(),
               samples.tobytes(), int(sum(p["recv_rec"][1] for p in plan)), len(orecs)))
    finally:
        dist.destroy_process_group()


def _run(world, wl, n, stride, cap, bcap):
    tbl = _table(wl, world, n, stride)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, wl, n, stride, cap, bcap, tbl, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        item = q.get(timeout=600)
        res[item[0]] = item[1:]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # one rank's oracle over the whole stream
    a, o, l = _whole(wl, world, n, stride)
    _, recs, _, rb = oracle.parse(a, o, l, match_table=tbl)
    samples = oracle.FragAssembler().batch_readers(a, o, recs, tbl)[0]
    _, dels, ack = oracle.HistoryIngest(tbl).batch(a, o, recs, samples)
    # origin = (source rank, record index in that rank's parse); rank r parsed datagrams [r n, (r+1) n)
    first_rec = np.searchsorted(recs["dgram_idx"], np.arange(world) * n)
    got, spilled, items = [], 0, 0
    owner_ack = np.ones(len(ack), dtype=np.int64)
    for rank in range(world):
        d, k, orank, osrc, osamp, sp, ni = res[rank]
        d = np.frombuffer(d, DELIVERY_DTYPE)
        orank, osrc = np.frombuffer(orank, np.uint32), np.frombuffer(osrc, np.uint32)
        spilled += sp
        items += ni
        for x in d:
            j = int(x["rec_idx"])
            got.append((int(first_rec[int(orank[j])]) + int(osrc[j]), int(x["reader_slot"])))
        k = np.frombuffer(k, np.int64)
        moved = k != 1
        assert not (moved & (owner_ack != 1)).any(), "two owners advanced one proxy"
        owner_ack[moved] = k[moved]
    got.sort(key=lambda t: t[0])  # stable: set order inside a record
    exp = [(int(x["rec_idx"]), int(x["reader_slot"])) for x in dels]
    assert got == exp, (len(got), len(exp))
    assert np.array_equal(owner_ack, ack)
    assert len(exp) > 0
    return spilled, items


@pytest.mark.parametrize("world", [2, 3])
def test_owner_ingest_c3_at_c5_indices(world):
    """C3 mix (DATA / HEARTBEAT / GAP with bitmaps / INFO_*) with the ranks' chunks at C5's
    generator indices; slots large enough for everything (no spill)."""
    spilled, items = _run(world, oracle.WL_C3, 2500, C5_STRIDE, cap=12000, bcap=1 << 20)
    assert spilled == 0 and items > 5000


@pytest.mark.parametrize("world", [2, 3])
def test_owner_ingest_forced_small_cap(world):
    """Slots of 50 records / 256 blob bytes: most items cross in the exact spill round."""
    spilled, items = _run(world, oracle.WL_C3, 2500, C5_STRIDE, cap=50, bcap=256)
    assert spilled > items // 2


@pytest.mark.parametrize("cap,bcap", [(20000, 32 << 20), (64, 4096)])
def test_owner_reassembly_c4(cap, bcap):
    """DataFrag: 64-KiB samples whose fragments straddle the ranks' chunks; the owner
    reassembles them from the payload blobs and ingests the completed samples."""
    spilled, items = _run(2, oracle.WL_C4, 3000, 3000, cap=cap, bcap=bcap)
    assert (spilled > 0) == (cap == 64)
