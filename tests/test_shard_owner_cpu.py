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
import types

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle
from rtps_rx.records import RECORD_DTYPE, DELIVERY_DTYPE, FRAG_SAMPLE_DTYPE, pack_match_table, WRITER_KINDS
from rtps_rx.shard import spill_plan
from shard_ref import COUNTS_DTYPE, ITEM_DTYPE, balanced_owner_table, shard_pack_np, shard_unpack_np

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
        # the shard's default owner table (RTPS_OWNER_BALANCED): the table's writers dealt evenly
        table = balanced_owner_table([bytes(t["writer_guid"]) for t in tbl], world)
        packed = shard_pack_np(arena, off, recs, world, cap, bcap, table)
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


def test_aborted_communicator_is_forgotten():
    """after RTPS_RX_EABORTED the library has freed the communicator, so the owning
    Exchange / OwnerShard drops its handle and every later call raises instead of handing RCCL a
    freed ncclComm_t."""
    import rtps_rx
    from rtps_rx import shard
    owner = types.SimpleNamespace(comm=object())
    shard._COMMS[("test", 0)] = owner.comm
    with pytest.raises(rtps_rx.RtpsRxError):
        shard._check_comm(rtps_rx.RTPS_RX_EABORTED, owner)
    assert owner.comm is None and ("test", 0) not in shard._COMMS
    with pytest.raises(rtps_rx.RtpsRxError):
        shard._live_comm(owner)


def _lpt_mirror(writers, n_ranks, weights=None, groups=None):
    """Python restatement of rtps_rx_owner_assign: groups by total weight, largest first (ties:
    the group's smallest GUID), each to the least-loaded owner (ties: the lowest rank)."""
    n = len(writers)
    weights = [1] * n if weights is None else list(weights)
    groups = list(range(n)) if groups is None else list(groups)
    members = {}
    for w, g in enumerate(groups):
        members.setdefault(g, []).append(w)
    keyed = sorted(members.values(), key=lambda m: (-sum(weights[w] for w in m), min(bytes(writers[w]) for w in m)))
    load, owner = [0] * n_ranks, [0] * n
    for m in keyed:
        best = min(range(n_ranks), key=lambda r: (load[r], r))
        load[best] += sum(weights[w] for w in m)
        for w in m:
            owner[w] = best
    return owner


def test_owner_assign_balances_the_workload_writers():
    """the writers of T / C3 (16 GUIDs from the generator, weighted by their
    records in a batch) dealt over 2 / 4 / 8 owners: max / mean records per owner <= 1.1 and
    no idle owner, where the GUID hash left one of 8 idle and another at 1.5x the mean."""
    from rtps_rx.shard import owner_assign
    from rtps_rx.records import DATA, HEARTBEAT, GAP
    for wl in (oracle.WL_T, oracle.WL_C3):
        a, o, l = oracle.gen(wl, 20000)
        _, recs, _, _ = oracle.parse(a, o, l, threads=8)
        recs = recs[np.isin(recs["kind"], (DATA, HEARTBEAT, GAP))]
        keys = [bytes(p) + bytes(w) for p, w in zip(recs["prefix"], recs["writer_id"])]
        writers = sorted(set(keys))
        assert len(writers) >= 16  # T: 16 writer GUIDs; C3: 16 prefixes x 16 writer ids
        per = {g: 0 for g in writers}
        for k in keys:
            per[k] += 1
        for n in (2, 4, 8):
            own = owner_assign(writers, n)
            assert list(own) == _lpt_mirror(writers, n)
            load = np.bincount(own, weights=[per[g] for g in writers], minlength=n)
            assert load.min() > 0 and load.max() / load.mean() <= 1.1, (wl, n, load)
            # weighted by the records: as good or better
            wown = owner_assign(writers, n, weights=[per[g] for g in writers])
            assert list(wown) == _lpt_mirror(writers, n, [per[g] for g in writers])
            wload = np.bincount(wown, weights=[per[g] for g in writers], minlength=n)
            assert wload.max() <= load.max()


def test_owner_assign_order_free_groups_and_weights():
    """The deal depends on the writers, weights and groups, not on their order (every rank must
    get the same table); a group's writers share an owner; uneven weights go largest first."""
    from rtps_rx.shard import owner_assign
    rng = np.random.default_rng(3)
    writers = [bytes(rng.integers(0, 256, 16, dtype=np.uint8)) for _ in range(40)]
    weights = rng.integers(1, 1000, 40)
    groups = rng.integers(0, 12, 40)
    own = owner_assign(writers, 5, weights, groups)
    assert list(own) == _lpt_mirror(writers, 5, weights, groups)
    for g in set(groups.tolist()):
        assert len(set(own[groups == g].tolist())) == 1
    perm = rng.permutation(40)
    # the same groups under the permutation (group ids renamed to the permuted positions' own ids)
    own2 = owner_assign([writers[i] for i in perm], 5, weights[perm], groups[perm])
    assert [int(x) for x in own2] == [int(own[i]) for i in perm]
    assert list(owner_assign(writers, 1)) == [0] * 40
