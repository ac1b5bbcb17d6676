"""GPU checks of the owner-side exchange (rtps_rx_shard_*):

  * the device pack (shard_hist / shard_scan / shard_scatter) against the numpy
    model (tests/shard_ref.py): counts, cut, every slot and spill item (32-B
    rtps_shard_item), every blob byte (the records of non-DATA kinds and their
    consumers' bytes), for 1 / 2 / 3 / 8 destinations, slots large and small;
  * the device unpack against the model, with the receive buffers filled as W
    sources would fill them;
  * one rank end to end (pack -> host-driven exchange -> unpack -> reassembly +
    ingest on the owner batch) against the oracle, with forced spill;
  * two ranks on the box's GPU over gloo at C5's generator indices, and one rank
    through the library's RCCL rounds (scripts/owner_check.py);
  * the full C5 per-rank size (8M datagrams) through pack + the one-rank RCCL
    rounds + unpack, and through rtps_rx_bucket_by_writer_padded + rtps_rx_exchange
    (scripts/c5_full_check.py)."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

import oracle
from rtps_rx.records import RECORD_DTYPE, DELIVERY_DTYPE, pack_match_table, WRITER_KINDS, max_records
from shard_ref import COUNTS_DTYPE, ITEM_DTYPE, balanced_owner_table, shard_pack_np, shard_unpack_np

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def rx():
    import rtps_rx
    r = rtps_rx.MessageReceiver(oracle.OWN_PREFIX, max_datagrams=1 << 16)
    yield r
    r.close()


def _device_batch(rx, arena, off, ln, tbl=None):
    dev = torch.device("cuda", 0)
    A = torch.from_numpy(arena).to(dev)
    O = torch.from_numpy(off.view(np.int64)).to(dev)
    L = torch.from_numpy(ln.view(np.int32)).to(dev)
    rx.set_match_table(tbl if tbl is not None else [])
    outs = rx.alloc_outputs(len(ln), max_records(ln))
    rx.parse_batch_device(A, O, L, len(ln), outs)
    rx.sync()
    return A, O, outs


def _corpora():
    a3, o3, l3 = oracle.gen(oracle.WL_C3, 6000, first_idx=3 << 23)
    a4, o4, l4 = oracle.gen(oracle.WL_C4, 2000)
    return {"C3": (a3, o3, l3), "C4": (a4, o4, l4)}


CORPORA = _corpora()


@pytest.mark.parametrize("wl", ["C3", "C4"])
@pytest.mark.parametrize("world", [1, 2, 3, 8])
@pytest.mark.parametrize("small", [False, True])
def test_pack_matches_model(rx, wl, world, small):
    from rtps_rx.shard import OwnerShard, dev_to_numpy
    arena, off, ln = CORPORA[wl]
    A, O, outs = _device_batch(rx, arena, off, ln)
    _, recs, _, _ = oracle.parse(arena, off, ln)
    cap, bcap = (37, 1024) if small else (len(recs), 64 << 20)
    sh = OwnerShard(rx, world, None, torch.device("cuda", 0), cap, bcap)
    try:
        sh.pack(A, O, outs)
        rx.sync()
        exp = shard_pack_np(arena, off, recs, world, cap, bcap)
        b = sh.buffers()
        counts = dev_to_numpy(b.send_counts, 32 * world, COUNTS_DTYPE)
        slots = dev_to_numpy(b.send_slots, ITEM_DTYPE.itemsize * world * cap, ITEM_DTYPE)
        blob = dev_to_numpy(b.send_blob, world * bcap)
        tot_n = int(counts["n"].sum())
        tot_b = int(counts["bytes"].sum())
        spill = dev_to_numpy(b.send_spill, ITEM_DTYPE.itemsize * tot_n, ITEM_DTYPE)
        bspill = dev_to_numpy(b.send_blob_spill, tot_b)
        sb = sbb = 0
        spilled = 0
        for d in range(world):
            e, c = exp[d], counts[d]
            assert c.tobytes() == e["counts"][0].tobytes(), (d, c, e["counts"])
            cut, cb, n, nb = int(c["cut"]), int(c["cut_bytes"]), int(c["n"]), int(c["bytes"])
            assert slots[d * cap:d * cap + cut].tobytes() == e["slot_items"].tobytes()
            assert blob[d * bcap:d * bcap + cb].tobytes() == e["slot_blob"].tobytes()
            assert spill[sb + cut:sb + n].tobytes() == e["spill_items"].tobytes()
            assert bspill[sbb + cb:sbb + nb].tobytes() == e["spill_blob"].tobytes()
            sb += n
            sbb += nb
            spilled += n - cut
        assert (spilled > 0) == small
    finally:
        sh.close()


@pytest.mark.parametrize("world", [2, 8])
def test_owner_table_modes(rx, world):
    """the shard's writer -> owner table.  With readers set, the default deal
    (RTPS_OWNER_BALANCED) is the readers' writer GUIDs dealt by rtps_rx_owner_assign: the device
    pack equals the model with that table, no owner is idle and max / mean items per owner is
    <= 1.1 on T's 16 writers; RTPS_OWNER_TOPIC puts every writer of the one reader's topic cache
    on one owner; RTPS_OWNER_HASH is round 4's hash.  owner_of agrees with the pack."""
    from rtps_rx.shard import OwnerShard, dev_to_numpy, OWNER_BALANCED, OWNER_HASH, OWNER_TOPIC
    arena, off, ln = oracle.gen(oracle.WL_T, 8000)
    _, r0, _, _ = oracle.parse(arena, off, ln)
    guids = sorted({bytes(x["prefix"]) + bytes(x["writer_id"]) for x in r0})
    assert len(guids) == 16
    tbl = pack_match_table([(g, 100) for g in guids])
    A, O, outs = _device_batch(rx, arena, off, ln, tbl)
    _, recs, _, _ = oracle.parse(arena, off, ln, match_table=tbl)
    sh = OwnerShard(rx, world, None, torch.device("cuda", 0), len(recs), 1 << 20)
    try:
        for mode in (OWNER_BALANCED, OWNER_TOPIC, OWNER_HASH):
            sh.set_owners(mode)
            sh.pack(A, O, outs)
            rx.sync()
            table = {OWNER_BALANCED: balanced_owner_table(guids, world), OWNER_TOPIC: {g: 0 for g in guids},
                     OWNER_HASH: None}[mode]
            exp = shard_pack_np(arena, off, recs, world, len(recs), 1 << 20, table)
            counts = dev_to_numpy(sh.buffers().send_counts, 32 * world, COUNTS_DTYPE)
            assert counts.tobytes() == np.concatenate([e["counts"] for e in exp]).tobytes(), mode
            n = counts["n"].astype(np.int64)
            if mode == OWNER_BALANCED:
                assert n.min() > 0 and n.max() / n.mean() <= 1.1, n
            if mode == OWNER_TOPIC:
                assert n[0] == n.sum()
            for g in guids:
                want = table[g] if table else sh.owner_of(g)
                assert sh.owner_of(g) == want
    finally:
        sh.close()
        rx.set_match_table([])


def test_owner_table_sticky_device(rx):
    """the default table follows the readers STICKILY.  A writer whose GUID
    sorts before every other joins the readers; the next pack keeps every earlier writer's
    owner (owner_of answers the pending table the same way before the pack commits it), the
    newcomer goes to the least-loaded rank, and the device pack equals the model with that table."""
    from rtps_rx.shard import OwnerShard, dev_to_numpy
    arena, off, ln = oracle.gen(oracle.WL_T, 8000)
    _, r0, _, _ = oracle.parse(arena, off, ln)
    guids = sorted({bytes(x["prefix"]) + bytes(x["writer_id"]) for x in r0})
    world = 4
    A, O, outs = _device_batch(rx, arena, off, ln, pack_match_table([(g, 100) for g in guids]))
    sh = OwnerShard(rx, world, None, torch.device("cuda", 0), len(r0) + 16, 1 << 20)
    try:
        sh.pack(A, O, outs)
        rx.sync()
        before = {g: sh.owner_of(g) for g in guids}
        assert before == balanced_owner_table(guids, world)
        first = b"\x00" * 12 + bytes([0, 0, 1, 2])
        tbl = pack_match_table([(first, 100)] + [(g, 100) for g in guids])
        rx.set_match_table(tbl)
        assert {g: sh.owner_of(g) for g in guids} == before  # pending table, not committed
        sh.pack(A, O, outs)
        rx.sync()
        assert {g: sh.owner_of(g) for g in guids} == before
        load = np.bincount(list(before.values()), minlength=world)
        assert sh.owner_of(first) == int(np.argmin(load))
        table = dict(before)
        table[first] = sh.owner_of(first)
        _, recs, _, _ = oracle.parse(arena, off, ln, match_table=tbl)
        exp = shard_pack_np(arena, off, recs, world, len(r0) + 16, 1 << 20, table)
        counts = dev_to_numpy(sh.buffers().send_counts, 32 * world, COUNTS_DTYPE)
        assert counts.tobytes() == np.concatenate([e["counts"] for e in exp]).tobytes()
    finally:
        sh.close()
        rx.set_match_table([])


def test_owner_topic_default_and_refusal(rx):
    """once topics are set, the shard's default deal is RTPS_OWNER_TOPIC: its
    table (writer GUIDs and entity keys) equals tests/shard_ref.topic_owner_table, a writer
    without a proxy follows its entity id's group, and the device pack equals the model.  Under
    an explicit RTPS_OWNER_BALANCED deal over 2 ranks the ingest refuses the topic caches
    (RTPS_RX_EINVAL); a one-rank shard and RTPS_OWNER_TOPIC take them."""
    import rtps_rx
    from rtps_rx.shard import OwnerShard, dev_to_numpy, OWNER_BALANCED, OWNER_TOPIC
    from shard_ref import topic_owner_table, EKEY
    from test_shard_owner_cpu import _topic_setup
    import ingest_ref as R
    tbl, topics, dgrams = _topic_setup()
    arena, off, ln = oracle.pack(dgrams[:2000], align=16)
    rx.set_readers(tbl)
    rx.set_topics(*topics)
    dev = torch.device("cuda", 0)
    A = torch.from_numpy(arena).to(dev)
    O = torch.from_numpy(off.view(np.int64)).to(dev)
    L = torch.from_numpy(ln.view(np.int32)).to(dev)
    outs = rx.alloc_outputs(len(ln), max_records(ln))
    rx.parse_batch_device(A, O, L, len(ln), outs)
    rx.sync()
    _, recs, _, _ = oracle.parse(arena, off, ln, match_table=tbl)
    sh = OwnerShard(rx, 2, None, dev, len(recs), 1 << 20)
    one = None
    try:
        table = topic_owner_table(tbl, topics[1], 2)
        for k, v in table.items():
            if not k.startswith(EKEY):
                assert sh.owner_of(k) == v, k
        stray = R.PREFIXES[2] + R.BUILTIN_KIND_KEY  # no proxy: by its entity id's group
        assert sh.owner_of(stray) == table[EKEY + R.BUILTIN_KIND_KEY]
        sh.pack(A, O, outs)
        rx.sync()
        exp = shard_pack_np(arena, off, recs, 2, len(recs), 1 << 20, table)
        counts = dev_to_numpy(sh.buffers().send_counts, 64, COUNTS_DTYPE)
        assert counts.tobytes() == np.concatenate([e["counts"] for e in exp]).tobytes()
        rx.ingest_batch(arena, off, ln, tbl.n_proxies, topic_cache=True)  # TOPIC (the default): accepted
        sh.set_owners(OWNER_BALANCED)
        with pytest.raises(rtps_rx.RtpsRxError):
            rx.ingest_batch(arena, off, ln, tbl.n_proxies, topic_cache=True)
        rx.ingest_batch(arena, off, ln, tbl.n_proxies)  # without the topic caches: fine
        sh.set_owners(OWNER_TOPIC)
        rx.ingest_batch(arena, off, ln, tbl.n_proxies, topic_cache=True)
        sh.close()
        one = OwnerShard(rx, 1, None, dev, len(recs), 1 << 20)
        one.set_owners(OWNER_BALANCED)
        rx.ingest_batch(arena, off, ln, tbl.n_proxies, topic_cache=True)  # one rank splits nothing
    finally:
        sh.close()
        if one is not None:
            one.close()
        rx.set_topics([], [])
        rx.ingest_reset()
        rx.topic_reset()
        rx.set_match_table([])


@pytest.mark.parametrize("wl", ["C3", "C4"])
@pytest.mark.parametrize("small", [False, True])
def test_unpack_matches_model(rx, wl, small):
    """Receive buffers filled as 3 sources (3 chunks of the stream) would fill them."""
    from rtps_rx.shard import OwnerShard, dev_copy, dev_to_numpy
    world = 3
    arena, off, ln = CORPORA[wl]
    cap, bcap = (29, 512) if small else (20000, 64 << 20)
    sh = OwnerShard(rx, world, None, torch.device("cuda", 0), cap, bcap)
    try:
        received = []
        per = len(ln) // world
        for s in range(world):
            o, l = off[s * per:(s + 1) * per], ln[s * per:(s + 1) * per]
            _, recs, _, _ = oracle.parse(arena, o, l)
            received.append(shard_pack_np(arena, o, recs, world, cap, bcap)[1])  # what owner 1 gets from source s
        b = sh.buffers()
        rc = np.concatenate([x["counts"] for x in received])
        sp = sum(int(c["n"] - c["cut"]) for c in rc)
        spb = sum(int(c["bytes"] - c["cut_bytes"]) for c in rc)
        from rtps_rx.shard import shard_lib
        assert shard_lib().rtps_rx_shard_reserve_spill(sh._h, sp, spb) == 0
        b = sh.buffers()
        dev_copy(b.recv_counts, rc.ctypes.data, rc.nbytes)
        rs = rbs = 0
        for s, x in enumerate(received):
            dev_copy(b.recv_slots + s * cap * ITEM_DTYPE.itemsize, x["slot_items"].ctypes.data, x["slot_items"].nbytes)
            dev_copy(b.recv_blob + s * bcap, x["slot_blob"].ctypes.data, x["slot_blob"].nbytes)
            sr = np.ascontiguousarray(x["spill_items"])
            dev_copy((b.recv_spill or 0) + rs * ITEM_DTYPE.itemsize, sr.ctypes.data, sr.nbytes)
            dev_copy((b.recv_blob_spill or 0) + rbs, x["spill_blob"].ctypes.data, x["spill_blob"].nbytes)
            rs += len(sr)
            rbs += len(x["spill_blob"])
        assert (rs > 0) == small
        ob = sh.unpack()
        erecs, eoff, earena, (erank, edidx) = shard_unpack_np(received)
        assert ob.n_records == len(erecs) > 100
        assert ob.records().tobytes() == erecs.tobytes()
        assert np.array_equal(ob.dgram_off(), eoff)
        assert ob.arena_bytes()[:len(earena)].tobytes() == earena.tobytes()
        grank, gdidx = ob.origin()
        assert np.array_equal(grank, erank) and np.array_equal(gdidx, edidx)
        n_dev = dev_to_numpy(ob.outs["n_records"].ptr, 8, np.uint64)
        assert int(n_dev[0]) == ob.n_records
    finally:
        sh.close()


@pytest.mark.parametrize("wl,cap,bcap", [("C3", 100000, 1 << 20), ("C3", 300, 512), ("C4", 100, 4096)])
def test_one_rank_owner_pipeline(rx, wl, cap, bcap):
    """pack -> exchange (one rank: the host transport copies) -> unpack -> frag + ingest on the
    owner batch == the oracle's reassembly + ingest of the batch itself."""
    from rtps_rx.shard import OwnerShard
    from rtps_rx.records import FRAG_SAMPLE_DTYPE
    arena, off, ln = CORPORA[wl]
    _, r0, _, _ = oracle.parse(arena, off, ln)
    guids = sorted({bytes(r["prefix"]) + bytes(r["writer_id"]) for r in r0[np.isin(r0["kind"], WRITER_KINDS)]})
    tbl = pack_match_table([(g, 5) for g in guids] + [(g, 6) for g in guids[1::3]])
    A, O, outs = _device_batch(rx, arena, off, ln, tbl)
    rx.ingest_reset()
    rx.frag_reset()
    sh = OwnerShard(rx, 1, None, torch.device("cuda", 0), cap, bcap)
    try:
        sh.pack(A, O, outs)
        sh.exchange()
        sh.finish()
        ob = sh.unpack()
        m = ob.n_records
        fouts = rx.alloc_frag_outputs(max(m, 1), ob.arena.nbytes + 16 * m + (1 << 20))
        iouts = rx.alloc_ingest_outputs(max(m, 1), len(tbl))
        rx.frag_assemble(ob.arena, ob.off, ob.outs, fouts)
        rx.ingest(ob.arena, ob.off, ob.outs, iouts, fouts)
        rx.sync()
        na = int(iouts["n_accepted"].item())
        dels = iouts["accepted"][:na].cpu().numpy().reshape(-1).view(DELIVERY_DTYPE)
        ack = iouts["ack_base"][:len(tbl)].cpu().numpy()
        # oracle on the whole batch; its deliveries name records of the whole batch
        _, recs, _, _ = oracle.parse(arena, off, ln, match_table=tbl)
        samples = oracle.FragAssembler().batch_readers(arena, off, recs, tbl)[0]
        _, odels, oack = oracle.HistoryIngest(tbl).batch(arena, off, recs, samples)
        _, src = ob.origin()  # each owner record's index in the (one) source's parse output
        got = [(int(src[int(d["rec_idx"])]), int(d["reader_slot"])) for d in dels]
        assert got == [(int(d["rec_idx"]), int(d["reader_slot"])) for d in odels]
        assert np.array_equal(ack, oack) and na > (20 if wl == "C4" else 100)
        if wl == "C4":
            ns = int(fouts["n_samples"].item())
            assert ns == len(samples) > 10
            s = fouts["samples"][:ns].cpu().numpy().reshape(-1).view(FRAG_SAMPLE_DTYPE)
            assert np.array_equal(s["sn"], samples["sn"]) and np.array_equal(s["writer_guid"], samples["writer_guid"])
    finally:
        sh.close()
        rx.set_match_table([])


def _torchrun(nproc, script, args, timeout=600):
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
                        "--master-addr=127.0.0.1", f"--master-port={port}", os.path.join(REPO, "scripts", script)]
                       + args, capture_output=True, text=True, timeout=timeout, env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    return r.stdout


@pytest.mark.parametrize("args", [["gloo", "c3"], ["gloo", "c3", "small"], ["gloo", "c4"], ["gloo", "c4", "small"]])
def test_owner_two_ranks_gloo(args):
    """two ranks at C5 generator indices (rank * 8M; C4: consecutive chunks so
    samples straddle them), device parse -> pack -> exchange -> unpack -> reassembly + ingest on
    each owner; every owner's deliveries and ack_base equal the single-rank oracle ingest of the
    whole stream for its writers; "small" forces most items through the spill round."""
    out = _torchrun(2, "owner_check.py", args)
    assert out.count(" OK") == 2, out


def test_owner_one_rank_rccl():
    """The library's RCCL rounds (rtps_rx_shard_exchange / _finish) with a one-rank communicator,
    slots small enough that the spill round runs too."""
    out = _torchrun(1, "owner_check.py", ["nccl", "c3", "small"])
    assert out.count(" OK") == 1 and "library RCCL" in out, out


def test_c5_full_per_rank_size():
    """8M C3 datagrams (C5's per-rank size at 8 GPUs) through pack + the
    one-rank RCCL rounds + unpack, and through bucket_by_writer_padded + rtps_rx_exchange:
    no overflow, no truncation, every item received intact."""
    out = _torchrun(1, "c5_full_check.py", [], timeout=900)
    assert "C5 full OK" in out, out
