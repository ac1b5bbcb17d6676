"""Receive side end to end on the GPU: datagrams sent over UDP loopback land in
the slots of a pinned host arena (io_uring buffer ring, or recvmmsg), and the
device parses that arena in place (zero-copy from host memory) — bit-exact with
the CPU oracle on the same slots; then the received batch goes through the
history-cache ingest."""
import numpy as np
import pytest

import oracle
from rtps_rx.records import pack_match_table, DATA

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


def _receive_all(rxu, sent, burst=64):  # a burst must fit the socket buffer (rmem_max)
    from rtps_rx import udp
    offs, lens = [], []
    for k in range(0, len(sent), burst):
        packed, poff, plen = oracle.pack(sent[k:k + burst])
        assert udp.send_batch("127.0.0.1", rxu.port, packed, poff, plen) == len(poff)
        got = 0
        while got < len(poff):
            o, n = rxu.recv_batch(4096, timeout_ms=2000)
            assert len(o) > 0, f"burst {k}: {got} of {len(poff)}"
            offs.append(o.copy())
            lens.append(n.copy())
            got += len(o)
    return np.concatenate(offs), np.concatenate(lens)


@pytest.mark.parametrize("force_recvmmsg", [False, True])
def test_loopback_zero_copy_parse(force_recvmmsg):
    import rtps_rx
    from rtps_rx import udp
    slot, nslot = 2048, 8192
    arena = torch.zeros(slot * nslot, dtype=torch.uint8, pin_memory=True)
    rxu = udp.UdpReceiver(arena, slot_bytes=slot, force_recvmmsg=force_recvmmsg, rcvbuf_bytes=4 << 20)
    a, o0, l0 = oracle.gen(oracle.WL_C3, 6000)
    sent = [a[int(x):int(x) + int(y)].tobytes() for x, y in zip(o0, l0)]
    off, ln = _receive_all(rxu, sent)
    host = arena.numpy()
    assert [host[int(x):int(x) + int(y)].tobytes() for x, y in zip(off, ln)] == sent
    n = len(off)
    rx = rtps_rx.MessageReceiver(oracle.OWN_PREFIX, max_datagrams=n)
    st, recs, _, rb = oracle.parse(host, off, ln, threads=8)
    wk = recs["kind"] == DATA
    guids = sorted({bytes(r["prefix"]) + bytes(r["writer_id"]) for r in recs[wk]})
    tbl = pack_match_table([(g, i) for i, g in enumerate(guids)])
    rx.set_match_table(tbl)
    st, recs, (t_off, t_ent), rb = oracle.parse(host, off, ln, match_table=tbl, threads=8)
    # offsets / lengths in pinned memory too: the whole input is read over PCIe in place
    off_t = torch.from_numpy(off.view(np.int64)).pin_memory()
    ln_t = torch.from_numpy(ln.view(np.int32)).pin_memory()
    cap = rtps_rx.max_records(ln)
    outs = rx.alloc_outputs(n, cap)
    iouts = rx.alloc_ingest_outputs(cap, len(tbl))
    rx.parse_batch_device(arena, off_t, ln_t, n, outs)
    rx.ingest(arena, off_t, outs, iouts)
    rx.sync()
    m = int(outs["n_records"].item())
    assert m == len(recs)
    assert np.array_equal(outs["status"][:n].cpu().numpy(), st)
    assert outs["records"][:m].cpu().numpy().tobytes() == recs.tobytes()
    g_off, g_ent = rx.expand_targets(outs["target"][:m].cpu().numpy().view(np.uint32))
    assert np.array_equal(g_off, t_off) and g_ent.tobytes() == t_ent.tobytes()
    ing = oracle.HistoryIngest(tbl)
    o_acc, o_accepted, o_ack = ing.batch(host, off, recs)
    assert np.array_equal(iouts["accept"][:m].cpu().numpy(), o_acc)
    assert np.array_equal(iouts["ack_base"][:len(tbl)].cpu().numpy(), o_ack)
    rxu.release(off)
    rxu.close()
    rx.close()
