"""Native receive loop (rtps_rx_pump) on the GPU: datagrams sent over UDP
loopback are received into a pinned arena, parsed in place, ingested into the
history cache and CDR-decoded, batch by batch, with two batches in flight.
Every batch is checked inside its callback (while its slots still hold the
datagrams) against the CPU oracle run on the same slots: status, records,
target readers, accept counts and deliveries (the oracle's writer proxies
carried across the same batch split) and decoded rows.  Edges: batches cut by the record capacity,
stop_after, an idle link, a callback that stops the loop."""
import threading
import time

import numpy as np
import pytest

import oracle
from rtps_rx.records import pack_match_table, DATA, DELIVERY_DTYPE

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


def _sender(rxu, stats, sent, burst=64, window=128):
    """Publisher thread: bursts of `burst` datagrams, at most `window` ahead of what
    the pump has taken (the socket buffer must hold them: rmem_max)."""
    from rtps_rx import udp

    def run():
        k = 0
        while k < len(sent):
            while k - stats.datagrams > window:
                time.sleep(0.0002)
            packed, poff, plen = oracle.pack(sent[k:k + burst])
            k += udp.send_batch("127.0.0.1", rxu.port, packed, poff, plen)
    t = threading.Thread(target=run, daemon=True)  # never outlives a failed test
    t.start()
    return t


def _hello_type():
    from rtps_rx import cdr
    return cdr.CdrType([("user_id", "i32"), ("message", cdr.String(60))])


class _Checker:
    """on_batch: compare one batch with the oracle on the same arena slots."""

    def __init__(self, host, tbl, sample_type=None, ingest=True, rx=None):
        self.host, self.tbl, self.t, self.rx = host, tbl, sample_type, rx
        self.ing = oracle.HistoryIngest(tbl) if ingest else None
        self.got = []
        self.batches = 0
        self.records = 0
        self.accepted = 0
        self.decoded = 0

    def __call__(self, b):
        n = b.n_datagrams
        off, ln = b.off, b.len
        self.got += [self.host[int(x):int(x) + int(y)].tobytes() for x, y in zip(off, ln)]
        st, recs, (t_off, t_ent), _ = oracle.parse(self.host, off, ln, match_table=self.tbl)
        m = b.n_records
        assert m == len(recs), f"batch {b.seq}: {m} records, oracle {len(recs)}"
        assert np.array_equal(b.outs["status"][:n].cpu().numpy(), st), f"batch {b.seq}: status"
        assert b.outs["records"][:m].cpu().numpy().tobytes() == recs.tobytes(), f"batch {b.seq}: records"
        g_off, g_ent = self.rx.expand_targets(b.outs["target"][:m].cpu().numpy().view(np.uint32))
        assert np.array_equal(g_off, t_off) and g_ent.tobytes() == t_ent.tobytes(), f"batch {b.seq}: targets"
        if self.ing is not None:
            o_acc, o_accepted, _ = self.ing.batch(self.host, off, recs)
            assert np.array_equal(b.iouts["accept"][:m].cpu().numpy(), o_acc), f"batch {b.seq}: accept"
            assert b.n_accepted == len(o_accepted)
            got = b.iouts["accepted"][:b.n_accepted].cpu().numpy().reshape(-1).view(DELIVERY_DTYPE)
            assert got.tobytes() == o_accepted.tobytes(), f"batch {b.seq}: deliveries"
            self.accepted += b.n_accepted
        if self.t is not None:
            o_rows, o_status = oracle.cdr_decode(self.t, self.host, off, recs)
            assert np.array_equal(b.row_status[:m].cpu().numpy(), o_status), f"batch {b.seq}: row status"
            if m:
                assert np.array_equal(b.rows[:m].cpu().numpy(), o_rows.reshape(m, -1)), f"batch {b.seq}: rows"
            self.decoded += int((o_status == 0).sum())
        self.batches += 1
        self.records += m
        return False


def _setup(nslot=8192, slot=2048):
    import rtps_rx
    from rtps_rx import udp
    arena = torch.zeros(slot * nslot, dtype=torch.uint8, pin_memory=True)
    rxu = udp.UdpReceiver(arena, slot_bytes=slot, rcvbuf_bytes=4 << 20)
    rx = rtps_rx.MessageReceiver(oracle.OWN_PREFIX, max_datagrams=4096)
    return rtps_rx, udp, arena, rxu, rx


def _c3_traffic(n):
    a, o0, l0 = oracle.gen(oracle.WL_C3, n)
    sent = [a[int(x):int(x) + int(y)].tobytes() for x, y in zip(o0, l0)]
    st, recs, _, _ = oracle.parse(a, o0, l0, threads=8)
    guids = sorted({bytes(r["prefix"]) + bytes(r["writer_id"]) for r in recs[recs["kind"] == DATA]})
    return sent, pack_match_table([(g, i) for i, g in enumerate(guids)])


@pytest.mark.parametrize("cut", [False, True])
def test_pump_c3_ingest_decode(cut):
    rtps_rx, udp, arena, rxu, rx = _setup()
    sent, tbl = _c3_traffic(6000)
    rx.set_match_table(tbl)
    from rtps_rx import cdr
    t = cdr.CdrType([("a", "u8"), ("b", "i32"), ("c", "u16"), ("d", "f64")])  # decodes C3's random payloads
    # cut: a record capacity of 3000 cuts most batches (C3 bounds are up to 370 per datagram)
    pump = udp.Pump(rx, rxu, max_batch=4096, ingest=True, sample_type=t, max_recs=3000 if cut else None,
                    n_entries=len(tbl))
    chk = _Checker(arena.numpy(), tbl, t, rx=rx)
    th = _sender(rxu, pump.stats, sent)
    stats = pump.run(wait_ms=5, stop_after=len(sent), idle_stop_ms=10000, on_batch=chk)
    th.join()
    assert chk.got == sent
    assert stats.datagrams == stats.completed == len(sent)
    assert stats.batches == chk.batches and stats.records == chk.records and stats.accepted == chk.accepted
    assert chk.accepted > 0 and chk.decoded > 0
    if cut:
        assert stats.batches >= len(sent) * 100 // 3000
    rxu.close()
    rx.close()


def test_pump_hello_world_all_accepted_and_decoded():
    import bench
    rtps_rx, udp, arena, rxu, rx = _setup(slot=256)
    data, off, ln = bench.hello_world_datagrams(20000)
    sent = [data[int(x):int(x) + int(y)].tobytes() for x, y in zip(off, ln)]
    tbl = pack_match_table([(bench.HELLO_PREFIX + bench.HELLO_WRITER, 0)])
    rx.set_match_table(tbl)
    pump = udp.Pump(rx, rxu, max_batch=4096, ingest=True, sample_type=_hello_type(), n_entries=1)
    chk = _Checker(arena.numpy(), tbl, _hello_type(), rx=rx)
    th = _sender(rxu, pump.stats, sent, burst=512, window=2048)
    stats = pump.run(wait_ms=5, stop_after=len(sent), idle_stop_ms=10000, on_batch=chk)
    th.join()
    assert chk.got == sent
    assert stats.accepted == len(sent) and chk.decoded == len(sent)
    rxu.close()
    rx.close()


def test_pump_idle_and_callback_stop():
    rtps_rx, udp, arena, rxu, rx = _setup(nslot=1024)
    sent, tbl = _c3_traffic(100)  # ~80 KB: fits the socket buffer without a running receiver
    rx.set_match_table(tbl)
    pump = udp.Pump(rx, rxu, max_batch=16)
    t0 = time.perf_counter()
    stats = pump.run(wait_ms=2, idle_stop_ms=100)  # nothing sent: returns once idle
    assert stats.datagrams == 0 and stats.batches == 0
    assert time.perf_counter() - t0 < 5
    packed, poff, plen = oracle.pack(sent)
    assert udp.send_batch("127.0.0.1", rxu.port, packed, poff, plen) == len(sent)
    # a callback returning True stops the loop after the batches in flight
    seen = []
    stats = pump.run(wait_ms=50, idle_stop_ms=2000, on_batch=lambda b: seen.append(b.n_datagrams) or True)
    assert 1 <= len(seen) <= 2 and stats.completed == stats.datagrams == sum(seen) < len(sent)
    # the rest is still there for the next run, in order
    chk = _Checker(arena.numpy(), tbl, ingest=False, rx=rx)
    stats2 = pump.run(wait_ms=20, idle_stop_ms=300, on_batch=chk)
    assert stats.datagrams + stats2.datagrams == len(sent)
    assert chk.got == sent[stats.datagrams:]
    rxu.close()
    rx.close()
