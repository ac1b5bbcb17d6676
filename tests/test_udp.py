"""UDP batch receive (rtps_udp_*), CPU side: datagrams sent over loopback land
byte-exact in arena slots, in order, with both backends (io_uring multishot
recv on a provided-buffer ring, and recvmmsg), and the received batch parses
exactly like the datagrams that were sent (the CPU oracle on both).  Edges:
datagrams longer than a slot (dropped, counted), every slot in use (the
multishot recv re-arms after release), empty polls, bad configurations."""
import json
import os

import numpy as np
import pytest

import oracle
from rtps_rx import udp, RtpsRxError

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "vectors.json")


def _backends():
    return ["io_uring", "io_uring_sqpoll", "recvmmsg"]


def _open(arena, backend, **kw):
    rx = udp.UdpReceiver(arena, force_recvmmsg=backend == "recvmmsg", sqpoll=backend == "io_uring_sqpoll", **kw)
    want = {"io_uring": udp.IO_URING, "io_uring_sqpoll": udp.IO_URING_SQPOLL, "recvmmsg": udp.RECVMMSG}[backend]
    if rx.backend != want:
        rx.close()
        pytest.skip(f"{backend} not available here (got backend {rx.backend})")
    return rx


def _drain(rx, want, batch=512, release=True, timeout_ms=2000):
    got_off, got_len = [], []
    data = []
    while len(data) < want:
        off, ln = rx.recv_batch(batch, timeout_ms=timeout_ms)
        if len(off) == 0:
            break
        for o, n in zip(off, ln):
            data.append(rx.arena_np[int(o):int(o) + int(n)].tobytes())
        got_off.append(off.copy())
        got_len.append(ln.copy())
        if release:
            rx.release(off)
    return data


def _golden_datagrams():
    with open(GOLDEN) as f:
        v = json.load(f)
    return [bytes.fromhex(x["hex"]) for x in v["messages"]]


@pytest.mark.parametrize("backend", _backends())
def test_loopback_bytes_and_parse(backend):
    arena = np.zeros(2048 * 1024, dtype=np.uint8)
    rx = _open(arena, backend, slot_bytes=2048, rcvbuf_bytes=8 << 20)
    sent = _golden_datagrams()
    a, off, ln = oracle.gen(oracle.WL_C2, 120)
    sent += [a[int(o):int(o) + int(n)].tobytes() for o, n in zip(off, ln)]
    packed, poff, plen = oracle.pack(sent)
    assert udp.send_batch("127.0.0.1", rx.port, packed, poff, plen) == len(sent)
    got = []
    offs, lens = [], []
    while len(got) < len(sent):
        o, n = rx.recv_batch(64, timeout_ms=2000)
        assert len(o) > 0, f"received {len(got)} of {len(sent)}"
        offs.append(o.copy())
        lens.append(n.copy())
        got += [arena[int(x):int(x) + int(y)].tobytes() for x, y in zip(o, n)]
    assert got == sent
    # the batch, as received (slot offsets), parses like the datagrams that were sent
    o, n = np.concatenate(offs), np.concatenate(lens)
    st_a, rec_a, _, rb_a = oracle.parse(arena, o, n)
    st_b, rec_b, _, rb_b = oracle.parse(packed, poff, plen)
    assert np.array_equal(st_a, st_b) and np.array_equal(rb_a, rb_b)
    assert rec_a.tobytes() == rec_b.tobytes()
    rx.release(o)
    assert len(rx.recv_batch(16, timeout_ms=0)[0]) == 0
    rx.close()


@pytest.mark.parametrize("backend", _backends())
def test_truncated_datagrams_dropped(backend):
    arena = np.zeros(256 * 64, dtype=np.uint8)
    rx = _open(arena, backend, slot_bytes=256)
    sizes = [100, 300, 256, 257, 40, 1000, 16]
    sent = [bytes([i]) * s for i, s in enumerate(sizes)]
    packed, poff, plen = oracle.pack(sent)
    udp.send_batch("127.0.0.1", rx.port, packed, poff, plen)
    got = _drain(rx, 4)
    assert got == [s for s in sent if len(s) <= 256]
    assert rx.truncated.value == 3
    rx.close()


@pytest.mark.parametrize("backend", _backends())
def test_all_slots_in_use_then_release(backend):
    arena = np.zeros(128 * 16, dtype=np.uint8)
    rx = _open(arena, backend, slot_bytes=128, rcvbuf_bytes=1 << 20)
    sent = [i.to_bytes(4, "little") * 20 for i in range(60)]
    packed, poff, plen = oracle.pack(sent)
    udp.send_batch("127.0.0.1", rx.port, packed, poff, plen)
    got, held = [], []
    o, n = rx.recv_batch(100, timeout_ms=2000)
    got += [arena[int(x):int(x) + int(y)].tobytes() for x, y in zip(o, n)]
    assert 0 < len(o) <= 16
    held.append(o.copy())
    o2, _ = rx.recv_batch(100, timeout_ms=0)  # every slot is out: nothing can be received
    assert len(o2) == 0
    rx.release(np.concatenate(held))
    got += _drain(rx, 60 - len(got), batch=8)
    assert got == sent
    rx.close()


def test_bad_configuration():
    arena = np.zeros(4096, dtype=np.uint8)
    for kw in [dict(slot_bytes=100), dict(slot_bytes=24), dict(slot_bytes=4096 * 2)]:
        with pytest.raises(RtpsRxError):
            udp.UdpReceiver(arena, **kw)
    with pytest.raises(RtpsRxError):
        udp.UdpReceiver(np.zeros(48 * 3, dtype=np.uint8), slot_bytes=48)  # 3 slots: not a power of two


def test_pump_refuses_unpinned_arena():
    """The native receive loop parses the arena in place on the GPU: a numpy
    (pageable) arena is refused before anything touches the device."""
    arena = np.zeros(2048 * 16, dtype=np.uint8)
    rx = udp.UdpReceiver(arena, slot_bytes=2048)
    with pytest.raises(RtpsRxError):
        udp.Pump(None, rx, max_batch=16)
    rx.close()
