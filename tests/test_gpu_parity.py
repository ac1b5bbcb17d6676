"""GPU parity: the HIP parser (through the C ABI) vs the CPU oracle, bit-exact.

Every record byte, every status byte, every record's target readers (the
GPU's target set expanded through the library's set table against the
oracle's literal available_readers scan), rec_begin and the record count must
be identical.  Inputs: the reference's golden vectors,
the four synthetic BASELINE workloads (generated on the device and copied
back for the oracle), misaligned packing, byte-flip fuzz, edge cases
(empty batch, 64 KiB datagrams, max-records datagrams, arena tail), and the
full 1M-datagram configs.
"""
import os
import struct

import numpy as np
import pytest

import oracle
from golden_cases import cases, check_case, shape_type_from_payload
import rtps_rx.records as rtps_records
from rtps_rx.records import record_to_dict, RECORD_DTYPE, DGRAM_OK, DATA, max_records, NO_TARGET

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def rx():
    import rtps_rx
    r = rtps_rx.MessageReceiver(oracle.OWN_PREFIX, max_datagrams=1 << 21)
    yield r
    r.close()


def _assert_same(gpu, ora, label, rx=None):
    st, recs, tg, rb = ora
    assert np.array_equal(gpu.status, st), f"{label}: status differs at {np.nonzero(gpu.status != st)[0][:10]}"
    assert gpu.n_records == len(recs), f"{label}: {gpu.n_records} records vs oracle {len(recs)}"
    g = gpu.records.view(np.uint8).reshape(-1, 64)
    o = recs.view(np.uint8).reshape(-1, 64)
    if not np.array_equal(g, o):
        bad = np.nonzero((g != o).any(axis=1))[0]
        i = int(bad[0])
        raise AssertionError(f"{label}: {len(bad)} records differ; first #{i}: gpu {record_to_dict(gpu.records[i])}"
                             f" oracle {record_to_dict(recs[i])}")
    assert np.array_equal(gpu.rec_begin, rb), f"{label}: rec_begin differs"
    if rx is not None and tg is not None:
        g_off, g_ent = rx.expand_targets(gpu.target)
        o_off, o_ent = tg
        assert np.array_equal(g_off, o_off), f"{label}: target counts differ at {np.nonzero(g_off != o_off)[0][:10]}"
        assert g_ent.tobytes() == o_ent.tobytes(), f"{label}: target readers differ"


def _parity(rx, arena, off, ln, label, own=None, table=None):
    if table is not None:
        if isinstance(table, rtps_records.Readers):
            rx.set_readers(table)
        else:
            rx.set_match_table(table)
    try:
        gpu = rx.handle_received_batch(arena, off, ln)
        ora = oracle.parse(arena, off, ln, own=own or oracle.OWN_PREFIX, match_table=table, threads=8)
        _assert_same(gpu, ora, label, rx)
    finally:
        if table is not None:
            rx.set_match_table([])
    return gpu


def test_golden_vectors(rx):
    cs = [c for c in cases() if c[2] == oracle.OWN_PREFIX]
    arena, off, ln = oracle.pack([c[1] for c in cs])
    gpu = _parity(rx, arena, off, ln, "golden")
    for i, c in enumerate(cs):
        check_case(c, int(gpu.status[i]), gpu.submessages(i), record_to_dict)


def test_golden_shape_type_red(rx):
    c = next(c for c in cases() if c[0] == "mr_shapes_red")
    arena, off, ln = oracle.pack([c[1]])
    gpu = rx.handle_received_batch(arena, off, ln)
    d = [record_to_dict(r) for r in gpu.records if r["kind"] == DATA][0]
    assert shape_type_from_payload(c[1][d["pl_off"]:d["pl_off"] + d["pl_len"]]) == ("RED", 105, 23, 30)
    assert len(gpu.submessages(0)) == 4  # message_receiver.rs:1223


def test_golden_zero_own_prefix():
    """mr_test_submsg_count uses GUID::default() as own prefix (message_receiver.rs:1280)."""
    import rtps_rx
    r = rtps_rx.MessageReceiver(bytes(12), max_datagrams=64)
    cs = [c for c in cases() if c[2] == bytes(12)]
    arena, off, ln = oracle.pack([c[1] for c in cs])
    gpu = r.handle_received_batch(arena, off, ln)
    _assert_same(gpu, oracle.parse(arena, off, ln, own=bytes(12)), "zero-own")
    assert [len(gpu.submessages(i)) for i in range(len(cs))] == [4, 2]
    r.close()


def _device_gen(rx, wl, n, first_idx=0, n_writers=16):
    import rtps_rx
    off, ln, size = rtps_rx.gen_layout(wl, n, first_idx=first_idx, n_writers=n_writers)
    dev = torch.device("cuda", 0)
    arena_t = torch.zeros(max(size, 16), dtype=torch.uint8, device=dev)
    off_t = torch.from_numpy(off.view(np.int64)).to(dev)
    ln_t = torch.from_numpy(ln.view(np.int32)).to(dev)
    rx.generate(wl, arena_t, off_t, ln_t, n, first_idx=first_idx, n_writers=n_writers)
    rx.sync()
    return arena_t.cpu().numpy(), off, ln


@pytest.mark.parametrize("wl,name", [(1, "T"), (2, "C2"), (3, "C3"), (4, "C4")])
def test_workload_parity(rx, wl, name):
    n = 20000
    arena, off, ln = _device_gen(rx, wl, n, first_idx=12345)
    h_arena, h_off, h_ln = oracle.gen(wl, n, first_idx=12345)
    assert np.array_equal(h_off, off) and np.array_equal(h_ln, ln)
    assert np.array_equal(h_arena[:len(arena)], arena[:len(h_arena)]), "device generator != host generator"
    _parity(rx, arena, off, ln, name)


@pytest.mark.parametrize("hint", [0, 1, 2, 4, 7])
def test_spec_hint_never_changes_results(rx, hint):
    """The speculative single-pass tiles and the two-pass fix-up give identical output."""
    arena, off, ln = oracle.gen(oracle.WL_C3, 30000)
    # splice one-DATA datagrams (T) in front so some tiles are speculative for hint 1
    a2, o2, l2 = oracle.gen(oracle.WL_C2, 3000)
    dg = [a2[int(o):int(o) + int(l)].tobytes() for o, l in zip(o2, l2)] + \
         [arena[int(o):int(o) + int(l)].tobytes() for o, l in zip(off, ln)] + \
         [a2[int(o):int(o) + int(l)].tobytes() for o, l in zip(o2, l2)]
    A, O, L = oracle.pack(dg)
    rx.set_spec_hint(hint)
    try:
        _parity(rx, A, O, L, f"hint{hint}")
    finally:
        rx.set_spec_hint(1)


def test_match_table(rx):
    import rtps_rx
    arena, off, ln = oracle.gen(oracle.WL_C3, 20000)
    # matched writers: 10 of the 16 generated writers, slot = writer index; plus duplicates (first wins)
    st, recs, _, _ = oracle.parse(arena, off, ln)
    guids = sorted({bytes(r["prefix"]) + bytes(r["writer_id"]) for r in recs if r["kind"] == DATA})
    # compatibility form; guids[0] also goes to a second reader (slot 99): one writer, two readers
    entries = [(g, i % 7) for i, g in enumerate(guids[:40])] + [(guids[0], 99)]
    table = rtps_rx.pack_match_table(entries)
    gpu = _parity(rx, arena, off, ln, "match", table=table)
    assert (gpu.target != NO_TARGET).sum() > 0


def _c3_reader_sets(recs):
    """Readers for C3 traffic (a15): two readers on the same writers, a stateless reader
    with proxies, a BestEffort reader matched to writers of a foreign prefix (its
    records are targeted by entity id only), readers listed out of EntityId order."""
    from rtps_rx.records import READER_STATELESS, READER_BEST_EFFORT
    guids = sorted({bytes(r["prefix"]) + bytes(r["writer_id"]) for r in recs if r["kind"] == DATA})
    readers = [(bytes([0, 0, 5, 0x07]), 3, 0), (bytes([0, 0, 1, 0x07]), 1, 0),
               (bytes([0, 0, 2, 0x04]), 2, READER_STATELESS), (bytes([0, 0, 4, 0x07]), 4, READER_BEST_EFFORT)]
    foreign = sorted({bytes([0x55] * 12) + g[12:] for g in guids[10:]})
    proxies = [(g, 1) for g in guids[::2]] + [(g, 0) for g in guids[:6]] + [(g, 2) for g in guids[6:10]] + \
              [(g, 3) for g in foreign]
    return rtps_records.Readers(readers, proxies)


def test_reader_sets(rx):
    """a15 (dp_event_loop.rs:266-327, reader.rs:474-484, 712-739): one writer to several
    readers, stateless readers never targeted, writers known by entity id only, builtin-
    and vendor-kind writers: every record's target readers == the oracle's scan."""
    import ingest_ref as R
    A, O, L = oracle.pack(R.a15_stream(6000, 3), align=1)
    gpu = _parity(rx, A, O, L, "a15 stream", table=R.a15_readers())
    assert (gpu.target != NO_TARGET).sum() > 1000
    arena, off, ln = oracle.gen(oracle.WL_C3, 30000)
    _, recs, _, _ = oracle.parse(arena, off, ln)
    _parity(rx, arena, off, ln, "C3 reader sets", table=_c3_reader_sets(recs))


@pytest.mark.parametrize("hint", [1, 0])
def test_reader_sets_full_size_c3(rx, hint):
    """1M C3 datagrams with the multi-reader table, speculative and chained launches."""
    n = 1 << 20
    arena, off, ln = _device_gen(rx, 3, n)
    _, recs, _, _ = oracle.parse(arena[:4 << 20], off[:2000], ln[:2000])
    rx.set_spec_hint(hint)
    try:
        _parity(rx, arena, off, ln, f"C3-1M reader sets hint {hint}", table=_c3_reader_sets(recs))
    finally:
        rx.set_spec_hint(1)


def test_misaligned_packing(rx):
    arena, off, ln = oracle.gen(oracle.WL_C3, 5000)
    dg = [arena[int(o):int(o) + int(l)].tobytes() for o, l in zip(off, ln)]
    for align in (1, 2, 3):
        a2, o2, l2 = oracle.pack(dg, align=align) if align > 1 else oracle.pack(dg, align=1)
        if align == 3:  # odd start
            a2 = np.concatenate([np.zeros(3, np.uint8), a2])
            o2 = o2 + 3
        _parity(rx, a2, o2, l2, f"align{align}")


def test_fuzz_byte_flips(rx):
    rng = np.random.default_rng(7)
    arena, off, ln = oracle.gen(oracle.WL_C3, 20000)
    arena = arena.copy()
    for _ in range(4):
        a = arena.copy()
        k = len(a) // 40
        pos = rng.integers(0, len(a), k)
        a[pos] = rng.integers(0, 256, k).astype(np.uint8)
        _parity(rx, a, off, ln, "fuzz")
    # header-region flips hit the walk hardest
    a = arena.copy()
    for o, l in zip(off[::3], ln[::3]):
        p = int(o) + int(rng.integers(0, min(int(l), 64)))
        a[p] = rng.integers(0, 256)
    _parity(rx, a, off, ln, "fuzz-headers")


def test_random_submessage_soup(rx):
    """Random kinds/lengths/flags: exercises every error path of every reader."""
    arena, off, ln = _soup(20000)
    _parity(rx, arena, off, ln, "soup")


def test_edge_cases(rx):
    dg = []
    dg.append(b"")                                              # empty datagram
    dg.append(b"RTPS")                                          # short
    dg.append(b"RTPS\x02\x04\x01\x12\x00DDSPING")               # 16-B ping
    dg.append(b"RTPX" + bytes(16))                              # RTPX
    dg.append(b"RTPS\x03\x00" + bytes(14))                      # version 3
    dg.append(b"RTPS\x02\x04" + bytes(14))                      # header only: OK, 0 records
    dg.append(b"RTPS\x02\x04" + bytes(14) + b"\x09\x01")         # trailing 2 bytes
    hdr = b"RTPS\x02\x04\x01\x12" + bytes(range(1, 13))
    # max records: INFO_TS with Invalidate and length 0, repeated to 64 KiB
    dg.append(hdr + b"\x09\x03\x00\x00" * ((65536 - 20) // 4))
    # 64 KiB datagram: one DATA with octetsToNextHeader = 0 (extends to the end)
    body = b"\x00\x00\x10\x00" + bytes(4) + b"\x00\x00\x01\x02" + struct.pack("<iI", 0, 5) + b"\x00\x01\x00\x00"
    big = hdr + b"\x15\x05\x00\x00" + body
    dg.append(big + bytes(65536 - len(big)))
    dg.append(big + bytes(65537 - len(big)))                    # too long for the record layout
    # PAD / INFO_TS with length 0 in the middle
    dg.append(hdr + b"\x01\x01\x00\x00" + b"\x09\x03\x00\x00" + b"\x07\x01\x1c\x00" + bytes(28))
    arena, off, ln = oracle.pack(dg)
    gpu = _parity(rx, arena, off, ln, "edge")
    assert gpu.status.tolist()[:7] == [1, 1, 2, 3, 5, 0, 6]
    assert len(gpu.submessages(7)) == (65536 - 20) // 4
    assert gpu.status[9] == 7


def test_arena_tail_exact(rx):
    """Last datagram ends exactly at the arena end: the window loads must not lose bytes."""
    arena, off, ln = oracle.gen(oracle.WL_C3, 300)
    dg = [arena[int(o):int(o) + int(l)].tobytes() for o, l in zip(off, ln)]
    a2, o2, l2 = oracle.pack(dg, align=1)
    a2 = a2[:int(o2[-1]) + int(l2[-1])]
    _parity(rx, a2, o2, l2, "tail")


def test_empty_batch(rx):
    gpu = rx.handle_received_batch(np.zeros(16, np.uint8), np.zeros(0, np.uint64), np.zeros(0, np.uint32))
    assert gpu.n_records == 0 and len(gpu.status) == 0


@pytest.mark.parametrize("wl,name", [(1, "T"), (2, "C2"), (3, "C3"), (4, "C4")])
def test_full_size_parity(rx, wl, name):
    """BASELINE full sizes (1M datagrams): bit-exact vs the oracle on all datagrams."""
    n = 1 << 20
    arena, off, ln = _device_gen(rx, wl, n)
    gpu = _parity(rx, arena, off, ln, f"{name}-1M")
    if wl in (1, 2):  # size-independent properties of the one-DATA-per-datagram configs
        assert (gpu.status == DGRAM_OK).all() and gpu.n_records == n
        assert np.array_equal(gpu.records["dgram_idx"], np.arange(n, dtype=np.uint32))
        assert np.array_equal(gpu.records["sn"], np.arange(n) // 16 + 1)
        u = gpu.records["u"].view(np.uint16).reshape(-1, 8)
        assert (u[:, 1] == (980 if wl == 1 else 256)).all()


# The pass for mixed traffic: the product library has the item pass (E / S / W2) only.  The
# measured, rejected passes (chained lane walk C, LDS tiles D, record slabs E' / W', round 4's
# record pass W) live in diagnostic builds (-DRTPS_DIAG_PASSES, csrc/diag/mixed_passes.inc);
# with RTPS_RX_LIB naming such a build and RTPS_RX_DIAG_PASSES=1 these tests cover them too,
# and tests/diag_mixed_passes.py holds the chained pass's own tests.
DIAG_PASSES = os.environ.get("RTPS_RX_DIAG_PASSES") == "1"
MIXED_PASSES = [(2, "item")] + ([(3, "rslab"), (0, "chain"), (1, "lds")] if DIAG_PASSES else [])
RECORD_PASSES = [2] + ([1] if DIAG_PASSES else [])


@pytest.mark.parametrize("mp", [m for m, _ in MIXED_PASSES if m in (2, 0)])
@pytest.mark.parametrize("wl,name", [(3, "C3"), (1, "T")])
def test_mixed_launch_full_size(rx, wl, name, mp):
    """Spec hint 0 (mixed traffic): the item pass (E / S / W2), bit-exact at 1M datagrams
    (C3: 1M + 64K, 4352 tiles of 256; T forced through the mixed pass)."""
    n = (1 << 20) + (1 << 16 if wl == 3 else 0)
    arena, off, ln = _device_gen(rx, wl, n)
    rx.set_spec_hint(0)
    rx.debug_set_mixed_pass(mp)
    try:
        _parity(rx, arena, off, ln, f"{name}-1M-{dict(MIXED_PASSES)[mp]}")
    finally:
        rx.debug_set_mixed_pass(2)
        rx.set_spec_hint(1)


@pytest.mark.parametrize("mp,mname", MIXED_PASSES)
@pytest.mark.parametrize("wl", [3, 1])
def test_mixed_passes_agree(rx, wl, mp, mname):
    """The three passes for mixed traffic, the item pass (E/S/W), LDS tiles (D) and the
    chained lane walk (C), bit-exact with the oracle on the same batch (C3, and one-DATA
    traffic forced through the mixed pass), misaligned packing included."""
    a, o, l = oracle.gen(wl, 60000, first_idx=777)
    dg = [a[int(x):int(x) + int(y)].tobytes() for x, y in zip(o[:3000], l[:3000])]
    rx.set_spec_hint(0)
    rx.debug_set_mixed_pass(mp)
    try:
        _parity(rx, a, o, l, f"wl {wl} {mname}")
        for align in (1, 2, 3):
            A, O, L = oracle.pack(dg, align=align)
            O = O + align  # offsets = align mod 16, unaligned for the 16-B staging loads
            A2 = np.zeros(len(A) + 16, np.uint8)
            A2[align:align + len(A)] = A
            _parity(rx, A2, O, L, f"wl {wl} {mname} align {align}")
    finally:
        rx.debug_set_mixed_pass(2)
        rx.set_spec_hint(1)


@pytest.mark.parametrize("mp", [m for m, _ in MIXED_PASSES if m in (1, 2)])
def test_lds_tile_fallbacks(rx, mp):
    """Tiles the LDS pass cannot stage (bytes beyond the image: 64 KiB datagrams; more
    materialised submessages than item slots: INFO_TS-only datagrams) take the lane
    walk inside the same kernel; neighbouring tiles stay on the LDS path.  The same batch
    through the item pass: the wave holding the 1000-record datagram overflows its item
    slab (512) and the record pass walks that wave's datagrams instead."""
    a, o, l = oracle.gen(oracle.WL_C3, 500)
    c3 = [a[int(x):int(x) + int(y)].tobytes() for x, y in zip(o, l)]
    hdr = b"RTPS\x02\x04\x01\x0f" + bytes(range(12))
    many = hdr + b"\x09\x03\x00\x00" * 1000          # 1000 INFO_TS (Invalidate): 1000 records
    big_data = hdr + bytes([0x15, 0x05]) + (65000 - 24).to_bytes(2, "little") + bytes(2) + \
        (16).to_bytes(2, "little") + bytes(16) + b"\x00\x01\x00\x00" + bytes(65000 - 48)
    assert len(big_data) == 65000
    dg = c3[:100] + [many] + c3[100:230] + [big_data, big_data[:64000]] * 2 + c3[230:]
    A, O, L = oracle.pack(dg, align=4)
    rx.set_spec_hint(0)
    rx.debug_set_mixed_pass(mp)
    try:
        gpu = _parity(rx, A, O, L, "LDS fallbacks" if mp == 1 else "item-slab overflow")
        assert int(gpu.status[100]) == DGRAM_OK and len(gpu.submessages(100)) == 1000
        assert int(gpu.status[231]) == DGRAM_OK and int(gpu.status[232]) != DGRAM_OK
    finally:
        rx.debug_set_mixed_pass(2)
        rx.set_spec_hint(1)


def _soup(n, seed=11):
    rng = np.random.default_rng(seed)
    kinds = [0x01, 0x06, 0x07, 0x08, 0x09, 0x0c, 0x0d, 0x0e, 0x0f, 0x12, 0x13, 0x15, 0x16, 0x30, 0x80, 0x02]
    dgrams = []
    for i in range(n):
        d = bytearray(b"RTPS\x02\x04\x01\x12") + bytearray(rng.integers(0, 256, 12, dtype=np.uint8))
        for _ in range(int(rng.integers(1, 6))):
            kind = int(rng.choice(kinds))
            le = int(rng.integers(0, 2))
            flags = int(rng.integers(0, 256)) & ~1 | le
            blen = int(rng.choice([0, 4, 8, 12, 16, 20, 24, 28, 32, 36, 40, 44, 48, 60, 64, int(rng.integers(0, 90))]))
            body = bytearray(rng.integers(0, 256, blen, dtype=np.uint8))
            if blen >= 4 and rng.random() < 0.7:  # plausible otq / numBits
                struct.pack_into("<H" if le else ">H", body, 2, int(rng.choice([16, 28, 17, 30, 8, 0])))
            if kind in (0x06, 0x08, 0x12) and blen >= 28 and rng.random() < 0.7:
                struct.pack_into("<I" if le else ">I", body, {0x06: 16, 0x08: 24, 0x12: 20}[kind],
                                 int(rng.choice([0, 1, 31, 32, 33, 64, 256, 257])))
            if kind in (0x15, 0x16) and blen >= 36 and rng.random() < 0.5:  # inline QoS params
                flags |= 2
            declared = blen if rng.random() < 0.9 else int(rng.integers(0, 120))
            d += bytes([kind, flags]) + struct.pack("<H" if le else ">H", declared) + body
        if rng.random() < 0.05:
            d += bytes(rng.integers(0, 256, int(rng.integers(1, 4)), dtype=np.uint8))
        dgrams.append(bytes(d))
    return oracle.pack(dgrams)


@pytest.mark.parametrize("mp,mname", MIXED_PASSES)
def test_mixed_pass_malformed_inputs(rx, mp, mname):
    """Every pass for mixed traffic on the inputs that hit the error paths: the random
    submessage soup (a datagram dropped after some of its submessages already produced
    items), header byte flips, INFO_SRC / INFO_DST / INFO_TS interleavings of the a15
    reader-set stream, all bit-exact against the oracle."""
    import ingest_ref as R
    rx.set_spec_hint(0)
    rx.debug_set_mixed_pass(mp)
    try:
        arena, off, ln = _soup(12000, seed=23)
        _parity(rx, arena, off, ln, f"soup {mname}")
        rng = np.random.default_rng(5)
        a, o, l = oracle.gen(oracle.WL_C3, 12000)
        a = a.copy()
        for x, y in zip(o[::2], l[::2]):
            a[int(x) + int(rng.integers(0, min(int(y), 96)))] = rng.integers(0, 256)
        _parity(rx, a, o, l, f"fuzz-headers {mname}")
        A, O, L = oracle.pack(R.a15_stream(4000, 5), align=1)
        _parity(rx, A, O, L, f"a15 stream {mname}", table=R.a15_readers())
    finally:
        rx.debug_set_mixed_pass(2)
        rx.set_spec_hint(1)


@pytest.mark.parametrize("emit", RECORD_PASSES)
def test_record_passes_agree(rx, emit):
    """The item pass's record pass W2 (rtps_parse_emit2_kernel; with a diagnostic build also
    round 4's rtps_parse_emit_kernel), bit-exact on mixed traffic with a reader table, the
    malformed soup (items of datagrams dropped later in their walk), misaligned packing and a
    wave whose items overflow its slab (1000 records in one datagram: that wave is walked)."""
    import ingest_ref as R
    rx.set_spec_hint(0)
    rx.debug_set_mixed_pass(2)
    prev = rx.debug_emit(emit)
    try:
        a, o, l = oracle.gen(oracle.WL_C3, 70000, first_idx=99)
        _parity(rx, a, o, l, f"C3 emit {emit}", table=R.a15_readers())
        arena, off, ln = _soup(12000, seed=31)
        _parity(rx, arena, off, ln, f"soup emit {emit}")
        c3 = [a[int(x):int(x) + int(y)].tobytes() for x, y in zip(o[:600], l[:600])]
        hdr = b"RTPS\x02\x04\x01\x0f" + bytes(range(12))
        many = hdr + b"\x09\x03\x00\x00" * 1000
        A, O, L = oracle.pack(c3[:300] + [many] + c3[300:], align=1)
        gpu = _parity(rx, A, O, L, f"slab overflow emit {emit}")
        assert len(gpu.submessages(300)) == 1000
    finally:
        rx.debug_emit(prev)
        rx.set_spec_hint(1)


def test_launch_choice_follows_traffic(rx):
    """The speculative / chained choice follows the previous batch's mix (a lagging
    hint): a mixed batch after mixed ones, a one-DATA batch after mixed ones (chained
    with a stale hint), then one-DATA again; every batch bit-exact."""
    c3 = oracle.gen(oracle.WL_C3, 16 * 256 + 77)
    c2 = oracle.gen(oracle.WL_C2, 20 * 256 + 5)
    for label, (a, o, l) in [("C3 first", c3), ("C3 again", c3), ("C2 after C3", c2), ("C2 again", c2),
                             ("C3 after C2", c3)]:
        _parity(rx, a, o, l, label)


@pytest.mark.parametrize("world", [2, 3, 8])
def test_bucket_by_writer_matches_reference(rx, world):
    from shard_ref import bucket_np
    arena, off, ln = oracle.gen(oracle.WL_C3, 20000)
    dev = torch.device("cuda", 0)
    A = torch.from_numpy(arena).to(dev)
    O = torch.from_numpy(off.view(np.int64)).to(dev)
    L = torch.from_numpy(ln.view(np.int32)).to(dev)
    cap = max_records(ln)
    outs = rx.alloc_outputs(len(ln), cap)
    torch.cuda.synchronize()
    rx.parse_batch_device(A, O, L, len(ln), outs)
    bucketed = torch.empty((cap, 64), dtype=torch.uint8, device=dev)
    counts = torch.zeros(world, dtype=torch.int64, device=dev)
    rx.bucket_by_writer(outs, world, bucketed, counts)
    rx.sync()
    _, recs, _, _ = oracle.parse(arena, off, ln)
    exp, exp_counts = bucket_np(recs, world)
    assert counts.cpu().numpy().tolist() == exp_counts.tolist()
    got = bucketed[:int(exp_counts.sum())].cpu().numpy()
    assert got.tobytes() == exp.view(np.uint8).tobytes()
    # padded buckets: a roomy capacity keeps everything, a tight one keeps each bucket's prefix
    start = np.concatenate([[0], np.cumsum(exp_counts)[:-1]])
    raw = exp.view(np.uint8).reshape(-1, 64)
    for pcap in (int(exp_counts.max()) + 5, max(int(exp_counts.min()) // 2, 1)):
        padded = torch.zeros((world * pcap, 64), dtype=torch.uint8, device=dev)
        pc = torch.zeros(world, dtype=torch.int64, device=dev)
        rx.bucket_by_writer_padded(outs, world, pcap, padded, pc)
        rx.sync()
        assert pc.cpu().numpy().tolist() == exp_counts.tolist()
        pn = padded.cpu().numpy()
        for d in range(world):
            k = min(int(exp_counts[d]), pcap)
            assert pn[d * pcap:d * pcap + k].tobytes() == raw[start[d]:start[d] + k].tobytes(), (pcap, d)
            assert not pn[d * pcap + k:(d + 1) * pcap].any()


@pytest.mark.parametrize("world", [2, 3, 8])
def test_bucket_descriptors_matches_reference(rx, world):
    from shard_ref import desc_bucket_np
    from rtps_rx.records import MATCH_DTYPE, XDESC_DTYPE
    arena, off, ln = oracle.gen(oracle.WL_C3, 20000)
    _, recs0, _, _ = oracle.parse(arena, off, ln)
    guids = sorted({(bytes(r["prefix"]) + bytes(r["writer_id"])) for r in recs0[:4000]})
    table_guids = guids[:max(3, len(guids) * 2 // 3)]  # some writers matched, some not
    tbl = np.zeros(len(table_guids), dtype=MATCH_DTYPE)
    for k, g in enumerate(table_guids):
        tbl[k]["writer_guid"] = np.frombuffer(g, dtype=np.uint8)
        tbl[k]["reader_slot"] = k % 5
    rx.set_match_table(tbl)
    try:
        dev = torch.device("cuda", 0)
        A = torch.from_numpy(arena).to(dev)
        O = torch.from_numpy(off.view(np.int64)).to(dev)
        L = torch.from_numpy(ln.view(np.int32)).to(dev)
        cap = max_records(ln)
        outs = rx.alloc_outputs(len(ln), cap)
        torch.cuda.synchronize()
        rx.parse_batch_device(A, O, L, len(ln), outs)
        _, recs, _, _ = oracle.parse(arena, off, ln, match_table=tbl)
        # TARGETED-only records (the unmatched writers share entity ids with matched ones) go to
        # the owner of their entity set; their set numbers come from the parse's target output,
        # itself held to the oracle's target readers by test_reader_sets
        from rtps_rx.records import ROUTE_MATCHED, ROUTE_TARGETED
        sets = outs["target"][:len(recs)].cpu().numpy().view(np.uint32)
        only_t = ((recs["route"] & ROUTE_TARGETED) != 0) & ((recs["route"] & ROUTE_MATCHED) == 0)
        assert only_t.sum() > 100
        exp = desc_bucket_np(recs, table_guids, world, entity_sets=sets)
        sizes = [len(e) for e in exp]
        assert sum(sizes) > 1000
        for pcap in (max(sizes) + 3, max(min(sizes) // 2, 1)):
            out = torch.zeros((world * pcap, 16), dtype=torch.uint8, device=dev)
            cnt = torch.zeros(world, dtype=torch.int64, device=dev)
            rx.bucket_descriptors(outs, world, pcap, out, cnt)
            rx.sync()
            assert cnt.cpu().numpy().tolist() == sizes
            got = out.cpu().numpy().reshape(-1).view(XDESC_DTYPE)
            for d in range(world):
                k = min(sizes[d], pcap)
                assert got[d * pcap:d * pcap + k].tobytes() == exp[d][:k].tobytes(), (pcap, d)
    finally:
        rx.set_match_table([])


@pytest.mark.parametrize("mode", ["", "padded", "desc", "padded c5"])
def test_sharded_path_two_ranks_gloo(mode):
    """Full N=2 path (device parse + device bucket + all-to-all) on one GPU with gloo;
    "padded" = fixed-capacity buckets with the equal-split exchange; "c5" = the ranks'
    chunks at C5's generator indices (rank * 8M): every owner's received record
    multiset equals the oracle's."""
    _shard_check(2, "gloo", mode.split())


def test_rccl_exchange_one_rank():
    """The library's own RCCL exchange (rtps_rx_exchange, what a Rust host binds) on the
    box's one GPU: a one-rank communicator sends every bucket to itself."""
    out = _shard_check(1, "nccl", ["padded", "c5"])
    assert "library RCCL exchange" in out


def _shard_check(nproc, backend, args):
    import os
    import socket
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
                        "--master-addr=127.0.0.1", f"--master-port={port}",
                        os.path.join(repo, "scripts", "shard_check.py"), backend] + args,
                       capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert r.stdout.count(" OK") == nproc, r.stdout
    return r.stdout


@pytest.mark.parametrize("wl", [1, 3])
def test_zero_copy_host_memory(rx, wl):
    """Arena, offsets, lengths and all outputs in pinned host memory (zero-copy over PCIe)."""
    arena, off, ln = oracle.gen(wl, 20000)
    A = torch.from_numpy(arena).pin_memory()
    O = torch.from_numpy(off.view(np.int64)).pin_memory()
    L = torch.from_numpy(ln.view(np.int32)).pin_memory()
    cap = max_records(ln)
    outs = {"status": torch.empty(len(ln), dtype=torch.uint8).pin_memory(),
            "records": torch.empty((cap, 64), dtype=torch.uint8).pin_memory(),
            "target": torch.empty(cap, dtype=torch.int32).pin_memory(),
            "rec_begin": torch.empty(len(ln), dtype=torch.int32).pin_memory(),
            "n_records": torch.zeros(1, dtype=torch.int64).pin_memory(), "max_records": cap}
    rx.parse_batch_device(A, O, L, len(ln), outs)
    rx.sync()
    st, recs, match, rb = oracle.parse(arena, off, ln)
    n = int(outs["n_records"][0])
    assert n == len(recs)
    assert np.array_equal(outs["status"].numpy(), st)
    assert outs["records"][:n].numpy().tobytes() == recs.view(np.uint8).tobytes()
    assert np.array_equal(outs["rec_begin"].numpy().view(np.uint32), rb)
