"""GPU parity of the batch CDR decode (a18) through the C ABI
(rtps_rx_cdr_decode) vs the CPU oracle (rtps_oracle_cdr_decode): every row
byte and every row status identical."""
import numpy as np
import pytest

import cdr_ref
import oracle
from golden_cases import cases
from rtps_rx import cdr
from rtps_rx.records import DATA
from test_cdr_oracle import TYPES

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def rx():
    import rtps_rx
    r = rtps_rx.MessageReceiver(oracle.OWN_PREFIX, max_datagrams=1 << 21)
    yield r
    r.close()


def _check(rx, t, arena, off, ln, label):
    res, rows, status = rx.take_batch(t, arena, off, ln)
    st, recs, _, _ = oracle.parse(arena, off, ln, threads=8)
    assert res.n_records == len(recs)
    o_rows, o_status = oracle.cdr_decode(t, arena, off, recs)
    bad = np.nonzero(status != o_status)[0]
    assert len(bad) == 0, f"{label}: row status differs at {bad[:8]}: gpu {status[bad[:8]]} oracle {o_status[bad[:8]]}"
    g = rows.view(np.uint8).reshape(len(recs), t.row_bytes) if len(recs) else rows
    if len(recs):
        diff = np.nonzero((g != o_rows).any(axis=1))[0]
        assert len(diff) == 0, f"{label}: {len(diff)} rows differ, first {diff[:8]}"
    return rows, status


def test_shape_type_red(rx):
    dgram = next(c[1] for c in cases() if c[0] == "mr_shapes_red")
    arena, off, ln = oracle.pack([dgram])
    res, rows, status = rx.take_batch(cdr.ShapeType, arena, off, ln)
    i = [k for k, r in enumerate(res.records) if r["kind"] == DATA][0]
    assert status[i] == cdr.CDR_OK
    assert cdr.ShapeType.to_python(rows[i]) == {"color": "RED", "x": 105, "y": 23, "shapesize": 30}


@pytest.mark.parametrize("name", sorted(TYPES))
def test_corpus_parity(rx, name):
    t = TYPES[name]
    dgrams = cdr_ref.corpus(t, 3000, seed=100 + len(name))
    arena, off, ln = oracle.pack(dgrams, align=1)  # unaligned payloads
    _, status = _check(rx, t, arena, off, ln, name)
    if name != "empty":
        assert np.bincount(status, minlength=7)[[0, 1, 2, 3]].all()


@pytest.mark.parametrize("name,clean", [("segs", True), ("segs", False), ("mixed", True), ("shape", True)])
def test_little_endian_chunks(rx, name, clean):
    """All-little-endian batches take the block-copy path for segments (and clean ones the
    all-OK path); mixed-status LE batches mix it with the per-slot path."""
    t = TYPES[name]
    dgrams = cdr_ref.corpus(t, 5000, seed=7, le_only=True, clean=clean)
    arena, off, ln = oracle.pack(dgrams, align=1)
    _, status = _check(rx, t, arena, off, ln, f"{name}-le{'-clean' if clean else ''}")
    if clean:
        assert (status[status != cdr.CDR_NOT_DATA] == cdr.CDR_OK).all()


def test_bad_program_rejected(rx):
    import rtps_rx
    dev = torch.device("cuda", 0)
    outs = rx.alloc_outputs(1, 4)
    rows, st = rx.alloc_rows(cdr.ShapeType, 4)
    arena = torch.zeros(64, dtype=torch.uint8, device=dev)
    off = torch.zeros(1, dtype=torch.int64, device=dev)
    bad = cdr.CdrType([("x", "u32")])
    bad.ops = bad.ops.copy()
    bad.ops["size"] = 3
    with pytest.raises(rtps_rx.RtpsRxError):
        rx.cdr_decode(bad, arena, off, outs, rows, st)
    bad.ops["size"] = 4
    bad.ops["out_off"] = bad.row_bytes  # field past the row
    with pytest.raises(rtps_rx.RtpsRxError):
        rx.cdr_decode(bad, arena, off, outs, rows, st)


def _device_gen(rx, wl, n):
    import rtps_rx
    off, ln, size = rtps_rx.gen_layout(wl, n)
    dev = torch.device("cuda", 0)
    arena_t = torch.zeros(max(size, 16), dtype=torch.uint8, device=dev)
    off_t = torch.from_numpy(off.view(np.int64)).to(dev)
    ln_t = torch.from_numpy(ln.view(np.int32)).to(dev)
    rx.generate(wl, arena_t, off_t, ln_t, n)
    rx.sync()
    return arena_t.cpu().numpy(), off, ln


@pytest.mark.parametrize("wl,t", [(2, "C2Sample"), (1, "TSample"), (3, "ShapeType"), (3, "MIXED"), (4, "C2Sample")])
def test_workload_decode_parity(rx, wl, t):
    typ = cdr_ref.MIXED if t == "MIXED" else getattr(cdr, t)
    arena, off, ln = _device_gen(rx, wl, 20000)
    _check(rx, typ, arena, off, ln, f"wl{wl}-{t}")


def test_c2_full_size(rx):
    """1M C2 datagrams: every record decodes (payload of primitives), bit-exact vs the oracle,
    and the rows are the payload bytes themselves (LE wire = host order)."""
    n = 1 << 20
    arena, off, ln = _device_gen(rx, 2, n)
    rows, status = _check(rx, cdr.C2Sample, arena, off, ln, "C2-1M")
    assert (status == cdr.CDR_OK).all()
    raw = rows.view(np.uint8).reshape(n, -1)
    k = np.arange(0, n, 4099)
    for i in k[:64]:
        base = int(off[i]) + 44 + 4
        assert np.array_equal(raw[i], arena[base:base + cdr.C2Sample.row_bytes])


@pytest.mark.parametrize("wl,t", [(3, "ShapeType"), (1, "TSample"), (3, "MIXED")])
def test_list_decode_parity(rx, wl, t):
    """Compact rows (rtps_rx_cdr_decode_list): row k decodes the record of list entry k.  The
    list is every DATA sample's record index (the rows the per-record layout fills), then the
    same list with a stride of 8 (the rtps_delivery layout) and with entries that name
    non-sample records and out-of-range indices (RTPS_CDR_NOT_DATA, zero rows)."""
    typ = cdr_ref.MIXED if t == "MIXED" else getattr(cdr, t)
    arena, off, ln = _device_gen(rx, wl, 20000)
    st, recs, _, _ = oracle.parse(arena, off, ln, threads=8)
    o_rows, o_status = oracle.cdr_decode(typ, arena, off, recs)
    dev = torch.device("cuda", 0)
    a_t = torch.from_numpy(arena).to(dev)
    off_t = torch.from_numpy(off.view(np.int64)).to(dev)
    ln_t = torch.from_numpy(ln.view(np.int32)).to(dev)
    outs = rx.alloc_outputs(len(ln), max(len(recs), 1))
    rx.parse_batch_device(a_t, off_t, ln_t, len(ln), outs)
    samples = np.nonzero(o_status != cdr.CDR_NOT_DATA)[0].astype(np.uint32)
    others = np.nonzero(o_status == cdr.CDR_NOT_DATA)[0][:50].astype(np.uint32)
    mixed = np.concatenate([samples[:300], others, np.array([len(recs), 0xFFFFFFFF], np.uint32), samples[300:]])
    for lst, stride in ((samples, 4), (mixed, 8)):
        wide = np.zeros((len(lst), stride // 4), np.uint32)
        wide[:, 0] = lst
        wide[:, 1:] = 0xABCDEF01  # the rest of a delivery entry is not read
        l_t = torch.from_numpy(wide.reshape(-1).view(np.int32)).to(dev)
        n_t = torch.tensor([len(lst)], dtype=torch.int64, device=dev)
        rows, rst = rx.alloc_rows(typ, len(lst))
        rx.cdr_decode_list(typ, a_t, off_t, outs, l_t, stride, n_t, len(lst), rows, rst)
        torch.cuda.synchronize()
        rows = rows.cpu().numpy()[:len(lst)]
        rst = rst.cpu().numpy()[:len(lst)]
        ok = lst < len(recs)
        exp_st = np.full(len(lst), cdr.CDR_NOT_DATA, np.uint8)
        exp_st[ok] = o_status[lst[ok]]
        assert np.array_equal(rst, exp_st), f"list stride {stride}: row status differs"
        exp_rows = np.zeros((len(lst), typ.row_bytes), np.uint8)
        exp_rows[ok] = o_rows[lst[ok]]
        assert np.array_equal(rows, exp_rows), f"list stride {stride}: rows differ"


def test_list_decode_without_records(rx):
    """list entries when the batch has no decodable records (max_records = 0, or
    *n_records = 0) are RTPS_CDR_NOT_DATA with zero rows, and the kernel loads no record."""
    typ = cdr.ShapeType
    arena, off, ln = _device_gen(rx, 3, 600)
    dev = torch.device("cuda", 0)
    a_t = torch.from_numpy(arena).to(dev)
    off_t = torch.from_numpy(off.view(np.int64)).to(dev)
    ln_t = torch.from_numpy(ln.view(np.int32)).to(dev)
    outs = rx.alloc_outputs(len(ln), 4 * len(ln))
    rx.parse_batch_device(a_t, off_t, ln_t, len(ln), outs)
    lst = torch.arange(0, 64, dtype=torch.int32, device=dev)
    n_t = torch.tensor([64], dtype=torch.int64, device=dev)
    for label, o in (("max_records 0", dict(outs, max_records=0)),
                     ("n_records 0", dict(outs, n_records=torch.zeros(1, dtype=torch.int64, device=dev)))):
        rows, rst = rx.alloc_rows(typ, 64)
        rows.fill_(0x5A)
        rx.cdr_decode_list(typ, a_t, off_t, o, lst, 4, n_t, 64, rows, rst)
        torch.cuda.synchronize()
        assert (rst.cpu().numpy()[:64] == cdr.CDR_NOT_DATA).all(), label
        assert not rows.cpu().numpy().view(np.uint8).reshape(64, -1)[:64].any(), label


@pytest.mark.parametrize("name", ["polygon", "nested"])
def test_composite_list_parity(rx, name):
    """Composite programs (lane-per-row kernel) in list mode: every DATA sample, then a
    shuffled list with non-sample and out-of-range entries, against the oracle."""
    t = TYPES[name]
    dgrams = cdr_ref.corpus(t, 4000, seed=31)
    arena, off, ln = oracle.pack(dgrams, align=1)
    st, recs, _, _ = oracle.parse(arena, off, ln, threads=8)
    o_rows, o_status = oracle.cdr_decode(t, arena, off, recs)
    dev = torch.device("cuda", 0)
    a_t = torch.from_numpy(arena).to(dev)
    off_t = torch.from_numpy(off.view(np.int64)).to(dev)
    ln_t = torch.from_numpy(ln.view(np.int32)).to(dev)
    outs = rx.alloc_outputs(len(ln), max(len(recs), 1))
    rx.parse_batch_device(a_t, off_t, ln_t, len(ln), outs)
    rng = np.random.default_rng(3)
    lst = np.concatenate([np.arange(len(recs)), [len(recs), 0xFFFFFFFF]]).astype(np.uint32)
    rng.shuffle(lst)
    l_t = torch.from_numpy(lst.view(np.int32)).to(dev)
    n_t = torch.tensor([len(lst)], dtype=torch.int64, device=dev)
    rows, rst = rx.alloc_rows(t, len(lst))
    rx.cdr_decode_list(t, a_t, off_t, outs, l_t, 4, n_t, len(lst), rows, rst)
    torch.cuda.synchronize()
    rows = rows.cpu().numpy().view(np.uint8).reshape(-1, t.row_bytes)[:len(lst)]
    rst = rst.cpu().numpy()[:len(lst)]
    ok = lst < len(recs)
    exp_st = np.full(len(lst), cdr.CDR_NOT_DATA, np.uint8)
    exp_st[ok] = o_status[lst[ok]]
    assert np.array_equal(rst, exp_st)
    exp_rows = np.zeros((len(lst), t.row_bytes), np.uint8)
    exp_rows[ok] = o_rows[lst[ok]]
    assert np.array_equal(rows, exp_rows)
    assert (o_status == cdr.CDR_OK).sum() > 500


def test_bad_composite_program_rejected(rx):
    """Host validation of composite programs: unmatched BEGIN / END, a stride that is not a
    multiple of 4, an element slot past its stride, overlapping slots, depth > 4."""
    import rtps_rx
    dev = torch.device("cuda", 0)
    outs = rx.alloc_outputs(1, 4)
    arena = torch.zeros(64, dtype=torch.uint8, device=dev)
    off = torch.zeros(1, dtype=torch.int64, device=dev)
    good = cdr_ref.POLYGON
    rows, st = rx.alloc_rows(good, 4)
    rx.cdr_decode(good, arena, off, outs, rows, st)  # accepted as built
    b = [int(k) for k in good.ops["kind"]].index(cdr.OP_SEQ_BEGIN)
    e = [int(k) for k in good.ops["kind"]].index(cdr.OP_END)

    def bad(edit):
        t = cdr_ref.POLYGON
        saved = t.ops
        t.ops = t.ops.copy()
        try:
            edit(t.ops)
            with pytest.raises(rtps_rx.RtpsRxError):
                rx.cdr_decode(t, arena, off, outs, rows, st)
        finally:
            t.ops = saved
    bad(lambda o: o.__setitem__(e, (cdr.OP_PRIM, 4, 0, 1, 0)))                       # BEGIN never closed
    bad(lambda o: o.__setitem__(b, (cdr.OP_PRIM, 4, 0, 1, int(o[b]["out_off"]))))    # stray END
    bad(lambda o: o["stride"].__setitem__(b, 6))                                       # stride % 4
    bad(lambda o: o["out_off"].__setitem__(b + 2, 8))                                  # y past the 8-B element
    bad(lambda o: o["out_off"].__setitem__(b + 2, 0))                                  # y over x
    bad(lambda o: o["count"].__setitem__(b, 1 << 20))                                  # slot past the row
    deep = cdr.CdrType([("d", cdr.Seq(cdr.Seq(cdr.Seq(cdr.Seq(cdr.String(1), 1), 1), 1), 1))])
    r2, s2 = rx.alloc_rows(deep, 4)
    rx.cdr_decode(deep, arena, off, outs, r2, s2)  # depth 4 accepted
    ops = deep.ops.copy()
    wrap = np.array([(cdr.OP_ARRAY_BEGIN, 0, deep.row_bytes, 1, 0)], dtype=cdr.OP_DTYPE)  # fits, but depth 5
    deep.ops = np.concatenate([wrap, ops, ops[-1:]])
    with pytest.raises(rtps_rx.RtpsRxError):
        rx.cdr_decode(deep, arena, off, outs, r2, s2)


@pytest.mark.parametrize("seed", range(6))
def test_random_composite_types_gpu(rx, seed):
    """The GPU against the oracle on random types (test_cdr_oracle.test_random_composite_types)."""
    rng = np.random.default_rng(1000 + seed)
    t = cdr_ref.random_type(rng)
    dgrams = cdr_ref.corpus(t, 1500, seed=seed)
    arena, off, ln = oracle.pack(dgrams, align=1)
    _check(rx, t, arena, off, ln, f"random-{seed}")


def test_wide_elements_gpu(rx):
    """cdr_ref.WIDE on the GPU: statuses and rows equal the oracle's, in bounded time."""
    t = cdr_ref.WIDE
    dgrams, want = [], []
    for i, (label, value, st) in enumerate(cdr_ref.wide_payloads()):
        pad = (-len(value)) % 4
        dgrams.append(cdr_ref.data_datagram(cdr_ref.REP_CDR_LE + bytes([0, pad]) + value + bytes(pad), sn=i + 1))
        want.append(st)
    arena, off, ln = oracle.pack(dgrams * 16, align=1)
    _, status = _check(rx, t, arena, off, ln, "wide")
    assert list(status[:4]) == want
