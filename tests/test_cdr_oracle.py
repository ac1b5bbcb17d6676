"""CPU checks of the CDR decode oracle (a18): the reference's ShapeType vector,
an independent Python restatement on mixed corpora (every error class, LE/BE),
round trips through the encoder and edge cases of the classic-CDR rules."""
import struct

import numpy as np
import pytest

import cdr_ref
import oracle
from golden_cases import cases
from rtps_rx import cdr
from rtps_rx.records import DATA

TYPES = {
    "shape": cdr.ShapeType,
    "mixed": cdr_ref.MIXED,
    "prims": cdr.CdrType([("a", "u8"), ("b", "u64"), ("c", "i16"), ("d", "f32"), ("e", "i8"), ("f", "f64")]),
    "seqs": cdr.CdrType([("s", cdr.Seq("f64", 4)), ("t", cdr.Seq("u8", 9)), ("n", cdr.String(3)),
                         ("v", cdr.Seq("i32", 0))]),
    "empty": cdr.CdrType([]),
    "segs": cdr_ref.SEGS,
    # composite elements (SEQ_BEGIN / ARRAY_BEGIN ... END): parity unpinned (no reference vector)
    "polygon": cdr_ref.POLYGON,
    "nested": cdr_ref.NESTED,
}


def _decode_corpus(t, n, seed):
    dgrams = cdr_ref.corpus(t, n, seed)
    arena, off, ln = oracle.pack(dgrams)
    st, recs, _, _ = oracle.parse(arena, off, ln)
    assert (st == 0).all()
    return arena, off, recs


def test_shape_type_red_known_answer():
    """rtps/message_receiver.rs:1250-1254 decodes the DATA payload as ShapeType with color "RED"."""
    dgram = next(c[1] for c in cases() if c[0] == "mr_shapes_red")
    arena, off, ln = oracle.pack([dgram])
    st, recs, _, _ = oracle.parse(arena, off, ln)
    rows, status = oracle.cdr_decode(cdr.ShapeType, arena, off, recs)
    data = [i for i, r in enumerate(recs) if r["kind"] == DATA]
    assert len(data) == 1 and status[data[0]] == cdr.CDR_OK
    assert all(status[i] == cdr.CDR_NOT_DATA for i in range(len(recs)) if i not in data)
    v = cdr.ShapeType.to_python(cdr.ShapeType.rows(rows)[data[0]])
    assert v == {"color": "RED", "x": 105, "y": 23, "shapesize": 30}
    assert not rows[[i for i in range(len(recs)) if i not in data]].any()


@pytest.mark.parametrize("name", sorted(TYPES))
def test_oracle_matches_python_restatement(name):
    t = TYPES[name]
    arena, off, recs = _decode_corpus(t, 600, seed=len(name))
    rows, status = oracle.cdr_decode(t, arena, off, recs)
    exp_rows, exp_status = cdr_ref.expected_rows(t, arena, off, recs)
    bad = np.nonzero(status != exp_status)[0]
    assert len(bad) == 0, f"{name}: status differs at {bad[:8]}: {status[bad[:8]]} vs {exp_status[bad[:8]]}"
    assert np.array_equal(rows, exp_rows), f"{name}: rows differ at {np.nonzero((rows != exp_rows).any(1))[0][:8]}"
    if name != "empty":
        hist = np.bincount(status, minlength=7)
        assert hist[cdr.CDR_OK] > 0 and hist[cdr.CDR_NOT_DATA] > 0 and hist[cdr.CDR_BAD_ENCODING] > 0


@pytest.mark.parametrize("le", [True, False])
@pytest.mark.parametrize("name", ["mixed", "polygon", "nested"])
def test_round_trip(le, name):
    t = TYPES[name]
    rng = np.random.default_rng(7 + le)
    vals = [cdr_ref.random_values(t, rng) for _ in range(64)]
    dgrams = [cdr_ref.data_datagram(cdr_ref.payload(t, v, le), sn=i + 1) for i, v in enumerate(vals)]
    arena, off, ln = oracle.pack(dgrams)
    st, recs, _, _ = oracle.parse(arena, off, ln)
    rows, status = oracle.cdr_decode(t, arena, off, recs)
    assert (status == cdr.CDR_OK).all()
    for v, row in zip(vals, t.rows(rows)):
        got = t.to_python(row)
        for k in v:
            want = v[k]
            if isinstance(want, float):
                assert struct.pack("<d", got[k]) == struct.pack("<d", want) or got[k] == want, k
            elif name != "mixed":  # composite values: float32 elements round-trip through f32
                assert _approx(got[k], want), (k, got[k], want)
            else:
                assert got[k] == (list(want) if isinstance(want, list) else want), (k, got[k], want)


def _approx(a, b):
    if isinstance(b, dict):
        return a.keys() == b.keys() and all(_approx(a[k], b[k]) for k in b)
    if isinstance(b, (list, tuple)):
        return len(a) == len(b) and all(_approx(x, y) for x, y in zip(a, b))
    if isinstance(b, float):
        return float(np.float32(b)) == a or a == b
    return a == b


def _one(t, value, rep=cdr_ref.REP_CDR_LE):
    dg = cdr_ref.data_datagram(rep + b"\x00\x00" + value)
    arena, off, ln = oracle.pack([dg])
    st, recs, _, _ = oracle.parse(arena, off, ln)
    rows, status = oracle.cdr_decode(t, arena, off, recs)
    return int(status[0]), rows[0]


def test_edge_rules():
    S = cdr.CdrType([("s", cdr.String(8))])
    assert _one(S, struct.pack("<I", 0))[0] == cdr.CDR_OK              # length 0: empty string
    assert _one(S, struct.pack("<I", 1) + b"\x00")[0] == cdr.CDR_OK    # "" with NUL
    st, row = _one(S, struct.pack("<I", 3) + b"hiX")                  # last byte dropped, NUL not checked
    assert st == cdr.CDR_OK and bytes(row[4:6]) == b"hi" and row[0] == 2
    assert _one(S, struct.pack("<I", 10) + b"12345678\x00")[0] == cdr.CDR_EOF
    assert _one(S, struct.pack("<I", 10) + b"123456789\x00")[0] == cdr.CDR_TOO_LONG
    assert _one(S, struct.pack("<I", 3) + b"\xc3\xa9\x00")[0] == cdr.CDR_OK  # é
    assert _one(S, struct.pack("<I", 2) + b"\xc3\x00")[0] == cdr.CDR_BAD_UTF8
    # empty sequence of 8-byte elements: no alignment padding is consumed
    Q = cdr.CdrType([("q", cdr.Seq("u64", 2)), ("x", "u32")])
    st, row = _one(Q, struct.pack("<II", 0, 77))
    assert st == cdr.CDR_OK and struct.unpack_from("<I", row, Q.ops[1]["out_off"])[0] == 77
    st, row = _one(Q, struct.pack("<IIQI", 1, 0, 5, 9))                # pad 4 before the u64
    assert st == cdr.CDR_OK and struct.unpack_from("<IQ", row, 0)[0] == 1
    # trailing bytes after the type are ignored (bytes_consumed is only reported)
    P = cdr.CdrType([("a", "u16")])
    assert _one(P, b"\x01\x02\xff\xff\xff\xff")[0] == cdr.CDR_OK
    assert _one(P, b"\x01")[0] == cdr.CDR_EOF
    B = cdr.CdrType([("b", "bool")])
    assert [_one(B, bytes([x]))[0] for x in (0, 1, 2, 255)] == [0, 0, cdr.CDR_BAD_BOOL, cdr.CDR_BAD_BOOL]
    # rep ids: CDR_BE / CDR_LE / PL_CDR_LE accepted (cdr_adapters.rs:96-100), PL_CDR_BE refused
    U = cdr.CdrType([("u", "u32")])
    st, row = _one(U, b"\x00\x00\x01\x02", rep=cdr_ref.REP_CDR_BE)
    assert st == 0 and bytes(row[:4]) == b"\x02\x01\x00\x00"
    assert _one(U, b"\x00\x00\x01\x02", rep=cdr_ref.REP_PL_CDR_LE)[0] == 0
    assert _one(U, b"\x00\x00\x01\x02", rep=cdr_ref.REP_PL_CDR_BE)[0] == cdr.CDR_BAD_ENCODING


def test_type_layout():
    t = cdr_ref.MIXED
    assert t.row_bytes % 4 == 0 and t.row_dtype.itemsize == t.row_bytes
    assert (t.ops["out_off"] % 4 == 0).all() and (np.diff(t.ops["out_off"].astype(int)) > 0).all()
    assert cdr.ShapeType.row_bytes == 144
    with pytest.raises(ValueError):
        cdr.CdrType([(f"f{i}", "u8") for i in range(cdr.MAX_OPS + 1)])


def test_composite_rules():
    """Sequences / arrays of strings and structs (serde Vec<T> / [T; N] through cdr-encoding):
    a u32 count aligned to 4, elements with no alignment of their own, each primitive
    aligned to its size from the value start; TOO_LONG only after the elements validate."""
    Tg = cdr.CdrType([("t", cdr.Seq(cdr.String(4), 2))])
    s3 = lambda a, b, c: struct.pack("<I", 3) + b"".join(  # noqa: E731
        struct.pack("<I", len(x) + 1) + x + b"\x00" + bytes((-(len(x) + 1)) % 4) for x in (a, b, c))
    st, row = _one(Tg, struct.pack("<I", 2) + struct.pack("<I", 3) + b"ab\x00\x00" + struct.pack("<I", 1) + b"\x00")
    assert st == cdr.CDR_OK and Tg.to_python(Tg.rows(row)[0]) == {"t": ["ab", ""]}
    assert _one(Tg, s3(b"a", b"b", b"c"))[0] == cdr.CDR_TOO_LONG           # n = 3 > 2, all valid
    assert _one(Tg, s3(b"a", b"b", b"\xff"))[0] == cdr.CDR_BAD_UTF8        # the element's own error first
    assert _one(Tg, s3(b"a", b"b", b"c")[:-4])[0] == cdr.CDR_EOF
    assert _one(Tg, s3(b"a", b"abcde", b"c"))[0] == cdr.CDR_TOO_LONG       # a string past its slot
    # struct elements: u8 then f64 aligned to 8 from the value start
    E = cdr.CdrType([("e", cdr.Seq(cdr.CdrType([("a", "u8"), ("b", "f64")]), 3)), ("z", "u16")])
    v = struct.pack("<IB3xdB7xdH", 2, 7, 1.5, 9, -2.0, 5)
    st, row = _one(E, v)
    assert st == cdr.CDR_OK
    assert E.to_python(E.rows(row)[0]) == {"e": [{"a": 7, "b": 1.5}, {"a": 9, "b": -2.0}], "z": 5}
    # empty sequence of 8-aligned elements: no padding consumed
    assert E.to_python(E.rows(_one(E, struct.pack("<IH", 0, 3))[1])[0]) == {"e": [], "z": 3}
    # elements that read no bytes cannot fail: n > count is TOO_LONG at once (no 2^32 loop)
    Z = cdr.CdrType([("q", cdr.Seq(cdr.Array("u32", 0), 3)), ("x", "u8")])
    assert _one(Z, struct.pack("<IB", 0xFFFFFFFF, 1))[0] == cdr.CDR_TOO_LONG
    st, row = _one(Z, struct.pack("<IB", 2, 1))
    assert st == cdr.CDR_OK and Z.to_python(Z.rows(row)[0]) == {"q": [[], []], "x": 1}
    # a huge count of non-empty elements ends at EOF after the bytes run out
    assert _one(E, struct.pack("<I", 0xFFFFFFFF) + bytes(64))[0] == cdr.CDR_EOF
    # arrays of structs: no count; nested sequences
    A = cdr.CdrType([("p", cdr.Array(cdr.CdrType([("x", "i16"), ("ok", "bool")]), 2)),
                     ("m", cdr.Seq(cdr.Seq("u16", 2), 2))])
    v = struct.pack("<hBxhB", -3, 1, 4, 0) + bytes(1) + struct.pack("<IIHHIH", 2, 2, 10, 11, 1, 12)
    st, row = _one(A, v)
    assert st == cdr.CDR_OK, st
    assert A.to_python(A.rows(row)[0]) == {"p": [{"x": -3, "ok": True}, {"x": 4, "ok": False}], "m": [[10, 11], [12]]}
    assert _one(A, struct.pack("<hBxhB", -3, 2, 4, 0))[0] == cdr.CDR_BAD_BOOL


def test_composite_layout():
    t = cdr_ref.POLYGON
    kinds = [int(k) for k in t.ops["kind"]]
    assert kinds.count(cdr.OP_SEQ_BEGIN) == 2 and kinds.count(cdr.OP_END) == 2
    b = kinds.index(cdr.OP_SEQ_BEGIN)
    assert int(t.ops[b]["stride"]) == 8 and int(t.ops[b]["count"]) == 8
    assert t.row_dtype.itemsize == t.row_bytes == t.row_dtype["pts"].itemsize + 20 + 4 + 4 * 16 + 4
    with pytest.raises(ValueError):  # depth > RTPS_CDR_MAX_DEPTH
        cdr.CdrType([("d", cdr.Seq(cdr.Seq(cdr.Seq(cdr.Seq(cdr.Seq(cdr.String(1), 1), 1), 1), 1), 1))])


@pytest.mark.parametrize("seed", range(12))
def test_random_composite_types(seed):
    """Random types (composite elements up to 4 deep): the C oracle's iterative walk against
    the independent recursive Python restatement, on corpora with every error class."""
    rng = np.random.default_rng(1000 + seed)
    t = cdr_ref.random_type(rng)
    arena, off, recs = _decode_corpus(t, 300, seed=seed)
    rows, status = oracle.cdr_decode(t, arena, off, recs)
    exp_rows, exp_status = cdr_ref.expected_rows(t, arena, off, recs)
    assert np.array_equal(status, exp_status), f"seed {seed}: statuses differ"
    assert np.array_equal(rows, exp_rows), f"seed {seed}: rows differ"
    assert (status == cdr.CDR_OK).any()


def test_wide_elements_past_the_slot():
    """cdr_ref.WIDE: 40,000 one-byte elements of a 64,004-byte element row walked past a
    one-element slot (the oracle; the GPU in test_cdr_gpu.py::test_wide_elements_gpu)."""
    for label, value, want in cdr_ref.wide_payloads():
        st, row = _one(cdr_ref.WIDE, value)
        assert st == want, label
        if want == cdr.CDR_OK:
            assert cdr_ref.WIDE.to_python(cdr_ref.WIDE.rows(row)[0])["t"] == 7
