"""Test-side CDR helpers for the batch decode (a18).

serialize(): classic CDR encoder with the rules of the reference's serializer
(cdr-encoding 0.10 CdrSerializer, used by CDRSerializerAdapter
serialization/cdr_adapters.rs:120-180): each primitive aligned to its size
from the start of the value, string = u32 (len+1) + bytes + NUL, sequence =
u32 count + elements, arrays without length, bool = one byte.

decode(): an independent pure-Python restatement of the decoder, used to
cross-check the C oracle (oracle/rtps_oracle.c rtps_oracle_cdr_decode) on
small corpora.  Its rules (alignment, padding only when an element is read,
str::from_utf8, bool 0/1) are cdr-encoding's published behaviour; the only
reference vector is the shapes-demo ShapeType "RED" payload
(rtps/message_receiver.rs:1250-1254), everything else is parity unpinned.
"""
import struct

import numpy as np

from rtps_rx import cdr

_FMT = {"u8": "B", "i8": "b", "u16": "H", "i16": "h", "u32": "I", "i32": "i", "f32": "f",
        "u64": "Q", "i64": "q", "f64": "d"}
REP_CDR_BE, REP_CDR_LE, REP_PL_CDR_BE, REP_PL_CDR_LE = b"\x00\x00", b"\x00\x01", b"\x00\x02", b"\x00\x03"


def _pad(buf, a):
    while len(buf) % a:
        buf.append(0)


def serialize(t, values, le=True):
    """values: {flat field name: value} for CdrType t -> CDR value bytes (no encapsulation header).
    A composite Seq / Array value is a list of element values (dicts for struct elements)."""
    buf = bytearray()
    _ser(t, values, "<" if le else ">", buf)
    return bytes(buf)


def _ser(t, values, e, buf):
    for name, kind, spec in t._layout:
        v = values[name]
        if kind == cdr.OP_PRIM:
            f = _FMT[spec]
            _pad(buf, struct.calcsize(f))
            buf += struct.pack(e + f, v)
        elif kind == cdr.OP_BOOL:
            buf.append(v if type(v) is int else (1 if v else 0))  # ints > 1 make invalid bools
        elif kind == cdr.OP_STRING:
            raw = v.encode() if isinstance(v, str) else bytes(v)
            _pad(buf, 4)
            buf += struct.pack(e + "I", len(raw) + 1) + raw + b"\x00"
        elif kind == cdr.OP_SEQ:
            f = _FMT[spec.prim]
            _pad(buf, 4)
            buf += struct.pack(e + "I", len(v))
            if len(v):
                _pad(buf, struct.calcsize(f))
                buf += struct.pack(e + f * len(v), *v)
        elif kind == cdr.OP_ARRAY:
            f = _FMT[spec.prim]
            if spec.n:
                _pad(buf, struct.calcsize(f))
                buf += struct.pack(e + f * spec.n, *v)
        elif kind in (cdr.OP_SEQ_BEGIN, cdr.OP_ARRAY_BEGIN):
            if kind == cdr.OP_SEQ_BEGIN:  # serde serialize_seq: u32 length, then the elements
                _pad(buf, 4)
                buf += struct.pack(e + "I", len(v))
            for x in v:
                _ser(spec.elem_type, {"v": x} if spec.wrapped else x, e, buf)


def payload(t, values, le=True, rep=None):
    """SerializedPayload bytes: rep id + options + value, padded to 4 (serialized_payload.rs:60-84)."""
    body = serialize(t, values, le)
    rep = rep if rep is not None else (REP_CDR_LE if le else REP_CDR_BE)
    padding = (-len(body)) % 4
    return rep + bytes([0, padding]) + body + bytes(padding)


def _utf8_ok(b):
    try:
        b.decode("utf-8", errors="strict")
    except UnicodeDecodeError:
        return False
    return True


def min_wire(t):
    """The fewest value bytes t can consume (0: it reads nothing, so it cannot fail)."""
    m = 0
    for _, kind, spec in t._layout:
        if kind == cdr.OP_PRIM:
            m += struct.calcsize(_FMT[spec])
        elif kind == cdr.OP_BOOL:
            m += 1
        elif kind in (cdr.OP_STRING, cdr.OP_SEQ, cdr.OP_SEQ_BEGIN):
            m += 4
        elif kind == cdr.OP_ARRAY:
            m += spec.n * struct.calcsize(_FMT[spec.prim])
        elif kind == cdr.OP_ARRAY_BEGIN:
            m += spec.n * min_wire(spec.elem_type)
    return m


class _Fail(Exception):
    def __init__(self, st):
        self.st = st


def decode(t, value, le):
    """(status, {name: value}, expected row bytes) for value bytes (after the 4-byte header).
    The row is built from raw (byte-swapped) element bytes, so floats compare bit-exactly.
    Composite sequences: the elements are read recursively; elements past the slot
    (n > cap) are read but not stored, and the sequence is TOO_LONG after them (at once
    when an element reads no bytes at all, as it cannot fail)."""
    row = bytearray(t.row_bytes)
    cur = [0]
    try:
        out = _dec(t, bytes(value), "<" if le else ">", le, cur, row, 0, True)
    except _Fail as f:
        return f.st, None, bytes(t.row_bytes)
    return cdr.CDR_OK, out, bytes(row)


def _dec(t, value, e, le, cur, row, base, write):
    n = len(value)
    out = {}

    def put(off, raw, sz):  # raw element bytes in wire order -> host (LE) order in the row
        if not write:
            return
        for k in range(0, len(raw), sz):
            el = raw[k:k + sz]
            row[base + off + k:base + off + k + sz] = el if le else el[::-1]

    def put_raw(off, raw):
        if write:
            row[base + off:base + off + len(raw)] = raw

    def u32():
        cur[0] += (-cur[0]) % 4
        if cur[0] + 4 > n:
            raise _Fail(cdr.CDR_EOF)
        x = struct.unpack_from(e + "I", value, cur[0])[0]
        cur[0] += 4
        return x

    off = 0
    for name, kind, spec in t._layout:
        o = off
        if kind in (cdr.OP_PRIM, cdr.OP_ARRAY):
            prim = spec if kind == cdr.OP_PRIM else spec.prim
            f = _FMT[prim]
            sz = struct.calcsize(f)
            cnt = 1 if kind == cdr.OP_PRIM else spec.n
            off += _slot(kind, spec)
            if cnt == 0:
                out[name] = []
                continue
            pos = cur[0]
            pad = (-pos) % sz
            if pos + pad + cnt * sz > n:
                raise _Fail(cdr.CDR_EOF)
            pos += pad
            vals = list(struct.unpack_from(e + f * cnt, value, pos))
            put(o, value[pos:pos + cnt * sz], sz)
            out[name] = vals[0] if kind == cdr.OP_PRIM else vals
            cur[0] = pos + cnt * sz
        elif kind == cdr.OP_BOOL:
            off += 4
            if cur[0] + 1 > n:
                raise _Fail(cdr.CDR_EOF)
            if value[cur[0]] > 1:
                raise _Fail(cdr.CDR_BAD_BOOL)
            out[name] = value[cur[0]] == 1
            put_raw(o, value[cur[0]:cur[0] + 1])
            cur[0] += 1
        elif kind == cdr.OP_STRING:
            off += _slot(kind, spec)
            ln = u32()
            if cur[0] + ln > n:
                raise _Fail(cdr.CDR_EOF)
            sb = value[cur[0]:cur[0] + max(ln - 1, 0)]
            if not _utf8_ok(sb):
                raise _Fail(cdr.CDR_BAD_UTF8)
            if len(sb) > spec.cap:
                raise _Fail(cdr.CDR_TOO_LONG)
            out[name] = sb.decode()
            put_raw(o, struct.pack("<I", len(sb)) + sb)
            cur[0] += ln
        elif kind == cdr.OP_SEQ:
            off += _slot(kind, spec)
            f = _FMT[spec.prim]
            sz = struct.calcsize(f)
            cnt = u32()
            vals = []
            if cnt:
                pad = (-cur[0]) % sz
                if cur[0] + pad + cnt * sz > n:
                    raise _Fail(cdr.CDR_EOF)
                if cnt > spec.cap:
                    raise _Fail(cdr.CDR_TOO_LONG)
                cur[0] += pad
                vals = list(struct.unpack_from(e + f * cnt, value, cur[0]))
                put(o + 4, value[cur[0]:cur[0] + cnt * sz], sz)
                cur[0] += cnt * sz
            put_raw(o, struct.pack("<I", cnt))
            out[name] = vals
        elif kind in (cdr.OP_SEQ_BEGIN, cdr.OP_ARRAY_BEGIN):
            off += _slot(kind, spec)
            et = spec.elem_type
            seq = kind == cdr.OP_SEQ_BEGIN
            cap = spec.cap if seq else spec.n
            cnt = u32() if seq else cap
            if seq:
                put_raw(o, struct.pack("<I", cnt))
            if cnt > cap and min_wire(et) == 0:
                raise _Fail(cdr.CDR_TOO_LONG)
            els = []
            for i in range(cnt):
                x = _dec(et, value, e, le, cur, row, base + o + (4 if seq else 0) + i * et.row_bytes,
                         write and i < cap)
                els.append(x["v"] if spec.wrapped else x)
            if cnt > cap:
                raise _Fail(cdr.CDR_TOO_LONG)
            out[name] = els
    return out


def _slot(kind, spec):
    """Row bytes of one field's slot (include/rtps_rx.h row layout)."""
    a4 = lambda x: (x + 3) // 4 * 4  # noqa: E731
    if kind == cdr.OP_PRIM:
        return a4(struct.calcsize(_FMT[spec]))
    if kind == cdr.OP_BOOL:
        return 4
    if kind == cdr.OP_STRING:
        return 4 + a4(spec.cap)
    if kind == cdr.OP_SEQ:
        return 4 + a4(struct.calcsize(_FMT[spec.prim]) * spec.cap)
    if kind == cdr.OP_ARRAY:
        return a4(struct.calcsize(_FMT[spec.prim]) * spec.n)
    if kind == cdr.OP_SEQ_BEGIN:
        return 4 + spec.cap * spec.elem_type.row_bytes
    return spec.n * spec.elem_type.row_bytes


def expected_rows(t, arena, offs, recs):
    """(rows u8[m, row_bytes], status u8[m]) computed record by record with decode()."""
    from rtps_rx.records import DATA, PK_DATA
    m = len(recs)
    rows = np.zeros((m, t.row_bytes), dtype=np.uint8)
    status = np.zeros(m, dtype=np.uint8)
    for r in range(m):
        rec = recs[r]
        if int(rec["kind"]) != DATA or int(rec["payload_kind"]) != PK_DATA:
            status[r] = cdr.CDR_NOT_DATA
            continue
        u = rec["u"].tobytes()
        pl_off, pl_len = struct.unpack_from("<HH", u, 0)
        rep = u[4:6]
        if rep not in (REP_CDR_BE, REP_CDR_LE, REP_PL_CDR_LE):
            status[r] = cdr.CDR_BAD_ENCODING
            continue
        base = int(offs[int(rec["dgram_idx"])]) + pl_off
        value = bytes(arena[base + 4:base + pl_len])
        st, _, row = decode(t, value, rep != REP_CDR_BE)
        status[r] = st
        rows[r] = np.frombuffer(row, dtype=np.uint8)
    return rows, status


def data_datagram(payload_bytes, sn=1, le=True, writer_key=b"\x00\x00\x01", prefix=bytes(range(1, 13)),
                  flags_extra=0x04):
    """RTPS message with one DATA (reader UNKNOWN, writer user-defined with key) carrying payload_bytes."""
    e = "<" if le else ">"
    body = struct.pack(e + "HH", 0, 16) + b"\x00\x00\x00\x00" + writer_key + b"\x02" + \
        struct.pack(e + "iI", sn >> 32, sn & 0xFFFFFFFF) + payload_bytes
    hdr = b"RTPS" + b"\x02\x04" + b"\x01\x0f" + prefix
    return hdr + bytes([0x15, (1 if le else 0) | flags_extra]) + struct.pack(e + "H", len(body)) + body


def random_values(t, rng, str_alphabet=("a", "Z", "0", " ", "é", "ß", "€", "😀", "\x00")):
    """Random field values that fit t's slots."""
    vals = {}
    for name, kind, spec in t._layout:
        if kind == cdr.OP_PRIM:
            vals[name] = _rand_prim(spec, rng)
        elif kind == cdr.OP_BOOL:
            vals[name] = bool(rng.integers(0, 2))
        elif kind == cdr.OP_STRING:
            s = ""
            while True:
                c = str_alphabet[rng.integers(0, len(str_alphabet))]
                if len((s + c).encode()) > spec.cap or rng.random() < 0.08:
                    break
                s += c
            vals[name] = s
        elif kind == cdr.OP_SEQ:
            vals[name] = [_rand_prim(spec.prim, rng) for _ in range(int(rng.integers(0, spec.cap + 1)))]
        elif kind == cdr.OP_ARRAY:
            vals[name] = [_rand_prim(spec.prim, rng) for _ in range(spec.n)]
        elif kind in (cdr.OP_SEQ_BEGIN, cdr.OP_ARRAY_BEGIN):
            cnt = int(rng.integers(0, spec.cap + 1)) if kind == cdr.OP_SEQ_BEGIN else spec.n
            vals[name] = [_rand_elem(spec, rng, str_alphabet) for _ in range(cnt)]
    return vals


def _rand_elem(spec, rng, str_alphabet):
    x = random_values(spec.elem_type, rng, str_alphabet)
    return x["v"] if spec.wrapped else x


def _rand_prim(p, rng):
    f = _FMT[p]
    if f in "fd":
        x = float(rng.standard_normal() * 1e3)
        return float(np.float32(x)) if f == "f" else x
    bits = struct.calcsize(f) * 8
    if f.isupper():
        return int(rng.integers(0, 1 << bits, dtype=np.uint64)) if bits == 64 else int(rng.integers(0, 1 << bits))
    lo = -(1 << (bits - 1))
    return int(rng.integers(lo, -lo, dtype=np.int64))


BAD_UTF8 = [b"\xc0\x80", b"\xed\xa0\x80", b"\x80", b"\xf0\x80\x80\x80", b"\xf4\x90\x80\x80", b"abc\xe2\x82",
            b"\xff", b"\xe0\x9f\xbf", b"\xc2", b"ok\xf5\x80\x80\x80"]
HB = bytes.fromhex("07010000" "00000000" "00000102" "0000000001000000" "0000000005000000" "01000000")


def corpus(t, n, seed, prefix=bytes(range(1, 13)), le_only=False, clean=False):
    """n datagrams carrying t-typed payloads: clean LE/BE samples plus every error class
    (truncation, byte corruption, bad UTF-8, over-long strings/sequences, bad bool,
    unsupported rep ids, KEY payloads and non-DATA submessages)."""
    rng = np.random.default_rng(seed)
    has = {k for _, k, _ in t._layout}
    out = []
    for i in range(n):
        le = True if le_only else bool(rng.integers(0, 2))
        vals = random_values(t, rng)
        mode = 0 if clean else int(rng.integers(0, 12))
        rep = None
        flags = 0x04
        if mode == 4 and cdr.OP_STRING in has:    # invalid UTF-8 inside a string
            name = next(nm for nm, k, _ in t._layout if k == cdr.OP_STRING)
            vals[name] = BAD_UTF8[int(rng.integers(0, len(BAD_UTF8)))]
        elif mode == 5 and cdr.OP_STRING in has:  # longer than the slot
            name, _, spec = next(x for x in t._layout if x[1] == cdr.OP_STRING)
            vals[name] = "x" * (spec.cap + 1 + int(rng.integers(0, 3)))
        elif mode == 6 and cdr.OP_SEQ in has:     # more elements than the slot
            name, _, spec = next(x for x in t._layout if x[1] == cdr.OP_SEQ)
            vals[name] = [0] * (spec.cap + 1)
        elif mode == 6 and cdr.OP_SEQ_BEGIN in has:
            seqs = [x for x in t._layout if x[1] == cdr.OP_SEQ_BEGIN]
            name, _, spec = seqs[int(rng.integers(0, len(seqs)))]
            vals[name] = [_rand_elem(spec, rng, ("a", "é")) for _ in range(spec.cap + 1 + int(rng.integers(0, 3)))]
        elif mode == 7:
            rep = [REP_PL_CDR_BE, b"\x00\x06", b"\x01\x00", b"\x00\x0a"][int(rng.integers(0, 4))]
        elif mode == 8:
            flags = 0x08  # KEY payload -> not a DATA sample
        elif mode == 3 and cdr.OP_BOOL in has:    # invalid bool byte
            names = [nm for nm, k, _ in t._layout if k == cdr.OP_BOOL]
            vals[names[int(rng.integers(0, len(names)))]] = int(rng.integers(2, 256))
        body = serialize(t, vals, le)
        if mode == 2 and body:                    # truncation
            body = body[:int(rng.integers(0, len(body)))]
        elif mode == 3 and cdr.OP_BOOL not in has and body:  # corrupt one byte
            b = bytearray(body)
            b[int(rng.integers(0, len(b)))] = int(rng.integers(2, 256))
            body = bytes(b)
        elif mode == 9 and body:                  # several random bytes
            b = bytearray(body)
            for _ in range(int(rng.integers(1, 5))):
                b[int(rng.integers(0, len(b)))] = int(rng.integers(0, 256))
            body = bytes(b)
        rep = rep if rep is not None else (REP_CDR_LE if le else REP_CDR_BE)
        if mode in (1, 10) and le and le_only:
            rep = REP_PL_CDR_LE if mode == 10 else rep
        elif mode == 10 and le:
            rep = REP_PL_CDR_LE                   # accepted, little-endian
        pad = (-len(body)) % 4
        pl = rep + bytes([0, pad]) + body + bytes(pad)
        dg = data_datagram(pl, sn=i + 1, le=bool(rng.integers(0, 2)), prefix=prefix, flags_extra=flags)
        if mode == 11:                            # a HEARTBEAT after the DATA: NOT_DATA record
            dg = dg + HB
        out.append(dg)
    return out


# A type exercising every op kind, alignment step and slot tail
MIXED = cdr.CdrType([("id", "u8"), ("temp", "f64"), ("flag", "bool"), ("name", cdr.String(24)),
                     ("hist", cdr.Seq("u16", 6)), ("big", cdr.Seq("i64", 3)), ("pos", cdr.Array("f32", 3)),
                     ("c", "i8"), ("t", "i16"), ("ok", "bool"), ("inner", cdr.ShapeType),
                     ("tail", cdr.Array("u64", 2))])


# Leading run of 4/8-byte fields contiguous on the wire and in the row: decoded
# little-endian chunks copy it as one block (a "segment"), others field by field
SEGS = cdr.CdrType([("a", "u64"), ("b", "f64"), ("c", cdr.Array("i32", 5)), ("d", "u32"), ("s", cdr.String(8)),
                    ("e", "u64"), ("f", cdr.Array("u16", 3))])


# Composite elements: a polygon (sequence of structs, sequence of strings) and
# deeper nesting (sequences of sequences, an array of structs holding a
# sequence, strings three levels down)
POLYGON = cdr.CdrType([("name", cdr.String(16)), ("pts", cdr.Seq(cdr.CdrType([("x", "f32"), ("y", "f32")]), 8)),
                       ("tags", cdr.Seq(cdr.String(12), 4)), ("k", "u8")])
NESTED = cdr.CdrType([("a", "u8"), ("m", cdr.Seq(cdr.Seq("u16", 3), 4)),
                      ("grid", cdr.Array(cdr.CdrType([("id", "u8"), ("v", cdr.Seq("f64", 2)), ("ok", "bool")]), 3)),
                      ("deep", cdr.Seq(cdr.Seq(cdr.Array(cdr.String(5), 2), 2), 2)), ("z", "i64")])


def random_type(rng, depth=0, budget=None):
    """A random sample type of primitives, bools, strings, sequences, arrays and nested
    structs, with composite sequences / arrays up to 4 levels deep (at most MAX_OPS ops)."""
    budget = budget if budget is not None else [cdr.MAX_OPS - 4]
    prims = list(cdr.PRIMS)
    fields = []
    for k in range(int(rng.integers(2, 6))):
        if budget[0] <= 2:
            break
        r = rng.random()
        if r < 0.25:
            spec = prims[int(rng.integers(0, len(prims)))]
        elif r < 0.30:
            spec = "bool"
        elif r < 0.40:
            spec = cdr.String(int(rng.integers(0, 13)))
        elif r < 0.48:
            spec = cdr.Seq(prims[int(rng.integers(0, len(prims)))], int(rng.integers(0, 5)))
        elif r < 0.53:
            spec = cdr.Array(prims[int(rng.integers(0, len(prims)))], int(rng.integers(0, 4)))
        elif depth < cdr.MAX_DEPTH and budget[0] > 6:
            budget[0] -= 2  # BEGIN + END
            elem = random_type(rng, depth + 1, budget) if rng.random() < 0.6 else cdr.String(int(rng.integers(0, 9)))
            spec = (cdr.Seq(elem, int(rng.integers(0, 4))) if rng.random() < 0.6
                    else cdr.Array(elem, int(rng.integers(1, 3))))
        else:
            spec = prims[int(rng.integers(0, len(prims)))]
        budget[0] -= 1
        fields.append((f"f{depth}_{k}", spec))
    return cdr.CdrType(fields)


# A crafted type for the walk's bounds: elements of 64,004 row bytes holding an array of
# 16,000 zero-width structs, one byte on the wire each.  A 40,000-element sequence of them
# (slot: one element) walks 39,999 elements past its slot; the zero-width arrays read and
# store nothing and are skipped, so the walk stays O(bytes).
WIDE_EL = cdr.CdrType([("b", "bool"), ("z", cdr.Array(cdr.CdrType([("q", cdr.Array("u32", 0))]), 16000))])
WIDE = cdr.CdrType([("s", cdr.Seq(WIDE_EL, 1)), ("t", "u8")])


def wide_payloads():
    """(label, value bytes, expected status) for WIDE."""
    import struct as st
    return [("ok", st.pack("<I", 1) + b"\x01" + b"\x07", cdr.CDR_OK),
            ("too_long", st.pack("<I", 40000) + b"\x01" * 40000 + b"\x07", cdr.CDR_TOO_LONG),
            ("bad_bool", st.pack("<I", 40000) + b"\x01" * 39000 + b"\x02" + b"\x00" * 999 + b"\x07",
             cdr.CDR_BAD_BOOL),
            ("eof", st.pack("<I", 40000) + b"\x01" * 30000, cdr.CDR_EOF)]
