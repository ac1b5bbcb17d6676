"""The sample's ChangeKind in the DATA record (rtps_record.u.data.change_kind):
Reader::deduce_change_kind (reference src/io_uring/rtps/reader.rs:1158-1182),
called for key payloads (:779-785) and key-hash-only DATA (:787-813); Data is
Alive (dds/ddsdata.rs:45-50).  InlineQos::status_info (elements/inline_qos.rs:27-42)
takes the first PID_STATUS_INFO or StatusInfo::empty(); StatusInfo::read_from reads
four u8 (:139-147); StatusInfo::change_kind (:164-175).

Known answers below are derived by hand from those lines; the StatusInfo bytes the
reference's own test uses (inline_qos.rs:198-238, `inline_qos_status_info`: the four
octets 00 00 00 03 read as Disposed | Unregistered under both CDR_LE and CDR_BE) are
the "si both" case, in both byte orders of the submessage, whose change kind follows
from StatusInfo::change_kind (:164-175: Disposed first).  The CPU test checks the
oracle against them, the GPU test the device against the oracle on the same
datagrams, both byte orders."""
import struct

import numpy as np
import pytest

import oracle
from ingest_ref import RTPS_HDR, ZERO_EID, _sn
from rtps_rx.records import (CK_ALIVE, CK_NONE, CK_NOT_ALIVE_DISPOSED, CK_NOT_ALIVE_UNREGISTERED, DATA,
                             PK_DATA, PK_ERR_AMBIGUOUS, PK_ERR_NO_CONTENT, PK_KEY, PK_KEY_HASH, U_DATA)

PREFIX = bytes(range(40, 52))
WKEY = b"\x00\x00\x07\x02"
KH = bytes(range(100, 116))


def _param(e, pid, value):
    return struct.pack(e + "HH", pid, len(value)) + value


def _data(le, dflag, kflag, params=None, payload=b"\x00\x01\x00\x00abcd"):
    """DATA with the given D / K flags, optional inline QoS parameters (list of (pid, value))."""
    e = "<" if le else ">"
    flags = (1 if le else 0) | (0x04 if dflag else 0) | (0x08 if kflag else 0)
    qos = b""
    if params is not None:
        flags |= 0x02
        qos = b"".join(_param(e, p, v) for p, v in params) + struct.pack(e + "HH", 1, 0)
    body = struct.pack(e + "HH", 0, 16) + ZERO_EID + WKEY + _sn(e, 5) + qos + (payload if (dflag or kflag) else b"")
    return bytes([0x15, flags]) + struct.pack(e + "H", len(body)) + body


REF_SI_BYTES = bytes([0x00, 0x00, 0x00, 0x03])  # inline_qos.rs:207, 227 (LE and BE alike: four octets)


def _si(flags, n=4):
    return (b"\x00\x00\x00" + bytes([flags]))[:n] if n <= 4 else b"\x00\x00\x00" + bytes([flags]) + bytes(n - 4)


# (name, D, K, inline-QoS parameters or None, payload kind, change kind)
CASES = [
    ("data", 1, 0, None, PK_DATA, CK_ALIVE),
    ("data with disposed si", 1, 0, [(0x71, _si(1))], PK_DATA, CK_ALIVE),              # Data is always Alive
    ("key, no qos", 0, 1, None, PK_KEY, CK_NOT_ALIVE_DISPOSED),                        # inline_qos None
    ("key, qos without si", 0, 1, [(0x0F, b"\x01\x02\x03\x04")], PK_KEY, CK_ALIVE),    # StatusInfo::empty()
    ("key, si disposed", 0, 1, [(0x71, _si(1))], PK_KEY, CK_NOT_ALIVE_DISPOSED),
    ("key, si unregistered", 0, 1, [(0x71, _si(2))], PK_KEY, CK_NOT_ALIVE_UNREGISTERED),
    # the reference's vector (inline_qos.rs:198-238): 00 00 00 03 = Disposed | Unregistered; Disposed first
    ("key, si both", 0, 1, [(0x71, REF_SI_BYTES)], PK_KEY, CK_NOT_ALIVE_DISPOSED),
    ("key, si filtered", 0, 1, [(0x71, _si(4))], PK_KEY, CK_ALIVE),
    ("key, si unknown bits", 0, 1, [(0x71, _si(0xF8 | 2))], PK_KEY, CK_NOT_ALIVE_UNREGISTERED),  # truncated bits
    ("key, si short", 0, 1, [(0x71, _si(2, 3))], PK_KEY, CK_NOT_ALIVE_DISPOSED),       # read error -> None
    ("key, si empty", 0, 1, [(0x71, b"")], PK_KEY, CK_NOT_ALIVE_DISPOSED),
    ("key, si long", 0, 1, [(0x71, _si(2, 8))], PK_KEY, CK_NOT_ALIVE_UNREGISTERED),     # four u8 read, rest ignored
    ("key, first si wins", 0, 1, [(0x71, _si(2)), (0x71, _si(1))], PK_KEY, CK_NOT_ALIVE_UNREGISTERED),
    ("key hash, si unregistered", 0, 0, [(0x70, KH), (0x71, _si(2))], PK_KEY_HASH, CK_NOT_ALIVE_UNREGISTERED),
    ("key hash, no si", 0, 0, [(0x70, KH)], PK_KEY_HASH, CK_ALIVE),
    ("key hash after si", 0, 0, [(0x71, _si(1)), (0x70, KH)], PK_KEY_HASH, CK_NOT_ALIVE_DISPOSED),
    ("no content", 0, 0, [(0x71, _si(2))], PK_ERR_NO_CONTENT, CK_NONE),
    ("ambiguous", 1, 1, [(0x71, _si(2))], PK_ERR_AMBIGUOUS, CK_NONE),
]


def _datagrams():
    out = []
    for le in (True, False):
        for name, d, k, params, pk, ck in CASES:
            out.append(RTPS_HDR + PREFIX + _data(le, d, k, params))
    return out


def _expected():
    return [(pk, ck) for _ in (0, 1) for _, _, _, _, pk, ck in CASES]


def _kinds(recs):
    assert (recs["kind"] == DATA).all()
    u = recs["u"].copy().view(U_DATA).reshape(-1)
    return list(zip(recs["payload_kind"].tolist(), u["change_kind"].tolist()))


def test_oracle_change_kind_known_answers():
    a, o, l = oracle.pack(_datagrams())
    st, recs, _, _ = oracle.parse(a, o, l)
    assert (st == 0).all() and len(recs) == len(l)
    got = _kinds(recs)
    names = [n for _ in (0, 1) for n, *_ in CASES]
    for name, g, e in zip(names, got, _expected()):
        assert g == e, f"{name}: (payload kind, change kind) {g} != {e}"


@pytest.mark.gpu
def test_device_change_kind_matches_oracle():
    import rtps_rx
    rx = rtps_rx.MessageReceiver(oracle.OWN_PREFIX, max_datagrams=1024)
    try:
        dg = _datagrams() * 8
        for align in (16, 1):
            a, o, l = oracle.pack(dg, align=align)
            res = rx.handle_received_batch(a, o, l)
            st, recs, _, _ = oracle.parse(a, o, l)
            assert np.array_equal(res.status, st)
            assert res.records.tobytes() == recs.tobytes(), f"align {align}: records differ"
            assert _kinds(res.records) == _expected() * 8
    finally:
        rx.close()
