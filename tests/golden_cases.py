"""Golden parse cases built from the reference's own wire vectors.

Inputs: tests/golden/vectors.json (bytes copied out of the reference's tests
by tests/golden/make_golden.py, each with its file:line).  Expected results:
transcribed below from the reference's assertions and struct literals
(SURVEY.md appendix B), so that the oracle is checked against the
reference, not against itself.
"""
import json
import os
import struct

from rtps_rx.records import (DGRAM_OK, DGRAM_SUBMSG_ERR, DATA, HEARTBEAT, ACKNACK, GAP, INFO_TS, INFO_DST,
                             INFO_SRC, NACK_FRAG, HEARTBEAT_FRAG, ROUTE_PASS, ROUTE_BUILTIN, ROUTE_HAS_QOS,
                             ROUTE_HAS_PAYLOAD, ROUTE_TS_VALID, PK_DATA)

HERE = os.path.dirname(os.path.abspath(__file__))
OWN = bytes.fromhex("0103000c292d31a228200208")  # rtps/message_receiver.rs:1138-1140
ZERO12 = bytes(12)                               # GUID::default().prefix (message_receiver.rs:1280)
SHAPES_PREFIX = "010f99067834000001000000"
# RTPS header used to wrap submessage-level vectors (the shapes-demo header, rtps/message.rs:591)
WRAP_HEADER = bytes.fromhex("52545053" "0203" "010f" + SHAPES_PREFIX)


def vectors():
    with open(os.path.join(HERE, "golden", "vectors.json")) as f:
        return json.load(f)


def _hb(first, last, count, rid="000003c7", wid="000003c2"):
    return {"reader_id": rid, "writer_id": wid, "sn": first, "last_sn": last, "count": count}


# message-level expectations: status, [(sub_off, kind)], {sub_off: {field: value}}
MESSAGES = {
    "msg_shapes_dst_ts_data_hb": (DGRAM_OK, [(20, INFO_DST), (36, INFO_TS), (48, DATA), (96, HEARTBEAT)], {
        20: {"prefix": "0103000c292d31a228200208"},
        36: {"ts_sec": 1592988954, "ts_frac": 335268864},
        48: {"prefix": SHAPES_PREFIX, "writer_id": "00000102", "reader_id": "00000007", "sn": 91,
             "pl_off": 72, "pl_len": 24, "payload_kind": PK_DATA, "ts_sec": 1592988954,
             "route_set": ROUTE_PASS | ROUTE_HAS_PAYLOAD | ROUTE_TS_VALID},
        96: dict(_hb(91, 91, 31, "00000007", "00000102"), prefix=SHAPES_PREFIX)}),
    "msg_shapes_datap_len0": (DGRAM_OK, [(20, DATA)], {
        20: {"prefix": "0103000c292d31a228200208", "writer_id": "000100c2", "reader_id": "00000000", "sn": 35,
             "pl_off": 44, "pl_len": 272, "route_set": ROUTE_PASS | ROUTE_BUILTIN}}),
    "msg_shapes_infots_datap": (DGRAM_OK, [(20, INFO_TS), (32, DATA)], {
        32: {"prefix": SHAPES_PREFIX, "writer_id": "000100c2", "reader_id": "000100c7", "sn": 1,
             "pl_off": 56, "pl_len": 148}}),
    "msg_shapes_dst_3acknack": (DGRAM_OK, [(20, INFO_DST), (36, ACKNACK), (64, ACKNACK), (92, ACKNACK)], {
        20: {"prefix": SHAPES_PREFIX},
        36: {"prefix": "0103000c292d31a228200208", "reader_id": "000003c7", "writer_id": "000003c2", "sn": 1,
             "num_bits": 0, "count": 1, "route_set": ROUTE_PASS | ROUTE_BUILTIN},
        64: {"reader_id": "000004c7", "writer_id": "000004c2", "sn": 1, "count": 1},
        92: {"reader_id": "000200c7", "writer_id": "000200c2", "sn": 1, "count": 1}}),
    "msg_infots_datap": (DGRAM_OK, [(20, INFO_TS), (32, DATA)], {
        32: {"writer_id": "000100c2", "reader_id": "000100c7", "sn": 1, "pl_off": 56, "pl_len": 148}}),
    "msg_dst_ts_dataw_hb": (DGRAM_OK, [(20, INFO_DST), (36, INFO_TS), (48, DATA), (320, HEARTBEAT)], {
        48: {"prefix": SHAPES_PREFIX, "writer_id": "000003c2", "reader_id": "000003c7", "sn": 1,
             "pl_off": 72, "pl_len": 248, "route_set": ROUTE_PASS | ROUTE_BUILTIN},
        320: _hb(1, 1, 2)}),
    "msg_fuzz_rtps": (DGRAM_SUBMSG_ERR, [], {}),
    "mr_shapes_red": (DGRAM_OK, [(20, INFO_DST), (36, INFO_TS), (48, DATA), (96, HEARTBEAT)], {
        48: {"sn": 91, "pl_off": 72, "pl_len": 24}}),
    "mr_submsg_count_1": (DGRAM_OK, [(20, INFO_DST), (36, INFO_TS), (48, DATA), (96, HEARTBEAT)], {
        48: {"sn": 67}, 96: _hb(67, 67, 7, "00000007", "00000102")}),
    "mr_submsg_count_2": (DGRAM_OK, [(20, INFO_DST), (36, ACKNACK)], {
        36: {"reader_id": "000004c7", "writer_id": "000004c2", "sn": 2, "num_bits": 0, "count": 3,
             "prefix": SHAPES_PREFIX, "route_set": ROUTE_PASS}}),
    "td_spdp_participant": (DGRAM_OK, [(20, INFO_TS), (32, DATA)], {
        32: {"writer_id": "000100c2", "reader_id": "000100c7", "sn": 1, "pl_off": 56, "pl_len": 148}}),
    "td_spdp_subscription": (DGRAM_OK, [(20, INFO_TS), (32, DATA)], {
        32: {"prefix": "0103000c292d31a228200208", "writer_id": "000004c2", "reader_id": "00000000", "sn": 1,
             "pl_off": 56, "pl_len": 192}}),
    "td_spdp_publication": (DGRAM_OK, [(20, INFO_DST), (36, INFO_TS), (48, DATA), (320, HEARTBEAT)], {
        48: {"writer_id": "000003c2", "reader_id": "000003c7", "sn": 1, "pl_off": 72, "pl_len": 248},
        320: _hb(1, 1, 2)}),
    "sedp_reader_raw": (DGRAM_OK, [(20, INFO_TS), (32, DATA)], {
        32: {"prefix": "39bcd6b14fa24972817dd454", "writer_id": "000004c2", "reader_id": "000004c7", "sn": 1,
             "pl_off": 56, "pl_len": 200}}),
    "spdp_evil_1": (DGRAM_OK, [(20, DATA)], {
        20: {"flags": 0x07, "prefix": "010f45d2b3f558b901000000", "writer_id": "000100c2", "sn": 0, "aux16": 4,
             "pl_off": 48, "pl_len": 6, "route_set": ROUTE_HAS_QOS | ROUTE_HAS_PAYLOAD}}),
    "spdp_evil_2": (DGRAM_OK, [(20, DATA)], {20: {"sn": 2, "pl_off": 44, "pl_len": 5}}),
    "spdp_evil_3": (DGRAM_SUBMSG_ERR, [], {}),
}
# mr_test_submsg_count runs its receiver with GUID::default() (all-zero prefix)
OWN_OVERRIDE = {"mr_submsg_count_1": ZERO12, "mr_submsg_count_2": ZERO12}

SUBMESSAGES = {
    "sub_data_red": (DGRAM_OK, [(20, DATA)], {20: {"sn": 91, "writer_id": "00000102", "reader_id": "00000007",
                                                   "pl_off": 44, "pl_len": 24}}),
    "sub_heartbeat": (DGRAM_OK, [(20, HEARTBEAT)], {20: _hb(91, 91, 31, "00000007", "00000102")}),
    "sub_info_dst": (DGRAM_OK, [(20, INFO_DST)], {20: {"prefix": "0103000c292d31a228200208"}}),
    "sub_acknack_fuzz": (DGRAM_SUBMSG_ERR, [], {}),  # submessage.rs:450: is_err()
}

RID, WID = "000003c7", "000003c2"
# serialization_test! bodies: kind, expected fields (from the struct literals)
BODIES = {
    "body_heartbeat": (HEARTBEAT, _hb(42, 7, 9)),
    "body_acknack": (ACKNACK, {"reader_id": RID, "writer_id": WID, "sn": 0, "num_bits": 0, "count": 1}),
    "body_gap": (GAP, {"reader_id": RID, "writer_id": WID, "sn": 42, "list_base": 7, "num_bits": 0}),
    "body_nack_frag": (NACK_FRAG, {"reader_id": RID, "writer_id": WID, "sn": 42, "fns_base": 1000,
                                   "num_bits": 0, "count": 6}),
    "body_heartbeat_frag": (HEARTBEAT_FRAG, {"reader_id": RID, "writer_id": WID, "sn": 42,
                                             "last_frag_num": 99, "count": 6}),
    "body_info_source": (INFO_SRC, {"version": [2, 2], "vendor": [0xFF, 0xAA],
                                    "prefix": "01026d3f7e07000001000000"}),
    "body_info_destination": (INFO_DST, {"prefix": "01026d3f7e07000001000000"}),
    "body_ts_zero": (INFO_TS, {"ts_sec": 0, "ts_frac": 0}),
    "body_ts_invalid": (INFO_TS, {"ts_sec": 0xFFFFFFFF, "ts_frac": 0xFFFFFFFF}),
    "body_ts_infinite": (INFO_TS, {"ts_sec": 0x7FFFFFFF, "ts_frac": 0xFFFFFFFF}),
    "body_ts_current": (INFO_TS, {"ts_sec": 1537045491, "ts_frac": 0}),
    "body_ts_wireshark": (INFO_TS, {"ts_sec": 1519152760, "ts_frac": 1328210046}),
}
# element vectors placed into a submessage body: (kind, wrapper, expected)
SNSETS = {"snset_empty": (42, 0), "snset_one": (1, 1), "snset_manual": (1, 25), "snset_multiword": (10, 64)}
FNSETS = {"fnset_empty": (42, 0), "fnset_manual": (1000, 14)}
SNS = {"sn_default": 1, "sn_unknown": -(1 << 32), "sn_non_zero": 0x0011223344556677}


def _sub(kind, le, body, extra_flags=0):
    flags = (1 if le else 0) | extra_flags
    ln = struct.pack("<H" if le else ">H", len(body))
    return WRAP_HEADER + bytes([kind, flags]) + ln + body


# S1 (speedy read_from_buffer accepts trailing bytes): Message::read_from_buffer reads the
# 20-B Header with speedy's Header::read_from_buffer over the WHOLE datagram
# (rtps/message.rs:66-67), and the reference's own capture tests unwrap() that
# (message.rs:584-794): the speedy readers ignore bytes past the value.  The
# fixed-size bodies use the same reader on the submessage's content
# (Heartbeat::read_from_buffer_with_ctx, rtps/submessage.rs:183; AckNack :167;
# Gap :159; InfoDestination :200; InfoSource :207), so a body longer than its
# fields parses, with the same field values.  Derived from the reference's vectors:
TRAILING = {  # name: (source body vector, kind, extra bytes)
    "s1_heartbeat_trailing": ("body_heartbeat", HEARTBEAT, 4),
    "s1_heartbeat_trailing_odd": ("body_heartbeat", HEARTBEAT, 3),
    "s1_info_destination_trailing": ("body_info_destination", INFO_DST, 8),
    "s1_info_source_trailing": ("body_info_source", INFO_SRC, 1),
}


def cases():
    """[(name, datagram, own_prefix, status, [(off, kind)], {off: fields})]"""
    v = vectors()
    out = []
    for m in v["messages"]:
        st, kinds, fields = MESSAGES[m["name"]]
        out.append((m["name"], bytes.fromhex(m["hex"]), OWN_OVERRIDE.get(m["name"], OWN), st, kinds, fields))
    for m in v["submessages"]:
        st, kinds, fields = SUBMESSAGES[m["name"]]
        out.append((m["name"], WRAP_HEADER + bytes.fromhex(m["hex"]), OWN, st, kinds, fields))
    bodies = {b["name"]: b for b in v["bodies"]}
    for name, (kind, exp) in BODIES.items():
        for le in (True, False):
            body = bytes.fromhex(bodies[name]["le" if le else "be"])
            out.append((f"{name}_{'le' if le else 'be'}", _sub(kind, le, body), OWN, DGRAM_OK, [(20, kind)],
                        {20: exp}))
    for name, (src, kind, extra) in TRAILING.items():
        for le in (True, False):
            body = bytes.fromhex(bodies[src]["le" if le else "be"]) + bytes(range(0xA0, 0xA0 + extra))
            out.append((f"{name}_{'le' if le else 'be'}", _sub(kind, le, body), OWN, DGRAM_OK, [(20, kind)],
                        {20: BODIES[src][1]}))
    rid, wid = bytes.fromhex(RID), bytes.fromhex(WID)
    for name, (base, nb) in SNSETS.items():
        for le in (True, False):
            e = "<" if le else ">"
            body = rid + wid + bytes.fromhex(bodies[name]["le" if le else "be"]) + struct.pack(e + "i", 5)
            out.append((f"{name}_{'le' if le else 'be'}", _sub(ACKNACK, le, body), OWN, DGRAM_OK, [(20, ACKNACK)],
                        {20: {"sn": base, "num_bits": nb, "count": 5, "bitmap_off": 44}}))
    for name, (base, nb) in FNSETS.items():
        for le in (True, False):
            e = "<" if le else ">"
            body = rid + wid + struct.pack(e + "iI", 0, 42) + bytes.fromhex(bodies[name]["le" if le else "be"]) \
                + struct.pack(e + "i", 6)
            out.append((f"{name}_{'le' if le else 'be'}", _sub(NACK_FRAG, le, body), OWN, DGRAM_OK,
                        [(20, NACK_FRAG)], {20: {"sn": 42, "fns_base": base, "num_bits": nb, "count": 6}}))
    for name, value in SNS.items():
        for le in (True, False):
            e = "<" if le else ">"
            sn = bytes.fromhex(bodies[name]["le" if le else "be"])
            body = rid + wid + sn + sn + struct.pack(e + "i", 3)
            out.append((f"{name}_{'le' if le else 'be'}", _sub(HEARTBEAT, le, body), OWN, DGRAM_OK,
                        [(20, HEARTBEAT)], {20: {"sn": value, "last_sn": value, "count": 3}}))
    return out


def check_case(case, status, recs, to_dict):
    """Assert one case against a parser's status and its records (for that datagram)."""
    name, dgram, own, exp_status, kinds, fields = case
    assert status == exp_status, f"{name}: status {status} != {exp_status}"
    got = [(int(r["sub_off"]), int(r["kind"])) for r in recs]
    assert got == kinds, f"{name}: submessages {got} != {kinds}"
    by_off = {int(r["sub_off"]): to_dict(r) for r in recs}
    for off, exp in fields.items():
        d = by_off[off]
        for k, val in exp.items():
            if k == "route_set":
                assert d["route"] & val == val, f"{name}@{off}: route {d['route']:#x} lacks {val:#x}"
            else:
                assert d[k] == val, f"{name}@{off}: {k} = {d[k]!r}, expected {val!r}"


def shape_type_from_payload(payload):
    """CDR_LE ShapeType {color: string, x, y, size: i32} (rtps/message_receiver.rs:1240-1254)."""
    assert payload[:4] == b"\x00\x01\x00\x00"  # CDR_LE encapsulation
    v = payload[4:]
    n = struct.unpack_from("<I", v, 0)[0]
    color = v[4:4 + n - 1].decode()
    off = 4 + n
    off = (off + 3) // 4 * 4
    x, y, size = struct.unpack_from("<iii", v, off)
    return color, x, y, size
