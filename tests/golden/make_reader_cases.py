#!/usr/bin/env python3
"""Known answers of the reference's own Reader unit tests, as wire event streams.

The reference's reader tests (io_uring/rtps/reader.rs:1537-1988, the same tests
in rtps/reader.rs:1464-1974) drive a Reader with submessage structs built from
literals and assert what its writer proxy and topic cache hold afterwards.
This script re-encodes every one of those literal submessages as an RTPS
datagram (the wire form the receive path parses: header with the test's
source GuidPrefix, then the submessage with the flags the test passes) and
writes, per case, the readers / proxies the test sets up and the values the
test asserts after each step.  Only the literal field values and the
assertions are transcribed (no reference source text is stored); each case
carries the file:line of the test it comes from.

Literals the tests use (cited):
  GUID::dummy_test_guid(kind)   prefix b"FakeTestGUID", entity key [1,2,3]   structure/guid.rs:587-595
  EntityKind READER_NO_KEY_USER_DEFINED 0x04, WRITER_NO_KEY_USER_DEFINED 0x03 structure/guid.rs:115-116
  Data::default()               reader_id UNKNOWN, writer_sn 1, no inline QoS,
                                payload = SerializedPayload::default()       test/test_properties.rs:28-37
  SerializedPayload::default()  CDR_LE, value b"fake data"                    test/test_properties.rs:22-26
  SequenceNumber::default()     1                                             structure/sequence_number.rs:193-197
  Timestamp::INVALID            (0xFFFFFFFF, 0xFFFFFFFF)                      structure/time.rs:49-52
  BitFlags::from_flag(DATA_Flags::Data): flags = D only (0x04), big-endian    submessage_flag.rs:64-70
  QosPolicies::qos_none() -> reliability None -> BestEffort reader            io_uring/rtps/reader.rs:173-176

Output: tests/golden/reader_known_answers.json.  Usage: python3 make_reader_cases.py
"""
import json
import os
import struct

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "reader_known_answers.json")

PREFIX = b"FakeTestGUID"
READER_EID = bytes([1, 2, 3, 0x04])
WRITER_EID = bytes([1, 2, 3, 0x03])
WRITER_GUID = PREFIX + WRITER_EID
UNKNOWN = bytes(4)
PAYLOAD_DEFAULT = bytes([0x00, 0x01, 0x00, 0x00]) + b"fake data"
RTPS_HDR = b"RTPS\x02\x04\x01\x0f"  # protocol 2.4, vendor 0x010f (any vendor is accepted)

READER_BEST_EFFORT, READER_STATELESS = 0x2, 0x1


def _sn(e, sn):
    return struct.pack(e + "iI", sn >> 32, sn & 0xFFFFFFFF)


def sub(kind, flags, body):
    e = "<" if flags & 1 else ">"
    return bytes([kind, flags]) + struct.pack(e + "H", len(body)) + body


def data(reader_id, sn, flags=0x04, payload=PAYLOAD_DEFAULT):
    e = "<" if flags & 1 else ">"
    body = struct.pack(e + "HH", 0, 16) + reader_id + WRITER_EID + _sn(e, sn) + payload
    return sub(0x15, flags, body)


def heartbeat(first, last, count, final):
    flags = 0x01 | (0x02 if final else 0)
    return sub(0x07, flags, READER_EID + WRITER_EID + _sn("<", first) + _sn("<", last) + struct.pack("<i", count))


def gap(start, base, num_bits, members):
    words = [0] * ((num_bits + 31) // 32)
    for s in members:  # NumberSet::insert: bit (s - base), MSB first (sequence_number.rs:377-395)
        p = s - base
        words[p // 32] |= 1 << (31 - p % 32)
    body = READER_EID + WRITER_EID + _sn("<", start) + _sn("<", base) + struct.pack("<I", num_bits)
    body += b"".join(struct.pack("<I", w) for w in words)
    return sub(0x08, 0x01, body)


def info_ts(sec, frac):
    return sub(0x09, 0x01, struct.pack("<II", sec, frac))


def dgram(*subs):
    return (RTPS_HDR + PREFIX + b"".join(subs)).hex()


def reader(flags):
    return {"entity_id": READER_EID.hex(), "reader_slot": 7, "flags": flags}


PROXY = [{"writer_guid": WRITER_GUID.hex(), "reader": 0}]

CASES = [
    {
        "name": "reader_sends_notification_when_receiving_data",
        "source": "src/io_uring/rtps/reader.rs:1537-1603 (src/rtps/reader.rs:1464-1552)",
        "asserts": "handle_data_msg returns true (the change enters the cache)",
        "readers": [reader(READER_BEST_EFFORT)], "proxies": PROXY,
        "batches": [{"datagrams": [dgram(data(READER_EID, 1))],
                     "deliveries": [[0, 7]], "ack_base": [2]}],
    },
    {
        "name": "reader_sends_data_to_topic_cache",
        "source": "src/io_uring/rtps/reader.rs:1606-1686 (src/rtps/reader.rs:1554-1653)",
        "asserts": "the cache change holds writer_guid, sequence number 1, source timestamp INVALID and "
                   "the Data's serialized payload",
        "readers": [reader(READER_BEST_EFFORT)], "proxies": PROXY,
        "batches": [{"datagrams": [dgram(info_ts(0xFFFFFFFF, 0xFFFFFFFF), data(READER_EID, 1))],
                     "deliveries": [[1, 7]], "ack_base": [2],
                     "delivered": [{"writer_guid": WRITER_GUID.hex(), "sn": 1, "ts": [0xFFFFFFFF, 0xFFFFFFFF],
                                    "payload": PAYLOAD_DEFAULT.hex()}]}],
    },
    {
        "name": "reader_handles_heartbeats",
        "source": "src/io_uring/rtps/reader.rs:1689-1821 (src/rtps/reader.rs:1656-1766)",
        "asserts": "HEARTBEATs with counts 1, 2, 2 (duplicate: ignored), 3 and first_sn 1; a reliable reader. "
                   "Observable on the ingest boundary: no sample, all_ackable_before stays 1 "
                   "(irrelevant_changes_up_to(1) removes nothing)",
        "readers": [reader(0)], "proxies": PROXY,
        "batches": [{"datagrams": [dgram(heartbeat(1, 0, 1, True))], "deliveries": [], "ack_base": [1]},
                    {"datagrams": [dgram(heartbeat(1, 1, 2, False))], "deliveries": [], "ack_base": [1]},
                    {"datagrams": [dgram(heartbeat(1, 1, 2, False))], "deliveries": [], "ack_base": [1]},
                    {"datagrams": [dgram(heartbeat(1, 3, 3, False))], "deliveries": [], "ack_base": [1]}],
    },
    {
        "name": "reader_handles_gaps",
        "source": "src/io_uring/rtps/reader.rs:1823-1937 (src/rtps/reader.rs:1769-1902)",
        "asserts": "all_ackable_before == 3 after GAP(1, {base 3, 7 bits: 4}), == 5 after DATA sn 3, "
                   "== 6 after GAP(5, {base 5, 7 bits: 5})",
        "readers": [reader(READER_BEST_EFFORT)], "proxies": PROXY,
        "batches": [{"datagrams": [dgram(gap(1, 3, 7, [4]))], "deliveries": [], "ack_base": [3]},
                    {"datagrams": [dgram(data(UNKNOWN, 3))], "deliveries": [[0, 7]], "ack_base": [5]},
                    {"datagrams": [dgram(gap(5, 5, 7, [5]))], "deliveries": [], "ack_base": [6]}],
    },
    {
        "name": "reader_handles_gaps_one_batch",
        "source": "src/io_uring/rtps/reader.rs:1823-1937 (the same three events in one batch)",
        "asserts": "the final all_ackable_before == 6 and the DATA accepted, with all three events decided in "
                   "one parallel batch",
        "readers": [reader(READER_BEST_EFFORT)], "proxies": PROXY,
        "batches": [{"datagrams": [dgram(gap(1, 3, 7, [4])), dgram(data(UNKNOWN, 3)), dgram(gap(5, 5, 7, [5]))],
                     "deliveries": [[1, 7]], "ack_base": [6]}],
    },
    {
        "name": "stateless_reader_does_not_contain_writer_proxies",
        "source": "src/io_uring/rtps/reader.rs:1940-1988 (src/rtps/reader.rs:1905-1974)",
        "asserts": "matched_writer(writer_guid).is_none() for a like_stateless (BestEffort) reader: it "
                   "contains no writer, so no target set names it and a DATA of that writer reaches no reader",
        "readers": [reader(READER_STATELESS | READER_BEST_EFFORT)], "proxies": PROXY,
        "batches": [{"datagrams": [dgram(data(READER_EID, 1))], "deliveries": [], "no_target": True}],
    },
]


def main():
    with open(OUT, "w") as f:
        json.dump({"generator": "tests/golden/make_reader_cases.py", "cases": CASES}, f, indent=1)
        f.write("\n")


if __name__ == "__main__":
    main()
