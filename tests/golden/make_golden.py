#!/usr/bin/env python3
"""Extract the reference's own RTPS wire vectors into tests/golden/vectors.json.

Runs only where /root/reference exists (this build container).  It reads
the reference's Rust test sources AS TEXT and copies out the byte arrays
that the reference's tests feed to its parser (DATA: inputs), together with
the file:line they come from.  No reference source text is stored: only
the bytes and their citation.  The expected parse results live in
tests/test_oracle_golden.py (transcribed from the reference's assertions and
struct literals).

Usage:  python3 tests/golden/make_golden.py [/root/reference]
"""
import json
import os
import re
import sys

REF = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "vectors.json")

# whole datagrams the reference's tests parse with Message::read_from_buffer /
# handle_received_packet: (name, file, first line of the literal)
MESSAGES = [
    ("msg_shapes_dst_ts_data_hb", "src/rtps/message.rs", 590),
    ("msg_shapes_datap_len0", "src/rtps/message.rs", 615),
    ("msg_shapes_infots_datap", "src/rtps/message.rs", 654),
    ("msg_shapes_dst_3acknack", "src/rtps/message.rs", 686),
    ("msg_infots_datap", "src/rtps/message.rs", 712),
    ("msg_dst_ts_dataw_hb", "src/rtps/message.rs", 746),
    ("msg_fuzz_rtps", "src/rtps/message.rs", 801),
    ("mr_shapes_red", "src/rtps/message_receiver.rs", 1125),
    ("mr_submsg_count_1", "src/rtps/message_receiver.rs", 1260),
    ("mr_submsg_count_2", "src/rtps/message_receiver.rs", 1272),
    ("td_spdp_participant", "src/test/test_data.rs", 2),
    ("td_spdp_subscription", "src/test/test_data.rs", 23),
    ("td_spdp_publication", "src/test/test_data.rs", 46),
    ("sedp_reader_raw", "src/discovery/sedp_messages.rs", 1403),
    ("spdp_evil_1", "src/discovery/spdp_participant_data.rs", 745),
    ("spdp_evil_2", "src/discovery/spdp_participant_data.rs", 782),
    ("spdp_evil_3", "src/discovery/spdp_participant_data.rs", 820),
]

# single submessages (header + body) the reference's tests parse
SUBMESSAGES = [
    ("sub_data_red", "src/rtps/submessage.rs", 342),
    ("sub_heartbeat", "src/rtps/submessage.rs", 368),
    ("sub_info_dst", "src/rtps/submessage.rs", 394),
    ("sub_acknack_fuzz", "src/rtps/submessage.rs", 424),
]

# serialization_test! bodies: (name, kind, file, anchor) -> first le=[..], be=[..] after anchor
BODIES = [
    ("body_heartbeat", 0x07, "src/messages/submessages/heartbeat.rs", "heartbeat,"),
    ("body_acknack", 0x06, "src/messages/submessages/ack_nack.rs", "acknack,"),
    ("body_gap", 0x08, "src/messages/submessages/gap.rs", "gap,"),
    ("body_nack_frag", 0x12, "src/messages/submessages/nack_frag.rs", "nack_frag,"),
    ("body_heartbeat_frag", 0x13, "src/messages/submessages/heartbeat_frag.rs", "heartbeat_frag,"),
    ("body_info_source", 0x0C, "src/messages/submessages/info_source.rs", "info_source,"),
    ("body_info_destination", 0x0E, "src/messages/submessages/info_destination.rs", "info_destination,"),
    ("body_ts_zero", 0x09, "src/structure/time.rs", "time_zero,"),
    ("body_ts_invalid", 0x09, "src/structure/time.rs", "time_invalid,"),
    ("body_ts_infinite", 0x09, "src/structure/time.rs", "time_infinite,"),
    ("body_ts_current", 0x09, "src/structure/time.rs", "time_current_empty_fraction,"),
    ("body_ts_wireshark", 0x09, "src/structure/time.rs", "time_from_wireshark,"),
    ("snset_empty", None, "src/structure/sequence_number.rs", "sequence_number_set_empty,"),
    ("snset_one", None, "src/structure/sequence_number.rs", "sequence_number_set_one,"),
    ("snset_manual", None, "src/structure/sequence_number.rs", "sequence_number_set_manual,"),
    ("snset_multiword", None, "src/structure/sequence_number.rs", "sequence_number_set_multiword,"),
    ("fnset_empty", None, "src/structure/sequence_number.rs", "fragment_number_set_empty,"),
    ("fnset_manual", None, "src/structure/sequence_number.rs", "fragment_number_set_manual,"),
    ("sn_default", None, "src/structure/sequence_number.rs", "sequence_number_default,"),
    ("sn_unknown", None, "src/structure/sequence_number.rs", "sequence_number_unknown,"),
    ("sn_non_zero", None, "src/structure/sequence_number.rs", "sequence_number_non_zero,"),
]

HEX0X = re.compile(r"0x([0-9A-Fa-f]{2})")


def _lines(rel):
    with open(os.path.join(REF, rel), encoding="utf-8") as f:
        return f.read().split("\n")


def _strip_comment(line):
    i = line.find("//")
    return line if i < 0 else line[:i]


def literal_at(rel, first_line):
    """Bytes of the array / hex! literal that starts on first_line (1-based)."""
    lines = _lines(rel)
    i = first_line - 1
    if "hex!(" in lines[i]:
        j = i
        while '"' not in lines[j]:
            j += 1
        text = lines[j][lines[j].index('"') + 1:]
        if '"' in text:
            text = text[: text.index('"')]
        else:
            while True:
                j += 1
                if '"' in lines[j]:
                    text += " " + lines[j][: lines[j].index('"')]
                    break
                text += " " + lines[j]
        toks = [t for t in text.split() if re.fullmatch(r"[0-9A-Fa-f]{2}", t)]
        return bytes(int(t, 16) for t in toks), j + 1
    out, j = [], i
    while True:
        seg = _strip_comment(lines[j])
        if j == i:
            k = seg.index("= [") + 2 if "= [" in seg else seg.index("[")
            seg = seg[k + 1:]
        end = "]" in seg
        if end:
            seg = seg[: seg.index("]")]
        out += [int(h, 16) for h in HEX0X.findall(seg)]
        if end:
            return bytes(out), j + 1
        j += 1


def le_be_after(rel, anchor):
    lines = _lines(rel)
    start = next(k for k, l in enumerate(lines) if anchor in l)
    found = {}
    for k in range(start, len(lines)):
        for tag in ("le", "be"):
            if tag not in found and re.search(r"\b%s = \[" % tag, lines[k]):
                found[tag] = (k + 1,) + literal_at(rel, k + 1)
        if len(found) == 2:
            break
    return found


def main():
    doc = {"reference": "w-utter/rustdds-io_uring (read as text only)",
           "messages": [], "submessages": [], "bodies": []}
    for name, rel, line in MESSAGES:
        b, end = literal_at(rel, line)
        doc["messages"].append({"name": name, "source": f"{rel}:{line}-{end}", "hex": b.hex()})
    for name, rel, line in SUBMESSAGES:
        b, end = literal_at(rel, line)
        doc["submessages"].append({"name": name, "source": f"{rel}:{line}-{end}", "hex": b.hex()})
    for name, kind, rel, anchor in BODIES:
        f = le_be_after(rel, anchor)
        doc["bodies"].append({"name": name, "kind": kind,
                              "source": f"{rel}:{f['le'][0]} (le), :{f['be'][0]} (be)",
                              "le": f["le"][1].hex(), "be": f["be"][1].hex()})
    with open(OUT, "w") as fh:
        json.dump(doc, fh, indent=1)
        fh.write("\n")
    print("wrote", OUT, {k: len(v) for k, v in doc.items() if isinstance(v, list)})


if __name__ == "__main__":
    main()
