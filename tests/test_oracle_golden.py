"""Pin the CPU oracle to the reference's own wire vectors and assertions (CPU only)."""
import numpy as np
import pytest

import oracle
from golden_cases import cases, check_case, shape_type_from_payload, vectors
from rtps_rx.records import record_to_dict, DGRAM_OK, DATA

CASES = cases()


def _parse_one(dgram, own):
    arena, off, ln = oracle.pack([dgram])
    st, recs, match, rb = oracle.parse(arena, off, ln, own=own)
    return int(st[0]), recs


@pytest.mark.parametrize("case", CASES, ids=[c[0] for c in CASES])
def test_oracle_matches_reference_vector(case):
    st, recs = _parse_one(case[1], case[2])
    check_case(case, st, recs, record_to_dict)


def test_vector_inventory():
    v = vectors()
    assert len(v["messages"]) == 17 and len(v["submessages"]) == 4 and len(v["bodies"]) == 21
    for m in v["messages"]:
        assert m["source"].startswith("src/")


def test_shape_type_red():
    """rtps/message_receiver.rs:1250-1254: the DATA payload decodes to ShapeType color == "RED"."""
    name, dgram, own = next((c[0], c[1], c[2]) for c in CASES if c[0] == "mr_shapes_red")
    st, recs = _parse_one(dgram, own)
    d = [record_to_dict(r) for r in recs if r["kind"] == DATA][0]
    color, x, y, size = shape_type_from_payload(dgram[d["pl_off"]:d["pl_off"] + d["pl_len"]])
    assert (color, x, y, size) == ("RED", 105, 23, 30)


def test_submessage_counts():
    """message_receiver.rs:1223,1288,1291 — submessage_count 4 / 4 / 2."""
    by = {c[0]: c for c in CASES}
    for name, count in (("mr_shapes_red", 4), ("mr_submsg_count_1", 4), ("mr_submsg_count_2", 2)):
        st, recs = _parse_one(by[name][1], by[name][2])
        assert st == DGRAM_OK and len(recs) == count


def test_batch_equals_single():
    """Parsing all vectors as one batch gives the per-datagram results, in order."""
    dgrams = [c[1] for c in CASES if c[2] == oracle.OWN_PREFIX]
    arena, off, ln = oracle.pack(dgrams)
    st, recs, match, rb = oracle.parse(arena, off, ln)
    k = 0
    for i, d in enumerate(dgrams):
        s1, r1 = _parse_one(d, oracle.OWN_PREFIX)
        assert st[i] == s1
        r = recs[k:k + len(r1)].copy()
        r["dgram_idx"] = 0
        assert r.tobytes() == r1.tobytes()
        assert rb[i] == k
        k += len(r1)
    assert k == len(recs)


def test_threads_equal_single():
    arena, off, ln = oracle.gen(oracle.WL_C3, 3000)
    a = oracle.parse(arena, off, ln, threads=1)
    b = oracle.parse(arena, off, ln, threads=4)
    for x, y in zip(a, b):
        if isinstance(x, tuple):  # targets: (off, entries)
            assert all(np.array_equal(u, v) for u, v in zip(x, y))
        else:
            assert np.array_equal(x, y)


import reader_known  # noqa: E402

READER_CASES = reader_known.cases()


@pytest.mark.parametrize("case", READER_CASES, ids=[c["name"] for c in READER_CASES])
def test_oracle_reader_known_answers(case):
    """The reference's Reader unit tests (io_uring/rtps/reader.rs:1537-1988): all_ackable_before
    3 -> 5 -> 6 over GAP / DATA / GAP, duplicate HEARTBEAT counts ignored, no proxy in a stateless
    reader, the topic-cache change of a default DATA; through the oracle's parse + ingest."""
    reader_known.check(case, reader_known.oracle_batch_fn())
