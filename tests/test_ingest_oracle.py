"""History-cache ingest, CPU side: the oracle's sequential restatement
(rtps_oracle_ingest_batch) against hand-derived known answers from the
reference's writer-proxy rules and against an independent Python model
(tests/ingest_ref.py) on random corpora, batch after batch.

Parity pinning: the reference has no unit test for RtpsWriterProxy /
Reader::handle_*_msg with wire input, so these answers are derived from
rtps/rtps_writer_proxy.rs:202-355 and io_uring/rtps/reader.rs:514-1116
(parity unpinned by fixtures; two independent restatements agree)."""
import numpy as np
import pytest

import frag_ref
import ingest_ref as R
import oracle
from rtps_rx.records import pack_match_table, DATA_FRAG


def _run(dgrams, ing, best_effort=False, frag=None, pairs=False):
    """accepted: the deliveries' record indices (pairs: (record, reader slot) tuples)."""
    arena, off, ln = oracle.pack(dgrams, align=4)
    tbl = ing.table
    st, recs, _, _ = oracle.parse(arena, off, ln, match_table=tbl)
    samples = frag.batch(arena, off, recs)[0] if frag is not None else None
    acc, dels, ack = ing.h.batch(arena, off, recs, samples, best_effort=best_effort)
    accepted = _pairs(dels) if pairs else np.array(dels["rec_idx"], dtype=np.int64)
    return arena, off, recs, samples, acc, accepted, ack


def _pairs(dels):
    return [(int(d["rec_idx"]), int(d["reader_slot"])) for d in dels]


class _Ing:
    def __init__(self, tbl):
        self.table = tbl
        self.h = oracle.HistoryIngest(tbl)


def _one_writer():
    tbl = pack_match_table([(R.PREFIXES[0] + R.writer_key(0), 0), (R.PREFIXES[1] + R.writer_key(0), 1)])
    return _Ing(tbl)


def _data_dgrams(sns, p=0, k=0):
    return [R.datagram(R.PREFIXES[p], [R.data_sub(R.writer_key(k), s)]) for s in sns]


def test_duplicates_first_occurrence_wins():
    ing = _one_writer()
    *_, acc, accepted, ack = _run(_data_dgrams([1, 2, 2, 1, 3]), ing)
    assert accepted.tolist() == [0, 1, 4]
    assert ack.tolist() == [4, 1]


def test_out_of_order_and_persistence_across_batches():
    ing = _one_writer()
    *_, accepted, ack = _run(_data_dgrams([3, 1]), ing)
    assert accepted.tolist() == [0, 1] and ack.tolist() == [2, 1]  # 2 missing
    *_, accepted, ack = _run(_data_dgrams([3, 2, 0, -5, 4]), ing)
    assert accepted.tolist() == [1, 4] and ack.tolist() == [5, 1]


def test_heartbeat_first_sn_and_stale_count():
    ing = _one_writer()
    w = R.writer_key(0)
    d = [R.datagram(R.PREFIXES[0], [R.hb_sub(w, 5, 9, 1), R.data_sub(w, 3), R.data_sub(w, 5)]),
         R.datagram(R.PREFIXES[0], [R.hb_sub(w, 10, 12, 1), R.data_sub(w, 7)]),   # stale count: ignored
         R.datagram(R.PREFIXES[0], [R.hb_sub(w, 8, 12, 2), R.data_sub(w, 7)])]    # 7 < new ack_base 8... already have it
    *_, accepted, ack = _run(d, ing)
    assert accepted.tolist() == [2, 4]  # DATA 5, then DATA 7 (second copy ignored)
    assert ack.tolist() == [8, 1]


def test_best_effort_ignores_heartbeats():
    ing = _one_writer()
    w = R.writer_key(0)
    d = [R.datagram(R.PREFIXES[0], [R.hb_sub(w, 5, 9, 1), R.data_sub(w, 3)])]
    *_, accepted, ack = _run(d, ing, best_effort=True)
    assert accepted.tolist() == [1] and ack.tolist() == [1, 1]


def test_gap_range_and_list():
    ing = _one_writer()
    w = R.writer_key(0)
    d = [R.datagram(R.PREFIXES[0], [R.gap_sub(w, 2, 4, [True, False, True])]),  # 2, 3 + list {4, 6}
         R.datagram(R.PREFIXES[0], [R.data_sub(w, s) for s in (1, 3, 5, 6)]),
         R.datagram(R.PREFIXES[0], [R.gap_sub(w, 0, 9, [True])]),                 # invalid: gapStart <= 0
         R.datagram(R.PREFIXES[0], [R.data_sub(w, 8)])]
    *_, accepted, ack = _run(d, ing)
    assert accepted.tolist() == [1, 3, 6]
    assert ack.tolist() == [7, 1]  # 7 never arrived


def test_sample_kinds_and_unmatched():
    ing = _one_writer()
    w = R.writer_key(0)
    d = [R.datagram(R.PREFIXES[0], [R.data_sub(w, 1, key=True), R.data_sub(w, 2, both=True),
                                    R.data_sub(w, 2, key_hash=bytes(16)), R.data_sub(w, 3, le=False)]),
         R.datagram(R.PREFIXES[2], [R.data_sub(w, 1)]),                           # writer not in the table
         R.datagram(R.PREFIXES[1], [R.info_dst_sub(bytes([9] * 12)), R.data_sub(w, 1)])]  # not for us
    *_, acc, accepted, ack = _run(d, ing)
    assert accepted.tolist() == [0, 2, 3]
    assert acc.tolist() == [1, 0, 1, 1, 0, 0, 0]
    assert ack.tolist() == [4, 1]


@pytest.mark.parametrize("seed", [1, 2, 3, 4])
@pytest.mark.parametrize("best_effort", [False, True])
def test_oracle_matches_python_model(seed, best_effort):
    tbl, guids = R.table()
    ing = _Ing(tbl)
    model = R.IngestRef(tbl)
    dgrams = R.stream(1500, seed)
    for a, b in [(0, 1), (1, 400), (400, 401), (401, 1500)]:
        arena, off, recs, _, acc, accepted, ack = _run(dgrams[a:b], ing, best_effort=best_effort, pairs=True)
        m_acc, m_ack = model.batch(arena, off, recs, best_effort=best_effort)
        assert accepted == m_acc, f"seed {seed} batch {a}:{b}"
        assert ack.tolist() == m_ack, f"seed {seed} batch {a}:{b}"
        assert int(acc.sum()) == len(m_acc)


@pytest.mark.parametrize("seed", [5, 6, 7])
@pytest.mark.parametrize("best_effort", [False, True])
def test_reader_sets_oracle_matches_python_model(seed, best_effort):
    """a15: reader sets (two readers on one writer, stateless / BestEffort / participant
    readers, builtin- and vendor-kind writers, writers known by entity id only)."""
    rd = R.a15_readers()
    ing = _Ing(rd)
    model = R.IngestRef(rd)
    dgrams = R.a15_stream(2000, seed)
    for a, b in [(0, 700), (700, 701), (701, 2000)]:
        arena, off, recs, _, acc, accepted, ack = _run(dgrams[a:b], ing, best_effort=best_effort, pairs=True)
        m_acc, m_ack = model.batch(arena, off, recs, best_effort=best_effort)
        assert accepted == m_acc, f"seed {seed} batch {a}:{b}"
        assert ack.tolist() == m_ack, f"seed {seed} batch {a}:{b}"
        slots = {s for _, s in m_acc}
        assert 12 not in slots  # the stateless reader never receives


def test_reader_sets_known_answers():
    """Hand-derived from dp_event_loop.rs:266-327, reader.rs:474-484, 693-758: targets in
    EntityId order (slot 10 < 11 < 14), the participant reader accepts duplicates, a
    writer known only by entity id delivers only when its kind is not user-defined."""
    rd = R.a15_readers()
    ing = _Ing(rd)
    P, wk = R.PREFIXES, R.writer_key
    d = [R.datagram(P[0], [R.data_sub(wk(0), 1)]),                  # 0: readers 10, 11, 14 (all proxied)
         R.datagram(P[0], [R.data_sub(wk(0), 1)]),                  # 1: duplicate: only 14
         R.datagram(P[3], [R.data_sub(wk(0), 1)]),                  # 2: unknown prefix, user kind: none
         R.datagram(P[3], [R.data_sub(R.BUILTIN_KIND_KEY, 5)]),     # 3: builtin kind, no proxy: reader 10
         R.datagram(P[1], [R.data_sub(R.VENDOR_KIND_KEY, 2)] * 2),  # 4, 5: participant reader, dup ok
         R.datagram(P[0], [R.data_sub(wk(2), 1)]),                  # 6: only the stateless reader has it
         R.datagram(P[2], [R.hb_sub(wk(1), 9, 9, 1), R.data_sub(wk(1), 3)])]  # 7 HB: 11 no proxy, 13 BestEffort
    *_, acc, accepted, ack = _run(d, ing, pairs=True)
    assert accepted == [(0, 10), (0, 11), (0, 14), (1, 14), (3, 10), (4, 14), (5, 14), (8, 13)]  # 8: 11 has no proxy
    assert acc.tolist() == [3, 1, 0, 1, 1, 1, 0, 0, 1]
    # proxies: (P0 w0 r1) (P0 w0 r0) (P1 w0) (P0 w1) (stateless x2) (P2 w1 r3) (P0 bk) (P1 vk r4) (P0 w0 r4)
    assert ack.tolist() == [2, 2, 1, 1, 1, 1, 1, 1, 1, 2]


def test_completed_datafrag_samples():
    dgrams = frag_ref.soup(1200, 5)
    arena, off, ln = oracle.pack(dgrams, align=4)
    _, recs0, _, _ = oracle.parse(arena, off, ln)
    fr = recs0[recs0["kind"] == DATA_FRAG]
    guids = sorted({bytes(r["prefix"]) + bytes(r["writer_id"]) for r in fr})
    tbl = pack_match_table([(g, i) for i, g in enumerate(guids[:-1])])  # last writer unmatched
    ing = _Ing(tbl)
    model = R.IngestRef(tbl)
    fa = oracle.FragAssembler()
    for a, b in [(0, 500), (500, 1200)]:
        arena, off, recs, samples, acc, accepted, ack = _run(dgrams[a:b], ing, frag=fa, pairs=True)
        m_acc, m_ack = model.batch(arena, off, recs, samples)
        assert accepted == m_acc and ack.tolist() == m_ack
    assert len(accepted) > 0


def test_reader_sets_targets_and_route_bits():
    """The oracle's per-record target readers (rtps_oracle_targets) and the MATCHED /
    TARGETED route bits of its parse against the Python model's literal scan."""
    from rtps_rx.records import ROUTE_MATCHED, ROUTE_TARGETED, ROUTE_BUILTIN, WRITER_KINDS, NO_PROXY
    rd = R.a15_readers()
    model = R.IngestRef(rd)
    arena, off, ln = oracle.pack(R.a15_stream(800, 11), align=4)
    st, recs, (t_off, t_ent), _ = oracle.parse(arena, off, ln, match_table=rd)
    n_multi = 0
    for i, r in enumerate(recs):
        guid = bytes(r["prefix"]) + bytes(r["writer_id"])
        exp = []
        if int(r["kind"]) in WRITER_KINDS and not int(r["route"]) & ROUTE_BUILTIN:
            exp = [(model.slot[x], NO_PROXY if k is None else k) for x, k in model.targets(guid)]
        got = [(int(e["reader_slot"]), int(e["proxy"])) for e in t_ent[int(t_off[i]):int(t_off[i + 1])]]
        assert got == exp, i
        route = int(r["route"])
        assert bool(route & ROUTE_TARGETED) == bool(exp), i
        assert bool(route & ROUTE_MATCHED) == any(k != NO_PROXY for _, k in exp), i
        n_multi += len(exp) > 1
    assert n_multi > 100
