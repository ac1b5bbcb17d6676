"""GPU parity of the topic caches (rtps_rx_ingest with RTPS_INGEST_TOPIC_CACHE: the
deliveries' DELIVERY_CACHED flag, TopicCache::add_change, structure/dds_cache.rs:210-284)
against the CPU oracle: the writer-proxy restatement (rtps_oracle_ingest_*) followed by
the sequential add_change restatement (rtps_oracle_topics_*), batch after batch.

The four cases a delivery list alone gets wrong (each delivery is an on_read, but not
each is stored): two readers of one topic on one writer; a reader matched mid-stream
whose fresh proxy re-accepts SNs the topic still holds (or no longer holds, after the
GC); repeated SNs of a writer with no proxy whose kind is not user-defined; the SPDP
participant reader, which accepts duplicates.  Plus mixed topics with small caches
across batches with the periodic GC, and full-size C3."""
import numpy as np
import pytest

import ingest_ref as R
import oracle
from rtps_rx.records import Readers, DELIVERY_CACHED

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


@pytest.fixture
def rx():
    import rtps_rx
    r = rtps_rx.MessageReceiver(oracle.OWN_PREFIX, max_datagrams=1 << 21)
    yield r
    r.close()


def _batch(rx, ing, tcs, rd, dgrams, label):
    arena, off, ln = oracle.pack(dgrams, align=4)
    res, acc, dels, ack, ovf, _ = rx.ingest_batch(arena, off, ln, rd.n_proxies, topic_cache=True)
    st, recs, _, _ = oracle.parse(arena, off, ln, match_table=rd, threads=8)
    assert res.records.tobytes() == recs.tobytes(), f"{label}: parse differs"
    o_acc, o_dels, o_ack = ing.batch(arena, off, recs)
    o_dels = tcs.apply(recs, o_dels)
    assert np.array_equal(dels["rec_idx"], o_dels["rec_idx"]) and \
        np.array_equal(dels["reader_slot"], o_dels["reader_slot"]), f"{label}: deliveries differ"
    bad = np.nonzero(dels["flags"] != o_dels["flags"])[0]
    assert len(bad) == 0, (f"{label}: {len(bad)} cache flags differ, first at {bad[:6]}: "
                           f"gpu {dels['flags'][bad[:6]]} oracle {o_dels['flags'][bad[:6]]}")
    return dels


def _cached(d):
    return (d["flags"] & DELIVERY_CACHED) != 0


def _data_stream(prefix, wkey, sns, per_datagram=3):
    out, cur = [], []
    for sn in sns:
        cur.append(R.data_sub(wkey, int(sn)))
        if len(cur) == per_datagram:
            out.append(R.datagram(prefix, cur))
            cur = []
    if cur:
        out.append(R.datagram(prefix, cur))
    return out


def test_two_readers_of_one_topic(rx):
    P, wk = R.PREFIXES, R.writer_key
    rd = Readers([(bytes([0, 0, 1, 7]), 10, 0), (bytes([0, 0, 2, 7]), 11, 0)],
                 [(P[0] + wk(0), 0), (P[0] + wk(0), 1)])
    rx.set_readers(rd)
    rx.set_topics([(1, 64)], [(10, 1), (11, 1)])
    ing, tcs = oracle.HistoryIngest(rd), oracle.TopicCaches([(1, 64)], [(10, 1), (11, 1)])
    rng = np.random.default_rng(3)
    for b in range(3):
        sns = rng.integers(1, 400, 600)
        d = _batch(rx, ing, tcs, rd, _data_stream(P[0], wk(0), sns), f"batch {b}")
        assert (~_cached(d)).sum() > 0 and _cached(d).sum() > 0


@pytest.mark.parametrize("keep", [2000, 3])
def test_reader_matched_mid_stream(rx, keep):
    """A second reader of the topic is matched after SN 1..300 arrived; the writer then
    re-sends them (a reliable repair): the new reader's fresh proxy accepts every one (on_read),
    the topic stores those it no longer holds (max_keep 3: nearly all; 2000: none)."""
    P, wk = R.PREFIXES, R.writer_key
    r1 = [(bytes([0, 0, 1, 7]), 10, 0)]
    rd1 = Readers(r1, [(P[0] + wk(0), 0)])
    rd2 = Readers(r1 + [(bytes([0, 0, 2, 7]), 11, 0)], [(P[0] + wk(0), 0), (P[0] + wk(0), 1)])
    topics = [(1, keep)]
    rx.set_readers(rd1)
    rx.set_topics(topics, [(10, 1), (11, 1)])
    ing, tcs = oracle.HistoryIngest(rd1), oracle.TopicCaches(topics, [(10, 1), (11, 1)])
    _batch(rx, ing, tcs, rd1, _data_stream(P[0], wk(0), range(1, 301)), "before")
    rx.set_readers(rd2)
    ing.set_readers(rd2)
    d = _batch(rx, ing, tcs, rd2, _data_stream(P[0], wk(0), range(1, 301)), "resend")
    assert len(d) == 300 and (d["reader_slot"] == 11).all()
    stored = int(_cached(d).sum())
    assert (stored == 0) if keep == 2000 else (stored > 250)
    d = _batch(rx, ing, tcs, rd2, _data_stream(P[0], wk(0), range(290, 360)), "after")
    assert len(d) > 0


def test_proxy_less_builtin_kind_writer(rx):
    """A writer of builtin entity kind without a proxy: every sample is accepted (reader.rs:734-739),
    repeats included; the topic stores each (writer, SN) once while it holds it."""
    rd = R.a15_readers()
    rx.set_readers(rd)
    topics = [(1, 5)]
    rx.set_topics(topics, [(10, 1)])
    ing, tcs = oracle.HistoryIngest(rd), oracle.TopicCaches(topics, [(10, 1)])
    rng = np.random.default_rng(9)
    for b in range(3):
        dg = []
        for p in (1, 2, 3):
            dg += _data_stream(R.PREFIXES[p], R.BUILTIN_KIND_KEY, rng.integers(1, 90, 150), per_datagram=2)
        order = rng.permutation(len(dg))
        d = _batch(rx, ing, tcs, rd, [dg[i] for i in order], f"builtin-kind batch {b}")
        assert (~_cached(d)).sum() > 0


def test_spdp_reader_accepts_duplicates(rx):
    """The SPDP participant reader accepts duplicate samples (reader.rs:712-722); its topic cache
    stores a (writer, SN) only once while it holds it; max_keep 4 lets old ones back in."""
    P, wk = R.PREFIXES, R.writer_key
    rd = Readers([(R.SPDP_PARTICIPANT_READER, 14, 0)], [(P[0] + wk(0), 0)])
    rx.set_readers(rd)
    topics = [(9, 4)]
    rx.set_topics(topics, [(14, 9)])
    ing, tcs = oracle.HistoryIngest(rd), oracle.TopicCaches(topics, [(14, 9)])
    rng = np.random.default_rng(1)
    for b in range(3):
        sns = np.concatenate([rng.integers(1, 30, 200), np.arange(60, 70), [64, 64, 128, 1, 1]])
        d = _batch(rx, ing, tcs, rd, _data_stream(P[0], wk(0), sns), f"spdp batch {b}")
        assert len(d) == len(sns) and (~_cached(d)).sum() > 0


@pytest.mark.parametrize("seed", [5, 6])
def test_a15_topics_across_batches_with_gc(rx, seed):
    """Mixed: two readers of topic 1 (one with a proxy for the builtin-kind writer), the
    BestEffort and SPDP readers on topic 2 (max_keep 3), the rest private; the random a15
    stream (duplicates, GAPs, HEARTBEATs) in batches, the periodic GC between two of them."""
    rd = R.a15_readers()
    rx.set_readers(rd)
    topics = [(1, 6), (2, 3)]
    tr = [(10, 1), (11, 1), (13, 2), (14, 2)]
    rx.set_topics(topics, tr)
    ing, tcs = oracle.HistoryIngest(rd), oracle.TopicCaches(topics, tr)
    dgrams = R.a15_stream(8000, seed)
    for a, b in [(0, 1), (1, 3000), (3000, 3001), (3001, 8000)]:
        _batch(rx, ing, tcs, rd, dgrams[a:b], f"a15 seed {seed} {a}:{b}")
        if a == 1:
            rx.topic_gc()
            tcs.gc()


def test_ingest_reset_keeps_topic_caches(rx):
    """rtps_rx_ingest_reset re-creates the writer proxies but not the topic caches,
    as in the reference (fresh RtpsWriterProxy entries, rtps_writer_proxy.rs:62-90; the
    TopicCache outlives them): the re-sent SNs pass the fresh proxies and are dropped by
    add_change's find_by_sn while the topic still holds them (dds_cache.rs:241-276).  The
    oracle keeps one TopicCaches across a fresh HistoryIngest."""
    P, wk = R.PREFIXES, R.writer_key
    rd = Readers([(bytes([0, 0, 1, 7]), 10, 0), (bytes([0, 0, 2, 7]), 11, 0)],
                 [(P[0] + wk(0), 0), (P[0] + wk(0), 1)])
    rx.set_readers(rd)
    rx.set_topics([(1, 64)], [(10, 1), (11, 1)])
    tcs = oracle.TopicCaches([(1, 64)], [(10, 1), (11, 1)])
    dg = _data_stream(P[0], wk(0), range(1, 50))
    for k, want in ((0, 49), (1, 0)):
        ing = oracle.HistoryIngest(rd)
        d = _batch(rx, ing, tcs, rd, dg, f"after ingest reset {k}")
        assert len(d) == 2 * 49 and _cached(d).sum() == want
        rx.ingest_reset()
    # past max_keep the topic has let the oldest go: those SNs are stored again
    dg2 = _data_stream(P[0], wk(0), range(50, 130))
    _batch(rx, oracle.HistoryIngest(rd), tcs, rd, dg2, "beyond max_keep")
    rx.ingest_reset()
    d = _batch(rx, oracle.HistoryIngest(rd), tcs, rd, dg, "old SNs after GC")
    assert _cached(d).sum() > 0


def test_topic_reset_empties_topic_caches(rx):
    """rtps_rx_topic_reset empties every topic cache (the proxies keep their state): after it, a
    re-sent stream through reset proxies is stored again in full."""
    P, wk = R.PREFIXES, R.writer_key
    rd = Readers([(bytes([0, 0, 1, 7]), 10, 0), (bytes([0, 0, 2, 7]), 11, 0)],
                 [(P[0] + wk(0), 0), (P[0] + wk(0), 1)])
    rx.set_readers(rd)
    rx.set_topics([(1, 64)], [(10, 1), (11, 1)])
    dg = _data_stream(P[0], wk(0), range(1, 50))
    for k in range(2):
        ing, tcs = oracle.HistoryIngest(rd), oracle.TopicCaches([(1, 64)], [(10, 1), (11, 1)])
        d = _batch(rx, ing, tcs, rd, dg, f"after topic reset {k}")
        assert _cached(d).sum() == 49
        rx.ingest_reset()
        rx.topic_reset()


def test_full_size_c3_two_readers_per_topic(rx):
    """1M C3 datagrams, every writer matched by two readers of one topic (max_keep 64)."""
    import rtps_rx
    from test_gpu_parity import _device_gen
    n = 1 << 20
    arena, off, ln = _device_gen(rx, 3, n)
    _, recs0, _, _ = oracle.parse(arena[:4 << 20], off[:2000], ln[:2000])
    from rtps_rx.records import DATA
    guids = sorted({bytes(r["prefix"]) + bytes(r["writer_id"]) for r in recs0 if r["kind"] == DATA})
    rd = Readers([(bytes([0, 0, 1, 7]), 10, 0), (bytes([0, 0, 2, 7]), 11, 0)],
                 [(g, 0) for g in guids] + [(g, 1) for g in guids[::2]])
    rx.set_readers(rd)
    rx.set_topics([(1, 64)], [(10, 1), (11, 1)])
    ing, tcs = oracle.HistoryIngest(rd), oracle.TopicCaches([(1, 64)], [(10, 1), (11, 1)])
    res, acc, dels, ack, ovf, _ = rx.ingest_batch(arena, off, ln, rd.n_proxies, topic_cache=True)
    st, recs, _, _ = oracle.parse(arena, off, ln, match_table=rd, threads=8)
    o_acc, o_dels, o_ack = ing.batch(arena, off, recs)
    o_dels = tcs.apply(recs, o_dels)
    assert dels.tobytes() == o_dels.tobytes()
    assert _cached(dels).sum() < len(dels)


@pytest.mark.parametrize("pattern", ["pairs", "halves"])
def test_spdp_repeats_batch(rx, pattern):
    """The topic caches' adversarial batch (bench.py topic_cache_spdp_repeats
    at 1M): the SPDP participant reader accepts duplicates (reader.rs:712-722), so every delivery
    is a candidate, and >= 50 % of them repeat a key stored earlier in the same batch (the
    in-order tc_resolve): 'pairs' = every SN twice in a row, 'halves' = the second half repeats
    the first.  One topic, max_keep 64; bit-exact CACHED flags against the oracle."""
    P, wk = R.PREFIXES, R.writer_key
    rd = Readers([(R.SPDP_PARTICIPANT_READER, 14, 0)], [(P[0] + wk(0), 0)])
    rx.set_readers(rd)
    topics = [(9, 64)]
    rx.set_topics(topics, [(14, 9)])
    ing, tcs = oracle.HistoryIngest(rd), oracle.TopicCaches(topics, [(14, 9)])
    n = 60000
    sns = (np.arange(n) // 2 + 1) if pattern == "pairs" else (np.arange(n) % (n // 2) + 1)
    d = _batch(rx, ing, tcs, rd, _data_stream(P[0], wk(0), sns, per_datagram=1), f"spdp {pattern}")
    # pairs: each repeat finds its key held (dropped); halves: max_keep 64 let every key go long
    # before its repeat (stored again) -- both through the in-order repeat resolution
    assert len(d) == n and _cached(d).sum() == (n // 2 if pattern == "pairs" else n)
