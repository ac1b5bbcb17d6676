"""CPU: the topic-cache restatement (oracle rtps_oracle_topics_*, TopicCache::add_change,
structure/dds_cache.rs:210-284, 367-420) against

  * the reference's own known answer (dds_cache.rs:463-530: three changes of one writer,
    SN 1, 2, 3, all stored),
  * hand-derived cases: two readers of one topic, a GC at a multiple-of-64 SN evicting
    the oldest changes so that a later duplicate is stored again, the periodic GC,
  * a literal transcription of the reference's data structures (an insertion-ordered
    `changes` map keyed by instant, `sequence_numbers`, remove_changes_before with its
    must / may counts) on random streams: the oracle's [E, I) formulation must agree.
"""
import numpy as np
import pytest

import oracle
from rtps_rx.records import RECORD_DTYPE, DELIVERY_DTYPE, DELIVERY_CACHED, DATA


def _recs(items):
    """items: [(prefix byte, writer key, sn)] -> records (DATA)."""
    r = np.zeros(len(items), dtype=RECORD_DTYPE)
    for i, (p, w, sn) in enumerate(items):
        r[i]["kind"] = DATA
        r[i]["prefix"] = [p] * 12
        r[i]["writer_id"] = [0, 0, w, 0x02]
        r[i]["sn"] = sn
    return r


def _dels(pairs):
    d = np.zeros(len(pairs), dtype=DELIVERY_DTYPE)
    for i, (rec, slot) in enumerate(pairs):
        d[i]["rec_idx"], d[i]["reader_slot"] = rec, slot
    return d


def _cached(d):
    return ((d["flags"] & DELIVERY_CACHED) != 0).astype(int).tolist()


def test_reference_known_answer_three_changes():
    """dds_cache.rs:463-530: SN 1, 2, 3 of GUID_UNKNOWN added to one topic -> 3 changes held."""
    tc = oracle.TopicCaches([(7, 64)], [(0, 7)])
    recs = _recs([(0, 0, 1), (0, 0, 2), (0, 0, 3)])
    recs["prefix"] = 0
    recs["writer_id"] = 0  # GUID::GUID_UNKNOWN
    assert _cached(tc.apply(recs, _dels([(0, 0), (1, 0), (2, 0)]))) == [1, 1, 1]


def test_two_readers_one_topic():
    """Both readers accept every sample (their own proxies); the topic stores each (writer, SN) once."""
    tc = oracle.TopicCaches([(1, 64)], [(3, 1), (4, 1)])
    recs = _recs([(9, 1, sn) for sn in range(1, 6)])
    d = _dels([(i, s) for i in range(5) for s in (3, 4)])
    assert _cached(tc.apply(recs, d)) == [1, 0] * 5
    # another topic's reader of the same writer stores them in its own cache
    tc2 = oracle.TopicCaches([(1, 64), (2, 64)], [(3, 1), (4, 2)])
    assert _cached(tc2.apply(recs, d)) == [1, 1] * 5


def test_unmapped_readers_have_private_caches():
    tc = oracle.TopicCaches()
    recs = _recs([(9, 1, 5)])
    assert _cached(tc.apply(recs, _dels([(0, 1), (0, 2), (0, 1)]))) == [1, 1, 0]


def test_gc_at_multiple_of_64_evicts_oldest():
    """max_keep 2: SN 1, 2, 3 are stored (no GC: no SN % 64 == 0); a re-sent SN 1 is a duplicate;
    SN 64 triggers the GC first (4 changes > 2: the two oldest, SN 1 and 2, go), is stored; now
    SN 1 is stored again, SN 3 (still held) is not."""
    tc = oracle.TopicCaches([(1, 2)], [(0, 1)])
    recs = _recs([(9, 1, sn) for sn in (1, 2, 3, 1, 64, 1, 3, 2)])
    d = _dels([(i, 0) for i in range(len(recs))])
    assert _cached(tc.apply(recs, d)) == [1, 1, 1, 0, 1, 1, 0, 0]
    # cache now holds (insertion order) 3, 64, 1 -> the periodic GC trims to the newest 2: 64, 1.
    # Then SN 3 is stored (64, 1, 3); SN 64's own GC evicts the oldest, 64 itself, before the
    # duplicate check, so it is stored again (1, 3, 64); SN 1 is held: not stored.
    tc.gc()
    recs2 = _recs([(9, 1, sn) for sn in (3, 64, 1)])
    assert _cached(tc.apply(recs2, _dels([(0, 0), (1, 0), (2, 0)]))) == [1, 1, 0]


class LiteralTopicCache:
    """The reference's TopicCache, transcribed: changes (instant -> (guid, sn)), sequence_numbers,
    add_change_internal (:221-268), remove_changes_before(ZERO) (:367-420) with KeepLast(1)."""

    def __init__(self, max_keep):
        self.max_keep = max_keep
        self.changes = {}      # instant -> key; instants increase with every insert
        self.seq = {}          # key -> instant
        self.now = 0

    def remove_changes_before_zero(self):
        count = len(self.changes)
        must = max(count - self.max_keep, 0)
        may = max(max(count - 1, 0), must)  # KeepLast { depth: 1 }
        keys = sorted(self.changes)
        # skip_while(i < must || (ts < ZERO && i < may)): ts < ZERO never holds
        cut = 0
        while cut < len(keys) and (cut < must or (False and cut < may)):
            cut += 1
        for ts in keys[:cut]:
            k = self.changes.pop(ts)
            del self.seq[k]

    def add_change(self, key, sn):
        if sn % 64 == 0:
            self.remove_changes_before_zero()
        if key in self.seq:
            return False
        self.now += 1
        self.changes[self.now] = key
        self.seq[key] = self.now
        return True


@pytest.mark.parametrize("seed", range(6))
def test_random_streams_match_literal_transcription(seed):
    rng = np.random.default_rng(seed)
    topics = [(10, int(rng.integers(1, 6))), (11, int(rng.integers(1, 80)))]
    slots = {0: 10, 1: 10, 2: 11, 3: 11}
    tc = oracle.TopicCaches(topics, list(slots.items()))
    lit = {t: LiteralTopicCache(k) for t, k in topics}
    for batch in range(4):
        n = 400
        items = [(int(rng.integers(1, 3)), int(rng.integers(1, 3)), int(rng.integers(-2, 200))) for _ in range(n)]
        recs = _recs(items)
        pairs = []
        for i in range(n):
            for s in rng.choice(4, size=int(rng.integers(1, 4)), replace=False):
                pairs.append((i, int(s)))
        got = _cached(tc.apply(recs, _dels(pairs)))
        want = []
        for (i, s) in pairs:
            p, w, sn = items[i]
            want.append(1 if lit[slots[s]].add_change((p, w, sn), sn) else 0)
        assert got == want, f"batch {batch}"
        if batch == 2:
            tc.gc()
            for c in lit.values():
                c.remove_changes_before_zero()
