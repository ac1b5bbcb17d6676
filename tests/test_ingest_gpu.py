"""GPU parity of the history-cache ingest (rtps_rx_ingest) with the CPU
oracle's sequential writer-proxy restatement: every per-record accept count,
the delivery list (record, reader slot) and every proxy's all_ackable_before,
batch after batch (state carried in the context), on random reliable /
best-effort corpora, on both ingest paths, reader sets (several readers per writer, stateless /
BestEffort / participant readers, writers known by entity id only),
completed DataFrag samples, the C3 and T workloads at full size, and the
edges (window overflow, empty batches, reset, a growing table)."""
import numpy as np
import pytest

import frag_ref
import ingest_ref as R
import oracle
from rtps_rx.records import pack_match_table, DATA_FRAG, Readers, DELIVERY_DTYPE

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


@pytest.fixture(params=[1, 2, 3, 4], ids=["global", "per_proxy", "global_fcmerge", "per_proxy_radix"])
def rx(request):
    """Every test runs on every ingest path (forced): global marks / merge, one
    workgroup per proxy replaying its events in order against an LDS window (its
    events grouped by the proxy bucketing, or by the radix sort: per_proxy_radix), and the
    global path whose GAP-free batches merge their coverage from the first-cover keys
    (k_fcmerge, chosen by size for large batches over few proxies, forced here)."""
    import rtps_rx
    r = rtps_rx.MessageReceiver(oracle.OWN_PREFIX, max_datagrams=1 << 21)
    r.debug_ingest_path(request.param)
    yield r
    r.close()


def _n_proxies(tbl):
    return tbl.n_proxies if isinstance(tbl, Readers) else len(Readers.from_match(tbl).proxies)


def _batch(rx, ing, tbl, dgrams, label, frag=False, fa=None, best_effort=False, align=4):
    arena, off, ln = oracle.pack(dgrams, align=align)
    res, acc, accepted, ack, ovf, samples = rx.ingest_batch(arena, off, ln, _n_proxies(tbl), frag=frag,
                                                            best_effort=best_effort)
    st, recs, _, _ = oracle.parse(arena, off, ln, match_table=tbl, threads=8)
    assert res.records.tobytes() == recs.tobytes(), f"{label}: parse differs"
    o_samples = fa.batch_readers(arena, off, recs, tbl)[0] if frag else None
    o_acc, o_accepted, o_ack = ing.batch(arena, off, recs, o_samples, best_effort=best_effort)
    assert np.array_equal(acc, o_acc), f"{label}: accept flags differ at {np.nonzero(acc != o_acc)[0][:10]}"
    assert accepted.tobytes() == o_accepted.tobytes(), f"{label}: deliveries"
    assert np.array_equal(ack, o_ack), f"{label}: ack_base {ack[ack != o_ack][:5]} vs {o_ack[ack != o_ack][:5]}"
    assert ovf == 0
    return acc, accepted, ack


@pytest.mark.parametrize("seed", [5, 6])
@pytest.mark.parametrize("best_effort", [False, True])
def test_reader_sets_across_batches(rx, seed, best_effort):
    """a15: several target readers per record (expanded events), per-proxy state."""
    rd = R.a15_readers()
    rx.set_readers(rd)
    ing = oracle.HistoryIngest(rd)
    dgrams = R.a15_stream(6000, seed)
    multi = 0
    for a, b in [(0, 1), (1, 2500), (2500, 2501), (2501, 6000)]:
        acc, dels, _ = _batch(rx, ing, rd, dgrams[a:b], f"a15 seed {seed} {a}:{b}", best_effort=best_effort)
        multi += int((acc > 1).sum())
    assert multi > 0


@pytest.mark.parametrize("seed", [1, 2, 3])
@pytest.mark.parametrize("best_effort", [False, True])
def test_stream_across_batches(rx, seed, best_effort):
    tbl, _ = R.table()
    rx.set_match_table(tbl)
    ing = oracle.HistoryIngest(tbl)
    dgrams = R.stream(6000, seed)
    total = 0
    for a, b in [(0, 1), (1, 2000), (2000, 2001), (2001, 6000)]:
        _, accepted, _ = _batch(rx, ing, tbl, dgrams[a:b], f"seed {seed} {a}:{b}", best_effort=best_effort)
        total += len(accepted)
    assert total > 20


def test_gap_heavy_single_proxy(rx):
    """One writer whose chunks hold more GAPs than the per-proxy kernel's chunk GAP list
    (GCAP = 512 of 2048 events): the listed GAPs run one per thread, the rest stay with
    their threads; both must give the oracle's decisions and ack_base."""
    tbl, _ = R.table(n_prefix=1, n_writer=1)
    rx.set_match_table(tbl)
    ing = oracle.HistoryIngest(tbl)
    rng = np.random.default_rng(11)
    wk = R.writer_key(0)
    dgrams = []
    for _ in range(3000):
        subs = []
        for _ in range(3):
            sn = int(rng.integers(1, 4000))
            if rng.random() < 0.8:
                nb = int(rng.integers(0, 100))
                subs.append(R.gap_sub(wk, sn, sn + int(rng.integers(-2, 6)), [bool(b) for b in rng.random(nb) < 0.3],
                                      bool(rng.random() < 0.8)))
            else:
                subs.append(R.data_sub(wk, sn, bool(rng.random() < 0.8)))
        dgrams.append(R.datagram(R.PREFIXES[0], subs))
    for a, b in [(0, 1500), (1500, 3000)]:
        _batch(rx, ing, tbl, dgrams[a:b], f"gaps {a}:{b}")


def test_dense_duplicates_wide_sn(rx):
    tbl, _ = R.table()
    rx.set_match_table(tbl)
    ing = oracle.HistoryIngest(tbl)
    for k, hi in enumerate([5, 300, 5000]):
        _batch(rx, ing, tbl, R.stream(4000, 40 + k, sn_hi=hi), f"sn_hi {hi}", align=1)


def test_completed_datafrag_samples(rx):
    dgrams = frag_ref.soup(3000, 7)
    arena, off, ln = oracle.pack(dgrams, align=4)
    _, recs0, _, _ = oracle.parse(arena, off, ln)
    guids = sorted({bytes(r["prefix"]) + bytes(r["writer_id"]) for r in recs0[recs0["kind"] == DATA_FRAG]})
    tbl = pack_match_table([(g, i) for i, g in enumerate(guids[:-1])])
    rx.set_match_table(tbl)
    ing = oracle.HistoryIngest(tbl)
    fa = oracle.FragAssembler()
    n = 0
    for a, b in [(0, 1000), (1000, 3000)]:
        _, accepted, _ = _batch(rx, ing, tbl, dgrams[a:b], f"frag {a}:{b}", frag=True, fa=fa)
        n += len(accepted)
    assert n > 10


def _far_draw(g):
    """SNs for the far-set tests: near ones, the window's edge, three anchors far past the
    window (duplicates included), so that samples, HEARTBEAT firstSNs and GAPs land beyond it."""
    import rtps_rx
    W = rtps_rx.INGEST_WINDOW
    x = g.random()
    if x < 0.5:
        return int(g.integers(-1, 80))
    if x < 0.6:
        return W - 3 + int(g.integers(0, 8))
    return int(g.choice([W + 40, 2 * W + 7, 5 * W])) + int(g.integers(0, 40))


def _far_gap_len(g, start):
    return start + (int(g.integers(30, 120)) if g.random() < 0.1 else int(g.integers(-3, 8)))


def test_far_sample_exact(rx):
    """a sample further than RTPS_INGEST_WINDOW ahead of the window is
    decided exactly (the far set, rtps_writer_proxy.rs:202-224), not accepted unchecked: a
    re-sent far SN is a duplicate in the same batch and in the next one."""
    import rtps_rx
    tbl = pack_match_table([(R.PREFIXES[0] + R.writer_key(0), 0)])
    rx.set_match_table(tbl)
    ing = oracle.HistoryIngest(tbl)
    w = R.writer_key(0)
    far = 1 + rtps_rx.INGEST_WINDOW + 5
    d = [R.datagram(R.PREFIXES[0], [R.data_sub(w, 1), R.data_sub(w, far), R.data_sub(w, 2), R.data_sub(w, far)])]
    acc, dels, ack = _batch(rx, ing, tbl, d, "far, batch 1")
    assert dels["rec_idx"].tolist() == [0, 1, 2] and ack.tolist() == [3]
    d = [R.datagram(R.PREFIXES[0], [R.data_sub(w, far), R.data_sub(w, far + 1), R.data_sub(w, 3)])]
    acc, dels, ack = _batch(rx, ing, tbl, d, "far, batch 2")
    assert dels["rec_idx"].tolist() == [1, 2] and ack.tolist() == [4]


def test_far_window_filled_up_to_the_far_set(rx):
    """The window covered up to its end: all_ackable_before continues through the far set
    (advance_ack_base, rtps_writer_proxy.rs:338-355), and the re-anchored window takes the
    far SNs it now spans."""
    import rtps_rx
    W = rtps_rx.INGEST_WINDOW
    tbl = pack_match_table([(R.PREFIXES[0] + R.writer_key(0), 0)])
    rx.set_match_table(tbl)
    ing = oracle.HistoryIngest(tbl)
    w = R.writer_key(0)
    far = [W + 1, W + 2, W + 3, W + 5, 2 * W + 9, 3 * W]
    _batch(rx, ing, tbl, [R.datagram(R.PREFIXES[0], [R.data_sub(w, v) for v in far])], "far first")
    # a GAP covering [1, W + 1): the window fills, ack_base runs through W+1..W+3, stops at W+4
    _, _, ack = _batch(rx, ing, tbl, [R.datagram(R.PREFIXES[0], [R.gap_sub(w, 1, W + 1, [])])], "gap fills")
    assert ack.tolist() == [W + 4]
    d = [R.datagram(R.PREFIXES[0], [R.data_sub(w, v) for v in (W + 4, W + 5, 2 * W + 9, 2 * W + 8, 3 * W)])]
    _, dels, _ = _batch(rx, ing, tbl, d, "after the pull")
    assert dels["rec_idx"].tolist() == [0, 3]


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_far_stream_across_batches(rx, seed):
    """Random reliable traffic whose SNs, HEARTBEAT firstSNs and GAPs reach past the window
    (three anchors up to 5 W ahead, duplicates, GAP ranges crossing the window's end),
    batch after batch: bit-exact with the oracle's unbounded change sets, nothing counted."""
    tbl, _ = R.table()
    rx.set_match_table(tbl)
    ing = oracle.HistoryIngest(tbl)
    dgrams = R.stream(5000, 100 + seed, sn_draw=_far_draw, gap_len=_far_gap_len)
    for a, b in [(0, 1), (1, 1500), (1500, 1501), (1501, 5000)]:
        _batch(rx, ing, tbl, dgrams[a:b], f"far seed {seed} {a}:{b}")


def test_far_reader_sets(rx):
    """The same with several readers per record (expanded events) and the SPDP participant
    reader (DUPLICATES_OK: its far samples are all accepted and recorded)."""
    rd = R.a15_readers()
    rx.set_readers(rd)
    ing = oracle.HistoryIngest(rd)
    dgrams = R.stream(4000, 77, sn_draw=_far_draw, gap_len=_far_gap_len,
                      keys=[R.writer_key(0), R.writer_key(1), R.writer_key(2), R.BUILTIN_KIND_KEY])
    for a, b in [(0, 2000), (2000, 4000)]:
        _batch(rx, ing, rd, dgrams[a:b], f"far a15 {a}:{b}")


def _far_datagrams(subs, per=8):
    """the (prefix 0) submessages in datagrams of `per`, in the given order"""
    return [R.datagram(R.PREFIXES[0], subs[i:i + per]) for i in range(0, len(subs), per)]


def test_far_sets_past_former_caps(rx):
    """more than 1024 far SNs for one proxy and more than 8192 far events
    in one batch (round 4's per-proxy FCAP and per-batch FL_CAP), and far GAP ranges of
    thousands of SNs, batch after batch: bit-exact with the oracle's unbounded change sets
    (rtps_writer_proxy.rs:62 BTreeMap), n_window_overflow == 0 (_batch); then a GAP fills
    writer 0's window and all_ackable_before runs through its 6000 far SNs (far_extend), the
    re-anchored window takes them (far_pull) and re-sent ones are duplicates."""
    import rtps_rx
    W = rtps_rx.INGEST_WINDOW
    w0, w1 = R.writer_key(0), R.writer_key(1)
    tbl = pack_match_table([(R.PREFIXES[0] + w0, 0), (R.PREFIXES[0] + w1, 1)])
    rx.set_match_table(tbl)
    ing = oracle.HistoryIngest(tbl)
    g = np.random.default_rng(3)
    # batch 1: writer 0 sends W+1 .. W+3000 four times over in random order (12000 far events,
    # 3000 far SNs); writer 1 a GAP [2W, 2W + 5000) with a listed bitmap, and samples around it
    sns = np.repeat(np.arange(W + 1, W + 3001), 4)
    g.shuffle(sns)
    subs = [R.data_sub(w0, int(v)) for v in sns]
    s1 = [R.data_sub(w1, int(v)) for v in g.integers(2 * W - 10, 2 * W + 5100, 3000)]
    s1.insert(1500, R.gap_sub(w1, 2 * W, 2 * W + 5000, [bool(b) for b in g.random(64) < 0.5]))
    for k, sub in enumerate(s1):
        subs.insert(int(g.integers(0, len(subs) + 1)), sub)
    acc, dels, ack = _batch(rx, ing, tbl, _far_datagrams(subs), "far batch 1")
    assert len(dels) > 3000 and ack.tolist() == [1, 1]
    # batch 2: re-sent SNs of batch 1 (duplicates across batches) and W+3001 .. W+6000 twice
    sns = np.concatenate([g.integers(W + 1, W + 3001, 2000), np.repeat(np.arange(W + 3001, W + 6001), 2)])
    g.shuffle(sns)
    subs = [R.data_sub(w0, int(v)) for v in sns] + [R.data_sub(w1, int(v)) for v in range(2 * W - 5, 2 * W + 5)]
    acc, dels, ack = _batch(rx, ing, tbl, _far_datagrams(subs), "far batch 2")
    assert len(dels) >= 3000
    # batch 3: a GAP covering [1, W + 1) for writer 0: ack_base runs through the far set
    _, _, ack = _batch(rx, ing, tbl, [R.datagram(R.PREFIXES[0], [R.gap_sub(w0, 1, W + 1, [])])], "far gap fills")
    assert ack.tolist() == [W + 6001, 1]
    # batch 4: around the new ack_base, and writer 1 past its GAP again
    subs = [R.data_sub(w0, v) for v in range(W + 5990, W + 6010)] + \
           [R.data_sub(w1, int(v)) for v in g.integers(2 * W, 2 * W + 5200, 500)]
    _batch(rx, ing, tbl, _far_datagrams(subs), "far batch 4")


def test_far_sets_many_proxies(rx):
    """Far items spread over 48 proxies (several tables grown in one batch, one workgroup
    each on the per-proxy path, one k_far pass over all of them on the global one), over
    three batches; bit-exact, nothing counted."""
    import rtps_rx
    W = rtps_rx.INGEST_WINDOW
    keys = [R.writer_key(k) for k in range(48)]
    tbl = pack_match_table([(R.PREFIXES[0] + k, i) for i, k in enumerate(keys)])
    rx.set_match_table(tbl)
    ing = oracle.HistoryIngest(tbl)
    g = np.random.default_rng(8)
    for b in range(3):
        subs = []
        for k, w in enumerate(keys):
            base = (1 + k % 3) * W + 1000 * b
            subs += [R.data_sub(w, int(v)) for v in g.integers(base, base + 400 + 40 * k, 300)]
            if k % 5 == 0:
                subs.append(R.gap_sub(w, base + 100, base + 900, [bool(x) for x in g.random(40) < 0.5]))
        g.shuffle(subs)
        _batch(rx, ing, tbl, _far_datagrams(subs, per=5), f"far proxies batch {b}")


def test_late_joiner_gap_threshold(rx):
    """A reader that joins late: the writer's GAP [1, 10^6) starts at or below the proxy's
    all_ackable_before, so irrelevant_changes_range only moves it to 10^6
    (rtps_writer_proxy.rs:241-292) -- a threshold, with nothing to record SN by SN past the
    window (the per-proxy path takes such batches whatever the path).  Samples before the GAP in
    event order are accepted, those after it below 10^6 rejected; bit-exact with the oracle,
    nothing counted (_batch), across batches, next to a writer with ordinary far traffic."""
    import rtps_rx
    W = rtps_rx.INGEST_WINDOW
    w0, w1 = R.writer_key(0), R.writer_key(1)
    tbl = pack_match_table([(R.PREFIXES[0] + w0, 0), (R.PREFIXES[0] + w1, 1)])
    rx.set_match_table(tbl)
    ing = oracle.HistoryIngest(tbl)
    top = 1_000_000
    subs = [R.data_sub(w0, top - 7), R.data_sub(w0, 5),
            R.gap_sub(w0, 1, top, [True, False, True]),
            R.data_sub(w0, top - 7), R.data_sub(w0, top - 1), R.data_sub(w0, top + 1), R.data_sub(w0, top + 2),
            R.data_sub(w0, top), R.data_sub(w1, 3 * W), R.data_sub(w1, 3 * W), R.data_sub(w1, 1)]
    _, dels, ack = _batch(rx, ing, tbl, [R.datagram(R.PREFIXES[0], subs[i:i + 3]) for i in range(0, len(subs), 3)],
                          "late joiner")
    assert ack.tolist()[0] == top + 3
    # the next batch: below the new all_ackable_before, a second threshold GAP, fresh SNs
    subs = [R.data_sub(w0, top - 3), R.gap_sub(w0, 2, top + 2 * W, []), R.data_sub(w0, top + 2 * W - 1),
            R.data_sub(w0, top + 2 * W), R.data_sub(w1, 3 * W), R.data_sub(w1, 2)]
    _, dels, ack = _batch(rx, ing, tbl, [R.datagram(R.PREFIXES[0], subs)], "late joiner 2")
    assert ack.tolist()[0] == top + 2 * W + 1


@pytest.mark.parametrize("case", ["samples", "samples_hb", "hb_only", "small_gap", "two_chunks"])
def test_gap_threshold_moved_in_batch(rx, case):
    """a GAP whose range starts above all_ackable_before as it was at the
    batch's start, but at or below it when the GAP arrives (the batch's own DATA, HEARTBEAT or
    GAPs moved it), is irrelevant_changes_range's jump (rtps_writer_proxy.rs:241-292), not a
    range to insert SN by SN: DATA 1..5 then GAP [6, 10^6) in one batch; with a HEARTBEAT
    firstSN 100 before a GAP [50, 10^6); a small GAP closing the hole; 3000 samples so that the
    GAP sits in the per-proxy kernel's second chunk.  Bit-exact with the oracle and nothing
    counted in n_window_overflow (_batch), samples after the GAP decided against it."""
    top = 1_000_000
    w0, w1 = R.writer_key(0), R.writer_key(1)
    tbl = pack_match_table([(R.PREFIXES[0] + w0, 0), (R.PREFIXES[0] + w1, 1)])
    rx.set_match_table(tbl)
    ing = oracle.HistoryIngest(tbl)
    D = lambda sn: R.data_sub(w0, sn)
    if case == "samples":
        subs = [D(k) for k in range(1, 6)] + [R.gap_sub(w0, 6, top, [True, False, True])]
    elif case == "samples_hb":
        subs = [D(k) for k in range(1, 6)] + [R.hb_sub(w0, 100, 120, 1), R.gap_sub(w0, 50, top, [])]
    elif case == "hb_only":
        subs = [R.hb_sub(w0, 100, 120, 1), D(99), R.gap_sub(w0, 6, top, [])]
    elif case == "small_gap":
        subs = [D(1), D(2), D(3), R.gap_sub(w0, 4, 8, []), R.gap_sub(w0, 8, top, [False, True])]
    else:
        subs = [D(k) for k in range(1, 3001)] + [R.gap_sub(w0, 3001, top, [])]
    subs += [D(7), D(60), D(top - 1), D(top), D(top + 1), D(top + 1), R.data_sub(w1, 4), D(top + 3)]
    dg = [R.datagram(R.PREFIXES[0], subs[i:i + 3]) for i in range(0, len(subs), 3)]
    acc, dels, ack = _batch(rx, ing, tbl, dg, case)
    assert ack.tolist()[0] == (top + 4 if case == "samples" else top + 2)  # (the oracle's: the jump happened)
    # a second batch: the new all_ackable_before holds (below it rejected, above accepted once)
    dg = [R.datagram(R.PREFIXES[0], [D(top - 5), D(top + 2), D(top + 2), D(top + 4)])]
    _batch(rx, ing, tbl, dg, case + " next")


def test_big_far_set_grid_pass(rx):
    """far sets past FT_BIG slots are finished by the grid-wide k_fx_* pass.
    One writer sends 150,000 SNs past its window first (a far table of 2^20 slots), then SNs
    1..100 (all_ackable_before 101: the re-anchored window pulls the far SNs it now spans, the set
    is not extended), then the rest of the window (all_ackable_before runs through all 150,000
    far SNs), then re-sends of far SNs (rejected) and fresh ones; a second writer beside it stays
    small.  Bit-exact with the oracle on every ingest path, nothing counted."""
    import rtps_rx
    W = rtps_rx.INGEST_WINDOW
    w0, w1 = R.writer_key(0), R.writer_key(1)
    tbl = pack_match_table([(R.PREFIXES[0] + w0, 0), (R.PREFIXES[0] + w1, 1)])
    rx.set_match_table(tbl)
    ing = oracle.HistoryIngest(tbl)
    rng = np.random.default_rng(21)
    far = W + 10 + rng.permutation(150_000)

    def dgrams(sns, w=w0, per=4):
        return [R.datagram(R.PREFIXES[0], [R.data_sub(w, int(x)) for x in sns[i:i + per]])
                for i in range(0, len(sns), per)]
    _, _, ack = _batch(rx, ing, tbl, dgrams(far) + dgrams(np.arange(1, 30), w1), "far first")
    assert ack.tolist() == [1, 30]
    _, _, ack = _batch(rx, ing, tbl, dgrams(np.arange(1, 101)), "pull only")
    assert ack.tolist()[0] == 101
    rest = np.concatenate([np.arange(101, W + 10), far[:5], [W + 150_010 + 3, W + 150_010]])
    _, dels, ack = _batch(rx, ing, tbl, dgrams(rest), "extension")
    assert ack.tolist()[0] == W + 150_010 + 1
    _, dels, ack = _batch(rx, ing, tbl, dgrams(np.concatenate([far[-7:], [W + 150_012, W + 150_010 + 3]])), "after")
    assert len(dels) == 1 and ack.tolist()[0] == W + 150_011


def test_far_pool_out_counted(rx):
    """The one capacity left: a GAP covering more SNs past the window than the far-set pool
    keeps free (here 2^34) cannot be recorded SN by SN; that proxy's far samples of the batch
    are then accepted without the duplicate check and counted in n_window_overflow, the
    other proxy's stay exact, and nothing walks the range."""
    import rtps_rx
    W = rtps_rx.INGEST_WINDOW
    w0, w1 = R.writer_key(0), R.writer_key(1)
    tbl = pack_match_table([(R.PREFIXES[0] + w0, 0), (R.PREFIXES[0] + w1, 1)])
    rx.set_match_table(tbl)
    subs = [R.gap_sub(w0, 2 * W, 2 * W + (1 << 34), [])] + [R.data_sub(w0, 3 * W + k % 5) for k in range(10)] + \
           [R.data_sub(w1, 3 * W + k % 5) for k in range(10)]
    arena, off, ln = oracle.pack([R.datagram(R.PREFIXES[0], subs)])
    _, acc, accepted, ack, ovf, _ = rx.ingest_batch(arena, off, ln, 2)
    w1_dels = int((accepted["rec_idx"] >= 11).sum())
    assert ovf == 10 and w1_dels == 5 and len(accepted) == 15


def test_empty_and_eventless_batches(rx):
    tbl, _ = R.table()
    rx.set_match_table(tbl)
    ing = oracle.HistoryIngest(tbl)
    _batch(rx, ing, tbl, [], "empty")
    _batch(rx, ing, tbl, [R.datagram(R.PREFIXES[3], [R.data_sub(R.writer_key(0), 1)])], "unmatched only")
    _batch(rx, ing, tbl, R.stream(500, 9), "after empty")


def test_reset_and_growing_table(rx):
    tbl, guids = R.table(n_prefix=2, n_writer=2)
    rx.set_match_table(tbl)
    ing = oracle.HistoryIngest(tbl)
    dgrams = R.stream(3000, 21)
    _batch(rx, ing, tbl, dgrams[:1000], "small table")
    # append entries: existing proxies keep their state by position on both sides
    big, _ = R.table(n_prefix=4, n_writer=3)
    order = [bytes(g) for g in tbl["writer_guid"]]
    extra = [e for e in big if bytes(e["writer_guid"]) not in order]
    tbl2 = np.concatenate([tbl, np.array(extra, dtype=tbl.dtype)])
    rx.set_match_table(tbl2)
    ing.set_readers(tbl2)
    _batch(rx, ing, tbl2, dgrams[1000:3000], "grown table")
    rx.ingest_reset()
    _batch(rx, oracle.HistoryIngest(tbl2), tbl2, dgrams[:1000], "after reset")


def _device_batch(rx, wl, n):
    import rtps_rx
    off, ln, size = rtps_rx.gen_layout(wl, n)
    dev = torch.device("cuda", 0)
    arena = torch.zeros(size, dtype=torch.uint8, device=dev)
    off_t = torch.from_numpy(off.view(np.int64)).to(dev)
    ln_t = torch.from_numpy(ln.view(np.int32)).to(dev)
    rx.generate(wl, arena, off_t, ln_t, n)
    rx.sync()
    return arena, off_t, ln_t, off, ln


@pytest.mark.parametrize("wl,n,multi", [(3, 20000, False), (3, 1 << 20, False), (1, 1 << 20, False),
                                         (3, 1 << 20, True)])
def test_workload_parity(rx, wl, n, multi):
    import rtps_rx
    arena, off_t, ln_t, off, ln = _device_batch(rx, wl, n)
    host = arena.cpu().numpy()
    st, recs0, _, _ = oracle.parse(host, off, ln, threads=16)
    wk = np.isin(recs0["kind"], (0x15, 0x07, 0x08))
    guids = sorted({bytes(r["prefix"]) + bytes(r["writer_id"]) for r in recs0[wk]})
    tbl = pack_match_table([(g, i) for i, g in enumerate(guids)])
    if multi:  # every writer to reader 100, even writers to reader 101 too, odd ones to 102 (a15)
        tbl = pack_match_table([(g, 100) for g in guids] + [(g, 101) for g in guids[::2]] +
                               [(g, 102) for g in guids[1::2]])
    rx.set_match_table(tbl)
    cap = rtps_rx.max_records(ln)
    outs = rx.alloc_outputs(n, cap)
    iouts = rx.alloc_ingest_outputs(cap, len(tbl))
    ing = oracle.HistoryIngest(tbl)
    _, recs, _, _ = oracle.parse(host, off, ln, match_table=tbl, threads=16)
    for rep in range(2):  # the second pass sees every sample again: all duplicates
        rx.parse_batch_device(arena, off_t, ln_t, n, outs)
        rx.ingest(arena, off_t, outs, iouts)
        rx.sync()
        m = int(outs["n_records"].item())
        assert m == len(recs)
        o_acc, o_accepted, o_ack = ing.batch(host, off, recs)
        acc = iouts["accept"][:m].cpu().numpy()
        na = int(iouts["n_accepted"].item())
        assert np.array_equal(acc, o_acc), f"wl {wl} rep {rep}: accept"
        got = iouts["accepted"][:na].cpu().numpy().reshape(-1).view(DELIVERY_DTYPE)
        assert got.tobytes() == o_accepted.tobytes()
        assert np.array_equal(iouts["ack_base"][:len(tbl)].cpu().numpy(), o_ack)
        assert int(iouts["n_window_overflow"].item()) == 0
        if rep == 1:
            assert na == 0
        elif wl == 1:
            assert na == n
        elif multi:
            assert int((acc > 1).sum()) > 10000


import reader_known  # noqa: E402


@pytest.mark.parametrize("case", reader_known.cases(), ids=[c["name"] for c in reader_known.cases()])
def test_reader_known_answers(rx, case):
    """The reference's Reader unit tests (io_uring/rtps/reader.rs:1537-1988) through
    rtps_rx_parse_batch + rtps_rx_ingest on every ingest path: all_ackable_before 3 -> 5 -> 6
    (GAP, DATA, GAP), HEARTBEAT counts, the stateless reader, the delivered change's fields."""
    state = {}

    def fn(rd, arena, off, ln):
        if not state:
            rx.set_readers(rd)
            rx.ingest_reset()
            state["set"] = True
        res, acc, dels, ack, ovf, _ = rx.ingest_batch(arena, off, ln, rd.n_proxies)
        assert ovf == 0
        return res.records, dels, ack, res.target
    reader_known.check(case, fn)
