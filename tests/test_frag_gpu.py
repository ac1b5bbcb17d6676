"""GPU parity of the DataFrag reassembly (rtps_rx_frag_assemble) with the
CPU oracle: every sample descriptor, every heap byte, the sample count, heap
size and pending count, batch after batch (state carried in the context)."""
import numpy as np
import pytest

import frag_ref
import oracle

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


@pytest.fixture()
def rx():
    import rtps_rx
    r = rtps_rx.MessageReceiver(oracle.OWN_PREFIX, max_datagrams=1 << 21)
    yield r
    r.close()


def _compare(gpu, ora, label):
    res, samples, heap, ns, used, npend = gpu
    o_samples, o_heap, o_n, o_used = ora[:4]
    assert ns == o_n, f"{label}: {ns} samples vs oracle {o_n}"
    assert used == o_used, f"{label}: heap {used} vs {o_used}"
    assert samples.tobytes() == o_samples.tobytes(), f"{label}: sample descriptors differ"
    ok = samples["status"] != 2
    for s in samples[ok]:
        o, d = int(s["heap_off"]), int(s["data_size"])
        assert heap[o:o + d].tobytes() == o_heap[o:o + d].tobytes(), f"{label}: bytes of sample sn {s['sn']}"


def _run(rx, fa, dgrams_or_gen, label, **kw):
    if callable(dgrams_or_gen):
        arena, off, ln = dgrams_or_gen()
    else:
        arena, off, ln = oracle.pack(dgrams_or_gen, align=kw.pop("align", 16))
    gpu = rx.assemble_batch(arena, off, ln, **kw)
    st, recs, _, _ = oracle.parse(arena, off, ln, threads=8)
    ora = fa.batch(arena, off, recs, max_samples=kw.get("max_samples"), heap_bytes=kw.get("heap_bytes"))
    _compare(gpu, ora, label)
    assert gpu[5] == fa.pending(), f"{label}: pending {gpu[5]} vs {fa.pending()}"
    return gpu


@pytest.mark.parametrize("seed,sort", [(1, 0), (2, 0), (3, 0), (1, 1)])
def test_soup_single_batch(rx, seed, sort):
    rx.debug_frag_sort(sort)
    fa = oracle.FragAssembler()
    g = _run(rx, fa, frag_ref.soup(3000, seed), f"soup{seed}", align=1)
    assert g[3] > 100


def test_soup_across_batches(rx):
    dgrams = frag_ref.soup(4000, 11)
    fa = oracle.FragAssembler()
    bounds = [0, 1, 2, 700, 701, 1500, 2600, 4000]
    total = 0
    for a, b in zip(bounds[:-1], bounds[1:]):
        g = _run(rx, fa, dgrams[a:b], f"batch {a}:{b}")
        total += g[3]
    assert total > 100
    rx.frag_reset()
    fa2 = oracle.FragAssembler()
    _run(rx, fa2, dgrams[:1000], "after reset")


def test_capacity_limits(rx):
    dgrams = frag_ref.soup(2000, 5)
    fa = oracle.FragAssembler()
    _run(rx, fa, dgrams, "max_samples", max_samples=7)
    rx.frag_reset()
    fa = oracle.FragAssembler()
    _run(rx, fa, dgrams, "small heap", heap_bytes=4000)


def test_empty_and_no_frag_batches(rx):
    fa = oracle.FragAssembler()
    _run(rx, fa, frag_ref.soup(200, 3)[:0] or [b"RTPS\x02\x04\x01\x0f" + bytes(12)], "no records")
    _run(rx, fa, lambda: oracle.gen(oracle.WL_C3, 5000), "C3 (no DATA_FRAG)")


@pytest.mark.parametrize("n,batches,sort", [(20000, 1, 0), (20000, 7, 0), (1 << 20, 1, 0), (1 << 20, 1, 1)])
def test_c4_workload(rx, n, batches, sort):
    rx.debug_frag_sort(sort)  # 1: rocprim's device sort instead of the bucket sort
    arena, off, ln = oracle.gen(oracle.WL_C4, n)
    fa = oracle.FragAssembler()
    step = (n + batches - 1) // batches
    total = 0
    for k in range(batches):
        a, b = k * step, min(n, (k + 1) * step)
        sub_off = off[a:b] - off[a]
        end = int(off[b - 1] + ln[b - 1])
        sub = arena[int(off[a]):end]
        g = _run(rx, fa, lambda: (sub, sub_off, ln[a:b]), f"C4 {a}:{b}")
        total += g[3]
    assert total >= n // 49 - 16


def test_gc_across_batches(rx):
    """rtps_rx_frag_gc = garbage_collect_before (fragment_assembler.rs:216-224): batch b
    runs at clock t0 + b; after it the buffers last modified before t0 + b - 1 are
    dropped on the device and in the oracle; later fragments of a dropped (writer, SN)
    start new buffers, which the next batches' outputs then show."""
    dgrams = frag_ref.soup(4000, 11)
    fa = oracle.FragAssembler()
    t0 = 1_700_000_000 * 10**9
    dropped = 0
    for b, a in enumerate(range(0, len(dgrams), 250)):
        rx.frag_set_clock(t0 + b)
        fa.set_clock(t0 + b)
        g = _run(rx, fa, dgrams[a:a + 250], f"batch {b}")
        left = rx.frag_gc(t0 + b - 1)
        assert left == fa.gc(t0 + b - 1) == fa.pending(), f"batch {b}: {left} left vs {fa.pending()}"
        dropped += g[5] - left
    assert dropped > 0
    assert rx.frag_gc(t0 + 10**6) == 0 and fa.gc(t0 + 10**6) == 0  # everything expires


def test_c4_lossy_pending_bounded(rx):
    """A lossy C4 stream (1 % of datagrams lost: about 40 % of the 49-fragment samples never
    complete): without gc the pending buffers only grow; with gc after every batch
    (expiring what no fragment touched for two batches) n_pending stays bounded, and the
    samples and pending counts match the oracle batch after batch."""
    n, batches = 20000, 8
    rng = np.random.default_rng(5)
    fa = oracle.FragAssembler()
    t0 = 10**12
    pend, pend_nogc = [], []
    fa_nogc = oracle.FragAssembler()
    for b in range(batches):
        arena, off, ln = oracle.gen(oracle.WL_C4, n, first_idx=b * n)
        keep = rng.random(n) > 0.01
        sub = (arena, np.ascontiguousarray(off[keep]), np.ascontiguousarray(ln[keep]))
        rx.frag_set_clock(t0 + b)
        fa.set_clock(t0 + b)
        _run(rx, fa, lambda: sub, f"lossy C4 batch {b}")
        left = rx.frag_gc(t0 + b - 1)
        assert left == fa.gc(t0 + b - 1)
        pend.append(left)
        st, recs, _, _ = oracle.parse(*sub, threads=8)
        fa_nogc.batch(sub[0], sub[1], recs)
        pend_nogc.append(fa_nogc.pending())
    assert pend_nogc[-1] > 3 * max(pend[1:]), (pend, pend_nogc)
    assert max(pend[2:]) <= 3 * n // 49 // 2, pend  # about two batches of lost samples at most


def _key_hash(prefix, writer_key, sn):
    """The device's 32-bit sort key of (writer GUID, SN) (rtps_frag.hip key_hash), vectorised over sn."""
    g = np.frombuffer(bytes(prefix) + bytes(writer_key), dtype="<u4").astype(np.uint64)
    sn = np.asarray(sn, dtype=np.int64).view(np.uint64)
    m = np.uint64(0xFFFFFFFF)
    h = np.full(sn.shape, 0x811C9DC5, dtype=np.uint64)
    for x in (g[0], g[1], g[2], g[3], sn & m, (sn >> np.uint64(32)) & m):
        h = ((h ^ x) * np.uint64(0x01000193)) & m
    for sh, mul in ((16, 0x85EBCA6B), (13, 0xC2B2AE35)):
        h ^= h >> np.uint64(sh)
        h = (h * np.uint64(mul)) & m
    h ^= h >> np.uint64(16)
    return np.where(h == m, m - np.uint64(1), h)


@pytest.mark.parametrize("sort", [0, 1])
def test_bucket_sort_oversized_buckets(rx, sort):
    """The bucket sort's two large-bucket paths (rtps_bsort.h): 12000 fragments of one
    sample (one key: the bucket is already in key order) and 9000 one-fragment samples
    whose keys share their top byte, in shuffled SN order (an LSD pass per key byte),
    each beside a soup of other traffic; the same with rocprim's sort (sort=1)."""
    rx.debug_frag_sort(sort)
    rng = np.random.default_rng(7)
    prefix, wk = bytes(range(100, 112)), b"\x00\x01\x05\x02"
    fsz, nf = 16, 12000
    order = rng.permutation(nf) + 1
    payload = rng.integers(0, 256, nf * fsz, dtype=np.uint8).tobytes()
    big = [frag_ref.datagram(prefix, [frag_ref.datafrag_sub(wk, 77, int(f), 1, fsz, nf * fsz,
                                                            payload[(f - 1) * fsz:f * fsz])]) for f in order]
    fa = oracle.FragAssembler()
    g = _run(rx, fa, big, "one 12000-fragment sample")
    assert g[3] == 1
    sns = np.arange(1, 3_000_000, dtype=np.int64)
    hit = sns[(_key_hash(prefix, wk, sns) >> np.uint64(24)) == np.uint64(0x5A)][:9000]
    assert len(hit) == 9000
    rng.shuffle(hit)
    many = [frag_ref.datagram(prefix, [frag_ref.datafrag_sub(wk, int(sn), 1, 1, 8, 8, bytes([int(sn) & 255] * 8))])
            for sn in hit]
    mixed = many[:4500] + frag_ref.soup(600, 4) + many[4500:]
    rx.frag_reset()  # the writer's fragment size is fixed per context: start over with the oracle
    fa = oracle.FragAssembler()
    g = _run(rx, fa, mixed, "9000 keys in one bucket")
    assert g[3] >= 9000


@pytest.mark.parametrize("ingest_path,sets", [(1, "multi"), (2, "multi"), (1, "single"), (2, "single")])
def test_per_reader_assembly_and_ingest(rx, ingest_path, sets):
    """two readers of one writer, one with a Lifespan (reader.rs:578-589),
    a reader added mid-stream, a writer changing its fragment size: every (reader, writer)
    pair has its own assembler (reader.rs:617-619, 638-647).  Samples (with their reader),
    heap bytes, deliveries and every proxy's ack_base bit-exact against the oracle, on both
    ingest paths.  sets "single": the first batch's target sets hold one reader each (the
    in-place selection), the second one's two (the per-target expansion), with fragments
    pending across the switch."""
    from rtps_rx.records import FRAG_SAMPLE_DTYPE, DELIVERY_DTYPE, max_records
    dev = torch.device("cuda", 0)
    rx.debug_ingest_path(ingest_path)
    rx.set_reader_lifespan(12, frag_ref.RS_LIFESPAN[12])
    rx.frag_set_receive_time(frag_ref.RS_RECV_NS)
    fa = oracle.FragAssembler()
    ing = None
    per_reader = {}
    first = frag_ref.reader_scenario_readers(False) if sets == "multi" else frag_ref.reader_scenario_single_readers()
    batches = [(first, frag_ref.reader_scenario(400, 1, 1, 64)),
               (frag_ref.reader_scenario_readers(True), frag_ref.reader_scenario(600, 2, 200, 32))]
    for k, (rd, dgrams) in enumerate(batches):
        rx.set_readers(rd)
        if ing is None:
            ing = oracle.HistoryIngest(rd)
        else:
            ing.set_readers(rd)
        arena, off, ln = oracle.pack(dgrams, align=4)
        A = torch.from_numpy(arena).to(dev)
        O = torch.from_numpy(off.view(np.int64)).to(dev)
        L = torch.from_numpy(ln.view(np.int32)).to(dev)
        cap = max_records(ln)
        heap_bytes = 4 * len(arena) + (1 << 20)
        outs = rx.alloc_outputs(len(ln), cap)
        fouts = rx.alloc_frag_outputs(3 * cap, heap_bytes)
        iouts = rx.alloc_ingest_outputs(cap, rd.n_proxies)
        rx.parse_batch_device(A, O, L, len(ln), outs)
        rx.frag_assemble(A, O, outs, fouts)
        rx.ingest(A, O, outs, iouts, fouts)
        rx.sync()
        _, recs, _, _ = oracle.parse(arena, off, ln, match_table=rd)
        o_s, o_heap, o_n, o_used = fa.batch_readers(arena, off, recs, rd, frag_ref.RS_LIFESPAN, frag_ref.RS_RECV_NS,
                                                    max_samples=3 * cap, heap_bytes=heap_bytes)
        ns = int(fouts["n_samples"].item())
        assert ns == o_n > 0, (k, ns, o_n)
        assert int(fouts["heap_used"].item()) == o_used
        s = fouts["samples"][:ns].cpu().numpy().reshape(-1).view(FRAG_SAMPLE_DTYPE)
        assert s.tobytes() == o_s.tobytes(), f"batch {k}: sample descriptors differ"
        heap = fouts["heap"].cpu().numpy()
        for x in s:
            o, d = int(x["heap_off"]), int(x["data_size"])
            assert heap[o:o + d].tobytes() == o_heap[o:o + d].tobytes()
            per_reader[int(x["reader_slot"])] = per_reader.get(int(x["reader_slot"]), 0) + 1
        o_acc, o_dels, o_ack = ing.batch(arena, off, recs, o_s)
        na = int(iouts["n_accepted"].item())
        dels = iouts["accepted"][:na].cpu().numpy().reshape(-1).view(DELIVERY_DTYPE)
        assert dels.tobytes() == o_dels.tobytes(), f"batch {k}: deliveries differ"
        assert np.array_equal(iouts["accept"][:len(recs)].cpu().numpy(), o_acc)
        assert np.array_equal(iouts["ack_base"][:rd.n_proxies].cpu().numpy(), o_ack)
    assert per_reader[11] > 0 and per_reader[12] > 0 and per_reader.get(13, 0) > 0
    if sets == "multi":
        assert per_reader[11] > per_reader[12]


def test_target_set_past_64_readers(rx):
    """a target set of 70 readers on one writer, each with its own assembler (one
    with a Lifespan, so that the completions differ between readers): entries 64 and up take a
    completed sample exactly when their own assembler completed it (found among the record's
    samples), as the oracle's per-reader restatement does; deliveries and ack_base bit-exact."""
    from rtps_rx.records import FRAG_SAMPLE_DTYPE, DELIVERY_DTYPE, Readers, max_records
    dev = torch.device("cuda", 0)
    n_r = 70
    slots = [100 + k for k in range(n_r)]
    readers = [(bytes([0, 0, 1 + k, 0x07]), slots[k], 0) for k in range(n_r)]
    g1 = frag_ref.RS_PREFIX[0] + frag_ref.RS_WRITER[0]
    g2 = frag_ref.RS_PREFIX[1] + frag_ref.RS_WRITER[1]
    rd = Readers(readers, [(g1, k) for k in range(n_r)] + [(g2, k) for k in range(0, n_r, 3)])
    life = {slots[66]: 2 * 10**9, slots[3]: 2 * 10**9}
    rx.set_readers(rd)
    for sl, ns in life.items():
        rx.set_reader_lifespan(sl, ns)
    rx.frag_set_receive_time(frag_ref.RS_RECV_NS)
    fa = oracle.FragAssembler()
    ing = oracle.HistoryIngest(rd)
    dgrams = frag_ref.reader_scenario(300, 5, 1, 64)
    arena, off, ln = oracle.pack(dgrams, align=4)
    A = torch.from_numpy(arena).to(dev)
    O = torch.from_numpy(off.view(np.int64)).to(dev)
    L = torch.from_numpy(ln.view(np.int32)).to(dev)
    cap = max_records(ln)
    heap_bytes = 80 * len(arena) + (1 << 20)
    outs = rx.alloc_outputs(len(ln), cap)
    fouts = rx.alloc_frag_outputs(80 * cap, heap_bytes)
    iouts = rx.alloc_ingest_outputs(cap, rd.n_proxies)
    rx.parse_batch_device(A, O, L, len(ln), outs)
    rx.frag_assemble(A, O, outs, fouts)
    rx.ingest(A, O, outs, iouts, fouts)
    rx.sync()
    _, recs, _, _ = oracle.parse(arena, off, ln, match_table=rd)
    o_s, o_heap, o_n, o_used = fa.batch_readers(arena, off, recs, rd, life, frag_ref.RS_RECV_NS,
                                                max_samples=80 * cap, heap_bytes=heap_bytes)
    ns = int(fouts["n_samples"].item())
    assert ns == o_n > 0
    s = fouts["samples"][:ns].cpu().numpy().reshape(-1).view(FRAG_SAMPLE_DTYPE)
    assert s.tobytes() == o_s.tobytes()
    o_acc, o_dels, o_ack = ing.batch(arena, off, recs, o_s)
    na = int(iouts["n_accepted"].item())
    dels = iouts["accepted"][:na].cpu().numpy().reshape(-1).view(DELIVERY_DTYPE)
    assert dels.tobytes() == o_dels.tobytes()
    assert np.array_equal(iouts["ack_base"][:rd.n_proxies].cpu().numpy(), o_ack)
    late = np.isin(dels["reader_slot"], slots[64:])
    assert late.sum() > 0 and (dels["reader_slot"] == slots[66]).sum() < (dels["reader_slot"] == slots[65]).sum()
