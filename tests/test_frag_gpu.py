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


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_soup_single_batch(rx, seed):
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


@pytest.mark.parametrize("n,batches", [(20000, 1), (20000, 7), (1 << 20, 1)])
def test_c4_workload(rx, n, batches):
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
