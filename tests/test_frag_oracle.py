"""CPU checks of the DataFrag reassembly oracle:
against an independent Python model of the reference's FragmentAssembler on
an anomaly-rich corpus (single batch and split into batches), and on the C4
workload against the generator's own fragment layout (size-independent:
every 64 KiB sample is the concatenation of its 49 fragments)."""
import struct

import numpy as np
import pytest

import frag_ref
import oracle
from rtps_rx.records import DATA_FRAG, FRAG_OK, FRAG_SHORT, FRAG_NO_ROOM


def _parse(dgrams):
    arena, off, ln = oracle.pack(dgrams)
    st, recs, _, _ = oracle.parse(arena, off, ln)
    return arena, off, recs, st


def _check_against_model(samples, heap, model_out, label):
    assert len(samples) == len(model_out), f"{label}: {len(samples)} samples vs model {len(model_out)}"
    for s, (guid, sn, data, ri, flags) in zip(samples, model_out):
        assert bytes(s["writer_guid"]) == guid and int(s["sn"]) == sn, label
        assert int(s["rec_idx"]) == ri and int(s["flags"]) == flags, label
        assert int(s["data_size"]) == len(data), label
        assert int(s["status"]) == (FRAG_SHORT if len(data) < 4 else FRAG_OK), label
        o = int(s["heap_off"])
        assert heap[o:o + len(data)].tobytes() == data, f"{label}: bytes of sn {sn} differ"


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_oracle_matches_model_single_batch(seed):
    arena, off, recs, st = _parse(frag_ref.soup(1500, seed))
    assert (st == 0).all()
    f = oracle.FragAssembler()
    samples, heap, n, used = f.batch(arena, off, recs)
    model = frag_ref.FragRef()
    exp = model.batch(arena, off, recs)
    _check_against_model(samples, heap, exp, f"seed {seed}")
    assert f.pending() == model.pending()
    assert n > 50


def test_soup_covers_the_anomalies():
    short = key = irregular = 0
    for seed in (1, 2, 3):
        arena, off, recs, st = _parse(frag_ref.soup(1500, seed))
        exp = frag_ref.FragRef().batch(arena, off, recs)
        short += sum(len(e[2]) < 4 for e in exp)
        key += sum(bool(e[4] & 0x04) for e in exp)
        u = recs["u"].view(np.uint8).reshape(-1, 16)
        irregular += int((u[:, 8:10].copy().view("<u2")[:, 0] > 1).sum())  # several fragments per submessage
    assert short and key and irregular


@pytest.mark.parametrize("cuts", [[700], [1, 2, 3, 500, 1000], list(range(100, 1500, 100))])
def test_oracle_state_across_batches(cuts):
    dgrams = frag_ref.soup(1500, 9)
    f = oracle.FragAssembler()
    model = frag_ref.FragRef()
    bounds = [0] + cuts + [len(dgrams)]
    total = 0
    for a, b in zip(bounds[:-1], bounds[1:]):
        arena, off, recs, st = _parse(dgrams[a:b])
        samples, heap, n, used = f.batch(arena, off, recs)
        _check_against_model(samples, heap, model.batch(arena, off, recs), f"batch {a}:{b}")
        assert f.pending() == model.pending()
        total += n
    assert total > 50


@pytest.mark.parametrize("keep", [1, 2, 4])
def test_oracle_gc_across_batches(keep):
    """FragmentAssembler::garbage_collect_before (fragment_assembler.rs:216-224), called the
    way the reader does after each batch (reader.rs:1338-1340 with its expiry window): batch
    b runs at clock b; buffers last modified before b - keep + 1 are dropped, so their later
    fragments start fresh buffers that never complete."""
    dgrams = frag_ref.soup(2400, 11)
    f = oracle.FragAssembler()
    model = frag_ref.FragRef()
    step = 200
    dropped = 0
    t0 = 10**9  # ns clock (u64)
    for b, a in enumerate(range(0, len(dgrams), step)):
        f.set_clock(t0 + b)
        model.now = t0 + b
        arena, off, recs, st = _parse(dgrams[a:a + step])
        samples, heap, n, used = f.batch(arena, off, recs)
        _check_against_model(samples, heap, model.batch(arena, off, recs), f"batch {b}")
        before = model.pending()
        assert f.gc(t0 + b - keep + 1) == model.gc(t0 + b - keep + 1) == f.pending()
        dropped += before - model.pending()
    assert dropped > 0


def test_capacity_limits():
    arena, off, recs, st = _parse(frag_ref.soup(800, 4))
    full, fheap, n, used = oracle.FragAssembler().batch(arena, off, recs)
    # max_samples truncation: the count still reports every completed sample
    s2, _, n2, used2 = oracle.FragAssembler().batch(arena, off, recs, max_samples=10)
    assert n2 == n and len(s2) == 10 and used2 == used
    assert s2.tobytes() == full[:10].tobytes()
    # heap too small: descriptors kept, later samples NO_ROOM
    cap = int(full["heap_off"][n // 2])
    s3, h3, n3, used3 = oracle.FragAssembler().batch(arena, off, recs, heap_bytes=cap)
    assert n3 == n and used3 == used
    ok = full["heap_off"] + full["data_size"] <= cap
    assert (s3["status"][~ok] == FRAG_NO_ROOM).all() and (s3["status"][ok] == full["status"][ok]).all()


def test_c4_samples_are_their_fragments():
    n = 20000
    arena, off, ln = oracle.gen(oracle.WL_C4, n)
    st, recs, _, _ = oracle.parse(arena, off, ln)
    f = oracle.FragAssembler()
    samples, heap, ns, used = f.batch(arena, off, recs)
    assert ns >= n // 49 - 16 and (samples["status"] == FRAG_OK).all()
    assert (samples["data_size"] == 65536).all()
    u = recs["u"].view(np.uint8).reshape(-1, 16)
    pl_off = u[:, 0:2].copy().view("<u2")[:, 0]
    pl_len = u[:, 2:4].copy().view("<u2")[:, 0]
    fstart = u[:, 4:8].copy().view("<u4")[:, 0]
    guid = np.concatenate([recs["prefix"], recs["writer_id"]], axis=1)
    key = {}
    for i in range(len(recs)):
        key.setdefault((guid[i].tobytes(), int(recs["sn"][i])), []).append(i)
    for s in samples[::7]:
        idx = sorted(key[(s["writer_guid"].tobytes(), int(s["sn"]))], key=lambda i: fstart[i])
        assert [int(fstart[i]) for i in idx] == list(range(1, 50))
        data = b"".join(arena[int(off[recs["dgram_idx"][i]]) + int(pl_off[i]):
                              int(off[recs["dgram_idx"][i]]) + int(pl_off[i]) + int(pl_len[i])].tobytes()
                        for i in idx)
        o = int(s["heap_off"])
        assert heap[o:o + 65536].tobytes() == data
        assert int(s["rec_idx"]) == max(idx)  # the last fragment to arrive completes it


def _reader_batches():
    """Batch 1: readers A, B; batch 2: C added, W1 switches to 32-byte fragments."""
    import frag_ref as F
    return [(F.reader_scenario_readers(False), F.reader_scenario(400, 1, 1, 64)),
            (F.reader_scenario_readers(True), F.reader_scenario(600, 2, 200, 32))]


def test_oracle_per_reader_assembly_matches_model():
    """one assembler per (reader, writer) with the reader's own fragment
    size, the Lifespan drop (reader.rs:578-589) and a reader added mid-stream: the oracle
    (rtps_oracle_frag_batch_readers) against the independent Python model, batch after batch."""
    import frag_ref as F
    fa = oracle.FragAssembler()
    model = F.ReaderFragRef(F.reader_scenario_readers(False), F.RS_LIFESPAN, F.RS_RECV_NS)
    per_reader = {}
    for rd, dgrams in _reader_batches():
        model.set_readers(rd)
        arena, off, ln = oracle.pack(dgrams, align=4)
        _, recs, _, _ = oracle.parse(arena, off, ln, match_table=rd)
        samples, heap, n, used = fa.batch_readers(arena, off, recs, rd, F.RS_LIFESPAN, F.RS_RECV_NS)
        exp = model.batch(arena, off, recs)
        assert n == len(exp) > 0
        for s, (slot, g, sn, data, ri, fl) in zip(samples, exp):
            assert (int(s["reader_slot"]), bytes(s["writer_guid"]), int(s["sn"]), int(s["rec_idx"])) == (slot, g, sn, ri)
            assert heap[int(s["heap_off"]):int(s["heap_off"]) + int(s["data_size"])].tobytes() == data
            per_reader[slot] = per_reader.get(slot, 0) + 1
    # the scenario makes the readers differ: B loses samples to its Lifespan, C only has batch 2's
    assert per_reader[11] > per_reader[12] > 0 and per_reader.get(13, 0) > 0
