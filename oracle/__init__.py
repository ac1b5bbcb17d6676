"""ctypes binding of the CPU oracle (oracle/rtps_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, as the parity checker / CPU baseline.  The
product path (rustdds-io_uring_amd/) never imports this module.
"""
import ctypes
import os
import subprocess
import sys

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_REPO = os.path.dirname(_HERE)
sys.path.insert(0, os.path.join(_REPO, "rustdds-io_uring_amd"))
from rtps_rx.records import (RECORD_DTYPE, FRAG_SAMPLE_DTYPE, TARGET_DTYPE, DELIVERY_DTYPE,  # noqa: E402
                             max_records, as_readers)

LIB_PATH = os.path.join(_HERE, "librtps_oracle.so")
_lib = None

OWN_PREFIX = bytes([0x01, 0x03, 0x00, 0x0c, 0x29, 0x2d, 0x31, 0xa2, 0x28, 0x20, 0x02, 0x08])
SEED = 0x52545053
WL_T, WL_C2, WL_C3, WL_C4 = 1, 2, 3, 4


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        P = ctypes.c_void_p
        L.rtps_oracle_parse.restype = ctypes.c_uint64
        L.rtps_oracle_parse.argtypes = [P, P, P, ctypes.c_uint32, P, P, ctypes.c_uint32, P, ctypes.c_uint32,
                                        P, P, ctypes.c_uint64, P, ctypes.c_int]
        L.rtps_oracle_targets.restype = ctypes.c_uint64
        L.rtps_oracle_targets.argtypes = [P, ctypes.c_uint64, P, ctypes.c_uint32, P, ctypes.c_uint32, P, P,
                                          ctypes.c_uint64]
        L.rtps_oracle_gen_layout.restype = ctypes.c_uint64
        L.rtps_oracle_gen_layout.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32,
                                             ctypes.c_uint32, P, P]
        L.rtps_oracle_gen_fill.restype = None
        L.rtps_oracle_gen_fill.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32,
                                           ctypes.c_uint32, P, P]
        L.rtps_oracle_record_size.restype = ctypes.c_uint32
        L.rtps_oracle_frag_new.restype = P
        L.rtps_oracle_frag_free.argtypes = [P]
        L.rtps_oracle_frag_pending.restype = ctypes.c_uint64
        L.rtps_oracle_frag_pending.argtypes = [P]
        L.rtps_oracle_frag_set_clock.restype = None
        L.rtps_oracle_frag_set_clock.argtypes = [P, ctypes.c_uint64]
        L.rtps_oracle_frag_gc.restype = ctypes.c_uint64
        L.rtps_oracle_frag_gc.argtypes = [P, ctypes.c_uint64]
        L.rtps_oracle_frag_batch.restype = ctypes.c_uint64
        L.rtps_oracle_frag_batch.argtypes = [P, P, P, P, ctypes.c_uint64, P, ctypes.c_uint64, P, ctypes.c_uint64, P]
        L.rtps_oracle_frag_batch_readers.restype = ctypes.c_uint64
        L.rtps_oracle_frag_batch_readers.argtypes = [P, P, P, P, ctypes.c_uint64, P, P, P, ctypes.c_uint64, P,
                                                     ctypes.c_uint64, P, ctypes.c_uint64, P]
        L.rtps_oracle_ingest_new.restype = P
        L.rtps_oracle_ingest_new.argtypes = [P, ctypes.c_uint32, P, ctypes.c_uint32]
        L.rtps_oracle_ingest_free.argtypes = [P]
        L.rtps_oracle_ingest_set_readers.restype = None
        L.rtps_oracle_ingest_set_readers.argtypes = [P, P, ctypes.c_uint32, P, ctypes.c_uint32]
        L.rtps_oracle_ingest_batch.restype = ctypes.c_uint64
        L.rtps_oracle_ingest_batch.argtypes = [P, P, P, P, ctypes.c_uint64, P, ctypes.c_uint64, ctypes.c_uint32,
                                               P, P, ctypes.c_uint64, P]
        L.rtps_oracle_topics_new.restype = P
        L.rtps_oracle_topics_new.argtypes = [P, ctypes.c_uint32, P, ctypes.c_uint32]
        L.rtps_oracle_topics_free.argtypes = [P]
        L.rtps_oracle_topics_gc.restype = None
        L.rtps_oracle_topics_gc.argtypes = [P]
        L.rtps_oracle_topics_apply.restype = ctypes.c_uint64
        L.rtps_oracle_topics_apply.argtypes = [P, P, ctypes.c_uint64, P, ctypes.c_uint64]
        L.rtps_oracle_cdr_decode.restype = None
        L.rtps_oracle_cdr_decode.argtypes = [P, ctypes.c_uint32, ctypes.c_uint32, P, P, P, ctypes.c_uint64, P, P]
        assert L.rtps_oracle_record_size() == RECORD_DTYPE.itemsize
        _lib = L
    return _lib


def _ptr(a):
    return None if a is None else a.ctypes.data


def pack(datagrams, align=16):
    """list of bytes -> (arena u8, off u64, len u32) with `align`-byte aligned starts."""
    lens = np.array([len(d) for d in datagrams], dtype=np.uint32)
    offs = np.zeros(len(datagrams), dtype=np.uint64)
    pos = 0
    for i, d in enumerate(datagrams):
        offs[i] = pos
        pos += (len(d) + align - 1) // align * align if align > 1 else len(d)
    arena = np.zeros(max(pos, 1), dtype=np.uint8)
    for i, d in enumerate(datagrams):
        arena[int(offs[i]):int(offs[i]) + len(d)] = np.frombuffer(bytes(d), dtype=np.uint8)
    return arena, offs, lens


def _rt_args(table):
    rd = as_readers(table)
    r, p = rd.readers, rd.proxies
    return rd, (_ptr(r) if len(r) else None), len(r), (_ptr(p) if len(p) else None), len(p)


def parse(arena, offs, lens, own=OWN_PREFIX, match_table=None, threads=1, want_targets=True):
    """Returns (status u8[n], records RECORD_DTYPE[m], targets, rec_begin u32[n]).
    match_table: readers as rtps_rx.records.as_readers accepts (None: no readers);
    targets: (off u64[m+1], TARGET_DTYPE[k]) = the target readers of every record."""
    arena = np.ascontiguousarray(arena, dtype=np.uint8)
    offs = np.ascontiguousarray(offs, dtype=np.uint64)
    lens = np.ascontiguousarray(lens, dtype=np.uint32)
    n = len(lens)
    cap = max(max_records(lens), 1)
    status = np.zeros(n, dtype=np.uint8)
    recs = np.zeros(cap, dtype=RECORD_DTYPE)
    rec_begin = np.zeros(max(n, 1), dtype=np.uint32)
    own_a = np.frombuffer(bytes(own), dtype=np.uint8).copy()
    rd, rp, nr, pp, np_ = _rt_args(match_table)
    total = lib().rtps_oracle_parse(_ptr(arena), _ptr(offs), _ptr(lens), n, _ptr(own_a), rp, nr, pp, np_,
                                    _ptr(status), _ptr(recs), cap, _ptr(rec_begin), threads)
    recs = recs[:total]
    return status, recs, (targets(recs, rd) if want_targets else None), rec_begin[:n]


def targets(recs, table):
    """Target readers of every record (rtps_oracle_targets): (off u64[m+1], TARGET_DTYPE[k])."""
    recs = np.ascontiguousarray(recs, dtype=RECORD_DTYPE)
    m = len(recs)
    rd, rp, nr, pp, np_ = _rt_args(table)
    off = np.zeros(m + 1, dtype=np.uint64)
    cap = max(m * _widest(rd), 1)
    out = np.zeros(cap, dtype=TARGET_DTYPE)
    k = lib().rtps_oracle_targets(_ptr(recs) if m else None, m, rp, nr, pp, np_, _ptr(off), _ptr(out), cap)
    assert k <= cap
    return off, out[:int(k)]


def _widest(rd):
    """The most target readers a record can have: readers sharing one matched entity id."""
    from rtps_rx.records import READER_STATELESS
    by_eid = {}
    for p in rd.proxies:
        r = int(p["reader"])
        if not rd.readers[r]["flags"] & READER_STATELESS:
            by_eid.setdefault(bytes(p["writer_guid"][12:]), set()).add(r)
    return max((len(v) for v in by_eid.values()), default=0)


def gen(workload, n, seed=SEED, first_idx=0, n_writers=16):
    """Host build of the synthetic generator: (arena, off, len)."""
    offs = np.zeros(n, dtype=np.uint64)
    lens = np.zeros(n, dtype=np.uint32)
    size = lib().rtps_oracle_gen_layout(workload, seed, first_idx, n_writers, n, _ptr(offs), _ptr(lens))
    arena = np.zeros(max(int(size), 16), dtype=np.uint8)
    lib().rtps_oracle_gen_fill(workload, seed, first_idx, n_writers, n, _ptr(offs), _ptr(arena))
    return arena, offs, lens


def cdr_decode(sample_type, arena, offs, recs):
    """CDR-decode every record's DATA payload (rtps_oracle_cdr_decode) -> (rows u8[m, row_bytes], status u8[m])."""
    arena = np.ascontiguousarray(arena, dtype=np.uint8)
    offs = np.ascontiguousarray(offs, dtype=np.uint64)
    recs = np.ascontiguousarray(recs, dtype=RECORD_DTYPE)
    m = len(recs)
    rows = np.zeros((max(m, 1), sample_type.row_bytes), dtype=np.uint8)
    status = np.zeros(max(m, 1), dtype=np.uint8)
    ops = np.ascontiguousarray(sample_type.ops)
    lib().rtps_oracle_cdr_decode(_ptr(ops), len(ops), sample_type.row_bytes, _ptr(arena), _ptr(offs),
                                 _ptr(recs) if m else None, m, _ptr(rows), _ptr(status))
    return rows[:m], status[:m]


class FragAssembler:
    """Sequential DataFrag reassembly with state across batches (rtps_oracle_frag_*)."""

    def __init__(self):
        self.h = ctypes.c_void_p(lib().rtps_oracle_frag_new())

    def __del__(self):
        if getattr(self, "h", None):
            lib().rtps_oracle_frag_free(self.h)
            self.h = None

    def pending(self):
        return int(lib().rtps_oracle_frag_pending(self.h))

    def set_clock(self, now_ns):
        """The time the next batches stamp on the buffers they create or extend."""
        lib().rtps_oracle_frag_set_clock(self.h, now_ns)

    def gc(self, expire_before_ns):
        """garbage_collect_before: drop buffers last modified before expire_before; -> pending left."""
        return int(lib().rtps_oracle_frag_gc(self.h, expire_before_ns))

    def batch(self, arena, offs, recs, max_samples=None, heap_bytes=None):
        """-> (samples FRAG_SAMPLE_DTYPE[n], heap u8[heap_used], n_completed, heap_used)."""
        arena = np.ascontiguousarray(arena, dtype=np.uint8)
        offs = np.ascontiguousarray(offs, dtype=np.uint64)
        recs = np.ascontiguousarray(recs, dtype=RECORD_DTYPE)
        ms = len(recs) if max_samples is None else max_samples
        hb = (int(arena.nbytes) + 16 * len(recs) + (1 << 22)) if heap_bytes is None else heap_bytes
        samples = np.zeros(max(ms, 1), dtype=FRAG_SAMPLE_DTYPE)
        heap = np.zeros(max(hb, 1), dtype=np.uint8)
        used = ctypes.c_uint64()
        n = lib().rtps_oracle_frag_batch(self.h, _ptr(arena), _ptr(offs), _ptr(recs) if len(recs) else None,
                                         len(recs), _ptr(samples), ms, _ptr(heap), hb, ctypes.byref(used))
        return samples[:min(n, ms)], heap[:min(used.value, hb)], int(n), int(used.value)

    def batch_readers(self, arena, offs, recs, readers, lifespan_ns=None, recv_ns=0, max_samples=None,
                      heap_bytes=None):
        """With readers: one assembler per (reader, writer), each target reader fed in turn,
        Lifespans {reader_slot: ns} checked against the receive time recv_ns
        (rtps_oracle_frag_batch_readers) -> as batch()."""
        arena = np.ascontiguousarray(arena, dtype=np.uint8)
        offs = np.ascontiguousarray(offs, dtype=np.uint64)
        recs = np.ascontiguousarray(recs, dtype=RECORD_DTYPE)
        toff, tent = targets(recs, readers)
        tent = np.ascontiguousarray(tent) if len(tent) else np.zeros(1, dtype=TARGET_DTYPE)
        life = None
        if lifespan_ns:
            life = np.full(65536, np.iinfo(np.int64).max, dtype=np.int64)
            for slot, ns in lifespan_ns.items():
                life[slot] = duration_ticks(ns)
        ms = max(len(recs) * max(_widest(as_readers(readers)), 1), 1) if max_samples is None else max_samples
        hb = (int(arena.nbytes) * 4 + 16 * ms + (1 << 22)) if heap_bytes is None else heap_bytes
        samples = np.zeros(max(ms, 1), dtype=FRAG_SAMPLE_DTYPE)
        heap = np.zeros(max(hb, 1), dtype=np.uint8)
        used = ctypes.c_uint64()
        n = lib().rtps_oracle_frag_batch_readers(self.h, _ptr(arena), _ptr(offs), _ptr(recs) if len(recs) else None,
                                                 len(recs), _ptr(toff), _ptr(tent), _ptr(life),
                                                 timestamp_ticks(recv_ns), _ptr(samples), ms, _ptr(heap), hb,
                                                 ctypes.byref(used))
        return samples[:min(n, ms)], heap[:min(used.value, hb)], int(n), int(used.value)


def timestamp_ticks(unix_ns):
    """Timestamp::from_nanos (structure/time.rs:78-83) as ticks (seconds << 32 | fraction)."""
    return ((unix_ns // 10**9) << 32) + (((unix_ns % 10**9) << 32) // 10**9)


def duration_ticks(ns):
    """Duration::from_nanos (structure/duration.rs:60-67) as ticks (i64)."""
    sec, frac = int(ns) // 10**9, ((int(ns) % 10**9) << 32) // 10**9
    return (sec << 32) + frac


class HistoryIngest:
    """Sequential writer-proxy restatement with state across batches (rtps_oracle_ingest_*),
    one proxy per (reader, writer GUID) of the readers table."""

    def __init__(self, match_table):
        self.readers = as_readers(match_table)
        self.n = self.readers.n_proxies
        rd, rp, nr, pp, np_ = _rt_args(self.readers)
        self.h = ctypes.c_void_p(lib().rtps_oracle_ingest_new(rp, nr, pp, np_))

    def set_readers(self, match_table):
        """New readers / proxies; proxy state is kept by position (as on the device)."""
        self.readers = as_readers(match_table)
        self.n = self.readers.n_proxies
        rd, rp, nr, pp, np_ = _rt_args(self.readers)
        lib().rtps_oracle_ingest_set_readers(self.h, rp, nr, pp, np_)

    def __del__(self):
        if getattr(self, "h", None):
            lib().rtps_oracle_ingest_free(self.h)
            self.h = None

    def batch(self, arena, offs, recs, frag_samples=None, best_effort=False):
        """-> (accept u8[m], deliveries DELIVERY_DTYPE[k], ack_base i64[n_proxies])."""
        arena = np.ascontiguousarray(arena, dtype=np.uint8)
        offs = np.ascontiguousarray(offs, dtype=np.uint64)
        recs = np.ascontiguousarray(recs, dtype=RECORD_DTYPE)
        m = len(recs)
        fs = None if frag_samples is None else np.ascontiguousarray(frag_samples, dtype=FRAG_SAMPLE_DTYPE)
        accept = np.zeros(max(m, 1), dtype=np.uint8)
        cap = max(m * _widest(self.readers), 1)
        dels = np.zeros(cap, dtype=DELIVERY_DTYPE)
        ack = np.zeros(max(self.n, 1), dtype=np.int64)
        k = lib().rtps_oracle_ingest_batch(self.h, _ptr(arena), _ptr(offs), _ptr(recs) if m else None, m,
                                           _ptr(fs) if fs is not None and len(fs) else None,
                                           0 if fs is None else len(fs), 1 if best_effort else 0,
                                           _ptr(accept), _ptr(dels), cap, _ptr(ack))
        return accept[:m], dels[:int(k)], ack[:self.n]


def topic_args(topics, topic_readers):
    """(topics [(topic id, max_keep_samples)], readers [(reader slot, topic id)]) -> the two arrays."""
    from rtps_rx.records import TOPIC_DTYPE, TOPIC_READER_DTYPE
    t = np.zeros(len(topics), dtype=TOPIC_DTYPE)
    for i, (tid, k) in enumerate(topics):
        t[i] = (tid, k)
    r = np.zeros(len(topic_readers), dtype=TOPIC_READER_DTYPE)
    for i, (slot, tid) in enumerate(topic_readers):
        r[i]["reader_slot"], r[i]["topic"] = slot, tid
    return t, r


class TopicCaches:
    """Sequential TopicCache::add_change restatement (rtps_oracle_topics_*): one cache per topic,
    state across batches; apply() over a batch's deliveries (in order) sets DELIVERY_CACHED."""

    def __init__(self, topics=(), topic_readers=()):
        self.t, self.r = topic_args(topics, topic_readers)
        self.h = ctypes.c_void_p(lib().rtps_oracle_topics_new(_ptr(self.t) if len(self.t) else None, len(self.t),
                                                              _ptr(self.r) if len(self.r) else None, len(self.r)))

    def __del__(self):
        if getattr(self, "h", None):
            lib().rtps_oracle_topics_free(self.h)
            self.h = None

    def gc(self):
        lib().rtps_oracle_topics_gc(self.h)

    def apply(self, recs, deliveries):
        """-> a copy of deliveries with flags set (DELIVERY_CACHED where the change was stored)."""
        recs = np.ascontiguousarray(recs, dtype=RECORD_DTYPE)
        d = np.ascontiguousarray(deliveries, dtype=DELIVERY_DTYPE).copy()
        if len(d):
            lib().rtps_oracle_topics_apply(self.h, _ptr(recs) if len(recs) else None, len(recs), _ptr(d), len(d))
        return d
