"""Python host side of the MI355X RTPS receive-path parser.

Binds the C ABI of include/rtps_rx.h (librtps_rx.so, built from csrc/) with
ctypes; torch provides device memory and streams (plumbing only).  The
object model mirrors the reference's receive path:

  MessageReceiver(own_guid_prefix)         io_uring/rtps/message_receiver.rs:158-182
  .handle_received_batch(...)              batch form of handle_received_packet_2 (:232-287)
  BatchResult.passed_submessages(i)        SubmessageIter2::next -> PassedSubmessage (:56-119)

There is no CPU fallback: if the shared library (or a GPU) is missing the
constructor raises.
"""
import ctypes
import os

import numpy as np

from .records import (RECORD_DTYPE, MATCH_DTYPE, FRAG_SAMPLE_DTYPE, STATUS_NAMES, KIND_NAMES, WRITER_KINDS, READER_KINDS,
                      ROUTE_PASS, NO_MATCH, NO_TARGET, NO_PROXY, TARGET_DTYPE, DELIVERY_DTYPE, Readers, as_readers,
                      max_records, record_to_dict, pack_match_table)

_PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("RTPS_RX_LIB") or os.path.join(os.path.dirname(_PKG_DIR), "librtps_rx.so")
ABI_VERSION = 2

WL_T, WL_C2, WL_C3, WL_C4 = 1, 2, 3, 4
MIXED_CHAIN, MIXED_LDS, MIXED_ITEM, MIXED_RSLAB = 0, 1, 2, 3  # passes for mixed traffic (debug_set_mixed_pass)
WORKLOADS = {"T": WL_T, "C2": WL_C2, "C3": WL_C3, "C4": WL_C4}
SEED = 0x52545053

_lib = None


class RtpsRxError(RuntimeError):
    def __init__(self, msg, code=None):
        super().__init__(msg)
        self.code = code


RTPS_RX_EABORTED = -6  # the library aborted (and freed) an RCCL communicator


class _Config(ctypes.Structure):
    _fields_ = [("abi_version", ctypes.c_uint32), ("device", ctypes.c_int32),
                ("own_prefix", ctypes.c_uint8 * 12), ("max_datagrams", ctypes.c_uint32),
                ("flags", ctypes.c_uint32)]


class _FragOut(ctypes.Structure):
    _fields_ = [("samples", ctypes.c_void_p), ("max_samples", ctypes.c_uint64), ("heap", ctypes.c_void_p),
                ("heap_bytes", ctypes.c_uint64), ("n_samples", ctypes.c_void_p), ("heap_used", ctypes.c_void_p),
                ("n_pending", ctypes.c_void_p)]


class _IngestOut(ctypes.Structure):
    _fields_ = [("accept", ctypes.c_void_p), ("accepted", ctypes.c_void_p), ("max_accepted", ctypes.c_uint64),
                ("n_accepted", ctypes.c_void_p), ("ack_base", ctypes.c_void_p), ("n_window_overflow", ctypes.c_void_p)]


INGEST_BEST_EFFORT = 0x1
INGEST_TOPIC_CACHE = 0x2  # also run the topic caches' add_change (DELIVERY_CACHED on the deliveries)
INGEST_WINDOW = 1 << 17


class _Out(ctypes.Structure):
    _fields_ = [("status", ctypes.c_void_p), ("records", ctypes.c_void_p), ("max_records", ctypes.c_uint64),
                ("target", ctypes.c_void_p), ("rec_begin", ctypes.c_void_p), ("n_records", ctypes.c_void_p)]


EXPORTS = ["rtps_rx_create", "rtps_rx_destroy", "rtps_rx_set_stream", "rtps_rx_set_match_table",
           "rtps_rx_set_readers", "rtps_rx_target_table",
           "rtps_rx_parse_batch", "rtps_rx_sync", "rtps_rx_strerror", "rtps_rx_max_records_host",
           "rtps_rx_generate", "rtps_rx_bucket_by_writer", "rtps_rx_set_spec_hint", "rtps_rx_cdr_decode",
           "rtps_rx_bucket_by_writer_padded", "rtps_rx_frag_assemble", "rtps_rx_frag_reset",
           "rtps_rx_frag_set_clock", "rtps_rx_frag_gc",
           "rtps_rx_bucket_descriptors", "rtps_rx_ingest", "rtps_rx_ingest_reset", "rtps_udp_open", "rtps_udp_close",
           "rtps_udp_port", "rtps_udp_backend", "rtps_udp_recv_batch", "rtps_udp_release", "rtps_udp_send_batch",
           "rtps_rx_pump", "rtps_rx_set_topics", "rtps_rx_topic_gc", "rtps_rx_cdr_decode_list",
           "rtps_rx_topic_reset"]


def lib():
    """Load librtps_rx.so (raises if it was not built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RtpsRxError(f"{LIB_PATH} missing: run __graft_entry__.build() (make -C csrc)")
        L = ctypes.CDLL(LIB_PATH)
        P, U32, U64, I = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int
        L.rtps_rx_create.argtypes = [ctypes.POINTER(_Config), ctypes.POINTER(P)]
        L.rtps_rx_destroy.argtypes = [P]
        L.rtps_rx_set_stream.argtypes = [P, P]
        L.rtps_rx_set_match_table.argtypes = [P, P, U32]
        L.rtps_rx_set_readers.argtypes = [P, P, U32, P, U32]
        L.rtps_rx_set_readers.restype = I
        L.rtps_rx_target_table.argtypes = [P, ctypes.POINTER(P), ctypes.POINTER(P), ctypes.POINTER(U32)]
        L.rtps_rx_target_table.restype = I
        L.rtps_rx_parse_batch.argtypes = [P, P, U64, P, P, U32, ctypes.POINTER(_Out)]
        L.rtps_rx_sync.argtypes = [P]
        L.rtps_rx_strerror.argtypes = [I]
        L.rtps_rx_strerror.restype = ctypes.c_char_p
        L.rtps_rx_max_records_host.argtypes = [P, U32]
        L.rtps_rx_max_records_host.restype = U64
        L.rtps_rx_generate.argtypes = [P, I, U64, U64, U32, P, P, P, U32]
        L.rtps_rx_gen_layout_host.argtypes = [I, U64, U64, U32, U32, P, P]
        L.rtps_rx_gen_layout_host.restype = U64
        L.rtps_rx_record_size.restype = U32
        L.rtps_rx_bucket_by_writer.argtypes = [P, P, P, U64, U32, P, P]
        L.rtps_rx_bucket_by_writer.restype = I
        L.rtps_rx_bucket_by_writer_padded.argtypes = [P, P, P, U64, U32, U64, P, P]
        L.rtps_rx_bucket_by_writer_padded.restype = I
        L.rtps_rx_bucket_descriptors.argtypes = [P, P, P, U64, U32, U64, P, P]
        L.rtps_rx_bucket_descriptors.restype = I
        L.rtps_rx_frag_assemble.argtypes = [P, P, U64, P, P, P, U64, ctypes.POINTER(_FragOut)]
        L.rtps_rx_frag_assemble.restype = I
        L.rtps_rx_frag_reset.argtypes = [P]
        L.rtps_rx_frag_reset.restype = I
        L.rtps_rx_ingest.argtypes = [P, P, U64, P, P, P, U64, P, P, U64, U32, ctypes.POINTER(_IngestOut)]
        L.rtps_rx_ingest.restype = I
        L.rtps_rx_ingest_reset.argtypes = [P]
        L.rtps_rx_ingest_reset.restype = I
        L.rtps_rx_set_topics.argtypes = [P, P, U32, P, U32]
        L.rtps_rx_set_topics.restype = I
        L.rtps_rx_topic_gc.argtypes = [P]
        L.rtps_rx_topic_gc.restype = I
        L.rtps_rx_set_spec_hint.argtypes = [P, U32]
        L.rtps_rx_set_spec_hint.restype = I
        L.rtps_rx_cdr_decode.argtypes = [P, P, U32, U32, P, U64, P, P, P, U64, P, P]
        L.rtps_rx_cdr_decode.restype = I
        L.rtps_rx_cdr_decode_list.argtypes = [P, P, U32, U32, P, U64, P, P, P, U64, P, U32, P, U64, P, P]
        L.rtps_rx_cdr_decode_list.restype = I
        for fn in ("rtps_rx_create", "rtps_rx_destroy", "rtps_rx_set_stream", "rtps_rx_set_match_table",
                   "rtps_rx_parse_batch", "rtps_rx_sync", "rtps_rx_generate"):
            getattr(L, fn).restype = I
        assert L.rtps_rx_record_size() == RECORD_DTYPE.itemsize
        _lib = L
    return _lib


def _check(rc):
    if rc != 0:
        raise RtpsRxError(lib().rtps_rx_strerror(rc).decode(), rc)


def gen_layout(workload, n, seed=SEED, first_idx=0, n_writers=16):
    """Host layout of the synthetic generator: (off u64[n], len u32[n], arena_bytes)."""
    off = np.zeros(n, dtype=np.uint64)
    ln = np.zeros(n, dtype=np.uint32)
    size = lib().rtps_rx_gen_layout_host(workload, seed, first_idx, n_writers, n, off.ctypes.data, ln.ctypes.data)
    return off, ln, int(size)


class BatchResult:
    """Host copies of one batch's outputs (status, records, target sets, rec_begin)."""

    def __init__(self, status, records, target, rec_begin, n_records):
        self.status = status
        self.records = records
        self.target = target
        self.rec_begin = rec_begin
        self.n_records = n_records

    def submessages(self, i):
        """All materialised submessages of datagram i (Message.submessages order)."""
        if self.status[i] != 0:
            return self.records[0:0]
        lo = int(self.rec_begin[i])
        hi = int(self.rec_begin[i + 1]) if i + 1 < len(self.rec_begin) else self.n_records
        return self.records[lo:hi]

    def passed_submessages(self, i):
        """What SubmessageIter2::next yields for datagram i: writer/reader submessages with PASS."""
        r = self.submessages(i)
        return r[(r["route"] & ROUTE_PASS) != 0]


class MessageReceiver:
    """Batch receive-path parser bound to one GPU (one context = one stream)."""

    def __init__(self, own_guid_prefix, device=0, max_datagrams=1 << 20):
        import torch  # noqa: F401  (device memory / streams)
        if not torch.cuda.is_available():
            raise RtpsRxError("no GPU visible: the RTPS parser has no CPU fallback")
        cfg = _Config()
        cfg.abi_version = ABI_VERSION
        cfg.device = device
        own = bytes(own_guid_prefix)
        assert len(own) == 12
        for k in range(12):
            cfg.own_prefix[k] = own[k]
        cfg.max_datagrams = max_datagrams
        cfg.flags = 0
        h = ctypes.c_void_p()
        _check(lib().rtps_rx_create(ctypes.byref(cfg), ctypes.byref(h)))
        self._h = h
        self.device = device
        self.max_datagrams = max_datagrams
        self.own_guid_prefix = own
        self.readers = Readers()

    def close(self):
        if getattr(self, "_h", None):
            lib().rtps_rx_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_stream(self, stream):
        """Launch on a torch.cuda.Stream (its handle 0 = the HIP null stream);
        None = the context's own stream."""
        h = ctypes.c_void_p(-1) if stream is None else ctypes.c_void_p(stream.cuda_stream)
        _check(lib().rtps_rx_set_stream(self._h, h))

    def set_readers(self, readers):
        """The local readers and their writer proxies (a records.Readers, or what
        records.as_readers accepts): Domain registration + Reader::matched_writer_add."""
        rd = as_readers(readers)
        r, p = rd.readers, rd.proxies
        _check(lib().rtps_rx_set_readers(self._h, r.ctypes.data if len(r) else None, len(r),
                                         p.ctypes.data if len(p) else None, len(p)))
        self.readers = rd

    def set_match_table(self, entries):
        """Compatibility form: MATCH_DTYPE array or iterable of (writer_guid bytes[16], reader_slot);
        every distinct slot becomes a reader, every distinct pair one of its proxies."""
        t = entries if isinstance(entries, np.ndarray) else pack_match_table(entries)
        t = np.ascontiguousarray(t, dtype=MATCH_DTYPE)
        _check(lib().rtps_rx_set_match_table(self._h, t.ctypes.data if len(t) else None, len(t)))
        self.readers = as_readers(t)

    def target_table(self):
        """Host copy of the target sets: (first u32[n_sets + 1], entries TARGET_DTYPE)."""
        first, ent, n = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_uint32()
        _check(lib().rtps_rx_target_table(self._h, ctypes.byref(first), ctypes.byref(ent), ctypes.byref(n)))
        k = int(n.value)
        f = np.ctypeslib.as_array(ctypes.cast(first, ctypes.POINTER(ctypes.c_uint32)), shape=(k + 1,)).copy()
        total = int(f[-1])
        e = np.zeros(total, dtype=TARGET_DTYPE)
        if total:
            ctypes.memmove(e.ctypes.data, ent.value, total * TARGET_DTYPE.itemsize)
        return f, e

    def expand_targets(self, target):
        """Per-record target readers from per-record target set ids: (off u64[m+1], TARGET_DTYPE[k])."""
        first, ent = self.target_table()
        target = np.asarray(target, dtype=np.uint32)
        ok = target != NO_TARGET
        cnt = np.zeros(len(target), dtype=np.uint64)
        cnt[ok] = (first[target[ok] + 1] - first[target[ok]]).astype(np.uint64)
        off = np.zeros(len(target) + 1, dtype=np.uint64)
        np.cumsum(cnt, out=off[1:])
        starts = first[target[ok]].astype(np.int64)
        c = cnt[ok].astype(np.int64)
        total = int(c.sum())
        # entry j of record k: starts[k] + (j - first position of record k in the output)
        sel = np.repeat(starts - (np.cumsum(c) - c), c) + np.arange(total, dtype=np.int64)
        return off, ent[sel.astype(np.int64)]

    def set_spec_hint(self, records_per_datagram):
        """Performance hint only (results never depend on it): expected records per datagram."""
        _check(lib().rtps_rx_set_spec_hint(self._h, records_per_datagram))

    def sync(self):
        _check(lib().rtps_rx_sync(self._h))

    # ---- device-resident batch API (hot path) ----
    def alloc_outputs(self, n, max_recs):
        import torch
        dev = torch.device("cuda", self.device)
        return {
            "status": torch.empty(max(n, 1), dtype=torch.uint8, device=dev),
            "records": torch.empty((max(max_recs, 1), RECORD_DTYPE.itemsize), dtype=torch.uint8, device=dev),
            "target": torch.empty(max(max_recs, 1), dtype=torch.int32, device=dev),
            "rec_begin": torch.empty(max(n, 1), dtype=torch.int32, device=dev),
            "n_records": torch.zeros(1, dtype=torch.int64, device=dev),
            "max_records": max_recs,
        }

    def parse_batch_device(self, arena, off, lens, n, outs, want_target=True, want_rec_begin=True):
        """arena u8 / off i64 / lens i32 tensors (HBM, or pinned host memory for a
        zero-copy parse); outputs likewise.  Asynchronous on the context's stream."""
        key = (want_target, want_rec_begin)
        o = outs.get("_c_out", {}).get(key)
        if o is None:
            o = _Out()
            o.status = outs["status"].data_ptr()
            o.records = outs["records"].data_ptr()
            o.max_records = outs["max_records"]
            o.target = outs["target"].data_ptr() if want_target else None
            o.rec_begin = outs["rec_begin"].data_ptr() if want_rec_begin else None
            o.n_records = outs["n_records"].data_ptr()
            outs.setdefault("_c_out", {})[key] = o
        _check(lib().rtps_rx_parse_batch(self._h, arena.data_ptr(), arena.numel(), off.data_ptr(),
                                         lens.data_ptr(), n, ctypes.byref(o)))

    def debug_parse_phases(self, arena, off, lens, n, outs, phases):
        """Measurement hook: launch only the parse's first kernel (phases=1) or only the
        finishing kernels (phases=2); returns 1 (spec kernel A), 2 (chained lane walk C),
        3 (LDS tiles D) or 4 (the item pass: E, then S + W).
        Run two full parse_batch_device calls afterwards."""
        self.parse_batch_device(arena, off, lens, n, outs) if "_c_out" not in outs else None
        o = outs["_c_out"][(True, True)]
        L = lib()
        fn = L.rtps_rx_debug_parse_phases
        fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p,
                       ctypes.c_uint32, ctypes.POINTER(_Out), ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint32)]
        fn.restype = ctypes.c_int
        which = ctypes.c_uint32()
        _check(fn(self._h, arena.data_ptr(), arena.numel(), off.data_ptr(), lens.data_ptr(), n, ctypes.byref(o),
                  phases, ctypes.byref(which)))
        return int(which.value)

    def debug_ingest_path(self, path):
        """Ingest path: 0 chosen per batch, 1 global marks / merge, 2 one workgroup per proxy,
        3 global with the first-cover-key merge (k_fcmerge) forced for GAP-free batches."""
        fn = lib().rtps_rx_debug_ingest_path
        fn.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
        _check(fn(self._h, path))

    def debug_frag_sort(self, mode):
        """Reassembly key sort: 0 the bucket sort (default, up to 1.5M records), 1 rocprim's device sort."""
        fn = lib().rtps_rx_debug_frag_sort
        fn.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
        _check(fn(self._h, mode))

    def debug_set_mixed_pass(self, pass_):
        """The pass for mixed traffic (same results): MIXED_ITEM (2, the default: item walk,
        tile scan, record pass), MIXED_RSLAB (3: the walk builds the records into wave slabs,
        tile scan, slab copy), MIXED_CHAIN (0: chained lane walk) or MIXED_LDS (1: chained
        LDS tiles).  True / False select LDS tiles / the chained lane walk."""
        if pass_ is True or pass_ is False:
            pass_ = MIXED_LDS if pass_ else MIXED_CHAIN
        fn = lib().rtps_rx_debug_set_mixed_pass
        fn.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
        _check(fn(self._h, int(pass_)))

    def debug_emit(self, emit=0):
        """The item pass's record pass (same results): 1 = rtps_parse_emit_kernel, 2 =
        rtps_parse_emit2_kernel one workgroup per tile, 3 = rtps_parse_emit2_kernel persistent
        (the default); 0 selects nothing.  Returns the pass in effect."""
        fn = lib().rtps_rx_debug_emit
        fn.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
        fn.restype = ctypes.c_int
        r = fn(self._h, int(emit))
        if r < 0:
            _check(r)
        return r

    def generate(self, workload, arena, off, lens, n, seed=SEED, first_idx=0, n_writers=16):
        """Fill device arena with datagrams [first_idx, first_idx+n) of a synthetic workload."""
        _check(lib().rtps_rx_generate(self._h, workload, seed, first_idx, n_writers, arena.data_ptr(),
                                      off.data_ptr(), lens.data_ptr(), n))

    def bucket_by_writer(self, outs, n_dest, out_records, dest_counts):
        """Stable partition of outs["records"] by owner GPU (writer-GUID hash % n_dest); asynchronous."""
        _check(lib().rtps_rx_bucket_by_writer(self._h, outs["records"].data_ptr(), outs["n_records"].data_ptr(),
                                              outs["max_records"], n_dest, out_records.data_ptr(),
                                              dest_counts.data_ptr()))

    def alloc_rows(self, sample_type, max_recs):
        """Row buffers for cdr_decode: ([max_recs, row_bytes] u8, [max_recs] u8 status)."""
        import torch
        dev = torch.device("cuda", self.device)
        return (torch.empty((max(max_recs, 1), sample_type.row_bytes), dtype=torch.uint8, device=dev),
                torch.empty(max(max_recs, 1), dtype=torch.uint8, device=dev))

    def cdr_decode(self, sample_type, arena, off, outs, rows, row_status):
        """Decode every DATA payload of a parsed batch into fixed-layout rows of
        `sample_type` (a cdr.CdrType) on the device; asynchronous.  Row r belongs
        to record r; row_status[r] is a cdr.CDR_* code (OK rows only are filled)."""
        ops = sample_type.ops
        _check(lib().rtps_rx_cdr_decode(self._h, ops.ctypes.data, len(ops), sample_type.row_bytes,
                                        arena.data_ptr(), arena.numel(), off.data_ptr(), outs["records"].data_ptr(),
                                        outs["n_records"].data_ptr(), outs["max_records"], rows.data_ptr(),
                                        row_status.data_ptr()))

    def cdr_decode_list(self, sample_type, arena, off, outs, lst, stride, n_list, max_list, rows, row_status):
        """Compact decode: row k decodes the record named by the u32 at byte k * stride of the
        device tensor `lst` (e.g. the ingest deliveries: iouts["accepted"], stride 8, n_list =
        iouts["n_accepted"]), for k < min(n_list, max_list); row_status[k] a cdr.CDR_* code."""
        ops = sample_type.ops
        _check(lib().rtps_rx_cdr_decode_list(self._h, ops.ctypes.data, len(ops), sample_type.row_bytes,
                                             arena.data_ptr(), arena.numel(), off.data_ptr(),
                                             outs["records"].data_ptr(), outs["n_records"].data_ptr(),
                                             outs["max_records"], lst.data_ptr(), stride, n_list.data_ptr(),
                                             max_list, rows.data_ptr(), row_status.data_ptr()))

    def bucket_by_writer_padded(self, outs, n_dest, cap, out_records, dest_counts):
        """Same partition into n_dest fixed buckets of cap records (out_records[d*cap:(d+1)*cap]);
        dest_counts gets the true sizes (> cap = overflow, records past cap dropped)."""
        _check(lib().rtps_rx_bucket_by_writer_padded(self._h, outs["records"].data_ptr(),
                                                     outs["n_records"].data_ptr(), outs["max_records"], n_dest, cap,
                                                     out_records.data_ptr(), dest_counts.data_ptr()))

    def bucket_descriptors(self, outs, n_dest, cap, out_desc, dest_counts):
        """16-byte exchange descriptors of the MATCHED records in n_dest fixed buckets of cap
        (owner = writer set index % n_dest); needs readers."""
        _check(lib().rtps_rx_bucket_descriptors(self._h, outs["records"].data_ptr(), outs["n_records"].data_ptr(),
                                                outs["max_records"], n_dest, cap, out_desc.data_ptr(),
                                                dest_counts.data_ptr()))

    # ---- DataFrag reassembly (state persists in the context across batches) ----
    def alloc_frag_outputs(self, max_samples, heap_bytes):
        import torch
        dev = torch.device("cuda", self.device)
        return {"samples": torch.empty((max(max_samples, 1), FRAG_SAMPLE_DTYPE.itemsize), dtype=torch.uint8,
                                       device=dev),
                "max_samples": max_samples,
                "heap": torch.empty(max(heap_bytes, 1), dtype=torch.uint8, device=dev), "heap_bytes": heap_bytes,
                "n_samples": torch.zeros(1, dtype=torch.int64, device=dev),
                "heap_used": torch.zeros(1, dtype=torch.int64, device=dev),
                "n_pending": torch.zeros(1, dtype=torch.int64, device=dev)}

    def frag_assemble(self, arena, off, outs, fouts):
        """Reassemble the DATA_FRAG records of a parsed batch (asynchronous)."""
        o = fouts.get("_c")
        if o is None:
            o = _FragOut()
            o.samples = fouts["samples"].data_ptr()
            o.max_samples = fouts["max_samples"]
            o.heap = fouts["heap"].data_ptr()
            o.heap_bytes = fouts["heap_bytes"]
            o.n_samples = fouts["n_samples"].data_ptr()
            o.heap_used = fouts["heap_used"].data_ptr()
            o.n_pending = fouts["n_pending"].data_ptr()
            fouts["_c"] = o
        _check(lib().rtps_rx_frag_assemble(self._h, arena.data_ptr(), arena.numel(), off.data_ptr(),
                                           outs["records"].data_ptr(), outs["n_records"].data_ptr(),
                                           outs["max_records"], ctypes.byref(o)))

    def frag_reset(self):
        _check(lib().rtps_rx_frag_reset(self._h))

    def frag_set_clock(self, now_ns):
        """Clock (ns) the next batches stamp on the assembly buffers they create or extend."""
        L = lib()
        L.rtps_rx_frag_set_clock.argtypes = [ctypes.c_void_p, ctypes.c_uint64]
        _check(L.rtps_rx_frag_set_clock(self._h, now_ns))

    def set_reader_lifespan(self, reader_slot, lifespan_ns):
        """Lifespan QoS of a reader for the DataFrag assembly (reader.rs:578-589); None: none."""
        L = lib()
        L.rtps_rx_set_reader_lifespan.argtypes = [ctypes.c_void_p, ctypes.c_uint16, ctypes.c_int64]
        _check(L.rtps_rx_set_reader_lifespan(self._h, reader_slot, -1 if lifespan_ns is None else lifespan_ns))

    def frag_set_receive_time(self, unix_ns):
        """Timestamp::now() of the next batches for the Lifespan checks (0: the host clock)."""
        L = lib()
        L.rtps_rx_frag_set_receive_time.argtypes = [ctypes.c_void_p, ctypes.c_uint64]
        _check(L.rtps_rx_frag_set_receive_time(self._h, unix_ns))

    def frag_gc(self, expire_before_ns):
        """Drop the incomplete buffers last modified before expire_before_ns -> buffers left (host sync)."""
        import torch
        L = lib()
        L.rtps_rx_frag_gc.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p]
        n = torch.zeros(1, dtype=torch.int64, device=torch.device("cuda", self.device))
        _check(L.rtps_rx_frag_gc(self._h, expire_before_ns, n.data_ptr()))
        self.sync()
        return int(n.item())

    def assemble_batch(self, arena_np, off_np, len_np, max_samples=None, heap_bytes=None):
        """Parse + reassemble host arrays -> (BatchResult, samples FRAG_SAMPLE_DTYPE, heap u8, n_samples,
        heap_used, n_pending)."""
        import torch
        n = len(len_np)
        dev = torch.device("cuda", self.device)
        arena = torch.from_numpy(np.ascontiguousarray(arena_np, dtype=np.uint8)).to(dev)
        off = torch.from_numpy(np.ascontiguousarray(off_np, dtype=np.uint64).view(np.int64)).to(dev)
        lens = torch.from_numpy(np.ascontiguousarray(len_np, dtype=np.uint32).view(np.int32)).to(dev)
        cap = max_records(len_np)
        outs = self.alloc_outputs(n, cap)
        ms = cap if max_samples is None else max_samples
        hb = (int(arena.numel()) + 16 * cap + (1 << 22)) if heap_bytes is None else heap_bytes
        fouts = self.alloc_frag_outputs(ms, hb)
        torch.cuda.synchronize(dev)
        self.parse_batch_device(arena, off, lens, n, outs)
        self.frag_assemble(arena, off, outs, fouts)
        self.sync()
        total = int(outs["n_records"].item())
        kept = min(total, cap)
        recs = outs["records"][:kept].cpu().numpy().reshape(-1).view(RECORD_DTYPE)
        target = outs["target"][:kept].cpu().numpy().view(np.uint32)
        res = BatchResult(outs["status"][:n].cpu().numpy(), recs, target,
                          outs["rec_begin"][:n].cpu().numpy().view(np.uint32), total)
        ns = int(fouts["n_samples"].item())
        used = int(fouts["heap_used"].item())
        samples = fouts["samples"][:min(ns, ms)].cpu().numpy().reshape(-1).view(FRAG_SAMPLE_DTYPE)
        heap = fouts["heap"][:min(used, hb)].cpu().numpy()
        return res, samples, heap, ns, used, int(fouts["n_pending"].item())

    # ---- history-cache ingest (writer-proxy state persists in the context) ----
    def alloc_ingest_outputs(self, max_recs, n_proxies, max_accepted=None):
        """max_accepted: deliveries room (default max_recs x the largest target set)."""
        import torch
        dev = torch.device("cuda", self.device)
        if max_accepted is None:
            first, _ = self.target_table()
            widest = int(np.max(np.diff(first))) if len(first) > 1 else 1
            max_accepted = max_recs * max(widest, 1)
        return {"accept": torch.empty(max(max_recs, 1), dtype=torch.uint8, device=dev),
                "accepted": torch.empty((max(max_accepted, 1), DELIVERY_DTYPE.itemsize), dtype=torch.uint8, device=dev),
                "max_accepted": max_accepted,
                "n_accepted": torch.zeros(1, dtype=torch.int64, device=dev),
                "ack_base": torch.zeros(max(n_proxies, 1), dtype=torch.int64, device=dev),
                "n_window_overflow": torch.zeros(1, dtype=torch.int64, device=dev)}

    def set_topics(self, topics, topic_readers):
        """Topic caches: topics [(topic id, max_keep_samples)], topic_readers [(reader slot, topic id)];
        unmapped readers keep a cache of their own (max_keep 64).  Empties every topic cache."""
        from .records import TOPIC_DTYPE, TOPIC_READER_DTYPE
        t = np.zeros(len(topics), dtype=TOPIC_DTYPE)
        for i, (tid, k) in enumerate(topics):
            t[i] = (tid, k)
        r = np.zeros(len(topic_readers), dtype=TOPIC_READER_DTYPE)
        for i, (slot, tid) in enumerate(topic_readers):
            r[i]["reader_slot"], r[i]["topic"] = slot, tid
        _check(lib().rtps_rx_set_topics(self._h, t.ctypes.data if len(t) else None, len(t),
                                        r.ctypes.data if len(r) else None, len(r)))

    def topic_gc(self):
        """DDSCache::garbage_collect: every topic cache trimmed to its max_keep_samples newest changes."""
        _check(lib().rtps_rx_topic_gc(self._h))

    def ingest(self, arena, off, outs, iouts, fouts=None, best_effort=False, topic_cache=False):
        """Decide which samples of a parsed batch the readers accept (the stateful
        reader's writer proxies, Reader::handle_data_msg / _heartbeat_ / _gap_) and,
        with topic_cache, which of them their topic caches store (DELIVERY_CACHED);
        fouts: frag_assemble outputs of the same batch.  Asynchronous."""
        if iouts["accept"].numel() < max(outs["max_records"], 1):  # the ingest writes accept[0, max_records)
            raise ValueError(f"ingest: accept holds {iouts['accept'].numel()} bytes, the batch's record capacity "
                             f"is {outs['max_records']} (alloc_ingest_outputs(max_records, ...))")
        o = iouts.get("_c")
        if o is None:
            o = _IngestOut()
            o.accept = iouts["accept"].data_ptr()
            o.accepted = iouts["accepted"].data_ptr()
            o.max_accepted = iouts["max_accepted"]
            o.n_accepted = iouts["n_accepted"].data_ptr()
            o.ack_base = iouts["ack_base"].data_ptr()
            o.n_window_overflow = iouts["n_window_overflow"].data_ptr()
            iouts["_c"] = o
        frag = fouts["samples"].data_ptr() if fouts is not None else None
        nfrag = fouts["n_samples"].data_ptr() if fouts is not None else None
        mfrag = fouts["max_samples"] if fouts is not None else 0
        _check(lib().rtps_rx_ingest(self._h, arena.data_ptr(), arena.numel(), off.data_ptr(),
                                    outs["records"].data_ptr(), outs["n_records"].data_ptr(), outs["max_records"],
                                    frag, nfrag, mfrag, (INGEST_BEST_EFFORT if best_effort else 0) |
                                    (INGEST_TOPIC_CACHE if topic_cache else 0), ctypes.byref(o)))

    def ingest_reset(self):
        """Every writer proxy starts afresh; the topic caches keep their changes."""
        _check(lib().rtps_rx_ingest_reset(self._h))

    def topic_reset(self):
        """Empty every topic cache (the proxies keep their state)."""
        _check(lib().rtps_rx_topic_reset(self._h))

    def ingest_batch(self, arena_np, off_np, len_np, n_proxies, frag=False, best_effort=False, topic_cache=False):
        """Parse (+ reassemble) + ingest host arrays -> (BatchResult, accept u8[m], deliveries
        DELIVERY_DTYPE[k], ack_base i64[n_proxies], n_window_overflow, frag samples or None)."""
        import torch
        n = len(len_np)
        dev = torch.device("cuda", self.device)
        arena = torch.from_numpy(np.ascontiguousarray(arena_np, dtype=np.uint8)).to(dev)
        off = torch.from_numpy(np.ascontiguousarray(off_np, dtype=np.uint64).view(np.int64)).to(dev)
        lens = torch.from_numpy(np.ascontiguousarray(len_np, dtype=np.uint32).view(np.int32)).to(dev)
        cap = max_records(len_np)
        outs = self.alloc_outputs(n, cap)
        iouts = self.alloc_ingest_outputs(cap, n_proxies)
        fouts = self.alloc_frag_outputs(cap, int(arena.numel()) + 16 * cap + (1 << 20)) if frag else None
        torch.cuda.synchronize(dev)
        self.parse_batch_device(arena, off, lens, n, outs)
        if frag:
            self.frag_assemble(arena, off, outs, fouts)
        self.ingest(arena, off, outs, iouts, fouts, best_effort=best_effort, topic_cache=topic_cache)
        self.sync()
        total = int(outs["n_records"].item())
        kept = min(total, cap)
        recs = outs["records"][:kept].cpu().numpy().reshape(-1).view(RECORD_DTYPE)
        target = outs["target"][:kept].cpu().numpy().view(np.uint32)
        res = BatchResult(outs["status"][:n].cpu().numpy(), recs, target,
                          outs["rec_begin"][:n].cpu().numpy().view(np.uint32), total)
        na = int(iouts["n_accepted"].item())
        samples = None
        if frag:
            ns = min(int(fouts["n_samples"].item()), cap)
            samples = fouts["samples"][:ns].cpu().numpy().reshape(-1).view(FRAG_SAMPLE_DTYPE)
        dels = iouts["accepted"][:min(na, iouts["max_accepted"])].cpu().numpy().reshape(-1).view(DELIVERY_DTYPE)
        return (res, iouts["accept"][:kept].cpu().numpy(), dels,
                iouts["ack_base"][:n_proxies].cpu().numpy(), int(iouts["n_window_overflow"].item()), samples)

    # ---- convenience: host datagrams in, host results out ----
    def handle_received_batch(self, arena_np, off_np, len_np):
        """Parse host arrays on the GPU (H2D copy, parse, D2H copy) -> BatchResult."""
        import torch
        n = len(len_np)
        dev = torch.device("cuda", self.device)
        arena = torch.from_numpy(np.ascontiguousarray(arena_np, dtype=np.uint8)).to(dev)
        off = torch.from_numpy(np.ascontiguousarray(off_np, dtype=np.uint64).view(np.int64)).to(dev)
        lens = torch.from_numpy(np.ascontiguousarray(len_np, dtype=np.uint32).view(np.int32)).to(dev)
        cap = max_records(len_np)
        outs = self.alloc_outputs(n, cap)
        torch.cuda.synchronize(dev)
        self.parse_batch_device(arena, off, lens, n, outs)
        self.sync()
        total = int(outs["n_records"].item())
        kept = min(total, cap)
        recs = outs["records"][:kept].cpu().numpy().reshape(-1).view(RECORD_DTYPE)
        target = outs["target"][:kept].cpu().numpy().view(np.uint32)
        return BatchResult(outs["status"][:n].cpu().numpy(), recs, target,
                           outs["rec_begin"][:n].cpu().numpy().view(np.uint32), total)

    def take_batch(self, sample_type, arena_np, off_np, len_np):
        """Parse + CDR-decode host arrays on the GPU -> (BatchResult, rows, row_status):
        the batch form of DataReader::take's deserialize step (simpledatareader.rs:137-160)."""
        import torch
        n = len(len_np)
        dev = torch.device("cuda", self.device)
        arena = torch.from_numpy(np.ascontiguousarray(arena_np, dtype=np.uint8)).to(dev)
        off = torch.from_numpy(np.ascontiguousarray(off_np, dtype=np.uint64).view(np.int64)).to(dev)
        lens = torch.from_numpy(np.ascontiguousarray(len_np, dtype=np.uint32).view(np.int32)).to(dev)
        cap = max_records(len_np)
        outs = self.alloc_outputs(n, cap)
        rows, row_status = self.alloc_rows(sample_type, cap)
        torch.cuda.synchronize(dev)
        self.parse_batch_device(arena, off, lens, n, outs)
        self.cdr_decode(sample_type, arena, off, outs, rows, row_status)
        self.sync()
        total = int(outs["n_records"].item())
        kept = min(total, cap)
        recs = outs["records"][:kept].cpu().numpy().reshape(-1).view(RECORD_DTYPE)
        target = outs["target"][:kept].cpu().numpy().view(np.uint32)
        res = BatchResult(outs["status"][:n].cpu().numpy(), recs, target,
                          outs["rec_begin"][:n].cpu().numpy().view(np.uint32), total)
        return res, sample_type.rows(rows[:kept].cpu().numpy()), row_status[:kept].cpu().numpy()
