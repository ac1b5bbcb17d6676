"""Writer-GUID sharding of parsed records across GPUs.

Each rank parses its own contiguous chunk of datagrams; the records of the
writer and reader submessages are then partitioned by owner rank =
fmix32(fnv1a32(prefix || writer_id)) % world (stable, on the device:
rtps_rx_bucket_by_writer) and exchanged with ONE all-to-all.  The owner then
holds every record of its writers (ready for per-writer ordering, dedup and
fragment assembly).  The reference has a single process and no exchange;
this is the only collective of the path.

What crosses xGMI (item):
  * "records": the 64-byte records of every writer/reader submessage, owner =
    GUID hash % world (rtps_rx_bucket_by_writer[_padded]);
  * "descriptors": 16-byte rtps_xdesc of the records that reach a reader (MATCHED, or
    TARGETED by entity id only), owner = target set index % world
    (rtps_rx_bucket_descriptors): 4x fewer
    bytes, and owners balanced by the table order instead of a hash of a few
    writer GUIDs.  Full records and payloads stay on the source GPU.

Transport: with the "nccl" (RCCL) process group the buckets move through the
library's own RCCL exchange (rtps_rx_exchange: grouped ncclSend/ncclRecv per
peer on a dedicated HIP stream, the same entry point a Rust host binds;
torch.distributed only bootstraps the communicator's unique id).  The "gloo"
group (CPU tensors) rehearses several ranks on one GPU, which RCCL cannot.

Two modes:
  * contiguous (cap=None): buckets back to back, split sizes read back to the
    host (one device->host round trip per exchange); exact-size messages.
  * padded (cap=C): every bucket is a fixed slot of C records
    (rtps_rx_bucket_by_writer_padded), so the all-to-all has equal splits and
    the true counts travel in a second tiny all-to-all: no host round trip,
    fully asynchronous (exchange_async), so the exchange of batch k overlaps
    the parse of batch k+1.  Overflow (a bucket > C) is reported by
    overflowed(); C is sized from the previous batch's counts.
"""
import ctypes

import torch

RECORD_BYTES = 64
_COMMS = {}


def _forget_comm(comm):
    """The library aborted this communicator (RTPS_RX_EABORTED), which frees it: drop it from
    the cache so it is neither handed out again nor destroyed a second time."""
    for k, c in list(_COMMS.items()):
        if c is comm:
            del _COMMS[k]


def _check_comm(rc, owner):
    """_check for the calls that may abort the communicator of `owner` (an Exchange or an
    OwnerShard): on RTPS_RX_EABORTED the library has freed it, so the owner forgets it too and
    every later exchange call on that object raises instead of passing a freed handle."""
    from . import _check, RTPS_RX_EABORTED
    if rc == RTPS_RX_EABORTED:
        _forget_comm(owner.comm)
        owner.comm = None
        owner.comm_aborted = True
    _check(rc)


def _live_comm(owner):
    """The owner's communicator, or an error when an earlier call aborted it."""
    from . import RtpsRxError, RTPS_RX_EABORTED
    if getattr(owner, "comm_aborted", False):
        raise RtpsRxError("the RCCL communicator was aborted by an earlier failure; create a new exchange object",
                          RTPS_RX_EABORTED)
    return owner.comm


def destroy_comms():
    """Destroy the library RCCL communicators of this process (call before the process group goes)."""
    from . import lib
    while _COMMS:
        _, c = _COMMS.popitem()
        lib().rtps_rx_exchange_comm_destroy.argtypes = [ctypes.c_void_p]
        lib().rtps_rx_exchange_comm_destroy(c)


def rccl_comm(rx, dist, device):
    """This process's RCCL communicator for the library's exchange (one per world/rank):
    rank 0 makes the unique id, torch.distributed broadcasts it, every rank inits."""
    from . import lib, _check
    key = (dist.get_world_size(), dist.get_rank())
    if key not in _COMMS:
        L = lib()
        L.rtps_rx_exchange_unique_id.argtypes = [ctypes.c_void_p]
        L.rtps_rx_exchange_comm_init.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                                 ctypes.POINTER(ctypes.c_void_p)]
        uid = (ctypes.c_uint8 * 128)()
        if key[1] == 0:
            _check(L.rtps_rx_exchange_unique_id(uid))
        obj = [bytes(uid)]
        dist.broadcast_object_list(obj, src=0)
        uid = (ctypes.c_uint8 * 128).from_buffer_copy(obj[0])
        comm = ctypes.c_void_p()
        _check(L.rtps_rx_exchange_comm_init(uid, key[0], key[1], device.index, ctypes.byref(comm)))
        _COMMS[key] = comm
    return _COMMS[key]
ITEM_BYTES = {"records": 64, "descriptors": 16}
ITEM_BYTES_OWNER = 16  # rtps_shard_item: what the owner-side exchange moves per writer record


def owner_hash_words(words):
    """fnv1a32 over 4 little-endian u32 words, then the murmur3 finaliser fmix32 (the device's owner_hash)."""
    h = 0x811C9DC5
    for w in words:
        h = ((h ^ int(w)) * 0x01000193) & 0xFFFFFFFF
    h ^= h >> 16
    h = (h * 0x85EBCA6B) & 0xFFFFFFFF
    h ^= h >> 13
    h = (h * 0xC2B2AE35) & 0xFFFFFFFF
    return h ^ (h >> 16)


class _StreamWork:
    """wait(): the caller's current stream waits for the exchange (like a collective's Work)."""

    def __init__(self, event, device):
        self.event, self.device = event, device

    def wait(self):
        torch.cuda.current_stream(self.device).wait_event(self.event)


class Exchange:
    """Buffers + the exchange step for one rank."""

    def __init__(self, rx, max_records, world, dist, device, cap=None, item="records"):
        self.rx = rx
        self.world = world
        self.dist = dist
        self.device = device
        self.cap = cap
        self.item = item
        ib = ITEM_BYTES[item]
        assert item == "records" or cap, "descriptors are exchanged in padded buckets"
        slots = world * cap if cap else max(max_records, 1)
        self.bucketed = torch.empty((max(slots, 1), ib), dtype=torch.uint8, device=device)
        self.counts = torch.zeros(world, dtype=torch.int64, device=device)
        self.recv_counts = torch.zeros(world, dtype=torch.int64, device=device)
        self.received = torch.empty((max(slots, 1), ib), dtype=torch.uint8, device=device) if cap else None
        backend = dist.get_backend() if dist is not None else None
        self.host_collectives = backend == "gloo"  # gloo moves CPU tensors only
        # RCCL: the library's exchange on a dedicated stream (padded mode)
        self.comm = rccl_comm(rx, dist, device) if (dist is not None and not self.host_collectives and cap) else None
        self.xstream = torch.cuda.Stream(device) if self.comm is not None else None

    def bucket(self, outs):
        """Stable partition of this rank's records by owner rank (asynchronous)."""
        if self.item == "descriptors":
            self.rx.bucket_descriptors(outs, self.world, self.cap, self.bucketed, self.counts)
        elif self.cap:
            self.rx.bucket_by_writer_padded(outs, self.world, self.cap, self.bucketed, self.counts)
        else:
            self.rx.bucket_by_writer(outs, self.world, self.bucketed, self.counts)

    def exchange(self):
        """All-to-all of the bucketed records; returns (records [m, 64] u8, per-source counts list)."""
        if self.cap:
            for w in self.exchange_async():
                w.wait()
            return self.gather_received()
        dist = self.dist
        if self.host_collectives:
            counts = self.counts.cpu()
            recv_counts = torch.zeros_like(counts)
            dist.all_to_all_single(recv_counts, counts)
        else:
            dist.all_to_all_single(self.recv_counts, self.counts)
            counts, recv_counts = self.counts, self.recv_counts
        send = counts.tolist()
        recv = recv_counts.tolist()
        nsend = sum(send)
        if self.host_collectives:
            out = torch.empty((sum(recv), RECORD_BYTES), dtype=torch.uint8)
            dist.all_to_all_single(out, self.bucketed[:nsend].cpu(), recv, send)
            return out.to(self.device), recv
        out = torch.empty((sum(recv), RECORD_BYTES), dtype=torch.uint8, device=self.device)
        dist.all_to_all_single(out, self.bucketed[:nsend], recv, send)
        return out, recv

    # ---- padded mode ----
    def exchange_async(self):
        """Equal-split all-to-all of the padded buckets + their counts; returns the work handles
        (wait() on them orders the caller's stream after the exchange)."""
        assert self.cap, "exchange_async needs the padded mode"
        dist = self.dist
        if self.host_collectives:
            rc = torch.zeros(self.world, dtype=torch.int64)
            dist.all_to_all_single(rc, self.counts.cpu())
            rv = torch.empty_like(self.received, device="cpu")
            dist.all_to_all_single(rv, self.bucketed.cpu())
            self.recv_counts.copy_(rc)
            self.received.copy_(rv)
            return []
        from . import lib, _check
        cur = torch.cuda.current_stream(self.device)
        self.xstream.wait_stream(cur)  # the buckets are complete
        L = lib()
        L.rtps_rx_exchange.argtypes = [ctypes.c_void_p] * 5 + [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_void_p,
                                                               ctypes.c_void_p]
        _check_comm(L.rtps_rx_exchange(self.rx._h, _live_comm(self), ctypes.c_void_p(self.xstream.cuda_stream),
                                       self.bucketed.data_ptr(), self.counts.data_ptr(), self.cap,
                                       ITEM_BYTES[self.item], self.received.data_ptr(), self.recv_counts.data_ptr()),
                    self)
        done = torch.cuda.Event()
        done.record(self.xstream)
        return [_StreamWork(done, self.device)]

    def gather_received(self):
        """Host view after exchange_async completed: the valid items from every source in
        rank order ([m, item bytes] u8 on the device) and the per-source counts."""
        rc = self.recv_counts.cpu().tolist()
        parts = [self.received[s * self.cap:s * self.cap + min(c, self.cap)] for s, c in enumerate(rc)]
        return torch.cat(parts) if parts else self.received[:0], [min(c, self.cap) for c in rc]

    def overflowed(self):
        """True if a bucket of the last bucket() call had more than cap records (host sync)."""
        return bool(self.cap) and int(self.counts.max().item()) > self.cap


# ---------------------------------------------------------------------------
# Owner-side exchange (rtps_rx_shard_*, include/rtps_rx.h): every writer-kind
# record that passes goes to its writer's owner with the bytes the owner's
# fragment assembly and ingest read (GAP bitmaps, DATA_FRAG payloads), so the
# owner runs rtps_rx_frag_assemble / rtps_rx_ingest on all of its writers'
# submessages in stream order.  Fixed slots first (equal splits, no host round
# trip), then the exact spill of whatever did not fit: no record is dropped.
# ---------------------------------------------------------------------------
import numpy as _np

SHARD_COUNTS_DTYPE = _np.dtype([("n", "<u8"), ("bytes", "<u8"), ("cut", "<u8"), ("cut_bytes", "<u8")])
SHARD_LEAD = 65536
_HIP = None


def _hip():
    """HIP runtime (ctypes) for raw device-pointer copies of the library-owned buffers."""
    global _HIP
    if _HIP is None:
        _HIP = ctypes.CDLL("libamdhip64.so")
        _HIP.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
        _HIP.hipMemcpy.restype = ctypes.c_int
        _HIP.hipDeviceSynchronize.restype = ctypes.c_int
    return _HIP


def dev_copy(dst, src, nbytes):
    """hipMemcpy(dst, src, n, hipMemcpyDefault) between raw pointers (host or device), ordered
    after all work queued on the device and before what follows: the copy goes on the null
    stream, which does not wait for non-blocking streams (torch's, the context's)."""
    if nbytes:
        H = _hip()
        rc = H.hipDeviceSynchronize() or H.hipMemcpy(ctypes.c_void_p(dst), ctypes.c_void_p(src), nbytes, 4) \
            or H.hipDeviceSynchronize()
        if rc != 0:
            raise RuntimeError(f"hipMemcpy failed ({rc})")


def dev_to_numpy(ptr, nbytes, dtype=_np.uint8):
    a = _np.empty(nbytes, dtype=_np.uint8)
    dev_copy(a.ctypes.data, ptr, nbytes)
    return a.view(dtype)


class DevPtr:
    """A library-owned device buffer in the tensor shape the MessageReceiver methods take
    (data_ptr / numel)."""

    def __init__(self, ptr, nbytes):
        self.ptr, self.nbytes = int(ptr or 0), int(nbytes)

    def data_ptr(self):
        return self.ptr

    def numel(self):
        return self.nbytes


class _ShardBuffers(ctypes.Structure):
    _fields_ = [(n, ctypes.c_void_p) for n in ("send_slots", "send_blob", "send_counts", "recv_slots", "recv_blob",
                                               "recv_counts", "send_spill", "send_blob_spill", "recv_spill",
                                               "recv_blob_spill")] + \
               [("recv_spill_cap", ctypes.c_uint64), ("recv_blob_spill_cap", ctypes.c_uint64)]


class _OwnerBatch(ctypes.Structure):
    _fields_ = [("arena", ctypes.c_void_p), ("arena_len", ctypes.c_uint64), ("dgram_off", ctypes.c_void_p),
                ("records", ctypes.c_void_p), ("origin", ctypes.c_void_p), ("n_records_dev", ctypes.c_void_p),
                ("n_records", ctypes.c_uint64)]


class OwnerBatch:
    """The owner's received records as a batch for rx.frag_assemble / rx.ingest (device,
    library-owned, valid until the next unpack): `arena`, `off` and `outs` go where a parse's
    arena / offsets / outputs go."""

    def __init__(self, ob):
        n = int(ob.n_records)
        self.n_records = n
        self.arena = DevPtr(ob.arena, ob.arena_len)
        self.off = DevPtr(ob.dgram_off, 8 * n)
        self.origin_ptr = int(ob.origin or 0)
        self.outs = {"records": DevPtr(ob.records, 64 * n), "n_records": DevPtr(ob.n_records_dev, 8),
                     "max_records": n}

    def records(self):
        from .records import RECORD_DTYPE
        return dev_to_numpy(self.outs["records"].ptr, 64 * self.n_records, RECORD_DTYPE)

    def origin(self):
        """(source rank u32[n], the record's index in the source rank's parse output u32[n])."""
        o = dev_to_numpy(self.origin_ptr, 8 * self.n_records, _np.uint64)
        return (o >> _np.uint64(32)).astype(_np.uint32), (o & _np.uint64(0xFFFFFFFF)).astype(_np.uint32)

    def dgram_off(self):
        return dev_to_numpy(self.off.ptr, 8 * self.n_records, _np.uint64)

    def arena_bytes(self):
        return dev_to_numpy(self.arena.ptr, self.arena.nbytes)


def shard_lib():
    from . import lib
    L = lib()
    if not getattr(L, "_shard_bound", False):
        P, U32, U64 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64
        L.rtps_rx_shard_create.argtypes = [P, U32, U64, U64, ctypes.POINTER(P)]
        L.rtps_rx_shard_destroy.argtypes = [P]
        L.rtps_rx_shard_pack.argtypes = [P, P, U64, P, P, P, U64]
        L.rtps_rx_shard_exchange.argtypes = [P, P, P]
        L.rtps_rx_shard_finish.argtypes = [P, P, P]
        L.rtps_rx_shard_unpack.argtypes = [P, ctypes.POINTER(_OwnerBatch)]
        L.rtps_rx_shard_buffers.argtypes = [P, ctypes.POINTER(_ShardBuffers)]
        L.rtps_rx_shard_reserve_spill.argtypes = [P, U64, U64]
        L.rtps_rx_shard_set_owners.argtypes = [P, U32, P, P, U32]
        L.rtps_rx_shard_owner.argtypes = [P, P]
        L.rtps_rx_owner_assign.argtypes = [P, P, P, U32, U32, P]
        L.rtps_rx_owner_assign_sticky.argtypes = [P, P, P, U32, U32, P, P]
        for f in ("rtps_rx_shard_create", "rtps_rx_shard_destroy", "rtps_rx_shard_pack", "rtps_rx_shard_exchange",
                  "rtps_rx_shard_finish", "rtps_rx_shard_unpack", "rtps_rx_shard_buffers",
                  "rtps_rx_shard_reserve_spill", "rtps_rx_shard_set_owners", "rtps_rx_shard_owner",
                  "rtps_rx_owner_assign", "rtps_rx_owner_assign_sticky"):
            getattr(L, f).restype = ctypes.c_int
        L._shard_bound = True
    return L


OWNER_BALANCED, OWNER_HASH, OWNER_TOPIC = 0, 1, 2  # rtps_rx_shard_set_owners modes


def owner_assign(writers, n_ranks, weights=None, groups=None, prev=None):
    """rtps_rx_owner_assign (host, no GPU): writers = list of 16-byte GUIDs -> owner rank of each.
    Groups (list of group ids < n, optional) share an owner; weights (optional) per writer;
    prev (optional, rtps_rx_owner_assign_sticky): each writer's previous owner, -1 = new."""
    from . import _check
    n = len(writers)
    w = _np.frombuffer(b"".join(bytes(g) for g in writers), dtype=_np.uint8) if n else _np.zeros(16, _np.uint8)
    wt = None if weights is None else _np.ascontiguousarray(weights, dtype=_np.uint64)
    gr = None if groups is None else _np.ascontiguousarray(groups, dtype=_np.uint32)
    out = _np.zeros(max(n, 1), dtype=_np.uint32)
    args = (w.ctypes.data, None if wt is None else wt.ctypes.data, None if gr is None else gr.ctypes.data, n, n_ranks)
    if prev is None:
        _check(shard_lib().rtps_rx_owner_assign(*args, out.ctypes.data))
    else:
        pv = _np.ascontiguousarray(prev, dtype=_np.int32)
        assert len(pv) == n
        _check(shard_lib().rtps_rx_owner_assign_sticky(*args, pv.ctypes.data if n else None, out.ctypes.data))
    return out[:n]


def spill_plan(send_counts, recv_counts):
    """Round 1 of the protocol from round 0's counts (SHARD_COUNTS_DTYPE [world] each):
    per peer (send record range, send byte range) in the send spill's exact layout and
    (receive record offset + count, byte offset + count) in the receive spill."""
    s, r = send_counts, recv_counts
    sb = _np.concatenate([[0], _np.cumsum(s["n"].astype(_np.int64))[:-1]])
    sbb = _np.concatenate([[0], _np.cumsum(s["bytes"].astype(_np.int64))[:-1]])
    rn = (r["n"] - r["cut"]).astype(_np.int64)
    rb = (r["bytes"] - r["cut_bytes"]).astype(_np.int64)
    rs = _np.concatenate([[0], _np.cumsum(rn)[:-1]])
    rsb = _np.concatenate([[0], _np.cumsum(rb)[:-1]])
    plan = []
    for p in range(len(s)):
        plan.append({"send_rec": (int(sb[p] + s["cut"][p]), int(s["n"][p] - s["cut"][p])),
                     "send_bytes": (int(sbb[p] + s["cut_bytes"][p]), int(s["bytes"][p] - s["cut_bytes"][p])),
                     "recv_rec": (int(rs[p]), int(rn[p])), "recv_bytes": (int(rsb[p]), int(rb[p]))})
    return plan


class OwnerShard:
    """One rank's owner-side exchange (rtps_rx_shard_*).  Transport: the library's RCCL
    rounds (rtps_rx_shard_exchange / _finish) with the "nccl" group, or the same protocol
    moved by torch.distributed over host memory with "gloo" (one-GPU rehearsals)."""

    def __init__(self, rx, world, dist, device, cap, bcap):
        L = shard_lib()
        self.rx, self.world, self.dist, self.device = rx, world, dist, device
        self.cap, self.bcap = int(cap), int(bcap) + (-int(bcap)) % 16
        h = ctypes.c_void_p()
        from . import _check
        _check(L.rtps_rx_shard_create(rx._h, world, self.cap, self.bcap, ctypes.byref(h)))
        self._h = h
        backend = dist.get_backend() if dist is not None else "gloo"
        self.host_collectives = backend == "gloo"
        self.comm = None if self.host_collectives else rccl_comm(rx, dist, device)
        self.xstream = None if self.host_collectives else torch.cuda.Stream(device)
        self.last_spill = 0

    def close(self):
        if getattr(self, "_h", None):
            shard_lib().rtps_rx_shard_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def buffers(self):
        b = _ShardBuffers()
        from . import _check
        _check(shard_lib().rtps_rx_shard_buffers(self._h, ctypes.byref(b)))
        return b

    def set_owners(self, mode=OWNER_BALANCED, weights=None):
        """rtps_rx_shard_set_owners: the writer -> owner deal (OWNER_BALANCED, OWNER_TOPIC or
        OWNER_HASH); weights: {16-byte writer GUID: weight} (optional)."""
        from . import _check
        weights = weights or {}
        g = _np.frombuffer(b"".join(bytes(k) for k in weights), dtype=_np.uint8) if weights else None
        w = _np.array(list(weights.values()), dtype=_np.uint64) if weights else None
        _check(shard_lib().rtps_rx_shard_set_owners(self._h, mode, None if g is None else g.ctypes.data,
                                                    None if w is None else w.ctypes.data, len(weights)))

    def owner_of(self, guid):
        """The owner rank of a 16-byte writer GUID under the current deal."""
        from . import _check
        buf = (ctypes.c_uint8 * 16).from_buffer_copy(bytes(guid))
        r = shard_lib().rtps_rx_shard_owner(self._h, buf)
        if r < 0:
            _check(r)
        return r

    def pack(self, arena, off, outs):
        """Source side: this rank's parse output into the slots and the spill (asynchronous)."""
        from . import _check
        _check(shard_lib().rtps_rx_shard_pack(self._h, arena.data_ptr(), arena.numel(), off.data_ptr(),
                                              outs["records"].data_ptr(), outs["n_records"].data_ptr(),
                                              outs["max_records"]))

    def counts(self, side="send"):
        b = self.buffers()
        p = b.send_counts if side == "send" else b.recv_counts
        torch.cuda.synchronize(self.device)
        return dev_to_numpy(p, self.world * 32, SHARD_COUNTS_DTYPE)

    def exchange(self):
        """Round 0 (RCCL: asynchronous on the exchange stream; gloo: the whole protocol)."""
        if self.host_collectives:
            return self._exchange_host()
        _check_comm(shard_lib().rtps_rx_shard_exchange(self._h, _live_comm(self),
                                                       ctypes.c_void_p(self.xstream.cuda_stream)), self)

    def finish(self):
        """Waits for round 0's counts; moves any spill (RCCL).  No-op after a gloo exchange."""
        if self.host_collectives:
            return
        _check_comm(shard_lib().rtps_rx_shard_finish(self._h, _live_comm(self),
                                                     ctypes.c_void_p(self.xstream.cuda_stream)), self)

    def unpack(self):
        """Owner side -> OwnerBatch (host sync on the received counts)."""
        from . import _check
        ob = _OwnerBatch()
        _check(shard_lib().rtps_rx_shard_unpack(self._h, ctypes.byref(ob)))
        return OwnerBatch(ob)

    def _exchange_host(self):
        """The protocol over torch.distributed with CPU tensors (gloo): counts, slots and
        blob slots with equal splits, then the spill with the exact splits round 0's counts
        give, into the library's receive buffers."""
        dist, w = self.dist, self.world
        torch.cuda.synchronize(self.device)
        b = self.buffers()
        sc = dev_to_numpy(b.send_counts, w * 32, SHARD_COUNTS_DTYPE)
        rc = _np.zeros(w, dtype=SHARD_COUNTS_DTYPE)
        self._a2a(sc.view(_np.uint8), rc.view(_np.uint8))
        dev_copy(b.recv_counts, rc.ctypes.data, rc.nbytes)
        for sp, rp, nb in ((b.send_slots, b.recv_slots, self.cap * ITEM_BYTES_OWNER), (b.send_blob, b.recv_blob,
                                                                                        self.bcap)):
            if nb:
                s_host = dev_to_numpy(sp, w * nb)
                r_host = _np.empty(w * nb, dtype=_np.uint8)
                self._a2a(s_host, r_host)
                dev_copy(rp, r_host.ctypes.data, r_host.nbytes)
        plan = spill_plan(sc, rc)
        rn = sum(p["recv_rec"][1] for p in plan)
        rbn = sum(p["recv_bytes"][1] for p in plan)
        anyn = sum(p["send_rec"][1] + p["send_bytes"][1] for p in plan) + rn + rbn
        self.last_spill = rn
        if dist is not None:
            t = torch.tensor([anyn], dtype=torch.int64)
            dist.all_reduce(t)  # gloo's all_to_all needs every rank; skip round 1 only if nobody spills
            anyn = int(t.item())
        if anyn:
            from . import _check
            _check(shard_lib().rtps_rx_shard_reserve_spill(self._h, rn, rbn))
            b = self.buffers()
            for key, sp, rp, unit in (("rec", b.send_spill, b.recv_spill, ITEM_BYTES_OWNER),
                                      ("bytes", b.send_blob_spill, b.recv_blob_spill, 1)):
                sends = [dev_to_numpy(sp + p[f"send_{key}"][0] * unit, p[f"send_{key}"][1] * unit) for p in plan]
                recv = _np.empty(sum(p[f"recv_{key}"][1] for p in plan) * unit, dtype=_np.uint8)
                self._a2a(_np.concatenate(sends) if sends else _np.zeros(0, _np.uint8), recv,
                          [len(x) for x in sends], [p[f"recv_{key}"][1] * unit for p in plan])
                dev_copy(rp, recv.ctypes.data, recv.nbytes)
        torch.cuda.synchronize(self.device)

    def _a2a(self, send, recv, send_splits=None, recv_splits=None):
        if self.dist is None:  # one rank: the exchange is a copy
            recv[:] = send
            return
        out = torch.from_numpy(recv)
        self.dist.all_to_all_single(out, torch.from_numpy(_np.ascontiguousarray(send)), recv_splits, send_splits)
