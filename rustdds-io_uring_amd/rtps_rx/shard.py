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
  * "descriptors": 16-byte rtps_xdesc of the MATCHED records only, owner =
    writer set index % world (rtps_rx_bucket_descriptors): 4x fewer
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
        _check(L.rtps_rx_exchange(self.rx._h, self.comm, ctypes.c_void_p(self.xstream.cuda_stream),
                                  self.bucketed.data_ptr(), self.counts.data_ptr(), self.cap,
                                  ITEM_BYTES[self.item], self.received.data_ptr(), self.recv_counts.data_ptr()))
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
