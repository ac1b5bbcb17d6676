"""Writer-GUID sharding of parsed records across GPUs.

Each rank parses its own contiguous chunk of datagrams; the records of the
writer and reader submessages are then partitioned by owner rank =
fnv1a32(prefix || writer_id) % world (stable, on the device:
rtps_rx_bucket_by_writer) and exchanged with ONE all-to-all.  The owner then
holds every record of its writers (ready for per-writer ordering, dedup and
fragment assembly).  The reference has a single process and no exchange;
this is the only collective of the path.
"""
import torch

RECORD_BYTES = 64


def owner_hash_words(words):
    """fnv1a32 over 4 little-endian u32 words, then h ^ (h >> 15) (same as the device)."""
    h = 0x811C9DC5
    for w in words:
        h = ((h ^ int(w)) * 0x01000193) & 0xFFFFFFFF
    return h ^ (h >> 15)


class Exchange:
    """Buffers + the exchange step for one rank."""

    def __init__(self, rx, max_records, world, dist, device):
        self.rx = rx
        self.world = world
        self.dist = dist
        self.device = device
        self.bucketed = torch.empty((max(max_records, 1), RECORD_BYTES), dtype=torch.uint8, device=device)
        self.counts = torch.zeros(world, dtype=torch.int64, device=device)
        self.recv_counts = torch.zeros(world, dtype=torch.int64, device=device)
        backend = dist.get_backend() if dist is not None else None
        self.host_collectives = backend == "gloo"  # gloo moves CPU tensors only

    def bucket(self, outs):
        """Stable partition of this rank's records by owner rank (asynchronous)."""
        self.rx.bucket_by_writer(outs, self.world, self.bucketed, self.counts)

    def exchange(self):
        """All-to-all of the bucketed records; returns this rank's received records [m, 64] u8."""
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
