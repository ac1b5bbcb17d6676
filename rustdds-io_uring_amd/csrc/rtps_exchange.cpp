// rtps_exchange.cpp — the multi-GPU exchange of the sharded path over RCCL.
//
// One rank per GPU parses its contiguous chunk of datagrams; the writer /
// reader records are bucketed by owner rank on the device
// (rtps_rx_bucket_by_writer_padded: owner = fmix32(fnv1a32(prefix || writer_id))
// % world, or rtps_rx_bucket_descriptors) into fixed-capacity buckets, and this file
// moves bucket d to rank d: ONE grouped ncclSend / ncclRecv per peer
// (ncclGroupStart / ncclGroupEnd) of the equal-split buckets plus their true
// counts, on the context's stream.  Equal splits need no device-to-host round
// trip, so the exchange of batch k runs while batch k+1 is parsed.  The
// reference has one process and no collective; this is the path's only one.
// xGMI is point-to-point (one link per peer pair on an 8-GPU MI355X node), so
// per-peer send/recv is the natural all-to-all there.
//
// The owner-side exchange (rtps_rx_shard_exchange / _finish, state in
// rtps_shard.h) moves what the owner's fragment assembly and ingest consume:
// round 0 is the same equal-split group (counts, record slot, blob slot per
// peer); round 1 moves, only for the pairs whose items did not fit the slots,
// the exact remainder, whose size both ends read from round 0's counts.
//
// Failure: if enqueuing a send or receive fails part-way, the peers would wait
// for operations that were never posted, so the group is ended and the
// communicator aborted (ncclCommAbort, which frees it): the caller gets
// RTPS_RX_EABORTED, must forget the handle (never destroy it) and make a new
// communicator.  Every failure of rtps_rx_shard_finish aborts too: the peers post
// their spill rounds after round 0, so a rank that returns without its own would
// leave them waiting.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <string.h>

#include "../../include/rtps_rx.h"
#include "rtps_ctx.h"
#include "rtps_shard.h"

static_assert(RTPS_RX_EXCHANGE_ID_BYTES == NCCL_UNIQUE_ID_BYTES, "unique id size");

// Point-to-point messages are cut into pieces of at most XCHUNK bytes, posted in
// order inside the same group (NCCL matches a peer's sends and receives in
// order).  The cause (round 5, scripts/rccl_size_probe.py, profiles/r5_rccl_size_probe.json:
// ONE unchunked ncclSend + ncclRecv pair per size, pattern-filled, through
// rtps_rx_debug_rccl_p2p): this image's RCCL 2.26.6 delivers a single point-to-point
// message of up to 2^30 bytes whole, and of any larger size (2^30 + 4 B, 1.125, 1.25, 1.5,
// 2, 2.25 GiB) only its first half: the first wrong byte is at n / 2 every time.  It is
// RCCL's, not this library's size handling (the probe passes the byte count straight to
// ncclSend / ncclRecv as size_t).  So no message may exceed 2^30 bytes; 64-MB pieces keep
// well inside that and let the group's pieces pipeline.  (The probe is a self-send, the only
// pair a one-GPU box has; the exchanges no longer send to self: the own slot is a device copy.)
constexpr size_t XCHUNK = size_t(64) << 20;
static_assert(XCHUNK <= (size_t(1) << 30), "RCCL 2.26 delivers p2p messages of at most 2^30 bytes whole");
static bool send_bytes(const void* buf, size_t n, int peer, ncclComm_t c, hipStream_t st) {
  const uint8_t* p = static_cast<const uint8_t*>(buf);
  for (size_t o = 0; o < n; o += XCHUNK) {
    const size_t k = n - o < XCHUNK ? n - o : XCHUNK;
    if (ncclSend(p + o, k, ncclUint8, peer, c, st) != ncclSuccess) return false;
  }
  return true;
}
static bool recv_bytes(void* buf, size_t n, int peer, ncclComm_t c, hipStream_t st) {
  uint8_t* p = static_cast<uint8_t*>(buf);
  for (size_t o = 0; o < n; o += XCHUNK) {
    const size_t k = n - o < XCHUNK ? n - o : XCHUNK;
    if (ncclRecv(p + o, k, ncclUint8, peer, c, st) != ncclSuccess) return false;
  }
  return true;
}

// the communicator is unusable (a group was cut short): abort (frees it) and say so
static int abort_comm(ncclComm_t c) {
  (void)ncclCommAbort(c);
  return RTPS_RX_EABORTED;
}

extern "C" {

int rtps_rx_exchange_unique_id(uint8_t id[RTPS_RX_EXCHANGE_ID_BYTES]) {
  if (!id) return RTPS_RX_EINVAL;
  ncclUniqueId u;
  if (ncclGetUniqueId(&u) != ncclSuccess) return RTPS_RX_EHIP;
  memcpy(id, u.internal, NCCL_UNIQUE_ID_BYTES);
  return RTPS_RX_OK;
}

int rtps_rx_exchange_comm_init(const uint8_t id[RTPS_RX_EXCHANGE_ID_BYTES], int n_ranks, int rank, int device,
                               void** comm) {
  if (!id || !comm || n_ranks < 1 || rank < 0 || rank >= n_ranks) return RTPS_RX_EINVAL;
  if (hipSetDevice(device) != hipSuccess) return RTPS_RX_EHIP;
  ncclUniqueId u;
  memcpy(u.internal, id, NCCL_UNIQUE_ID_BYTES);
  ncclComm_t c = nullptr;
  if (ncclCommInitRank(&c, n_ranks, u, rank) != ncclSuccess) return RTPS_RX_EHIP;
  *comm = c;
  return RTPS_RX_OK;
}

int rtps_rx_exchange_comm_destroy(void* comm) {
  if (!comm) return RTPS_RX_EINVAL;
  return ncclCommDestroy((ncclComm_t)comm) == ncclSuccess ? RTPS_RX_OK : RTPS_RX_EHIP;
}

int rtps_rx_exchange(rtps_rx_ctx* ctx, void* comm, void* hip_stream, const void* send, const uint64_t* send_counts,
                     uint64_t cap, uint32_t item_bytes, void* recv, uint64_t* recv_counts) {
  if (!ctx || !comm || !send || !send_counts || !recv || !recv_counts || !cap || !item_bytes) return RTPS_RX_EINVAL;
  ncclComm_t c = (ncclComm_t)comm;
  int world = 0, me = 0;
  if (ncclCommCount(c, &world) != ncclSuccess || ncclCommUserRank(c, &me) != ncclSuccess) return RTPS_RX_EHIP;
  if (hipSetDevice(rtps_ctx_device(ctx)) != hipSuccess) return RTPS_RX_EHIP;
  hipStream_t st = hip_stream ? (hipStream_t)hip_stream : rtps_ctx_stream(ctx);
  const size_t bytes = (size_t)cap * item_bytes;
  const uint8_t* s = static_cast<const uint8_t*>(send);
  uint8_t* r = static_cast<uint8_t*>(recv);
  // this rank's own bucket: a device copy on the same stream, not an RCCL self-send
  if (hipMemcpyAsync(recv_counts + me, send_counts + me, sizeof(uint64_t), hipMemcpyDeviceToDevice, st) != hipSuccess ||
      hipMemcpyAsync(r + (size_t)me * bytes, s + (size_t)me * bytes, bytes, hipMemcpyDeviceToDevice, st) != hipSuccess)
    return RTPS_RX_EHIP;
  if (ncclGroupStart() != ncclSuccess) return RTPS_RX_EHIP;
  bool ok = true;
  for (int p = 0; p < world && ok; ++p) {
    if (p == me) continue;
    ok = ncclSend(send_counts + p, 1, ncclUint64, p, c, st) == ncclSuccess &&
         ncclRecv(recv_counts + p, 1, ncclUint64, p, c, st) == ncclSuccess &&
         send_bytes(s + (size_t)p * bytes, bytes, p, c, st) && recv_bytes(r + (size_t)p * bytes, bytes, p, c, st);
  }
  const bool ended = ncclGroupEnd() == ncclSuccess;
  if (!ok || !ended) return abort_comm(c);
  return RTPS_RX_OK;
}

int rtps_rx_shard_exchange(rtps_shard* s, void* comm, void* hip_stream) {
  if (!s || !comm) return RTPS_RX_EINVAL;
  ncclComm_t c = (ncclComm_t)comm;
  int world = 0, me = 0;
  if (ncclCommCount(c, &world) != ncclSuccess || ncclCommUserRank(c, &me) != ncclSuccess) return RTPS_RX_EHIP;
  if ((uint32_t)world != s->n_ranks) return RTPS_RX_EINVAL;
  if (hipSetDevice(s->device) != hipSuccess) return RTPS_RX_EHIP;
  hipStream_t st = hip_stream ? (hipStream_t)hip_stream : rtps_ctx_stream(s->ctx);
  if (hipStreamWaitEvent(st, s->packed, 0) != hipSuccess) return RTPS_RX_EHIP;  // the slots are complete
  const size_t rb = (size_t)s->cap * sizeof(shard_item), bb = (size_t)s->bcap;
  const size_t cw = sizeof(rtps_shard_counts) / sizeof(uint64_t);
  // this rank's own slot: device copies on the same stream, not an RCCL self-send
  if (hipMemcpyAsync(s->r_counts + me, s->s_counts + me, sizeof(rtps_shard_counts), hipMemcpyDeviceToDevice, st) !=
          hipSuccess ||
      hipMemcpyAsync(reinterpret_cast<uint8_t*>(s->r_slots) + me * rb,
                     reinterpret_cast<const uint8_t*>(s->s_slots) + me * rb, rb, hipMemcpyDeviceToDevice, st) !=
          hipSuccess ||
      hipMemcpyAsync(s->r_blob + me * bb, s->s_blob + me * bb, bb, hipMemcpyDeviceToDevice, st) != hipSuccess)
    return RTPS_RX_EHIP;
  if (ncclGroupStart() != ncclSuccess) return RTPS_RX_EHIP;
  bool ok = true;
  for (int p = 0; p < world && ok; ++p) {
    if (p == me) continue;
    ok = ncclSend(s->s_counts + p, cw, ncclUint64, p, c, st) == ncclSuccess &&
         ncclRecv(s->r_counts + p, cw, ncclUint64, p, c, st) == ncclSuccess &&
         send_bytes(reinterpret_cast<const uint8_t*>(s->s_slots) + p * rb, rb, p, c, st) &&
         recv_bytes(reinterpret_cast<uint8_t*>(s->r_slots) + p * rb, rb, p, c, st) &&
         send_bytes(s->s_blob + p * bb, bb, p, c, st) && recv_bytes(s->r_blob + p * bb, bb, p, c, st);
  }
  const bool ended = ncclGroupEnd() == ncclSuccess;
  if (!ok || !ended) return abort_comm(c);
  const size_t nb = (size_t)world * sizeof(rtps_shard_counts);
  if (hipMemcpyAsync(s->h_send, s->s_counts, nb, hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipMemcpyAsync(s->h_recv, s->r_counts, nb, hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipEventRecord(s->counts_ev, st) != hipSuccess || hipEventRecord(s->done, st) != hipSuccess)
    return RTPS_RX_EHIP;
  s->exchanged = true;
  s->finished = false;
  return RTPS_RX_OK;
}

int rtps_rx_shard_finish(rtps_shard* s, void* comm, void* hip_stream) {
  if (!s || !comm) return RTPS_RX_EINVAL;
  if (!s->exchanged) return RTPS_RX_EINVAL;  // no round 0 to finish
  ncclComm_t c = (ncclComm_t)comm;
  // from here on every failure aborts: the peers post their spill rounds regardless
  if (hipSetDevice(s->device) != hipSuccess) return abort_comm(c);
  hipStream_t st = hip_stream ? (hipStream_t)hip_stream : rtps_ctx_stream(s->ctx);
  if (hipEventSynchronize(s->counts_ev) != hipSuccess) return abort_comm(c);
  const uint32_t world = s->n_ranks;
  // spill sizes: what this rank still sends to each peer, what it still receives
  uint64_t need_r = 0, need_b = 0, any = 0;
  for (uint32_t p = 0; p < world; ++p) {
    const rtps_shard_counts& r = s->h_recv[p];
    const rtps_shard_counts& q = s->h_send[p];
    if (r.cut > r.n || r.cut_bytes > r.bytes || q.cut > q.n || q.cut_bytes > q.bytes) return abort_comm(c);
    need_r += r.n - r.cut;
    need_b += r.bytes - r.cut_bytes;
    any |= (r.n - r.cut) | (q.n - q.cut) | (r.bytes - r.cut_bytes) | (q.bytes - q.cut_bytes);
  }
  if (!any) {
    s->finished = true;
    return RTPS_RX_OK;
  }
  if (rtps_rx_shard_reserve_spill(s, need_r, need_b) != RTPS_RX_OK) return abort_comm(c);  // spill not receivable
  int me = 0;
  if (ncclCommUserRank(c, &me) != ncclSuccess) return abort_comm(c);
  if (ncclGroupStart() != ncclSuccess) return abort_comm(c);
  bool ok = true;
  uint64_t sb = 0, sbb = 0, rs = 0, rsb = 0;  // send-side exact-layout bases, receive-side spill offsets
  for (uint32_t p = 0; p < world && ok; ++p) {
    const rtps_shard_counts& q = s->h_send[p];
    const rtps_shard_counts& r = s->h_recv[p];
    const uint64_t sn = q.n - q.cut, sbytes = q.bytes - q.cut_bytes, rn = r.n - r.cut, rbytes = r.bytes - r.cut_bytes;
    if ((int)p == me)  // this rank's own spill (sn == rn): device copies, not an RCCL self-send
      ok = (!sn || hipMemcpyAsync(s->r_spill + rs, s->s_spill + sb + q.cut, sn * sizeof(shard_item),
                                  hipMemcpyDeviceToDevice, st) == hipSuccess) &&
           (!sbytes || hipMemcpyAsync(s->r_bspill + rsb, s->s_bspill + sbb + q.cut_bytes, sbytes,
                                      hipMemcpyDeviceToDevice, st) == hipSuccess);
    else
      ok = send_bytes(s->s_spill + sb + q.cut, sn * sizeof(shard_item), (int)p, c, st) &&
           send_bytes(s->s_bspill + sbb + q.cut_bytes, sbytes, (int)p, c, st) &&
           recv_bytes(s->r_spill + rs, rn * sizeof(shard_item), (int)p, c, st) &&
           recv_bytes(s->r_bspill + rsb, rbytes, (int)p, c, st);
    sb += q.n;
    sbb += q.bytes;
    rs += rn;
    rsb += rbytes;
  }
  const bool ended = ncclGroupEnd() == ncclSuccess;
  if (!ok || !ended) return abort_comm(c);
  if (hipEventRecord(s->done, st) != hipSuccess) return abort_comm(c);
  s->finished = true;
  return RTPS_RX_OK;
}

/* diagnostic hook (not in the public header; scripts/rccl_size_probe.py): ONE unchunked
   ncclSend + ncclRecv of `bytes` bytes between this rank and `peer` in one group on
   hip_stream, to find the message sizes RCCL delivers whole (the reason for XCHUNK). */
int rtps_rx_debug_rccl_p2p(void* comm, void* hip_stream, const void* send, void* recv, uint64_t bytes, int peer) {
  if (!comm || !send || !recv) return RTPS_RX_EINVAL;
  ncclComm_t c = (ncclComm_t)comm;
  hipStream_t st = (hipStream_t)hip_stream;
  if (ncclGroupStart() != ncclSuccess) return RTPS_RX_EHIP;
  const bool ok = ncclSend(send, (size_t)bytes, ncclUint8, peer, c, st) == ncclSuccess &&
                  ncclRecv(recv, (size_t)bytes, ncclUint8, peer, c, st) == ncclSuccess;
  const bool ended = ncclGroupEnd() == ncclSuccess;
  if (!ok || !ended) return abort_comm(c);
  return RTPS_RX_OK;
}

}  // extern "C"
