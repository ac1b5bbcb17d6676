// rtps_exchange.cpp — the multi-GPU exchange of the sharded path over RCCL.
//
// One rank per GPU parses its contiguous chunk of datagrams; the writer /
// reader records are bucketed by owner rank on the device
// (rtps_rx_bucket_by_writer_padded: owner = fnv1a32(prefix || writer_id) % world,
// or rtps_rx_bucket_descriptors) into fixed-capacity buckets, and this file
// moves bucket d to rank d: ONE grouped ncclSend / ncclRecv per peer
// (ncclGroupStart / ncclGroupEnd) of the equal-split buckets plus their true
// counts, on the context's stream.  Equal splits need no device-to-host round
// trip, so the exchange of batch k runs while batch k+1 is parsed.  The
// reference has one process and no collective; this is the path's only one.
// xGMI is point-to-point (one link per peer pair on an 8-GPU MI355X node), so
// per-peer send/recv is the natural all-to-all there.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <string.h>

#include "../../include/rtps_rx.h"
#include "rtps_ctx.h"

static_assert(RTPS_RX_EXCHANGE_ID_BYTES == NCCL_UNIQUE_ID_BYTES, "unique id size");

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
  (void)me;
  if (hipSetDevice(rtps_ctx_device(ctx)) != hipSuccess) return RTPS_RX_EHIP;
  hipStream_t st = hip_stream ? (hipStream_t)hip_stream : rtps_ctx_stream(ctx);
  const size_t bytes = (size_t)cap * item_bytes;
  const uint8_t* s = static_cast<const uint8_t*>(send);
  uint8_t* r = static_cast<uint8_t*>(recv);
  if (ncclGroupStart() != ncclSuccess) return RTPS_RX_EHIP;
  bool ok = true;
  for (int p = 0; p < world && ok; ++p) {
    ok = ncclSend(send_counts + p, 1, ncclUint64, p, c, st) == ncclSuccess &&
         ncclRecv(recv_counts + p, 1, ncclUint64, p, c, st) == ncclSuccess &&
         ncclSend(s + (size_t)p * bytes, bytes, ncclUint8, p, c, st) == ncclSuccess &&
         ncclRecv(r + (size_t)p * bytes, bytes, ncclUint8, p, c, st) == ncclSuccess;
  }
  const bool ended = ncclGroupEnd() == ncclSuccess;
  return ok && ended ? RTPS_RX_OK : RTPS_RX_EHIP;
}

}  // extern "C"
