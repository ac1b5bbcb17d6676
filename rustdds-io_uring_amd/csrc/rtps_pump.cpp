// rtps_pump.cpp — native receive loop: UDP arena -> GPU parse -> history-cache
// ingest -> CDR decode, batch by batch (include/rtps_rx.h, rtps_rx_pump).
//
// The reference's event loop handles one completion at a time
// (Domain::handle_event, io_uring/rtps/dp_event_loop.rs:162-211): take the
// provided buffer of the CQE, re-arm on ENOBUFS (traffic.rs:246-284), copy the
// datagram into a Bytes, parse it (handle_received_packet_2) and hand every
// submessage to its reader (dp_event_loop.rs:266-327).  Here one pass of the
// loop takes every datagram that has landed in the arena (rtps_udp_recv_batch),
// launches the batch's parse / ingest / decode on the context's stream, and
// only then finishes the previous batch (event wait, on_batch, slot release),
// so the host receives and the GPU works at the same time.  Batches size
// themselves to the traffic: a quiet link gives small, low-latency batches; a
// busy one fills max_batch.
#include <hip/hip_runtime_api.h>
#include <stdint.h>
#include <string.h>
#include <time.h>

#include <deque>
#include <utility>

#include "../../include/rtps_rx.h"
#include "rtps_ctx.h"

namespace {

uint64_t now_ns() {
  timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return (uint64_t)t.tv_sec * 1000000000ull + (uint64_t)t.tv_nsec;
}

void put(uint64_t* p, uint64_t v) { __atomic_store_n(p, v, __ATOMIC_RELAXED); }

struct Slot {              // host side of one in-flight batch
  uint64_t* off = nullptr;  // pinned [max_batch]: read by the GPU in place
  uint32_t* len = nullptr;
  uint64_t* cnt = nullptr;  // pinned [2]: n_records, n_accepted
  hipEvent_t ev = nullptr;
  uint32_t n = 0;
  uint64_t seq = 0;
  bool busy = false;
};

struct Pump {
  rtps_rx_ctx* ctx;
  rtps_udp_rx* udp;
  const uint8_t* arena;
  uint64_t arena_len;
  const rtps_pump_config* cfg;
  rtps_pump_stats* st;
  rtps_pump_stats acc{};
  hipStream_t stream;
  Slot slot[2];
  std::deque<std::pair<uint64_t, uint32_t>> carry;  // received, not yet in a batch (arrival order)
  uint64_t seq = 0;
  bool stop_requested = false;

  ~Pump() {
    for (Slot& s : slot) {
      if (s.off) (void)hipHostFree(s.off);
      if (s.len) (void)hipHostFree(s.len);
      if (s.cnt) (void)hipHostFree(s.cnt);
      if (s.ev) (void)hipEventDestroy(s.ev);
    }
  }

  void publish() {
    put(&st->datagrams, acc.datagrams);
    put(&st->completed, acc.completed);
    put(&st->batches, acc.batches);
    put(&st->records, acc.records);
    put(&st->accepted, acc.accepted);
    put(&st->truncated, acc.truncated);
    put(&st->first_ns, acc.first_ns);
    put(&st->last_ns, acc.last_ns);
  }

  int init() {
    const uint32_t mb = cfg->max_batch;
    for (Slot& s : slot) {
      if (hipHostMalloc(&s.off, mb * sizeof(uint64_t), hipHostMallocDefault) != hipSuccess ||
          hipHostMalloc(&s.len, mb * sizeof(uint32_t), hipHostMallocDefault) != hipSuccess ||
          hipHostMalloc(&s.cnt, 2 * sizeof(uint64_t), hipHostMallocDefault) != hipSuccess)
        return RTPS_RX_ENOMEM;
      if (hipEventCreateWithFlags(&s.ev, hipEventDisableTiming) != hipSuccess) return RTPS_RX_EHIP;
    }
    return RTPS_RX_OK;
  }

  // datagrams [k, n) of the batch do not fit its record capacity: back to the
  // front of the carry queue, ahead of anything received later
  void uncut(const Slot& s, uint32_t k, uint32_t n) {
    for (uint32_t i = n; i > k; --i) carry.emplace_front(s.off[i - 1], s.len[i - 1]);
  }

  int launch(Slot& s, uint32_t n, uint32_t b) {
    const rtps_pump_buffers& B = cfg->buffers[b];
    int rc = rtps_rx_parse_batch(ctx, arena, arena_len, s.off, s.len, n, &B.out);
    if (rc == RTPS_RX_OK && (cfg->flags & RTPS_PUMP_INGEST))
      rc = rtps_rx_ingest(ctx, arena, arena_len, s.off, B.out.records, B.out.n_records, B.out.max_records, nullptr,
                          nullptr, 0, cfg->ingest_flags, &B.ingest);
    if (rc == RTPS_RX_OK && (cfg->flags & RTPS_PUMP_CDR))
      rc = rtps_rx_cdr_decode(ctx, cfg->cdr_prog, cfg->cdr_n_ops, cfg->cdr_row_bytes, arena, arena_len, s.off,
                              B.out.records, B.out.n_records, B.out.max_records, B.rows, B.row_status);
    if (rc != RTPS_RX_OK) return rc;
    if (hipMemcpyAsync(&s.cnt[0], B.out.n_records, sizeof(uint64_t), hipMemcpyDeviceToHost, stream) != hipSuccess)
      return RTPS_RX_EHIP;
    s.cnt[1] = 0;
    if ((cfg->flags & RTPS_PUMP_INGEST) &&
        hipMemcpyAsync(&s.cnt[1], B.ingest.n_accepted, sizeof(uint64_t), hipMemcpyDeviceToHost, stream) != hipSuccess)
      return RTPS_RX_EHIP;
    if (hipEventRecord(s.ev, stream) != hipSuccess) return RTPS_RX_EHIP;
    s.n = n;
    s.seq = seq++;
    s.busy = true;
    acc.datagrams += n;
    acc.batches += 1;
    return RTPS_RX_OK;
  }

  int finish(Slot& s, uint32_t b) {
    if (!s.busy) return RTPS_RX_OK;
    s.busy = false;
    if (hipEventSynchronize(s.ev) != hipSuccess) return RTPS_RX_EHIP;
    acc.records += s.cnt[0];
    acc.accepted += s.cnt[1];
    if (cfg->on_batch) {
      rtps_pump_batch pb;
      pb.seq = s.seq;
      pb.buffer = b;
      pb.n_datagrams = s.n;
      pb.dgram_off = s.off;
      pb.dgram_len = s.len;
      pb.n_records = s.cnt[0];
      pb.n_accepted = s.cnt[1];
      if (cfg->on_batch(cfg->user, &pb) != 0) stop_requested = true;
    }
    int rc = rtps_udp_release(udp, s.off, s.n);
    acc.completed += s.n;
    acc.last_ns = now_ns();
    publish();
    return rc;
  }

  bool should_stop() const {
    if (stop_requested) return true;
    if (cfg->stop && *cfg->stop) return true;
    return cfg->stop_after && acc.datagrams >= cfg->stop_after;
  }

  int run() {
    uint32_t cur = 0;
    uint64_t idle_since = now_ns();
    int rc = RTPS_RX_OK;
    while (rc == RTPS_RX_OK && !should_stop()) {
      Slot& s = slot[cur];
      Slot& other = slot[cur ^ 1u];
      uint32_t want = cfg->max_batch;
      if (cfg->stop_after && cfg->stop_after - acc.datagrams < want) want = (uint32_t)(cfg->stop_after - acc.datagrams);
      uint32_t n = 0;
      while (n < want && !carry.empty()) {
        s.off[n] = carry.front().first;
        s.len[n] = carry.front().second;
        carry.pop_front();
        ++n;
      }
      if (n < want) {
        // wait for traffic only when nothing else is pending: an in-flight batch
        // is finished first so its outputs are not held back by a quiet link
        const int wait = (n || other.busy) ? 0 : cfg->wait_ms;
        uint64_t trunc = 0;
        const int r = rtps_udp_recv_batch(udp, s.off + n, s.len + n, want - n, wait, &trunc);
        if (r < 0) { rc = r; break; }
        acc.truncated += trunc;
        n += (uint32_t)r;
      }
      if (n == 0) {
        if (other.busy) { rc = finish(other, cur ^ 1u); continue; }
        publish();
        if (cfg->idle_stop_ms && now_ns() - idle_since >= (uint64_t)cfg->idle_stop_ms * 1000000ull) break;
        continue;
      }
      idle_since = now_ns();
      if (acc.first_ns == 0) acc.first_ns = idle_since;
      // cut the batch where its record bound would pass the output capacity
      const uint64_t cap = cfg->buffers[cur].out.max_records;
      uint64_t bound = 0;
      uint32_t k = 0;
      for (; k < n; ++k) {
        const uint32_t L = s.len[k];
        const uint64_t r = (L >= 20 && L <= RTPS_MAX_DATAGRAM) ? (L - 20u) / 4u : 0u;  // rtps_rx_max_records_host
        if (k && bound + r > cap) break;
        bound += r;
      }
      uncut(s, k, n);
      rc = launch(s, k, cur);
      if (rc != RTPS_RX_OK) {  // not in flight: wait for what was queued, then give its slots back
        (void)hipStreamSynchronize(stream);
        (void)rtps_udp_release(udp, s.off, k);
        break;
      }
      publish();
      cur ^= 1u;
      rc = finish(slot[cur], cur);  // the previous batch, while the GPU runs this one
    }
    // drain: finish what is in flight (oldest first), give back what was not batched
    const int rc0 = finish(slot[cur], cur);
    const int rc1 = finish(slot[cur ^ 1u], cur ^ 1u);
    if (rc == RTPS_RX_OK) rc = rc0 != RTPS_RX_OK ? rc0 : rc1;
    while (!carry.empty()) {
      uint64_t o = carry.front().first;
      carry.pop_front();
      (void)rtps_udp_release(udp, &o, 1);
    }
    publish();
    return rc;
  }
};

}  // namespace

extern "C" int rtps_rx_pump(rtps_rx_ctx* ctx, rtps_udp_rx* udp, const uint8_t* arena, uint64_t arena_len,
                            const rtps_pump_config* cfg, rtps_pump_stats* stats) {
  if (!ctx || !udp || !arena || !cfg || !stats || !cfg->buffers) return RTPS_RX_EINVAL;
  if (cfg->abi_version != RTPS_RX_ABI_VERSION) return RTPS_RX_EABI;
  if (cfg->flags & ~(RTPS_PUMP_INGEST | RTPS_PUMP_CDR)) return RTPS_RX_EINVAL;
  if (cfg->max_batch == 0 || cfg->max_batch > rtps_ctx_max_datagrams(ctx) || cfg->wait_ms < 0) return RTPS_RX_EINVAL;
  if ((cfg->flags & RTPS_PUMP_CDR) && (!cfg->cdr_prog || !cfg->cdr_n_ops)) return RTPS_RX_EINVAL;
  for (int b = 0; b < 2; ++b) {
    const rtps_pump_buffers& B = cfg->buffers[b];
    if (!B.out.status || !B.out.records || !B.out.n_records || !B.out.max_records) return RTPS_RX_EINVAL;
    if ((cfg->flags & RTPS_PUMP_INGEST) && (!B.ingest.accept || !B.ingest.accepted || !B.ingest.n_accepted))
      return RTPS_RX_EINVAL;
    if ((cfg->flags & RTPS_PUMP_CDR) && (!B.rows || !B.row_status)) return RTPS_RX_EINVAL;
  }
  memset(stats, 0, sizeof(*stats));
  (void)hipSetDevice(rtps_ctx_device(ctx));
  Pump p{ctx, udp, arena, arena_len, cfg, stats};
  p.stream = rtps_ctx_stream(ctx);
  int rc = p.init();
  if (rc != RTPS_RX_OK) return rc;
  return p.run();
}
