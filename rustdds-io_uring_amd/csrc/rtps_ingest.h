// rtps_ingest.h — internal interface of the history-cache ingest (rtps_ingest.hip)
// used by the C ABI in rtps_rx.hip.  Not installed; see include/rtps_rx.h.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/rtps_rx.h"
#include "rtps_readers.h"

struct IngestState;  // persistent per-proxy writer-proxy state + per-batch scratch

IngestState* rtps_ingest_state_new(int device);
void rtps_ingest_state_free(IngestState* s);
// Every writer proxy back to RtpsWriterProxy::new (asynchronous on `stream`).
int rtps_ingest_state_reset(IngestState* s, hipStream_t stream);
// Work queued behind a batch's deliveries (the topic caches): run(ctx, gate) queues it on the
// stream.  gate (device u64) non-null: the work must do nothing unless *gate != 0 when it runs.
struct IngestTail {
  int (*run)(void* ctx, const uint64_t* gate);
  void* ctx;
};
// One batch (asynchronous on `stream`); returns an RTPS_RX_* code.  `t`: the
// context's readers (target sets, proxies).  tail (optional): queued after the batch's
// deliveries.  The global identity path is queued before the host learns whether the batch
// takes it (its verdict on the device), and the tail right behind it, gated by that verdict, so
// that the device runs on without waiting for the host's launches; other paths queue it after
// their last launch, ungated.
int rtps_ingest_batch(IngestState* s, hipStream_t stream, const ReaderDev& t, const uint8_t* arena,
                      uint64_t arena_len, const uint64_t* dgram_off, const rtps_record* records,
                      const uint64_t* n_records, uint64_t max_records, const rtps_frag_sample* frag,
                      const uint64_t* n_frag, uint64_t max_frag, uint32_t flags, const rtps_ingest_out* out,
                      const IngestTail* tail = nullptr);
// Test / measurement hook: 0 = path chosen per batch, 1 = global marks / merge,
// 2 = per-proxy workgroups (results are the same).
void rtps_ingest_set_path(IngestState* s, uint32_t path);
// Tuning builds with RTPS_PROXY_STAMPS: the per-proxy phase sums of the last per-proxy batch.
int rtps_ingest_proxy_stamps(uint64_t* host, uint64_t n);
