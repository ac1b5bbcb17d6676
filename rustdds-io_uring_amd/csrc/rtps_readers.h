// rtps_readers.h — the context's local readers and writer proxies, turned into
// target sets (include/rtps_rx.h, "local readers and their writer proxies").
// Internal: used by the parse (rtps_rx.hip), the exchange buckets and the
// ingest (rtps_ingest.hip).  Host builder in rtps_readers.cpp.
//
// Classification restated (a15):
//   Domain::handle_event user path   io_uring/rtps/dp_event_loop.rs:266-327
//     available_readers.values_mut().filter(contains_writer(writer_entity_id))
//   Reader::contains_writer          io_uring/rtps/reader.rs:474-484
//   matched_writers lookup by GUID   io_uring/rtps/reader.rs:712-739
// Every possible outcome is precomputed on the host as a target set, so the
// device does one or two hash probes per writer record: the full writer GUID
// (writer sets), and on a miss its entity id (entity sets).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/rtps_rx.h"

// The six arrays are one device buffer, in this order and with no gaps (the LDS image of
// rt_stage, then set_first and set_ent): staging copies one flat range of gkeys.
struct ReaderDev {             // device view (kernel argument by value); gkeys == nullptr: no readers
  const uint32_t* gkeys;       // [gmask + 1] x 4 words: writer GUID keys (prefix || entity id, raw LE words)
  const uint32_t* gset;        // [gmask + 1] writer set of the slot, RTPS_NO_TARGET = empty slot
  const uint32_t* ekeys;       // [emask + 1] writer entity ids (raw LE word)
  const uint32_t* eset;        // [emask + 1] entity set of the slot, RTPS_NO_TARGET = empty slot
  const uint32_t* set_first;   // [n_sets + 1]
  const rtps_target* set_ent;  // [set_first[n_sets]]
  uint32_t gmask, emask;
  uint32_t n_writer_sets, n_sets, n_proxies, max_set;
  uint32_t n_ent;              // set_first[n_sets]: target entries of all sets
};

__host__ __device__ inline uint32_t rt_hash16(uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
  uint32_t h = 0x811c9dc5u;  // FNV-1a over the four words, then a fold
  h = (h ^ a) * 0x01000193u; h = (h ^ b) * 0x01000193u;
  h = (h ^ c) * 0x01000193u; h = (h ^ d) * 0x01000193u;
  return h ^ (h >> 15);
}
__host__ __device__ inline uint32_t rt_hash4(uint32_t e) {
  uint32_t h = (0x811c9dc5u ^ e) * 0x01000193u;
  h = (h ^ (h >> 13)) * 0x01000193u;
  return h ^ (h >> 15);
}

// LDS image of the two hash tables: gkeys (16 B), gset, ekeys, eset per slot.
__host__ __device__ constexpr uint32_t rt_lds_bytes(uint32_t gcap, uint32_t ecap) { return gcap * 20u + ecap * 8u; }
constexpr uint32_t RT_LDS_MAX = 48u * 1024u;  // larger tables are probed in global memory (L2)
// hash slots per key: 4 (load <= 1/4: short probe runs, a wave waits for its longest) while the
// tables fit RT_LDS_MAX, else 2
constexpr uint32_t RT_SLACK = 4u, RT_SLACK_MIN = 2u;
__host__ __device__ inline bool rt_fits_lds(const ReaderDev& r) {
  return r.gkeys != nullptr && rt_lds_bytes(r.gmask + 1u, r.emask + 1u) <= RT_LDS_MAX;
}

#ifdef __HIPCC__
// n words from src (global, 16-B aligned) to dst (LDS, 16-B aligned) by the workgroup: 16-B
// loads, four in flight per thread before their stores.  Caller syncs.
__device__ inline void rt_copy(uint32_t* dst, const uint32_t* src, uint32_t n) {
  const uint32_t n4 = n / 4u, bs = blockDim.x;
  const uint4* s4 = reinterpret_cast<const uint4*>(src);
  uint4* d4 = reinterpret_cast<uint4*>(dst);
  uint32_t k = threadIdx.x;
  for (; k + 3u * bs < n4; k += 4u * bs) {
    const uint4 a = s4[k], b = s4[k + bs], c = s4[k + 2u * bs], d = s4[k + 3u * bs];
    d4[k] = a; d4[k + bs] = b; d4[k + 2u * bs] = c; d4[k + 3u * bs] = d;
  }
  for (; k < n4; k += bs) d4[k] = s4[k];
  for (uint32_t i = n4 * 4u + threadIdx.x; i < n; i += bs) dst[i] = src[i];
}
// words of the tables' LDS image; with the target sets (set_first, set_ent) behind them
__host__ __device__ inline uint32_t rt_lds_words(const ReaderDev& r) { return rt_lds_bytes(r.gmask + 1u, r.emask + 1u) / 4u; }
__host__ __device__ inline uint32_t rt_image_words(const ReaderDev& r) { return rt_lds_words(r) + r.n_sets + 1u + 2u * r.n_ent; }
// Stage the tables into dynamic shared memory `lds` (uint32 words, 16-B aligned).  Caller syncs.
__device__ inline void rt_stage(const ReaderDev& r, uint32_t* lds) { rt_copy(lds, r.gkeys, rt_lds_words(r)); }
// writer set of the full GUID (a, b, c = prefix words, d = entity id), or RTPS_NO_TARGET
template <bool LDS>
__device__ __forceinline__ uint32_t rt_writer_set(const ReaderDev& r, const uint32_t* lds, uint32_t a, uint32_t b,
                                                  uint32_t c, uint32_t d) {
  const uint32_t* keys = LDS ? lds : r.gkeys;
  const uint32_t* sets = LDS ? lds + (r.gmask + 1u) * 4u : r.gset;
  uint32_t i = rt_hash16(a, b, c, d) & r.gmask;
  for (uint32_t probe = 0; probe <= r.gmask; ++probe) {
    // the slot's set and key loaded together (one LDS round trip per probe)
    const uint32_t s = sets[i];
    const uint4 k = *reinterpret_cast<const uint4*>(keys + 4u * i);
    if (s == RTPS_NO_TARGET) return RTPS_NO_TARGET;
    if (k.x == a && k.y == b && k.z == c && k.w == d) return s;
    i = (i + 1u) & r.gmask;
  }
  return RTPS_NO_TARGET;
}
template <bool LDS>
__device__ __forceinline__ uint32_t rt_entity_set(const ReaderDev& r, const uint32_t* lds, uint32_t d) {
  const uint32_t gcap = r.gmask + 1u;
  const uint32_t* keys = LDS ? lds + gcap * 5u : r.ekeys;
  const uint32_t* sets = LDS ? lds + gcap * 5u + r.emask + 1u : r.eset;
  uint32_t i = rt_hash4(d) & r.emask;
  for (uint32_t probe = 0; probe <= r.emask; ++probe) {
    const uint32_t s = sets[i], k = keys[i];
    if (s == RTPS_NO_TARGET) return RTPS_NO_TARGET;
    if (k == d) return s;
    i = (i + 1u) & r.emask;
  }
  return RTPS_NO_TARGET;
}
// Target set of a writer-kind record that is not a builtin pair; route gets
// RTPS_ROUTE_MATCHED | TARGETED (writer set) or TARGETED (entity set).
template <bool LDS>
__device__ __forceinline__ uint32_t rt_classify(const ReaderDev& r, const uint32_t* lds, uint32_t a, uint32_t b,
                                                uint32_t c, uint32_t d, uint32_t& route) {
  if (r.gkeys == nullptr) return RTPS_NO_TARGET;
  uint32_t t = rt_writer_set<LDS>(r, lds, a, b, c, d);
  if (t != RTPS_NO_TARGET) { route |= RTPS_ROUTE_MATCHED | RTPS_ROUTE_TARGETED; return t; }
  t = rt_entity_set<LDS>(r, lds, d);
  if (t != RTPS_NO_TARGET) route |= RTPS_ROUTE_TARGETED;
  return t;
}
#endif

// ---- host side (rtps_readers.cpp) ----
struct ReaderTable;
ReaderTable* rt_new();
void rt_free(ReaderTable* t);
// Validate and build the target sets; uploads the device tables (synchronous).
int rt_set(ReaderTable* t, const rtps_reader* readers, uint32_t n_readers, const rtps_proxy* proxies,
           uint32_t n_proxies, hipStream_t stream);
// The compatibility form (rtps_match pairs).
int rt_set_match(ReaderTable* t, const rtps_match* m, uint32_t n, hipStream_t stream);
ReaderDev rt_dev(const ReaderTable* t);  // gkeys == nullptr when no reader is set
void rt_host(const ReaderTable* t, const uint32_t** first, const rtps_target** ent, uint32_t* n_sets);
// the writer GUIDs of the writer sets 0 .. n-1 (16 bytes each, contiguous), nullptr when none
const uint8_t* rt_writer_guids(const ReaderTable* t, uint32_t* n);
// the writer entity ids of the entity sets n_writer_sets .. n_sets - 1 (4 bytes each), nullptr when none
const uint8_t* rt_entity_ids(const ReaderTable* t, uint32_t* n);
