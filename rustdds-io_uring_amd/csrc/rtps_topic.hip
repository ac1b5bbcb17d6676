// rtps_topic.hip — the topic caches' TopicCache::add_change on the device
// ("writer-proxy dedup and TopicCache::add_change").
//
// The reference hands every change a reader accepts (process_received_data ==
// true, io_uring/rtps/reader.rs:693-758) to the reader's topic cache
// (make_cache_change :1185-1205), whose add_change (structure/dds_cache.rs:210-284)
//   1. garbage-collects when the change's SN is a multiple of 64: the oldest
//      changes go until at most max_keep remain (remove_changes_before(ZERO),
//      :367-420: `ts < ZERO` never holds, so only the must-remove count applies);
//   2. stores the change unless the topic already holds (writer GUID, SN).
// The changes map is keyed by receive instant, i.e. insertion order, and only the
// oldest are ever removed, so with I = insertions so far and E = removals so far
// the live changes are exactly the insertions [E, I) and a GC sets
// E = max(E, I - max_keep).  A delivery's change is stored iff its key's last
// insertion index is < E at that moment (or it never was inserted).
//
// A batch's deliveries are decided at once:
//   * topic order: the deliveries are stably grouped by topic (radix sort of the
//     topic index; one topic: no sort), so that per-topic counts are scans;
//   * most deliveries cannot be duplicates: a topic with ONE reader that is not
//     the SPDP reader (DUPLICATES_OK) receives each user-kind (writer GUID, SN)
//     through that reader's writer proxy, which accepted it only if it never saw
//     it (rtps_rx_ingest), and the proxy has seen every change the topic holds
//     unless it was created or reset after they were stored (tracked per topic:
//     `until`).  Those deliveries are stored, unchecked ("certain");
//   * every other delivery is a candidate: a later delivery of the same record to
//     the same topic (another reader of it) is a duplicate whatever the GC does
//     (max_keep >= 1 keeps the change just stored); the first delivery of a key in
//     the batch that the topic does not hold live is stored; the rest, "repeats"
//     (the key was stored by an earlier record of this batch, or is held from an
//     earlier batch), are rare and decided by one thread per topic in order
//     (tc_resolve), with the topic's insertion count at any position from a scan
//     of the decided insertions and its E from the last GC position (a max-scan);
//   * the changes that survive the batch (index >= the new E) go into the live
//     index (a hash table key -> insertion index) that later batches consult.
// The CPU restatement the tests hold this to (oracle/, test-only) is the
// reference's sequential add_change.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <stdlib.h>
#include <string.h>

#include <chrono>
#include <new>
#include <vector>

#include "rtps_sort.h"
#include "rtps_topic.h"

namespace {

constexpr uint32_t TT = 256;
constexpr uint32_t NSLOT = 65536;
constexpr uint32_t NONE = 0xffffffffu;
constexpr uint64_t NO_IDX = ~0ull;
constexpr uint32_t DEFAULT_KEEP = 64;  // ResourceLimits::max_samples default (dds_cache.rs:175-183)

struct KeyP {  // one delivery's change
  uint32_t g[4];        // writer GUID: prefix || writer_id, raw words
  uint32_t snlo, snhi;  // SN
  uint32_t tid;         // topic (stable id)
  uint32_t rec;         // record index, NONE: no change (outside the batch)
};
static_assert(sizeof(KeyP) == 32, "KeyP");

// the live index: key -> index of the key's last insertion (live iff >= the topic's E)
struct PEnt {
  uint32_t fp;     // key fingerprint (| 1), 0 = empty
  uint32_t ready;  // the key fields are written
  uint32_t g[4];
  uint32_t snlo, snhi, tid, _p;
  uint64_t idx;
};
// the batch's candidates: key -> first position, the last in-batch insertion index
struct BEnt {
  uint64_t tag;    // epoch << 32 | fingerprint: claimed in this batch
  uint32_t ready;  // epoch once the key fields are written
  uint32_t minp;
  uint32_t g[4];
  uint32_t snlo, snhi, tid, _p;
  uint64_t last;   // NO_IDX until the resolver stores a repeat of the key
  uint32_t nrep;   // the key's repeats in this batch (tc_class)
  uint32_t _q;
};
static_assert(sizeof(PEnt) == 48 && sizeof(BEnt) == 64, "entries");

__device__ __forceinline__ uint64_t key_hash(const KeyP& k) {
  uint64_t h = 0xcbf29ce484222325ull ^ k.tid;
  h = (h ^ k.g[0]) * 0x100000001b3ull; h = (h ^ k.g[1]) * 0x100000001b3ull;
  h = (h ^ k.g[2]) * 0x100000001b3ull; h = (h ^ k.g[3]) * 0x100000001b3ull;
  h = (h ^ k.snlo) * 0x100000001b3ull; h = (h ^ k.snhi) * 0x100000001b3ull;
  h ^= h >> 33; h *= 0xff51afd7ed558ccdull; h ^= h >> 33;
  return h;
}
__device__ __forceinline__ uint32_t fp_of(uint64_t h) { return (uint32_t)(h >> 32) | 1u; }
template <class E>
__device__ __forceinline__ bool same_key(const E& e, const KeyP& k) {
  return e.g[0] == k.g[0] && e.g[1] == k.g[1] && e.g[2] == k.g[2] && e.g[3] == k.g[3] && e.snlo == k.snlo &&
         e.snhi == k.snhi && e.tid == k.tid;
}
template <class E>
__device__ __forceinline__ void put_key(E& e, const KeyP& k) {
  e.g[0] = k.g[0]; e.g[1] = k.g[1]; e.g[2] = k.g[2]; e.g[3] = k.g[3];
  e.snlo = k.snlo; e.snhi = k.snhi; e.tid = k.tid;
}
__device__ __forceinline__ uint32_t ld_acq(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_rel(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
}

// live-index lookup (entries written by earlier launches): the key's entry or nullptr
__device__ const PEnt* p_find(const PEnt* P, uint64_t mask, const KeyP& k) {
  const uint64_t h = key_hash(k);
  const uint32_t fp = fp_of(h);
  for (uint64_t j = h & mask, n = 0; n <= mask; j = (j + 1) & mask, ++n) {
    const PEnt& e = P[j];
    if (e.fp == 0u) return nullptr;
    if (e.fp == fp && same_key(e, k)) return &e;
  }
  return nullptr;
}
// Inserts below run as rounds over the wave's active lanes, each lane one probe step per
// round: a lane that finds a slot claimed by a lane of its own wave whose key is not yet
// written retries in the next round, after that lane's stores (a per-lane spin could be
// scheduled before them and never end).
//
// live-index insert / update (distinct keys per launch); false when the table is full
__device__ bool p_put(PEnt* P, uint64_t mask, const KeyP& k, uint64_t idx, uint64_t* n_used) {
  const uint64_t h = key_hash(k);
  const uint32_t fp = fp_of(h);
  uint64_t j = h & mask, n = 0;
  bool done = false, ok = false;
  while (__any(!done)) {
    if (done) continue;
    PEnt& e = P[j];
    const uint32_t cur = __hip_atomic_load(&e.fp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (cur == 0u) {
      if (atomicCAS(&e.fp, 0u, fp) == 0u) {
        put_key(e, k);
        e.idx = idx;
        st_rel(&e.ready, 1u);
        atomicAdd(reinterpret_cast<unsigned long long*>(n_used), 1ull);
        done = ok = true;
      }  // else: claimed meanwhile, look again next round
    } else if (cur == fp && ld_acq(&e.ready) == 0u) {
      // being written: next round
    } else if (cur == fp && same_key(e, k)) {
      e.idx = idx;  // a newer insertion of a dead key (one writer per key per launch)
      done = ok = true;
    } else if (++n > mask) {
      done = true;  // full
    } else {
      j = (j + 1) & mask;
    }
  }
  return ok;
}
// batch-map claim / min-position update (concurrent, same keys allowed)
__device__ void b_put(BEnt* B, uint64_t mask, uint32_t epoch, const KeyP& k, uint32_t p) {
  const uint64_t h = key_hash(k);
  const uint64_t tag = ((uint64_t)epoch << 32) | fp_of(h);
  uint64_t j = h & mask;
  bool done = false;
  while (__any(!done)) {
    if (done) continue;
    BEnt& e = B[j];
    const unsigned long long cur = __hip_atomic_load(reinterpret_cast<unsigned long long*>(&e.tag), __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_AGENT);
    if ((uint32_t)(cur >> 32) != epoch) {  // free in this batch
      if (atomicCAS(reinterpret_cast<unsigned long long*>(&e.tag), cur, (unsigned long long)tag) == cur) {
        put_key(e, k);
        e.last = NO_IDX;
        e.nrep = 0;
        atomicExch(&e.minp, p);
        st_rel(&e.ready, epoch);
        done = true;
      }
    } else if (cur == tag && ld_acq(&e.ready) != epoch) {
      // being written: next round
    } else if (cur == tag && same_key(e, k)) {
      atomicMin(&e.minp, p);
      done = true;
    } else {
      j = (j + 1) & mask;
    }
  }
}
__device__ BEnt* b_find(BEnt* B, uint64_t mask, uint32_t epoch, const KeyP& k) {
  const uint64_t h = key_hash(k);
  const uint64_t tag = ((uint64_t)epoch << 32) | fp_of(h);
  for (uint64_t j = h & mask, n = 0; n <= mask; j = (j + 1) & mask, ++n) {
    BEnt& e = B[j];
    if ((uint32_t)(e.tag >> 32) != epoch) return nullptr;
    if (e.tag == tag && same_key(e, k)) return &e;
  }
  return nullptr;
}

struct TDev {
  const uint32_t* slot_tid;  // [NSLOT] reader slot -> topic
  const uint32_t* slot_cid;  // [NSLOT] reader slot -> compact topic (sort key), nA = none
  const uint32_t* cid_tid;   // [nA]
  const uint8_t* simple;     // [nt] one reader, not DUPLICATES_OK
  const uint32_t* K;         // [nt] max_keep
  uint64_t *I, *E, *until;   // [nt]
  PEnt* P;
  uint64_t pmask;
  BEnt* B;
  uint64_t bmask;
  uint32_t epoch, nA;
  // the batch: a delivery's change is read from its record when needed (no per-delivery key copy)
  const rtps_record* recs;
  const uint64_t* n_records;
  uint64_t max_records;
  rtps_delivery* del;
  const uint64_t* n_del;
  uint64_t max_del;
  // batch scratch (positions p in topic order; only p < the batch's delivery count is read)
  uint32_t *skey, *skey2, *sval, *order;  // sort: compact topic, delivery index (order == nullptr: no sort)
  uint8_t* fl;        // FL_* per position
  uint32_t* kpre;     // [max + 1] stored (FL_INS) positions before p
  int32_t* lgc;       // last GC position <= p (-1: none)
  uint8_t* frins;     // a repeat (FL_REP) position's change stored (written for repeats only)
  uint32_t* frlist;   // repeat positions, ascending
  uint64_t* nfr;
  uint64_t* fridx;    // [max] insertion index of an inserted repeat
  uint32_t *segb, *sege;  // [nA] this batch's topic segments (one of two parity buffers)
  uint32_t *segb_next, *sege_next;  // the other buffer: cleared here for the next batch
  uint32_t *frb, *fre;  // [nA]
  uint64_t* ibase;    // [3 * nA] the resolve's per-topic values for tc_final: I at the batch start minus
                      // the stored positions before its segment (mod 2^64), the topic's new E, the first
                      // position whose change stays live
  uint64_t* n_full;   // live-index inserts that found no room (0)
  const uint64_t* ovf;  // the ingest's window overflows of the batch (nullptr: none): all candidates
  const uint64_t* gate; // (optional) the batch's kernels do nothing unless *gate != 0 (the prologue runs)
  // repeats decided in parallel (tc_rscan): per repeat j the decision, the exclusive count of the
  // sure stores before it; the undecided ones (AMB) in order, with their stores' running count
  uint8_t* rdec;      // [nfr] RD_HOLD / RD_STORE / RD_AMB
  uint32_t* rpre;     // [nfr + 1] sure stores before repeat j
  uint32_t* amb;      // [namb] the undecided repeats' j, ascending
  uint64_t* namb;
  uint32_t* acum;     // [namb] stored undecided repeats up to amb[a] (inclusive), written in order
  uint32_t *ab, *ae;  // [nA] the topic's range of amb[]
  uint64_t* n_used;   // claimed live-index slots
  uint64_t* h_used;   // pinned: n_used as the earlier batches left it (the batch's first kernel)
  // the single-pass scans (tc_cscan over positions, tc_rscan over repeats): tile tickets and
  // decoupled look-back words, cleared by the batch's first kernel
  uint32_t* ticket;         // [4]: tc_cscan's, tc_rscan's tickets, tc_rscan's finished workgroups
  unsigned long long* lb;   // [4 * ntl]: tc_cscan's count words, its GC words, tc_rscan's count words
  uint32_t ntl;
};
constexpr uint8_t FL_GC = 1, FL_CAND = 2, FL_REP0 = 4, FL_PLIVE = 8, FL_VALID = 16, FL_INS = 32, FL_REP = 64;

__device__ __forceinline__ uint32_t pos_k(const TDev& d, uint64_t p) { return d.order ? d.order[p] : (uint32_t)p; }
__device__ __forceinline__ uint32_t pos_cid(const TDev& d, uint64_t p) {
  return d.order ? d.skey2[p] : d.slot_cid[d.del[p].reader_slot];
}
__device__ __forceinline__ uint64_t n_deliveries(const TDev& d) { return *d.n_del < d.max_del ? *d.n_del : d.max_del; }
__device__ __forceinline__ bool gated_off(const TDev& d) { return d.gate && *d.gate == 0ull; }
__device__ __forceinline__ bool ins_at(const TDev& d, uint64_t p) { return (d.fl[p] & FL_INS) != 0; }
// delivery dl's change (writer GUID, SN, topic); rec = NONE when its record is outside the batch
__device__ __forceinline__ KeyP key_of(const TDev& d, const rtps_delivery& dl, uint32_t tid = NONE) {
  KeyP x{};
  x.rec = NONE;
  const uint64_t nrec = *d.n_records < d.max_records ? *d.n_records : d.max_records;
  if (dl.rec_idx < nrec) {
    const uint4* q = reinterpret_cast<const uint4*>(d.recs + dl.rec_idx);
    const uint4 a = q[0], b = q[1], c = q[2];
    x.g[0] = a.z; x.g[1] = a.w; x.g[2] = b.x; x.g[3] = b.y;  // prefix @8, writer_id @20
    x.snlo = c.x; x.snhi = c.y;                              // sn @32
    x.tid = tid != NONE ? tid : d.slot_tid[dl.reader_slot];
    x.rec = dl.rec_idx;
  }
  return x;
}

// The batch's first kernel also clears what the later ones count on: the other parity's topic
// segments (the next batch's), the scans' tickets and look-back words, and it publishes the live
// index's use as the earlier batches left it (pinned host memory, for reserve_live: read once
// this batch's event has passed, no copy on the stream).
__device__ __forceinline__ void batch_prologue(const TDev& d) {
  const uint32_t t0 = blockIdx.x * TT + threadIdx.x, st = gridDim.x * TT;
  for (uint32_t c = t0; c < d.nA; c += st) { d.segb_next[c] = NONE; d.sege_next[c] = 0u; }
  for (uint32_t k = t0; k < 3u * d.ntl; k += st) d.lb[k] = 0ull;
  if (t0 < 4u) d.ticket[t0] = 0u;
  if (t0 == 0) {
    if (d.h_used) __hip_atomic_store(d.h_used, *d.n_used, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    *d.nfr = 0ull;  // (tc_cscan sets it when the batch has deliveries)
    d.kpre[0] = 0u;
  }
}

// One position's flags (the change x of delivery dl, prev: the delivery before it in topic order,
// same topic): GC, certain (stored unchecked: FL_INS), the same record as the previous position,
// or a candidate (looked up in the live index, claimed in the batch map).
struct TopicFacts {  // what the marks read of a topic (loaded once per run of positions of one topic)
  uint32_t t;
  bool sure;      // its single non-DUPLICATES_OK reader's proxy saw everything it holds (no overflow)
  uint64_t E;
};
__device__ __forceinline__ TopicFacts facts_of(const TDev& d, uint32_t t) {
  TopicFacts z;
  z.t = t;
  z.E = d.E[t];
  // (a batch whose ingest overflowed its capacities may hold duplicates the proxies did not
  // see: every delivery is checked then)
  z.sure = d.simple[t] && z.E >= d.until[t] && !(d.ovf && *d.ovf != 0u);
  return z;
}
__device__ __forceinline__ uint8_t mark_one(const TDev& d, uint64_t p, const KeyP& x, bool same_rec_before,
                                            TopicFacts& tf) {
  if (x.rec == NONE) return 0;
  uint8_t f = FL_VALID;
  if ((x.snlo & 63u) == 0u) f |= FL_GC;  // (sn as usize) % 64 == 0 (:230-233)
  // the same record delivered earlier to this topic (another reader of it): the change it stored
  // (or found) is held now: max_keep >= 1 keeps the newest
  if (same_rec_before) return f | FL_REP0;
  if (tf.t != x.tid) tf = facts_of(d, x.tid);
  const bool user_kind = ((x.g[3] >> 24) & 0xf0u) == 0u;  // EntityKind::is_user_defined (guid.rs:168-170)
  if (tf.sure && user_kind) return f | FL_INS;
  f |= FL_CAND;
  const PEnt* e = p_find(d.P, d.pmask, x);
  if (e && e->idx >= tf.E) f |= FL_PLIVE;
  b_put(d.B, d.bmask, d.epoch, x, (uint32_t)p);
  return f;
}

// No sort (at most one topic receives): position = delivery.  The changes are read from the
// records, the positions marked, the topic's segment bounds found (atomics on the boundary
// positions only), in one launch.  GV positions per thread (their loads in flight together).
constexpr uint32_t GV = 4;
__device__ __forceinline__ void load_dels(const rtps_delivery* del, uint64_t p0, uint64_t nd, rtps_delivery* dv) {
  if (p0 + GV <= nd) {  // (hipMalloc-aligned, p0 a multiple of 4: two 16-B loads)
    const uint4 a = reinterpret_cast<const uint4*>(del + p0)[0], b = reinterpret_cast<const uint4*>(del + p0)[1];
    const uint32_t w[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
    for (uint32_t i = 0; i < GV; ++i) {
      dv[i].rec_idx = w[2 * i];
      dv[i].reader_slot = (uint16_t)(w[2 * i + 1] & 0xffffu);
      dv[i].flags = (uint16_t)(w[2 * i + 1] >> 16);
    }
  } else {
#pragma unroll
    for (uint32_t i = 0; i < GV; ++i) dv[i] = p0 + i < nd ? del[p0 + i] : rtps_delivery{NONE, 0, 0};
  }
}
__global__ __launch_bounds__(TT) void tc_gm(TDev d) {
  batch_prologue(d);  // (gated off too: the next batch's segment buffer is cleared here)
  if (gated_off(d)) return;
  const uint64_t nd = n_deliveries(d);
  if (d.nA == 0 || nd == 0) return;
  // every valid position is the one topic's: its facts loaded once, beside the first deliveries
  const uint32_t t0 = d.cid_tid[0];
  TopicFacts tf0 = facts_of(d, t0);
  for (uint64_t p0 = ((uint64_t)blockIdx.x * TT + threadIdx.x) * GV; p0 < nd; p0 += (uint64_t)gridDim.x * TT * GV) {
    rtps_delivery dv[GV];
    load_dels(d.del, p0, nd, dv);
    const rtps_delivery pv0 = p0 > 0 ? d.del[p0 - 1] : rtps_delivery{NONE, 0, 0};
    const uint32_t cprev = p0 > 0 ? d.slot_cid[pv0.reader_slot] : NONE;
    const uint32_t cnext = p0 + GV < nd ? d.slot_cid[d.del[p0 + GV].reader_slot] : NONE;
    uint32_t cid[GV];
    KeyP x[GV];
#pragma unroll
    for (uint32_t i = 0; i < GV; ++i) {
      cid[i] = p0 + i < nd ? d.slot_cid[dv[i].reader_slot] : NONE;
      x[i] = cid[i] < d.nA ? key_of(d, dv[i], t0) : KeyP{{0, 0, 0, 0}, 0, 0, 0, NONE};
    }
    uint32_t fw = 0;
    TopicFacts tf = tf0;
#pragma unroll
    for (uint32_t i = 0; i < GV; ++i) {
      const uint64_t p = p0 + i;
      const uint32_t c = cid[i];
      if (c >= d.nA) continue;
      const uint32_t cp = i ? cid[i - 1] : cprev, cn = i + 1 < GV ? cid[i + 1] : cnext;
      const uint32_t rp = i ? dv[i - 1].rec_idx : pv0.rec_idx;
      if (cp != c) atomicMin(&d.segb[c], (uint32_t)p);
      if (p + 1 == nd || cn != c) atomicMax(&d.sege[c], (uint32_t)p + 1u);
      fw |= (uint32_t)mark_one(d, p, x[i], cp == c && rp == dv[i].rec_idx, tf) << (8 * i);
    }
    if (p0 + GV <= nd) *reinterpret_cast<uint32_t*>(d.fl + p0) = fw;
    else
      for (uint32_t i = 0; p0 + i < nd; ++i) d.fl[p0 + i] = (uint8_t)(fw >> (8 * i));
  }
}

// (RTPS_TC_PROBE measurement kernels)
__global__ void tc_nop_big(TDev d) { if (threadIdx.x == 0 && blockIdx.x == 0 && d.gate == (const uint64_t*)1) d.fl[0] = 0; }
__global__ void tc_nop_small(uint8_t* p) { if (threadIdx.x == 0 && blockIdx.x == 0 && p == (uint8_t*)1) *p = 0; }
// Sort mode: deliveries -> the sort pairs (compact topic, delivery index)
__global__ __launch_bounds__(TT) void tc_gather(TDev d) {
  batch_prologue(d);
  if (gated_off(d)) return;
  const uint64_t nd = n_deliveries(d);
  for (uint64_t k = (uint64_t)blockIdx.x * TT + threadIdx.x; k < d.max_del; k += (uint64_t)gridDim.x * TT) {
    d.skey[k] = k < nd ? d.slot_cid[d.del[k].reader_slot] : d.nA;
    d.sval[k] = (uint32_t)k;
  }
}
// Sort mode: per position in topic order, the flags and the segment bounds
__global__ __launch_bounds__(TT) void tc_mark(TDev d) {
  if (gated_off(d)) return;
  const uint64_t nd = n_deliveries(d);
  for (uint64_t p = (uint64_t)blockIdx.x * TT + threadIdx.x; p < nd; p += (uint64_t)gridDim.x * TT) {
    const uint32_t c = d.skey2[p];
    uint8_t f = 0;
    if (c < d.nA) {
      const bool pv_same = p > 0 && d.skey2[p - 1] == c;
      if (!pv_same) d.segb[c] = (uint32_t)p;
      if (p + 1 == nd || d.skey2[p + 1] != c) d.sege[c] = (uint32_t)p + 1u;
      const rtps_delivery dl = d.del[d.order[p]];
      TopicFacts tf{NONE, false, 0};
      f = mark_one(d, p, key_of(d, dl), pv_same && d.del[d.order[p - 1]].rec_idx == dl.rec_idx, tf);
    }
    d.fl[p] = f;
  }
}

// ---- single-pass scans with decoupled look-back ----
// Workgroup t takes tile t (workgroups are dispatched in index order, so every earlier tile has
// started), publishes its aggregate, adds its predecessors' (walking back until an inclusive
// prefix), publishes its inclusive prefix.  A word: flag (1 aggregate, 2 inclusive) << 62 | value.
#ifndef RTPS_TC_CPT
#define RTPS_TC_CPT 8
#endif
constexpr uint32_t CPT = RTPS_TC_CPT, TS = TT * CPT;  // positions per thread / per tile
constexpr unsigned long long LB_AGG = 1ull << 62, LB_INC = 2ull << 62, LB_VAL = (1ull << 62) - 1ull;
constexpr unsigned long long M31 = (1ull << 31) - 1ull;
// The words are self-contained (no data rides on them), so relaxed agent-scope atomics suffice:
// no acquire / release fences (each would write back or invalidate the caches).
__device__ __forceinline__ unsigned long long lb_get(unsigned long long* w) {
  return __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void lb_put(unsigned long long* w, unsigned long long v) {
  __hip_atomic_store(w, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// Wave 0: the exclusive prefix of `tile` from its predecessors' words, 64 of them per step (lane l
// reads tile - 1 - l): the step waits until every word up to the newest inclusive one is
// published, then reduces them.  MAX: a running maximum, else the sum of two 31-bit halves
// (counts of at most 2^31 - 1 positions: no carry between them).
template <bool MAX>
__device__ unsigned long long lb_prefix(unsigned long long* words, uint32_t tile, uint32_t lane) {
  unsigned long long acc = 0;
  for (int64_t hi = (int64_t)tile - 1; hi >= 0; hi -= 64) {
    const int64_t t = hi - (int64_t)lane;
    unsigned long long v;
    uint32_t fi;
    for (;;) {
      v = t >= 0 ? lb_get(words + t) : LB_INC;  // (before tile 0: an inclusive zero)
      const uint64_t inc = __ballot((v >> 62) == 2ull), wait = __ballot((v >> 62) == 0ull);
      fi = inc ? (uint32_t)__builtin_ctzll(inc) : 64u;
      const uint64_t upto = fi >= 63u ? ~0ull : ((2ull << fi) - 1ull);
      if (!(wait & upto)) break;
      __builtin_amdgcn_s_sleep(1);
    }
    unsigned long long x = lane <= fi ? (v & LB_VAL) : 0ull;
#pragma unroll
    for (uint32_t d = 32; d >= 1; d >>= 1) {
      const unsigned long long y = __shfl_xor(x, d, 64);
      x = MAX ? (y > x ? y : x) : x + y;
    }
    acc = MAX ? (x > acc ? x : acc) : acc + x;
    if (fi < 64u) break;
  }
  return acc;
}
// block-wide exclusive scan of (a, b) sums and an inclusive max of m; totals to every thread
__device__ __forceinline__ void block_scan3(uint32_t& a, uint32_t& b, int32_t& m, uint32_t& ta, uint32_t& tb,
                                            int32_t& tm) {
  __shared__ uint32_t s_a[TT / 64], s_b[TT / 64];
  __shared__ int32_t s_m[TT / 64];
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  uint32_t ia = a, ib = b;
  int32_t im = m;
#pragma unroll
  for (uint32_t k = 1; k < 64; k <<= 1) {
    const uint32_t ya = (uint32_t)__shfl_up((int)ia, k, 64), yb = (uint32_t)__shfl_up((int)ib, k, 64);
    const int32_t ym = __shfl_up(im, k, 64);
    if (lane >= k) { ia += ya; ib += yb; im = ym > im ? ym : im; }
  }
  if (lane == 63u) { s_a[wave] = ia; s_b[wave] = ib; s_m[wave] = im; }
  __syncthreads();
  uint32_t pa = 0, pb = 0;
  int32_t pm = -1;
  ta = 0; tb = 0; tm = -1;
#pragma unroll
  for (uint32_t w = 0; w < TT / 64; ++w) {
    if (w < wave) { pa += s_a[w]; pb += s_b[w]; pm = s_m[w] > pm ? s_m[w] : pm; }
    ta += s_a[w]; tb += s_b[w]; tm = s_m[w] > tm ? s_m[w] : tm;
  }
  a = pa + ia - a;  // exclusive
  b = pb + ib - b;
  m = pm > im ? pm : im;  // inclusive
  __syncthreads();  // (the shared words are reused by the caller's next scan)
}

// candidates: first occurrence not held live -> stored; else a repeat (resolved below).  Then the
// scans every later pass reads: kpre (stored positions before p), lgc (last GC position <= p), the
// repeat list (frlist, nfr).  One launch, no host count.
__global__ __launch_bounds__(TT) void tc_cscan(TDev d) {
  __shared__ unsigned long long s_pre[2];
  const uint32_t tile = blockIdx.x;
  if (gated_off(d)) return;
  const uint64_t nd = n_deliveries(d);
  const uint64_t base = (uint64_t)tile * TS;
  if (base >= nd) return;  // (no later tile looks back at it)
  const uint64_t p0 = base + (uint64_t)threadIdx.x * CPT;
  uint8_t fv[CPT];
  {
    const uint2 w = p0 + CPT <= nd ? *reinterpret_cast<const uint2*>(d.fl + p0) : uint2{0u, 0u};
#pragma unroll
    for (uint32_t i = 0; i < CPT; ++i)
      fv[i] = p0 + CPT <= nd ? (uint8_t)((i < 4 ? w.x >> (8 * i) : w.y >> (8 * (i - 4))) & 0xffu)
                             : (p0 + i < nd ? d.fl[p0 + i] : (uint8_t)0);
  }
  uint32_t ins = 0, rep = 0;
  int32_t gc = -1;
#pragma unroll
  for (uint32_t i = 0; i < CPT; ++i) {
    const uint64_t p = p0 + i;
    uint8_t f = fv[i];
    if (f & FL_CAND) {
      const KeyP x = key_of(d, d.del[pos_k(d, p)]);
      BEnt* e = b_find(d.B, d.bmask, d.epoch, x);
      if ((e && e->minp < (uint32_t)p) || (f & FL_PLIVE)) {
        f |= FL_REP;
        if (e) atomicAdd(&e->nrep, 1u);
      } else {
        f |= FL_INS;
      }
      d.fl[p] = f;
      fv[i] = f;
    }
    ins += (f & FL_INS) ? 1u : 0u;
    rep += (f & FL_REP) ? 1u : 0u;
    if (f & FL_GC) gc = (int32_t)p;
  }
  // a stored position's delivery is flagged now (the ingest writes every delivery's flags as 0):
  // tc_final then visits only the repeats and the changes that stay live
#pragma unroll
  for (uint32_t i = 0; i < CPT; ++i)
    if (fv[i] & FL_INS) d.del[pos_k(d, p0 + i)].flags = (uint16_t)RTPS_DELIVERY_CACHED;
  uint32_t ta, tb;
  int32_t tm;
  uint32_t ea = ins, eb = rep;
  int32_t im = gc;
  block_scan3(ea, eb, im, ta, tb, tm);
  unsigned long long* const lw = d.lb;
  unsigned long long* const lg = d.lb + d.ntl;
  if (threadIdx.x < 64u) {
    const uint32_t lane = threadIdx.x;
    const unsigned long long agg = (unsigned long long)ta | ((unsigned long long)tb << 31);
    const unsigned long long gm = (unsigned long long)(tm + 1);
    if (tile == 0) {
      if (lane == 0) { lb_put(lw, LB_INC | agg); lb_put(lg, LB_INC | gm); s_pre[0] = 0; s_pre[1] = 0; }
    } else {
      if (lane == 0) { lb_put(lw + tile, LB_AGG | agg); lb_put(lg + tile, LB_AGG | gm); }
      const unsigned long long ex = lb_prefix<false>(lw, tile, lane), exm = lb_prefix<true>(lg, tile, lane);
      if (lane == 0) {
        lb_put(lw + tile, LB_INC | (ex + agg));
        lb_put(lg + tile, LB_INC | (exm > gm ? exm : gm));
        s_pre[0] = ex;
        s_pre[1] = exm;
      }
    }
  }
  __syncthreads();
  uint32_t ki = (uint32_t)(s_pre[0] & M31) + ea, kr = (uint32_t)(s_pre[0] >> 31) + eb;
  // the last GC position before this thread's first: the earlier tiles' (look-back), then the
  // earlier threads' (the block scan's inclusive value of the previous thread)
  const int32_t before = (int32_t)s_pre[1] - 1;
  int32_t cur;
  {
    __shared__ int32_t s_last[TT / 64];
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    const int32_t prev_incl = __shfl_up(im, 1, 64);
    if (lane == 63u) s_last[wave] = im;
    __syncthreads();
    const int32_t blk_ex = lane ? prev_incl : (wave ? s_last[wave - 1] : -1);
    cur = blk_ex > before ? blk_ex : before;
  }
  uint32_t kv[CPT];
  int32_t gv[CPT];
#pragma unroll
  for (uint32_t i = 0; i < CPT; ++i) {
    const uint64_t p = p0 + i;
    const uint8_t f = fv[i];
    kv[i] = ki;
    if (f & FL_GC) cur = (int32_t)p;
    gv[i] = cur;
    if (p < nd && (f & FL_REP)) d.frlist[kr++] = (uint32_t)p;
    ki += (f & FL_INS) ? 1u : 0u;
  }
  if (p0 + CPT <= nd) {
    reinterpret_cast<uint4*>(d.kpre + p0)[0] = uint4{kv[0], kv[1], kv[2], kv[3]};
    reinterpret_cast<uint4*>(d.kpre + p0)[1] = uint4{kv[4], kv[5], kv[6], kv[7]};
    reinterpret_cast<int4*>(d.lgc + p0)[0] = int4{gv[0], gv[1], gv[2], gv[3]};
    reinterpret_cast<int4*>(d.lgc + p0)[1] = int4{gv[4], gv[5], gv[6], gv[7]};
  } else {
#pragma unroll
    for (uint32_t i = 0; i < CPT; ++i)
      if (p0 + i < nd) { d.kpre[p0 + i] = kv[i]; d.lgc[p0 + i] = gv[i]; }
  }
  if (p0 < nd && nd <= p0 + CPT) {  // the thread holding the last position: the totals
    d.kpre[nd] = ki;
    *d.nfr = kr;
  }
}

__device__ __forceinline__ uint32_t lower_bound(const uint32_t* a, uint32_t lo, uint32_t hi, uint32_t v) {
  while (lo < hi) {
    const uint32_t m = (lo + hi) >> 1;
    if (a[m] < v) lo = m + 1; else hi = m;
  }
  return lo;
}

// Repeats.  Whether the topic still holds a repeat's key when it arrives depends on the
// insertions before it, repeats included, so the reference's add_change is sequential.  Most
// repeats are decided without that order: with I(q) the insertion count before position q (the
// sure insertions, kpre, plus the stored repeats before q, Rb(q)), the topic's E at p is
// max(E0, I(g) - K) for the last GC position g <= p of the segment (I is non-decreasing), and
// the key is held iff its last insertion L >= E.  For a key with ONE repeat in the batch, L is
// its first occurrence's insertion I(f) or its live-index entry; Rb(g) - Rb(f) lies in
// [0, repeats in [f, g)), so the decision is sure when both ends of that range agree:
//   first occurrence f < g:  held iff (kpre[g] - kpre[f]) + (Rb(g) - Rb(f)) <= K;
//   f >= g, or no GC yet:    held (I(f) >= I(g) >= I(g) - K, and I(f) >= I0 >= E0);
//   live entry idx (< I0):   held iff idx >= max(E0, I(g) - K), Rb(g) in [0, repeats before g].
// The rest (keys with several repeats, ranges that straddle K) go to tc_resolve, one thread per
// topic, in order: Rb then counts the sure stores (an exclusive scan) plus the undecided ones
// already stored.  (The SPDP reader with half of a 1M batch repeats: 1.9 s when every repeat
// was resolved in order, round 4's form.)
constexpr uint8_t RD_HOLD = 0, RD_STORE = 1, RD_AMB = 2;
__device__ __forceinline__ uint8_t rdec_one(const TDev& d, uint32_t j) {
  const uint32_t p = d.frlist[j];
  const uint32_t c = pos_cid(d, p);
  const uint32_t t = d.cid_tid[c];
  const uint32_t b = d.segb[c];
  const uint32_t jb = lower_bound(d.frlist, 0, j, b);  // the topic's first repeat
  const KeyP x = key_of(d, d.del[pos_k(d, p)]);
  const BEnt* be = b_find(d.B, d.bmask, d.epoch, x);
  uint8_t dec = RD_AMB;
  if (be && be->nrep == 1u) {
    const uint64_t K = d.K[t], E0 = d.E[t], I0 = d.I[t];
    const uint32_t kb = d.kpre[b];
    const int64_t g = d.lgc[p];
    const bool gc = g >= (int64_t)b;  // a GC of this topic at or before p
    const PEnt* pe = p_find(d.P, d.pmask, x);
    const uint32_t f = be->minp;
    const bool has_f = f < p && ins_at(d, f);
    // live entry: sure held / sure not held
    int live = -1;  // -1 none, 0 not held, 1 held, 2 unsure
    if (pe) {
      if (!gc) {
        live = pe->idx >= E0 ? 1 : 0;
      } else {
        const uint64_t Ig_lo = I0 + (d.kpre[g] - kb);
        const uint64_t Ig_hi = Ig_lo + (lower_bound(d.frlist, jb, j, (uint32_t)g) - jb);
        const uint64_t E_lo = Ig_lo > K && Ig_lo - K > E0 ? Ig_lo - K : E0;
        const uint64_t E_hi = Ig_hi > K && Ig_hi - K > E0 ? Ig_hi - K : E0;
        live = pe->idx >= E_hi ? 1 : pe->idx < E_lo ? 0 : 2;
      }
    }
    int first = -1;
    if (has_f) {
      if (!gc || f >= (uint32_t)g) {
        first = 1;
      } else {
        const uint64_t A = d.kpre[g] - d.kpre[f];
        const uint64_t D = lower_bound(d.frlist, jb, j, (uint32_t)g) - lower_bound(d.frlist, jb, j, f);
        first = A + D <= K ? 1 : A > K ? 0 : 2;
      }
    }
    if (live == 1 || first == 1) dec = RD_HOLD;                     // some last insertion is held
    else if (live != 2 && first != 2) dec = RD_STORE;                // none is (or there is none)
  }
  return dec;
}
// stored repeats of the topic before position q (q within the topic's segment; j: the first
// repeat at or past q is searched in [jb, jcur)): the sure ones plus the undecided ones stored
__device__ __forceinline__ uint32_t rep_before(const TDev& d, uint32_t q, uint32_t jb, uint32_t jcur, uint32_t ab,
                                               uint32_t acur) {
  const uint32_t jq = lower_bound(d.frlist, jb, jcur, q);
  const uint32_t aq = lower_bound(d.amb, ab, acur, jq);  // undecided repeats before jq
  return (d.rpre[jq] - d.rpre[jb]) + (aq > ab ? d.acum[aq - 1] : 0u);
}

// one thread per topic of the batch: its undecided repeats in order, then the new I / E
__device__ void resolve_topic(const TDev& d, uint32_t c) {
  const uint32_t t = d.cid_tid[c];
  const uint64_t I0 = d.I[t];
  const uint32_t b = d.segb[c], e = d.sege[c];
  if (b == NONE) { d.frb[c] = d.fre[c] = 0; d.ab[c] = d.ae[c] = 0; return; }
  d.ibase[c] = I0 - d.kpre[b];
  const uint64_t K = d.K[t], E0 = d.E[t];
  const uint32_t nfr = (uint32_t)*d.nfr, na = nfr ? (uint32_t)*d.namb : 0u;
  const uint32_t jb = lower_bound(d.frlist, 0, nfr, b), je = lower_bound(d.frlist, jb, nfr, e);
  const uint32_t ab = lower_bound(d.amb, 0, na, jb), ae = lower_bound(d.amb, ab, na, je);
  d.frb[c] = jb;
  d.fre[c] = je;
  d.ab[c] = ab;
  d.ae[c] = ae;
  const uint32_t kb = d.kpre[b];
  uint32_t RA = 0;  // undecided repeats stored so far
  auto E_at = [&](int64_t g, uint32_t jcur, uint32_t acur) -> uint64_t {  // E after the GCs up to g
    if (g < (int64_t)b) return E0;
    const uint64_t Ig = I0 + (d.kpre[g] - kb) + (nfr ? rep_before(d, (uint32_t)g, jb, jcur, ab, acur) : 0u);
    return Ig > K && Ig - K > E0 ? Ig - K : E0;
  };
  for (uint32_t a = ab; a < ae; ++a) {
    const uint32_t j = d.amb[a];
    const uint32_t p = d.frlist[j];
    const uint64_t E = E_at(d.lgc[p], j, a);
    const KeyP x = key_of(d, d.del[pos_k(d, p)]);
    BEnt* be = b_find(d.B, d.bmask, d.epoch, x);
    // the key's last insertion before p: a stored repeat, its first occurrence (stored unless a
    // repeat itself), or the live index
    uint64_t L = NO_IDX;
    const PEnt* pe = p_find(d.P, d.pmask, x);
    if (pe) L = pe->idx;
    if (be) {
      const uint32_t f = be->minp;
      if (f < p && ins_at(d, f)) {
        const uint64_t If = I0 + (d.kpre[f] - kb) + rep_before(d, f, jb, j, ab, a);
        if (L == NO_IDX || If > L) L = If;
      }
      if (be->last != NO_IDX && (L == NO_IDX || be->last > L)) L = be->last;
    }
    const bool held = L != NO_IDX && L >= E;  // find_by_sn (:241-252, 270-276)
    if (!held) {
      const uint64_t Ip = I0 + (d.kpre[p] - kb) + (d.rpre[j] - d.rpre[jb]) + RA;
      d.frins[p] = 1;
      d.fridx[p] = Ip;
      if (be) be->last = Ip;
      ++RA;
    }
    d.acum[a] = RA;
  }
  const uint64_t E = E_at(d.lgc[e - 1], je, ae);
  d.I[t] = I0 + (d.kpre[e] - kb) + (nfr ? d.rpre[je] - d.rpre[jb] : 0u) + RA;
  d.E[t] = E;
  d.ibase[d.nA + c] = E;
  // the first position whose change (if stored) stays live: the insertion count before p,
  // I0 + stored positions + stored repeats before p, is non-decreasing in p
  uint32_t lo = b, hi = e;
  while (lo < hi) {
    const uint32_t m = (lo + hi) >> 1;
    const uint64_t Im = I0 + (d.kpre[m] - kb) + (nfr ? rep_before(d, m, jb, je, ab, ae) : 0u);
    if (Im >= E) hi = m; else lo = m + 1;
  }
  d.ibase[2u * d.nA + c] = lo;
}

// per repeat the decision, then the scans: rpre (sure stores before j), the undecided list (amb,
// namb).  Single pass like tc_cscan; a batch without repeats costs one workgroup's ticket.
__device__ void rscan_tile(const TDev& d, uint32_t tile, uint32_t nfr);
// ... and the workgroup that finishes last resolves every topic (tc_resolve's pass: the topics'
// undecided repeats in order, their new I / E), so that a batch's repeats take one launch.
__global__ __launch_bounds__(TT) void tc_rscan(TDev d) {
  __shared__ uint32_t s_last;
  const uint32_t tile = blockIdx.x;
  if (gated_off(d)) return;
  const uint32_t nfr = (uint32_t)*d.nfr;
  const uint32_t n_work = nfr ? (uint32_t)((nfr + TS - 1) / TS) : 1u;  // workgroups with a tile
  if (tile >= n_work) return;
  if (nfr == 0u) {
    if (threadIdx.x == 0) { d.rpre[0] = 0u; *d.namb = 0ull; }
  } else {
    rscan_tile(d, tile, nfr);
  }
  __syncthreads();
  if (n_work > 1u) {  // the last of the working workgroups to finish resolves (release / acquire)
    if (threadIdx.x == 0)
      s_last = __hip_atomic_fetch_add(&d.ticket[2], 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT) == n_work - 1u;
    __syncthreads();
    if (!s_last) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  }
  for (uint32_t c = threadIdx.x; c < d.nA; c += TT) resolve_topic(d, c);
}
__device__ void rscan_tile(const TDev& d, uint32_t tile, uint32_t nfr) {
  __shared__ unsigned long long s_pre;
  const uint64_t base = (uint64_t)tile * TS;
  const uint64_t j0 = base + (uint64_t)threadIdx.x * CPT;
  uint8_t dv[CPT];
  uint32_t ns = 0, na = 0;
#pragma unroll
  for (uint32_t i = 0; i < CPT; ++i) {
    const uint64_t j = j0 + i;
    uint8_t dec = RD_HOLD;
    if (j < nfr) {
      dec = rdec_one(d, (uint32_t)j);
      d.rdec[j] = dec;
      d.frins[d.frlist[j]] = 0;  // (the resolve sets it for the undecided repeats it stores)
    }
    dv[i] = j < nfr ? dec : (uint8_t)0xff;
    ns += dec == RD_STORE && j < nfr;
    na += dec == RD_AMB && j < nfr;
  }
  uint32_t ta, tb;
  int32_t tm, im = -1;
  uint32_t es = ns, ea = na;
  block_scan3(es, ea, im, ta, tb, tm);
  unsigned long long* const lw = d.lb + 2u * d.ntl;
  if (threadIdx.x < 64u) {
    const uint32_t lane = threadIdx.x;
    const unsigned long long agg = (unsigned long long)ta | ((unsigned long long)tb << 31);
    if (tile == 0) {
      if (lane == 0) { lb_put(lw, LB_INC | agg); s_pre = 0; }
    } else {
      if (lane == 0) lb_put(lw + tile, LB_AGG | agg);
      const unsigned long long ex = lb_prefix<false>(lw, tile, lane);
      if (lane == 0) { lb_put(lw + tile, LB_INC | (ex + agg)); s_pre = ex; }
    }
  }
  __syncthreads();
  uint32_t rs = (uint32_t)(s_pre & M31) + es, ra = (uint32_t)(s_pre >> 31) + ea;
#pragma unroll
  for (uint32_t i = 0; i < CPT; ++i) {
    const uint64_t j = j0 + i;
    if (j >= nfr) break;
    d.rpre[j] = rs;
    if (dv[i] == RD_STORE) ++rs;
    if (dv[i] == RD_AMB) d.amb[ra++] = (uint32_t)j;
  }
  if (j0 < nfr && nfr <= j0 + CPT) {  // the thread holding the last repeat: the totals
    d.rpre[nfr] = rs;
    *d.namb = ra;
  }
}


// per position: the flag on the delivery (its whole 8-B entry rewritten: full-line stores),
// survivors into the live index.  A change's insertion index: the topic's count at the batch
// start + the stored positions before it + the stored repeats before it (rep_before); an
// undecided repeat's comes from the resolve.
// The changes that stay live go into the live index; the stored repeats get their flag.
// Workgroups [0, nA): topic c's positions from its first live one (the resolve's binary search)
// to its segment's end, the stored ones inserted; workgroups [nA, grid): the repeats.
__global__ __launch_bounds__(TT) void tc_final(TDev d) {
  if (gated_off(d)) return;
  const uint64_t nd = n_deliveries(d);
  if (nd == 0) return;
  const uint32_t nfr = (uint32_t)*d.nfr;
  if (blockIdx.x < d.nA) {
    const uint32_t c = blockIdx.x;
    const uint32_t b = d.segb[c], e = d.sege[c];
    if (b == NONE) return;
    const uint64_t base = d.ibase[c], E = d.ibase[d.nA + c];
    const uint32_t first = (uint32_t)d.ibase[2u * d.nA + c];
    const uint32_t jb = nfr ? d.frb[c] : 0u, je = nfr ? d.fre[c] : 0u;
    const uint32_t ab = nfr ? d.ab[c] : 0u, ae = nfr ? d.ae[c] : 0u;
    for (uint32_t p = first + threadIdx.x; p < e; p += TT) {
      if (!(d.fl[p] & FL_INS)) continue;  // (stored repeats: below)
      const uint64_t idx = base + d.kpre[p] + (je > jb ? rep_before(d, p, jb, je, ab, ae) : 0u);
      if (idx >= E && !p_put(d.P, d.pmask, key_of(d, d.del[pos_k(d, p)]), idx, d.n_used))
        atomicAdd(reinterpret_cast<unsigned long long*>(d.n_full), 1ull);
    }
    return;
  }
  for (uint32_t j = (blockIdx.x - d.nA) * TT + threadIdx.x; j < nfr; j += (gridDim.x - d.nA) * TT) {
    const uint32_t p = d.frlist[j];
    const uint8_t dec = d.rdec[j];
    const uint32_t c = pos_cid(d, p);
    uint64_t idx;
    if (dec == RD_STORE) {
      idx = d.ibase[c] + d.kpre[p] + rep_before(d, p, d.frb[c], d.fre[c], d.ab[c], d.ae[c]);
    } else if (dec == RD_AMB && d.frins[p]) {
      idx = d.fridx[p];
    } else {
      continue;  // held: not stored
    }
    rtps_delivery* dl = d.del + pos_k(d, p);
    dl->flags = (uint16_t)RTPS_DELIVERY_CACHED;
    if (idx >= d.ibase[d.nA + c] && !p_put(d.P, d.pmask, key_of(d, *dl), idx, d.n_used))
      atomicAdd(reinterpret_cast<unsigned long long*>(d.n_full), 1ull);
  }
}

__global__ void tc_gc(uint32_t nt, const uint32_t* K, const uint64_t* I, uint64_t* E) {
  const uint32_t t = blockIdx.x * TT + threadIdx.x;
  if (t < nt && I[t] - E[t] > K[t]) E[t] = I[t] - K[t];
}
__global__ void tc_until(uint32_t nt, const uint64_t* I, uint64_t* until) {
  const uint32_t t = blockIdx.x * TT + threadIdx.x;
  if (t < nt) until[t] = I[t];
}
// rebuild: the live entries (idx >= E of their topic) into a fresh table
__global__ __launch_bounds__(TT) void tc_rebuild(const PEnt* old, uint64_t n_old, PEnt* P, uint64_t mask,
                                                 const uint64_t* E, uint64_t* n_used) {
  for (uint64_t j = (uint64_t)blockIdx.x * TT + threadIdx.x; j < n_old; j += (uint64_t)gridDim.x * TT) {
    const PEnt& e = old[j];
    if (e.fp == 0u || e.idx < E[e.tid]) continue;
    KeyP k{};
    k.g[0] = e.g[0]; k.g[1] = e.g[1]; k.g[2] = e.g[2]; k.g[3] = e.g[3];
    k.snlo = e.snlo; k.snhi = e.snhi; k.tid = e.tid;
    p_put(P, mask, k, e.idx, n_used);
  }
}

}  // namespace

struct TopicState {
  int device = 0;
  uint32_t n_cfg = 0, nt = 0, nA = 0;
  std::vector<uint32_t> cfg_keep;        // [n_cfg]
  std::vector<uint32_t> slot_cfg;        // [NSLOT] configured topic of a slot, NONE: private
  // device
  uint32_t *slot_tid = nullptr, *slot_cid = nullptr, *cid_tid = nullptr, *K = nullptr;
  uint8_t* simple = nullptr;
  uint64_t *I = nullptr, *E = nullptr, *until = nullptr;
  PEnt* P = nullptr;
  uint64_t pcap = 0;
  uint64_t* n_used = nullptr;       // device: claimed live-index slots
  uint64_t* h_used = nullptr;       // pinned (mapped): n_used before each batch (its tc_gather)
  uint64_t last_del = 0;            // max_del of the latest batch
  hipEvent_t used_ev = nullptr;     // that copy of the last batch
  bool used_pending = false;
  uint64_t used_known = 0;          // claimed slots when the last observed copy was made
  uint64_t used_inflight = 0;       // bound on the slots the batches since may have claimed
  BEnt* B = nullptr;
  uint64_t bcap = 0;
  uint32_t epoch = 0;
  uint64_t cap = 0;  // batch scratch capacity (deliveries)
  uint32_t *skey = nullptr, *skey2 = nullptr, *sval = nullptr, *order = nullptr, *kpre = nullptr;
  int32_t* lgc = nullptr;
  uint8_t *fl = nullptr, *frins = nullptr;
  uint32_t* ticket = nullptr;          // the single-pass scans' tile tickets [4]
  unsigned long long* lb = nullptr;    // their look-back words [3 * ntl]
  uint32_t ntl = 0;
  uint32_t* frlist = nullptr;
  uint64_t *fridx = nullptr, *nfr = nullptr, *n_full = nullptr;
  uint64_t* n_full_zero = nullptr;  // a device zero word (RTPS_TC_PROBE=2)
  uint32_t *segb = nullptr, *sege = nullptr, *frb = nullptr, *fre = nullptr;  // segb / sege: [2 * acap], by batch parity
  uint64_t* ibase = nullptr;
  uint8_t *rdec = nullptr, *ramb = nullptr;                         // [n] parallel repeat decisions
  uint32_t *rpre = nullptr, *amb = nullptr, *acum = nullptr;  // [n + 1]
  uint64_t* namb = nullptr;
  uint32_t *ab = nullptr, *ae = nullptr;  // [nA]
  uint32_t acap = 0;  // [nA] arrays' capacity
  void* tmp = nullptr;
  size_t tmp_bytes = 0;
};

static bool dmalloc(void** p, size_t n) { return hipMalloc(p, n ? n : 16) == hipSuccess; }
template <class T>
static void dfree(T*& p) {
  if (p) (void)hipFree(p);
  p = nullptr;
}

static void free_scratch(TopicState* s) {
  dfree(s->skey); dfree(s->skey2); dfree(s->sval); dfree(s->order); dfree(s->kpre);
  dfree(s->lgc); dfree(s->fl); dfree(s->frins); dfree(s->frlist);
  dfree(s->fridx); dfree(s->B); dfree(s->tmp); dfree(s->lb);
  dfree(s->rdec); dfree(s->rpre); dfree(s->amb); dfree(s->acum);
  s->cap = 0; s->bcap = 0; s->tmp_bytes = 0; s->ntl = 0;
}

TopicState* rtps_topic_state_new(int device) {
  TopicState* s = new (std::nothrow) TopicState();
  if (!s) return nullptr;
  s->device = device;
  s->slot_cfg.assign(NSLOT, NONE);
  s->nt = NSLOT;  // no configured topics: every slot its own
  bool ok = dmalloc((void**)&s->slot_tid, NSLOT * 4) && dmalloc((void**)&s->slot_cid, NSLOT * 4) &&
            dmalloc((void**)&s->nfr, 8) && dmalloc((void**)&s->n_full, 8) && dmalloc((void**)&s->n_used, 8) &&
            dmalloc((void**)&s->ticket, 16) && dmalloc((void**)&s->n_full_zero, 8) &&
            hipMemset(s->n_full_zero, 0, 8) == hipSuccess &&
            dmalloc((void**)&s->namb, 8) &&
            hipMemset(s->n_full, 0, 8) == hipSuccess && hipMemset(s->n_used, 0, 8) == hipSuccess &&
            hipHostMalloc((void**)&s->h_used, 8, hipHostMallocCoherent | hipHostMallocMapped) == hipSuccess &&
            hipEventCreateWithFlags(&s->used_ev, hipEventDisableTiming) == hipSuccess;
  if (!ok) { rtps_topic_state_free(s); return nullptr; }
  return s;
}

void rtps_topic_state_free(TopicState* s) {
  if (!s) return;
  free_scratch(s);
  dfree(s->slot_tid); dfree(s->slot_cid); dfree(s->cid_tid); dfree(s->K); dfree(s->simple); dfree(s->I);
  dfree(s->E); dfree(s->until); dfree(s->P); dfree(s->nfr); dfree(s->n_full); dfree(s->segb); dfree(s->sege);
  dfree(s->frb); dfree(s->fre); dfree(s->ibase); dfree(s->n_used); dfree(s->ticket); dfree(s->n_full_zero);
  if (s->h_used) (void)hipHostFree(s->h_used);
  if (s->used_ev) (void)hipEventDestroy(s->used_ev);
  delete s;
}

// topic of a slot: the configured one, else the slot's private topic n_cfg + slot
static uint32_t tid_of(const TopicState* s, uint32_t slot) {
  return s->slot_cfg[slot] != NONE ? s->slot_cfg[slot] : s->n_cfg + slot;
}

// (re)build the per-topic tables from the current readers; `fresh`: empty every cache
static int build(TopicState* s, const uint32_t* set_first, const rtps_target* ent, uint32_t n_sets, bool fresh,
                 hipStream_t st) {
  const uint32_t nt = s->n_cfg + NSLOT;
  if (fresh || nt != s->nt || !s->I) {
    dfree(s->K); dfree(s->simple); dfree(s->I); dfree(s->E); dfree(s->until);
    s->nt = nt;
    if (!dmalloc((void**)&s->K, nt * 4ull) || !dmalloc((void**)&s->simple, nt) || !dmalloc((void**)&s->I, nt * 8ull) ||
        !dmalloc((void**)&s->E, nt * 8ull) || !dmalloc((void**)&s->until, nt * 8ull))
      return RTPS_RX_ENOMEM;
    if (hipMemsetAsync(s->I, 0, nt * 8ull, st) != hipSuccess || hipMemsetAsync(s->E, 0, nt * 8ull, st) != hipSuccess ||
        hipMemsetAsync(s->until, 0, nt * 8ull, st) != hipSuccess)
      return RTPS_RX_EHIP;
    fresh = true;
  }
  // readers that can receive (every target entry), their flags
  std::vector<uint8_t> seen(NSLOT, 0), dup(NSLOT, 0);
  const uint32_t n_ent = n_sets ? set_first[n_sets] : 0u;
  for (uint32_t k = 0; k < n_ent; ++k) {
    seen[ent[k].reader_slot] = 1;
    if (ent[k].reader_flags & RTPS_TARGET_DUPLICATES_OK) dup[ent[k].reader_slot] = 1;
  }
  std::vector<uint32_t> readers_of(nt, 0), K(nt, DEFAULT_KEEP), slot_tid(NSLOT), slot_cid(NSLOT), cid_tid;
  std::vector<uint8_t> simple(nt, 1);
  for (uint32_t t = 0; t < s->n_cfg; ++t) K[t] = s->cfg_keep[t];
  std::vector<uint32_t> tid_cid(nt, NONE);
  for (uint32_t slot = 0; slot < NSLOT; ++slot) {
    const uint32_t t = tid_of(s, slot);
    slot_tid[slot] = t;
    if (!seen[slot]) continue;
    readers_of[t]++;
    if (dup[slot]) simple[t] = 0;
    if (tid_cid[t] == NONE) { tid_cid[t] = (uint32_t)cid_tid.size(); cid_tid.push_back(t); }
  }
  for (uint32_t t = 0; t < nt; ++t)
    if (readers_of[t] != 1) simple[t] = 0;
  s->nA = (uint32_t)cid_tid.size();
  for (uint32_t slot = 0; slot < NSLOT; ++slot) slot_cid[slot] = seen[slot] ? tid_cid[slot_tid[slot]] : s->nA;
  if (s->nA > s->acap || !s->segb) {
    dfree(s->cid_tid); dfree(s->segb); dfree(s->sege); dfree(s->frb); dfree(s->fre); dfree(s->ibase);
    dfree(s->ab); dfree(s->ae);
    const uint32_t a = s->nA ? s->nA : 1;
    if (!dmalloc((void**)&s->cid_tid, a * 4ull) || !dmalloc((void**)&s->segb, 2 * a * 4ull) ||
        !dmalloc((void**)&s->sege, 2 * a * 4ull) || !dmalloc((void**)&s->frb, a * 4ull) || !dmalloc((void**)&s->fre, a * 4ull) ||
        !dmalloc((void**)&s->ibase, 3 * a * 8ull) || !dmalloc((void**)&s->ab, a * 4ull) || !dmalloc((void**)&s->ae, a * 4ull))
      return RTPS_RX_ENOMEM;
    s->acap = a;
  }
  // both parity buffers of the topic segments start empty (each batch clears the next one's)
  if (hipMemsetAsync(s->segb, 0xff, 2 * s->acap * 4ull, st) != hipSuccess ||
      hipMemsetAsync(s->sege, 0, 2 * s->acap * 4ull, st) != hipSuccess)
    return RTPS_RX_EHIP;
  if (hipMemcpyAsync(s->K, K.data(), nt * 4ull, hipMemcpyHostToDevice, st) != hipSuccess ||
      hipMemcpyAsync(s->simple, simple.data(), nt, hipMemcpyHostToDevice, st) != hipSuccess ||
      hipMemcpyAsync(s->slot_tid, slot_tid.data(), NSLOT * 4ull, hipMemcpyHostToDevice, st) != hipSuccess ||
      hipMemcpyAsync(s->slot_cid, slot_cid.data(), NSLOT * 4ull, hipMemcpyHostToDevice, st) != hipSuccess ||
      (s->nA && hipMemcpyAsync(s->cid_tid, cid_tid.data(), s->nA * 4ull, hipMemcpyHostToDevice, st) != hipSuccess))
    return RTPS_RX_EHIP;
  if (fresh) {
    if (s->P && hipMemsetAsync(s->P, 0, s->pcap * sizeof(PEnt), st) != hipSuccess) return RTPS_RX_EHIP;
    if (hipMemsetAsync(s->n_used, 0, 8, st) != hipSuccess) return RTPS_RX_EHIP;
    s->used_known = s->used_inflight = 0;
    s->used_pending = false;
  } else {  // fresh proxies may accept what a topic still holds: check against the live changes
    hipLaunchKernelGGL(tc_until, dim3((nt + TT - 1) / TT), dim3(TT), 0, st, nt, s->I, s->until);
  }
  // (the host vectors above are read by the copies before this returns)
  return hipStreamSynchronize(st) == hipSuccess ? RTPS_RX_OK : RTPS_RX_EHIP;
}

int rtps_topic_configure(TopicState* s, const rtps_topic* topics, uint32_t n_topics, const rtps_topic_reader* readers,
                         uint32_t n_readers, const uint32_t* set_first, const rtps_target* ent, uint32_t n_sets,
                         hipStream_t st) {
  if (n_topics && !topics) return RTPS_RX_EINVAL;
  if (n_readers && !readers) return RTPS_RX_EINVAL;
  std::vector<uint32_t> keep(n_topics), scfg(NSLOT, NONE);
  for (uint32_t t = 0; t < n_topics; ++t) {
    if (topics[t].max_keep_samples < 1) return RTPS_RX_EINVAL;
    for (uint32_t u = 0; u < t; ++u)
      if (topics[u].topic == topics[t].topic) return RTPS_RX_EINVAL;  // repeated topic id
    keep[t] = topics[t].max_keep_samples;
  }
  for (uint32_t r = 0; r < n_readers; ++r) {
    uint32_t t = 0;
    while (t < n_topics && topics[t].topic != readers[r].topic) ++t;
    if (t == n_topics) return RTPS_RX_EINVAL;  // unknown topic
    scfg[readers[r].reader_slot] = t;
  }
  s->n_cfg = n_topics;
  s->cfg_keep = keep;
  s->slot_cfg = scfg;
  return build(s, set_first, ent, n_sets, true, st);
}

int rtps_topic_readers_changed(TopicState* s, const uint32_t* set_first, const rtps_target* ent, uint32_t n_sets,
                               hipStream_t st) {
  return build(s, set_first, ent, n_sets, false, st);
}

int rtps_topic_reset(TopicState* s, hipStream_t st) {
  if (!s->I) return RTPS_RX_OK;
  bool ok = hipMemsetAsync(s->I, 0, s->nt * 8ull, st) == hipSuccess &&
            hipMemsetAsync(s->E, 0, s->nt * 8ull, st) == hipSuccess &&
            hipMemsetAsync(s->until, 0, s->nt * 8ull, st) == hipSuccess &&
            (!s->P || hipMemsetAsync(s->P, 0, s->pcap * sizeof(PEnt), st) == hipSuccess) &&
            hipMemsetAsync(s->n_used, 0, 8, st) == hipSuccess;
  s->used_known = s->used_inflight = 0;
  s->used_pending = false;
  return ok ? RTPS_RX_OK : RTPS_RX_EHIP;
}

int rtps_topic_proxies_reset(TopicState* s, hipStream_t st) {
  if (!s->I) return RTPS_RX_OK;
  hipLaunchKernelGGL(tc_until, dim3((s->nt + TT - 1) / TT), dim3(TT), 0, st, s->nt, s->I, s->until);
  return hipGetLastError() == hipSuccess ? RTPS_RX_OK : RTPS_RX_EHIP;
}

uint32_t rtps_topic_of_slot(const TopicState* s, uint16_t slot) { return tid_of(s, slot); }
uint32_t rtps_topic_n_configured(const TopicState* s) { return s->n_cfg; }

int rtps_topic_gc(TopicState* s, hipStream_t st) {
  if (!s->I) return RTPS_RX_OK;
  hipLaunchKernelGGL(tc_gc, dim3((s->nt + TT - 1) / TT), dim3(TT), 0, st, s->nt, s->K, s->I, s->E);
  return hipGetLastError() == hipSuccess ? RTPS_RX_OK : RTPS_RX_EHIP;
}

static uint64_t pow2_at_least(uint64_t x) {
  uint64_t c = 1;
  while (c < x) c <<= 1;
  return c;
}

// the live index must hold what it holds plus one batch of survivors at load <= 1/2.  The
// claimed-slot count comes back to pinned memory after each batch (read without a sync
// once that batch is done); the batches still in flight are bounded by their sizes.
static int rebuild_live(TopicState* s, uint64_t ncap, hipStream_t st) {
  PEnt* np = nullptr;
  if (!dmalloc((void**)&np, ncap * sizeof(PEnt)) || hipMemsetAsync(np, 0, ncap * sizeof(PEnt), st) != hipSuccess) {
    if (np) (void)hipFree(np);
    return RTPS_RX_ENOMEM;
  }
  if (hipMemsetAsync(s->n_used, 0, 8, st) != hipSuccess) return RTPS_RX_EHIP;
  if (s->P) {  // the live entries only (idx >= E of their topic)
    const uint64_t b = (s->pcap + TT - 1) / TT;
    hipLaunchKernelGGL(tc_rebuild, dim3((uint32_t)(b < 8192 ? b : 8192)), dim3(TT), 0, st, s->P, s->pcap, np,
                       ncap - 1, s->E, s->n_used);
  }
  uint64_t used = 0;
  if (hipMemcpyAsync(&used, s->n_used, 8, hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipStreamSynchronize(st) != hipSuccess) {
    (void)hipFree(np);
    return RTPS_RX_EHIP;
  }
  if (s->P) (void)hipFree(s->P);
  s->P = np;
  s->pcap = ncap;
  s->used_known = used;
  s->used_inflight = 0;
  s->used_pending = false;
  return RTPS_RX_OK;
}
static int reserve_live(TopicState* s, uint64_t max_del, hipStream_t st) {
  if (s->used_pending && hipEventQuery(s->used_ev) == hipSuccess) {  // every batch so far is done
    s->used_known = *s->h_used;       // (before the latest batch: its tc_gather wrote it)
    s->used_inflight = s->last_del;   // what the latest batch may have claimed
    s->used_pending = false;
  }
  if (s->P && 2 * (s->used_known + s->used_inflight + max_del) <= s->pcap) return RTPS_RX_OK;
  if (hipStreamSynchronize(st) != hipSuccess) return RTPS_RX_EHIP;
  if (s->P) {  // exact count, then drop the dead entries
    if (hipMemcpy(&s->used_known, s->n_used, 8, hipMemcpyDeviceToHost) != hipSuccess) return RTPS_RX_EHIP;
    s->used_inflight = 0;
    s->used_pending = false;
    if (2 * (s->used_known + max_del) <= s->pcap) return RTPS_RX_OK;
    const int rc = rebuild_live(s, s->pcap, st);
    if (rc) return rc;
    if (2 * (s->used_known + max_del) <= s->pcap) return RTPS_RX_OK;
  }
  return rebuild_live(s, pow2_at_least(4 * (s->used_known + max_del) + 1024), st);
}

static int reserve_scratch(TopicState* s, uint64_t n, hipStream_t st) {
  if (n <= s->cap) return RTPS_RX_OK;
  if (hipStreamSynchronize(st) != hipSuccess) return RTPS_RX_EHIP;
  free_scratch(s);
  const uint64_t bcap = pow2_at_least(2 * n + 64);
  const uint32_t ntl = (uint32_t)((n + TS - 1) / TS);
  bool ok = dmalloc((void**)&s->skey, n * 4) && dmalloc((void**)&s->skey2, n * 4) && dmalloc((void**)&s->sval, n * 4) &&
            dmalloc((void**)&s->order, n * 4) && dmalloc((void**)&s->kpre, (n + 1) * 4) &&
            dmalloc((void**)&s->lgc, n * 4) && dmalloc((void**)&s->fl, n + 8) && dmalloc((void**)&s->frins, n) &&
            dmalloc((void**)&s->frlist, n * 4) &&
            dmalloc((void**)&s->fridx, n * 8) && dmalloc((void**)&s->B, bcap * sizeof(BEnt)) &&
            dmalloc((void**)&s->rdec, n) && dmalloc((void**)&s->rpre, (n + 1) * 4) &&
            dmalloc((void**)&s->amb, (n + 1) * 4) && dmalloc((void**)&s->acum, (n + 1) * 4) &&
            dmalloc((void**)&s->lb, 3ull * ntl * 8) &&
            hipMemsetAsync(s->B, 0, bcap * sizeof(BEnt), st) == hipSuccess;
  size_t tb = 0;  // the sort's temporary storage (more than one topic receives)
  ok = ok && rtps_sort_pairs(nullptr, tb, s->skey, s->skey2, s->sval, s->order, (uint32_t)n, 17, st) == hipSuccess;
  ok = ok && dmalloc(&s->tmp, tb);
  if (!ok) { free_scratch(s); return RTPS_RX_ENOMEM; }
  s->tmp_bytes = tb;
  s->cap = n;
  s->bcap = bcap;
  s->ntl = ntl;
  s->epoch = 0;
  return RTPS_RX_OK;
}

// A batch in four launches when at most one topic receives (no sort): tc_gm (changes + marks),
// tc_cscan (candidates + the position scans), tc_rscan (repeats' decisions + their scans, then
// the per-topic resolve), tc_final.  Every launch reads the delivery count on the device, so a
// batch sized by its capacity costs only its deliveries.
int rtps_topic_apply(TopicState* s, hipStream_t st, const rtps_record* recs, const uint64_t* n_records,
                     uint64_t max_records, rtps_delivery* del, const uint64_t* n_del, uint64_t max_del,
                     const uint64_t* ovf, const uint64_t* gate) {
  if (max_del == 0) return RTPS_RX_OK;
  if (max_del > 0x7fffffffull) return RTPS_RX_ETOOBIG;
  if (!s->I) return RTPS_RX_EINVAL;  // no readers known yet
  // measurement knob (tuning only; scripts/gpu_r6_iter.sh probe), bits: 1 queue nothing, 2 every
  // kernel gated off (a zero word), 4 no event record, 8 no pinned n_used store, 16 the first
  // kernel only, 32 / 64 an empty 1024-workgroup kernel with the TDev / an 8-B argument instead,
  // 128 a 20-us host spin instead, 256 / 512 one / three empty one-wave kernels instead.
  // Measured on T: the first kernel queued behind the ingest costs ~15 us of
  // device time whatever it is (one empty wave: +17 us, three: +23 us, a 20-us host delay: 0).
  static const int probe = [] { const char* e = getenv("RTPS_TC_PROBE"); return e ? atoi(e) : 0; }();
  if (probe & 128) {  // host time only: a 20-us spin, nothing queued
    const auto t0 = std::chrono::steady_clock::now();
    while (std::chrono::steady_clock::now() - t0 < std::chrono::microseconds(20)) {}
    return RTPS_RX_OK;
  }
  if (probe & 1) return RTPS_RX_OK;
  if (probe & 2) gate = s->n_full_zero;
  int rc = reserve_scratch(s, max_del, st);
  if (rc) return rc;
  rc = reserve_live(s, max_del, st);
  if (rc) return rc;
  if (++s->epoch == 0u) {  // batch-map tags would repeat: clear it (and restart the segment parity)
    if (hipMemsetAsync(s->B, 0, s->bcap * sizeof(BEnt), st) != hipSuccess ||
        hipMemsetAsync(s->segb, 0xff, 2 * s->acap * 4ull, st) != hipSuccess ||
        hipMemsetAsync(s->sege, 0, 2 * s->acap * 4ull, st) != hipSuccess)
      return RTPS_RX_EHIP;
    s->epoch = 1;
  }
  TDev d{};
  d.slot_tid = s->slot_tid; d.slot_cid = s->slot_cid; d.cid_tid = s->cid_tid; d.simple = s->simple; d.K = s->K;
  d.I = s->I; d.E = s->E; d.until = s->until; d.P = s->P; d.pmask = s->pcap - 1; d.B = s->B; d.bmask = s->bcap - 1;
  d.epoch = s->epoch; d.nA = s->nA;
  d.recs = recs; d.n_records = n_records; d.max_records = max_records; d.del = del; d.n_del = n_del; d.max_del = max_del;
  d.skey = s->skey; d.skey2 = s->skey2; d.sval = s->sval; d.order = s->nA > 1 ? s->order : nullptr;
  d.fl = s->fl; d.kpre = s->kpre; d.lgc = s->lgc; d.frins = s->frins;
  d.frlist = s->frlist; d.nfr = s->nfr; d.fridx = s->fridx;
  const uint32_t par = s->epoch & 1u;
  d.segb = s->segb + par * s->acap; d.sege = s->sege + par * s->acap;
  d.segb_next = s->segb + (par ^ 1u) * s->acap; d.sege_next = s->sege + (par ^ 1u) * s->acap;
  d.frb = s->frb; d.fre = s->fre; d.ibase = s->ibase; d.n_full = s->n_full;
  d.n_used = s->n_used;
  d.h_used = (probe & 8) ? nullptr : s->h_used;
  d.ovf = ovf;
  d.gate = gate;
  d.rdec = s->rdec; d.rpre = s->rpre; d.amb = s->amb; d.namb = s->namb;
  d.acum = s->acum; d.ab = s->ab; d.ae = s->ae;
  d.ticket = s->ticket; d.lb = s->lb;
  const uint32_t ntl = (uint32_t)((max_del + TS - 1) / TS);
  d.ntl = s->ntl;
  const uint32_t g = (uint32_t)((max_del + TT - 1) / TT < 8192 ? (max_del + TT - 1) / TT : 8192);
  if (probe & 32) { hipLaunchKernelGGL(tc_nop_big, dim3(1024), dim3(TT), 0, st, d); return RTPS_RX_OK; }
  if (probe & 64) { hipLaunchKernelGGL(tc_nop_small, dim3(1024), dim3(TT), 0, st, s->fl); return RTPS_RX_OK; }
  if (probe & 256) { hipLaunchKernelGGL(tc_nop_small, dim3(1), dim3(64), 0, st, s->fl); return RTPS_RX_OK; }
  if (probe & 512) {
    hipLaunchKernelGGL(tc_nop_small, dim3(1), dim3(64), 0, st, s->fl);
    hipLaunchKernelGGL(tc_nop_small, dim3(1), dim3(64), 0, st, s->fl);
    hipLaunchKernelGGL(tc_nop_small, dim3(1), dim3(64), 0, st, s->fl);
    return RTPS_RX_OK;
  }
  if (d.order) {
    hipLaunchKernelGGL(tc_gather, dim3(g), dim3(TT), 0, st, d);
    uint32_t bits = 1;
    while ((1u << bits) <= s->nA) ++bits;  // keys 0..nA (nA: no topic, sorts last)
    size_t tb = s->tmp_bytes;
    if (rtps_sort_pairs(s->tmp, tb, s->skey, s->skey2, s->sval, s->order, (uint32_t)max_del, (int)bits, st) !=
        hipSuccess)
      return RTPS_RX_EHIP;
    hipLaunchKernelGGL(tc_mark, dim3(g), dim3(TT), 0, st, d);
  } else {
    const uint64_t gq = (max_del + TT * GV - 1) / (TT * GV);
    hipLaunchKernelGGL(tc_gm, dim3((uint32_t)(gq < 8192 ? gq : 8192)), dim3(TT), 0, st, d);
  }
  if (probe & 16) return RTPS_RX_OK;
  hipLaunchKernelGGL(tc_cscan, dim3(ntl), dim3(TT), 0, st, d);
  // repeats: the sure ones decided in parallel, the undecided ones per topic in order
  hipLaunchKernelGGL(tc_rscan, dim3(ntl), dim3(TT), 0, st, d);
  {  // a workgroup per topic (its live tail), then the repeats' workgroups
    const uint64_t gr = (max_del + TT - 1) / TT;
    hipLaunchKernelGGL(tc_final, dim3(s->nA + (uint32_t)(gr < 1024 ? gr : 1024)), dim3(TT), 0, st, d);
  }
  s->used_inflight += max_del;
  s->last_del = max_del;
  if (!(probe & 4)) {
    if (hipEventRecord(s->used_ev, st) != hipSuccess) return RTPS_RX_EHIP;
    s->used_pending = true;
  }
  return hipGetLastError() == hipSuccess ? RTPS_RX_OK : RTPS_RX_EHIP;
}
