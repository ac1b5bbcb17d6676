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
#include <string.h>

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
  // batch scratch (positions p in topic order)
  KeyP* kp;           // [max] by delivery
  uint32_t *skey, *skey2, *sval, *order;  // sort: compact topic, delivery index
  uint8_t* fl;        // FL_* per position
  uint32_t *kins, *kpre;
  int32_t *gcpos, *lgc;
  uint8_t *fr, *frins;
  uint32_t* frlist;   // repeat positions, ascending
  uint64_t* nfr;
  uint32_t* frcum;    // inserted repeats of the topic up to frlist[j] (inclusive)
  uint64_t* fridx;    // [max] insertion index of an inserted repeat
  uint32_t *segb, *sege, *frb, *fre;  // [nA]
  uint64_t* ibase;    // [nA] I of the topic at the batch start
  uint64_t* n_full;   // live-index inserts that found no room (0)
  const uint64_t* ovf;  // the ingest's window overflows of the batch (nullptr: none): all candidates
  // repeats decided in parallel (tc_rdec): per repeat j the decision, the exclusive count of the
  // sure stores before it; the undecided ones (AMB) in order, with their stores' running count
  uint8_t* rdec;      // [nfr] RD_HOLD / RD_STORE / RD_AMB
  uint32_t *rst, *rpre;   // [nfr] 1 = sure store; exclusive scan of rst
  uint8_t* ramb;      // [nfr] 1 = undecided
  uint32_t* amb;      // [namb] the undecided repeats' j, ascending
  uint64_t* namb;
  uint32_t* acum;     // [namb] stored undecided repeats up to amb[a] (inclusive), written in order
  uint32_t *ab, *ae;  // [nA] the topic's range of amb[]
  uint64_t* n_used;   // claimed live-index slots
  uint64_t* h_used;   // pinned: n_used as the earlier batches left it (tc_gather)
};
constexpr uint8_t FL_GC = 1, FL_CAND = 2, FL_REP0 = 4, FL_PLIVE = 8, FL_VALID = 16;

__device__ __forceinline__ uint32_t pos_cid(const TDev& d, uint64_t p) { return d.order ? d.skey2[p] : d.skey[p]; }
__device__ __forceinline__ uint32_t pos_k(const TDev& d, uint64_t p) { return d.order ? d.order[p] : (uint32_t)p; }

// deliveries -> their changes (writer GUID, SN, topic) and the sort pairs
__global__ __launch_bounds__(TT) void tc_gather(TDev d, const rtps_record* recs, const uint64_t* n_records,
                                                uint64_t max_records, const rtps_delivery* del, const uint64_t* n_del,
                                                uint64_t max_del) {
  const uint64_t nrec = *n_records < max_records ? *n_records : max_records;
  const uint64_t nd = *n_del < max_del ? *n_del : max_del;
  // the topics' segment starts: none until tc_mark finds one
  for (uint32_t c = blockIdx.x * TT + threadIdx.x; c < d.nA; c += gridDim.x * TT) d.segb[c] = NONE;
  // the live index's use as the earlier batches left it, to pinned host memory for reserve_live
  // (read once this batch's event has passed: no copy on the stream)
  if (blockIdx.x == 0 && threadIdx.x == 0) __hip_atomic_store(d.h_used, *d.n_used, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  for (uint64_t k = (uint64_t)blockIdx.x * TT + threadIdx.x; k < max_del; k += (uint64_t)gridDim.x * TT) {
    KeyP x{};
    x.rec = NONE;
    uint32_t cid = d.nA;
    if (k < nd) {
      const rtps_delivery dl = del[k];
      cid = d.slot_cid[dl.reader_slot];
      if (dl.rec_idx < nrec) {
        const uint4* q = reinterpret_cast<const uint4*>(recs + dl.rec_idx);
        const uint4 a = q[0], b = q[1], c = q[2];
        x.g[0] = a.z; x.g[1] = a.w; x.g[2] = b.x; x.g[3] = b.y;  // prefix @8, writer_id @20
        x.snlo = c.x; x.snhi = c.y;                              // sn @32
        x.tid = d.slot_tid[dl.reader_slot];
        x.rec = dl.rec_idx;
      }
    }
    d.kp[k] = x;
    d.skey[k] = cid;
    d.sval[k] = (uint32_t)k;
  }
}

// per position: GC, segment bounds, certain / same-record / candidate, the batch map
__global__ __launch_bounds__(TT) void tc_mark(TDev d, uint64_t max_del) {
  for (uint64_t p = (uint64_t)blockIdx.x * TT + threadIdx.x; p < max_del; p += (uint64_t)gridDim.x * TT) {
    const uint32_t c = pos_cid(d, p);
    const KeyP x = d.kp[pos_k(d, p)];
    uint8_t f = 0;
    uint32_t kins = 0;
    int32_t gcp = -1;
    if (c < d.nA) {
      if (p == 0 || pos_cid(d, p - 1) != c) d.segb[c] = (uint32_t)p;
      if (p + 1 == max_del || pos_cid(d, p + 1) != c) d.sege[c] = (uint32_t)p + 1u;
    }
    if (c < d.nA && x.rec != NONE) {
      f = FL_VALID;
      if ((x.snlo & 63u) == 0u) { f |= FL_GC; gcp = (int32_t)p; }  // (sn as usize) % 64 == 0 (:230-233)
      // the same record delivered earlier to this topic (another reader of it): the change
      // it stored (or found) is held now: max_keep >= 1 keeps the newest
      const bool rep0 = p > 0 && pos_cid(d, p - 1) == c && d.kp[pos_k(d, p - 1)].rec == x.rec;
      const uint32_t t = x.tid;
      const bool user_kind = ((x.g[3] >> 24) & 0xf0u) == 0u;  // EntityKind::is_user_defined (guid.rs:168-170)
      // (a batch whose ingest overflowed its capacities may hold duplicates the proxies did not
      // see: every delivery is checked then)
      const bool cand = !d.simple[t] || d.E[t] < d.until[t] || !user_kind || (d.ovf && *d.ovf != 0u);
      if (rep0) {
        f |= FL_REP0;
      } else if (!cand) {
        kins = 1;
      } else {
        f |= FL_CAND;
        const PEnt* e = p_find(d.P, d.pmask, x);
        if (e && e->idx >= d.E[t]) f |= FL_PLIVE;
        b_put(d.B, d.bmask, d.epoch, x, (uint32_t)p);
      }
    }
    d.fl[p] = f;
    d.kins[p] = kins;
    d.gcpos[p] = gcp;
    d.fr[p] = 0;
    d.frins[p] = 0;
    d.rst[p] = 0;   // (tc_rdec's outputs for the repeats j < nfr <= p; the scans read all of them)
    d.ramb[p] = 0;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    d.rst[max_del] = 0;
    d.ramb[max_del] = 0;
  }
}

// candidates: first occurrence not held live -> stored; else a repeat (resolved in order)
__global__ __launch_bounds__(TT) void tc_class(TDev d, uint64_t max_del) {
  for (uint64_t p = (uint64_t)blockIdx.x * TT + threadIdx.x; p < max_del; p += (uint64_t)gridDim.x * TT) {
    const uint8_t f = d.fl[p];
    if (!(f & FL_CAND)) continue;
    const KeyP x = d.kp[pos_k(d, p)];
    BEnt* e = b_find(d.B, d.bmask, d.epoch, x);
    const bool rep = (e && e->minp < (uint32_t)p) || (f & FL_PLIVE);
    if (rep) {
      d.fr[p] = 1;
      if (e) atomicAdd(&e->nrep, 1u);
    } else {
      d.kins[p] = 1;
    }
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
__global__ __launch_bounds__(TT) void tc_rdec(TDev d) {
  const uint32_t nfr = (uint32_t)*d.nfr;
  for (uint32_t j = blockIdx.x * TT + threadIdx.x; j < nfr; j += gridDim.x * TT) {
    const uint32_t p = d.frlist[j];
    const uint32_t c = pos_cid(d, p);
    const uint32_t t = d.cid_tid[c];
    const uint32_t b = d.segb[c];
    const uint32_t jb = lower_bound(d.frlist, 0, j, b);  // the topic's first repeat
    const KeyP x = d.kp[pos_k(d, p)];
    const BEnt* be = b_find(d.B, d.bmask, d.epoch, x);
    uint8_t dec = RD_AMB;
    if (be && be->nrep == 1u) {
      const uint64_t K = d.K[t], E0 = d.E[t], I0 = d.I[t];
      const uint32_t kb = d.kpre[b];
      const int64_t g = d.lgc[p];
      const bool gc = g >= (int64_t)b;  // a GC of this topic at or before p
      const PEnt* pe = p_find(d.P, d.pmask, x);
      const uint32_t f = be->minp;
      const bool has_f = f < p && d.kins[f];
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
    d.rdec[j] = dec;
    d.rst[j] = dec == RD_STORE ? 1u : 0u;
    d.ramb[j] = dec == RD_AMB ? 1u : 0u;
  }
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
__global__ __launch_bounds__(TT) void tc_resolve(TDev d) {
  const uint32_t c = blockIdx.x * TT + threadIdx.x;
  if (c >= d.nA) return;
  const uint32_t t = d.cid_tid[c];
  const uint64_t I0 = d.I[t];
  d.ibase[c] = I0;
  const uint32_t b = d.segb[c], e = d.sege[c];
  if (b == NONE) { d.frb[c] = d.fre[c] = 0; d.ab[c] = d.ae[c] = 0; return; }
  const uint64_t K = d.K[t], E0 = d.E[t];
  const uint32_t nfr = (uint32_t)*d.nfr, na = (uint32_t)*d.namb;
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
    const uint64_t Ig = I0 + (d.kpre[g] - kb) + rep_before(d, (uint32_t)g, jb, jcur, ab, acur);
    return Ig > K && Ig - K > E0 ? Ig - K : E0;
  };
  for (uint32_t a = ab; a < ae; ++a) {
    const uint32_t j = d.amb[a];
    const uint32_t p = d.frlist[j];
    const uint64_t E = E_at(d.lgc[p], j, a);
    const KeyP x = d.kp[pos_k(d, p)];
    BEnt* be = b_find(d.B, d.bmask, d.epoch, x);
    // the key's last insertion before p: a stored repeat, its first occurrence (stored unless a
    // repeat itself), or the live index
    uint64_t L = NO_IDX;
    const PEnt* pe = p_find(d.P, d.pmask, x);
    if (pe) L = pe->idx;
    if (be) {
      const uint32_t f = be->minp;
      if (f < p && d.kins[f]) {
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
  d.I[t] = I0 + (d.kpre[e - 1] + d.kins[e - 1] - kb) + (d.rpre[je] - d.rpre[jb]) + RA;
  d.E[t] = E;
}

// per repeat: the sure stores' insertion (index: the insertions before it, repeats included)
// and every repeat's running count of stored repeats in its topic (frcum, for tc_final)
__global__ __launch_bounds__(TT) void tc_rfill(TDev d) {
  const uint32_t nfr = (uint32_t)*d.nfr;
  for (uint32_t j = blockIdx.x * TT + threadIdx.x; j < nfr; j += gridDim.x * TT) {
    const uint32_t p = d.frlist[j];
    const uint32_t c = pos_cid(d, p);
    const uint32_t jb = d.frb[c], ab = d.ab[c], ae = d.ae[c];
    const uint32_t aq = lower_bound(d.amb, ab, ae, j + 1u);  // undecided repeats up to j
    const uint32_t before = (d.rpre[j] - d.rpre[jb]) + (aq > ab ? d.acum[aq - 1] : 0u) -
                            ((aq > ab && d.amb[aq - 1] == j && d.frins[p]) ? 1u : 0u);
    if (d.rdec[j] == RD_STORE) {
      d.frins[p] = 1;
      d.fridx[p] = d.ibase[c] + (d.kpre[p] - d.kpre[d.segb[c]]) + before;
    }
    d.frcum[j] = before + (d.frins[p] ? 1u : 0u);
  }
}

// per position: the flag on the delivery, survivors into the live index
__global__ __launch_bounds__(TT) void tc_final(TDev d, rtps_delivery* del, uint64_t max_del) {
  for (uint64_t p = (uint64_t)blockIdx.x * TT + threadIdx.x; p < max_del; p += (uint64_t)gridDim.x * TT) {
    const uint8_t f = d.fl[p];
    if (!(f & FL_VALID)) continue;
    const uint32_t k = pos_k(d, p);
    const uint32_t c = pos_cid(d, p);
    const bool ins = d.kins[p] || d.frins[p];
    rtps_delivery* dl = del + k;
    dl->flags = (uint16_t)((dl->flags & ~RTPS_DELIVERY_CACHED) | (ins ? RTPS_DELIVERY_CACHED : 0u));
    if (!ins) continue;
    const KeyP x = d.kp[k];
    uint64_t idx;
    if (d.fr[p]) {
      idx = d.fridx[p];
    } else {
      const uint32_t jb = d.frb[c], je = d.fre[c];
      uint32_t r = 0;
      if (je > jb) {
        const uint32_t jq = lower_bound(d.frlist, jb, je, (uint32_t)p);
        r = jq > jb ? d.frcum[jq - 1] : 0u;
      }
      idx = d.ibase[c] + (d.kpre[p] - d.kpre[d.segb[c]]) + r;
    }
    if (idx >= d.E[x.tid] && !p_put(d.P, d.pmask, x, idx, d.n_used))
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
  KeyP* kp = nullptr;
  uint32_t *skey = nullptr, *skey2 = nullptr, *sval = nullptr, *order = nullptr, *kins = nullptr, *kpre = nullptr;
  int32_t *gcpos = nullptr, *lgc = nullptr;
  uint8_t *fl = nullptr, *fr = nullptr, *frins = nullptr;
  uint32_t *frlist = nullptr, *frcum = nullptr;
  uint64_t *fridx = nullptr, *nfr = nullptr, *n_full = nullptr;
  uint32_t *segb = nullptr, *sege = nullptr, *frb = nullptr, *fre = nullptr;
  uint64_t* ibase = nullptr;
  uint8_t *rdec = nullptr, *ramb = nullptr;                         // [n] parallel repeat decisions
  uint32_t *rst = nullptr, *rpre = nullptr, *amb = nullptr, *acum = nullptr;  // [n + 1]
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
  dfree(s->kp); dfree(s->skey); dfree(s->skey2); dfree(s->sval); dfree(s->order); dfree(s->kins); dfree(s->kpre);
  dfree(s->gcpos); dfree(s->lgc); dfree(s->fl); dfree(s->fr); dfree(s->frins); dfree(s->frlist); dfree(s->frcum);
  dfree(s->fridx); dfree(s->B); dfree(s->tmp);
  dfree(s->rdec); dfree(s->ramb); dfree(s->rst); dfree(s->rpre); dfree(s->amb); dfree(s->acum);
  s->cap = 0; s->bcap = 0; s->tmp_bytes = 0;
}

TopicState* rtps_topic_state_new(int device) {
  TopicState* s = new (std::nothrow) TopicState();
  if (!s) return nullptr;
  s->device = device;
  s->slot_cfg.assign(NSLOT, NONE);
  s->nt = NSLOT;  // no configured topics: every slot its own
  bool ok = dmalloc((void**)&s->slot_tid, NSLOT * 4) && dmalloc((void**)&s->slot_cid, NSLOT * 4) &&
            dmalloc((void**)&s->nfr, 8) && dmalloc((void**)&s->n_full, 8) && dmalloc((void**)&s->n_used, 8) &&
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
  dfree(s->frb); dfree(s->fre); dfree(s->ibase); dfree(s->n_used);
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
    if (!dmalloc((void**)&s->cid_tid, a * 4ull) || !dmalloc((void**)&s->segb, a * 4ull) ||
        !dmalloc((void**)&s->sege, a * 4ull) || !dmalloc((void**)&s->frb, a * 4ull) || !dmalloc((void**)&s->fre, a * 4ull) ||
        !dmalloc((void**)&s->ibase, a * 8ull) || !dmalloc((void**)&s->ab, a * 4ull) || !dmalloc((void**)&s->ae, a * 4ull))
      return RTPS_RX_ENOMEM;
    s->acap = a;
  }
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
  bool ok = dmalloc((void**)&s->kp, n * sizeof(KeyP)) && dmalloc((void**)&s->skey, n * 4) &&
            dmalloc((void**)&s->skey2, n * 4) && dmalloc((void**)&s->sval, n * 4) && dmalloc((void**)&s->order, n * 4) &&
            dmalloc((void**)&s->kins, n * 4) && dmalloc((void**)&s->kpre, n * 4) && dmalloc((void**)&s->gcpos, n * 4) &&
            dmalloc((void**)&s->lgc, n * 4) && dmalloc((void**)&s->fl, n) && dmalloc((void**)&s->fr, n) &&
            dmalloc((void**)&s->frins, n) && dmalloc((void**)&s->frlist, n * 4) && dmalloc((void**)&s->frcum, n * 4) &&
            dmalloc((void**)&s->fridx, n * 8) && dmalloc((void**)&s->B, bcap * sizeof(BEnt)) &&
            dmalloc((void**)&s->rdec, n) && dmalloc((void**)&s->ramb, n + 1) && dmalloc((void**)&s->rst, (n + 1) * 4) &&
            dmalloc((void**)&s->rpre, (n + 1) * 4) && dmalloc((void**)&s->amb, (n + 1) * 4) &&
            dmalloc((void**)&s->acum, (n + 1) * 4) &&
            hipMemsetAsync(s->B, 0, bcap * sizeof(BEnt), st) == hipSuccess;
  size_t b1 = 0, b2 = 0, b3 = 0, b4 = 0;
  ok = ok && rtps_sort_pairs(nullptr, b1, s->skey, s->skey2, s->sval, s->order, (uint32_t)n, 17, st) == hipSuccess;
  ok = ok && hipcub::DeviceScan::ExclusiveSum(nullptr, b2, s->kins, s->kpre, (int64_t)n, st) == hipSuccess;
  ok = ok && hipcub::DeviceScan::InclusiveScan(nullptr, b3, s->gcpos, s->lgc, hipcub::Max(), (int64_t)n, st) ==
                 hipSuccess;
  ok = ok && hipcub::DeviceSelect::Flagged(nullptr, b4, hipcub::CountingInputIterator<uint32_t>(0), s->fr, s->frlist,
                                           s->nfr, (int64_t)n, st) == hipSuccess;
  size_t b5 = 0, b6 = 0;
  ok = ok && hipcub::DeviceScan::ExclusiveSum(nullptr, b5, s->rst, s->rpre, (int64_t)n + 1, st) == hipSuccess;
  ok = ok && hipcub::DeviceSelect::Flagged(nullptr, b6, hipcub::CountingInputIterator<uint32_t>(0), s->ramb, s->amb,
                                           s->namb, (int64_t)n, st) == hipSuccess;
  size_t tb = b1;
  for (size_t b : {b2, b3, b4, b5, b6}) tb = b > tb ? b : tb;
  ok = ok && dmalloc(&s->tmp, tb);
  if (!ok) { free_scratch(s); return RTPS_RX_ENOMEM; }
  s->tmp_bytes = tb;
  s->cap = n;
  s->bcap = bcap;
  s->epoch = 0;
  return RTPS_RX_OK;
}

int rtps_topic_apply(TopicState* s, hipStream_t st, const rtps_record* recs, const uint64_t* n_records,
                     uint64_t max_records, rtps_delivery* del, const uint64_t* n_del, uint64_t max_del,
                     const uint64_t* ovf) {
  if (max_del == 0) return RTPS_RX_OK;
  if (max_del > 0x7fffffffull) return RTPS_RX_ETOOBIG;
  if (!s->I) return RTPS_RX_EINVAL;  // no readers known yet
  int rc = reserve_scratch(s, max_del, st);
  if (rc) return rc;
  rc = reserve_live(s, max_del, st);
  if (rc) return rc;
  if (++s->epoch == 0u) {  // batch-map tags would repeat: clear it
    if (hipMemsetAsync(s->B, 0, s->bcap * sizeof(BEnt), st) != hipSuccess) return RTPS_RX_EHIP;
    s->epoch = 1;
  }
  TDev d{};
  d.slot_tid = s->slot_tid; d.slot_cid = s->slot_cid; d.cid_tid = s->cid_tid; d.simple = s->simple; d.K = s->K;
  d.I = s->I; d.E = s->E; d.until = s->until; d.P = s->P; d.pmask = s->pcap - 1; d.B = s->B; d.bmask = s->bcap - 1;
  d.epoch = s->epoch; d.nA = s->nA;
  d.kp = s->kp; d.skey = s->skey; d.skey2 = s->skey2; d.sval = s->sval; d.order = s->nA > 1 ? s->order : nullptr;
  d.fl = s->fl; d.kins = s->kins; d.kpre = s->kpre; d.gcpos = s->gcpos; d.lgc = s->lgc; d.fr = s->fr;
  d.frins = s->frins; d.frlist = s->frlist; d.nfr = s->nfr; d.frcum = s->frcum; d.fridx = s->fridx;
  d.segb = s->segb; d.sege = s->sege; d.frb = s->frb; d.fre = s->fre; d.ibase = s->ibase; d.n_full = s->n_full;
  d.n_used = s->n_used;
  d.h_used = s->h_used;
  d.ovf = ovf;
  d.rdec = s->rdec; d.rst = s->rst; d.rpre = s->rpre; d.ramb = s->ramb; d.amb = s->amb; d.namb = s->namb;
  d.acum = s->acum; d.ab = s->ab; d.ae = s->ae;
  const uint32_t g = (uint32_t)((max_del + TT - 1) / TT < 8192 ? (max_del + TT - 1) / TT : 8192);
  hipLaunchKernelGGL(tc_gather, dim3(g), dim3(TT), 0, st, d, recs, n_records, max_records, del, n_del, max_del);
  if (d.order) {
    uint32_t bits = 1;
    while ((1u << bits) <= s->nA) ++bits;  // keys 0..nA (nA: no topic, sorts last)
    size_t tb = s->tmp_bytes;
    if (rtps_sort_pairs(s->tmp, tb, s->skey, s->skey2, s->sval, s->order, (uint32_t)max_del, (int)bits, st) !=
        hipSuccess)
      return RTPS_RX_EHIP;
  }
  hipLaunchKernelGGL(tc_mark, dim3(g), dim3(TT), 0, st, d, max_del);
  hipLaunchKernelGGL(tc_class, dim3(g), dim3(TT), 0, st, d, max_del);
  size_t tb = s->tmp_bytes;
  if (hipcub::DeviceScan::ExclusiveSum(s->tmp, tb, s->kins, s->kpre, (int64_t)max_del, st) != hipSuccess)
    return RTPS_RX_EHIP;
  tb = s->tmp_bytes;
  if (hipcub::DeviceScan::InclusiveScan(s->tmp, tb, s->gcpos, s->lgc, hipcub::Max(), (int64_t)max_del, st) !=
      hipSuccess)
    return RTPS_RX_EHIP;
  tb = s->tmp_bytes;
  if (hipcub::DeviceSelect::Flagged(s->tmp, tb, hipcub::CountingInputIterator<uint32_t>(0), s->fr, s->frlist, s->nfr,
                                    (int64_t)max_del, st) != hipSuccess)
    return RTPS_RX_EHIP;
  // repeats: the sure ones decided in parallel, the undecided ones per topic in order
  hipLaunchKernelGGL(tc_rdec, dim3(g), dim3(TT), 0, st, d);
  tb = s->tmp_bytes;
  if (hipcub::DeviceScan::ExclusiveSum(s->tmp, tb, s->rst, s->rpre, (int64_t)max_del + 1, st) != hipSuccess)
    return RTPS_RX_EHIP;
  tb = s->tmp_bytes;
  if (hipcub::DeviceSelect::Flagged(s->tmp, tb, hipcub::CountingInputIterator<uint32_t>(0), s->ramb, s->amb, s->namb,
                                    (int64_t)max_del, st) != hipSuccess)
    return RTPS_RX_EHIP;
  if (s->nA) hipLaunchKernelGGL(tc_resolve, dim3((s->nA + TT - 1) / TT), dim3(TT), 0, st, d);
  hipLaunchKernelGGL(tc_rfill, dim3(g), dim3(TT), 0, st, d);
  hipLaunchKernelGGL(tc_final, dim3(g), dim3(TT), 0, st, d, del, max_del);
  s->used_inflight += max_del;
  s->last_del = max_del;
  if (hipEventRecord(s->used_ev, st) != hipSuccess) return RTPS_RX_EHIP;
  s->used_pending = true;
  return hipGetLastError() == hipSuccess ? RTPS_RX_OK : RTPS_RX_EHIP;
}
