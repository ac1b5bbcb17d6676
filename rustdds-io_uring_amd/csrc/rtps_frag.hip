// rtps_frag.hip — DataFrag reassembly on the device.
//
// Replaces the per-reader FragmentAssembler / AssemblyBuffer
// (rtps/fragment_assembler.rs:23-214) driven by Reader::handle_datafrag_msg
// (io_uring/rtps/reader.rs:563-647).  The reference walks DATA_FRAG
// submessages one at a time; here a whole parsed batch is assembled at once,
// with the same result as the sequential walk in record order
// (the CPU restatement that tests/ check it against):
//
//  1 sort   every DATA_FRAG record with ROUTE_PASS is keyed by a 32-bit hash of
//           (writer GUID, SN); a stable sort (rtps_bsort.h: top-byte buckets,
//           then an LDS radix sort per bucket) groups each assembly buffer's
//           fragments in record order (hash collisions are resolved by the
//           walk, which compares full keys).
//  2 writers the fragment size of a writer is the one of its first DATA_FRAG
//           ever (FragmentAssembler::new): persistent open-addressing table,
//           atomicMin over the batch's first records of new writers.
//  3 walk   one thread per key run replays AssemblyBuffer::new / insert_frags /
//           is_complete on a bitmap (starting from the buffer carried over from
//           the previous batch, if any) and cuts the run into epochs: each
//           completed buffer, and at most one still incomplete.
//  4 place  completed samples are ranked by completing record (exclusive scans)
//           and get 16-byte-aligned heap offsets; incomplete buffers get room in
//           the next pending store.
//  5 copy   a regular epoch (no repeated fragment, fragment size equal to the
//           writer's, no clamping) tiles its buffer with its fragments' spans,
//           so every record copies its span (payload, then zeros for a short
//           payload) in parallel, two records per wave step, after the
//           carried-over bytes were copied.  Irregular epochs replay the copies in record
//           order in one workgroup each (rare).
//
// Roofline: HBM-bound.  Algorithmic bytes per DATA_FRAG record = its payload
// bytes read + the same bytes written + 64 B of the record read.
#include <hip/hip_runtime.h>

#include "rtps_bsort.h"
#include "rtps_sort.h"
#include <string.h>

#include <new>

#include "rtps_frag.h"

namespace {

constexpr uint32_t FT = 256;             // threads per block
constexpr uint32_t NONE = 0xffffffffu;
constexpr uint32_t SENT = 0xffffffffu;   // sort key of records that are not assembled
constexpr uint32_t FIXED = 0x80000000u;  // writer table: fragment size resolved
// Assembly keys are five words: the writer GUID (prefix || writer_id, record
// bytes 8..24) and a reader word, kept per batch position in rword[] by k_keys
// (FragSel):
//   mode 0, no readers: word 0, every DATA_FRAG that passes: one assembler per writer;
//   mode 1, readers, every target set of at most one reader: k_keys looks up the
//     record's reader (the target set, rtps_readers.h) and its Lifespan, word =
//     slot | 0x10000, records that reach no reader (or whose Lifespan has expired
//     for that reader) are not assembled;
//   mode 2, readers with larger sets: the batch is an expansion with one copy of a
//     DATA_FRAG record per target reader (rtps_rx.hip frag_x_*), the word in the
//     copy's reader_id field.
// So every (reader, writer) pair has its own assembler, as every Reader has its
// own FragmentAssembler per writer (io_uring/rtps/reader.rs:617-619, 638-647).
constexpr int KW = 5;

constexpr uint32_t WCAP = 1u << 16;      // writers
constexpr uint32_t PCAP = 1u << 16;      // pending buffers
constexpr uint32_t PTCAP = 2 * PCAP;     // pending hash table slots
constexpr uint64_t PBYTES = 1ull << 28;  // pending byte store (per side)
constexpr uint64_t PWORDS = 1ull << 22;  // pending bitmap words (per side)

// counters (device u64)
enum { C_OLD_N = 0, C_NEW_N, C_NEW_BYTES, C_NEW_WORDS, C_SPECIAL, C_POOL, C_OVERFLOW, C_LIVE, C_COUNT };

enum EpochState : uint32_t { E_PENDING = 0, E_DONE = 1, E_DEAD = 2 };  // DEAD: bitmap allocation failed
enum EpochFlags : uint32_t { EF_IRREGULAR = 1, EF_SKIP = 2 };  // SKIP: no bytes to write (no room)

struct Epoch {
  uint32_t guid[KW];
  int64_t sn;
  uint32_t data_size, count, nset, F;
  uint32_t state, eflags;
  uint32_t done_rec;   // completing record
  uint32_t rec_flags;  // DATA_FRAG flags of the completing record
  uint32_t old_pend;   // previous batch's pending entry it continues, or NONE
  uint32_t p0, p1;     // sorted-position range of its key run
  uint32_t new_pend;   // new pending entry (state PENDING)
  uint64_t bits;       // word offset of its bitmap in the walk pool
  uint64_t dst;        // heap offset (DONE) or new pending byte offset (PENDING)
};

struct Pend {
  uint32_t guid[KW];
  int64_t sn;
  uint32_t data_size, count, nset, consumed;  // consumed: continued by this batch, or expired by gc
  uint64_t bytes;     // offset in the pending byte store
  uint64_t bits;      // word offset in the pending bitmap store
  uint64_t modified;  // clock of the last batch that inserted fragments (AssemblyBuffer::modified_time)
};

__device__ __forceinline__ void guid_of(const rtps_record* r, uint32_t word, uint32_t g[KW]) {
  const uint4 v = *(const uint4*)((const uint8_t*)r + 8);  // prefix[12] @8, writer_id @20
  g[0] = v.x; g[1] = v.y; g[2] = v.z; g[3] = v.w;
  g[4] = word;
}
__device__ __forceinline__ uint32_t fmix32(uint32_t h) {
  h ^= h >> 16; h *= 0x85ebca6bu; h ^= h >> 13; h *= 0xc2b2ae35u; h ^= h >> 16;
  return h;
}
__device__ __forceinline__ uint32_t key_hash(const uint32_t g[KW], int64_t sn) {
  uint32_t h = 0x811c9dc5u;
  h = (h ^ g[0]) * 0x01000193u; h = (h ^ g[1]) * 0x01000193u; h = (h ^ g[2]) * 0x01000193u;
  h = (h ^ g[3]) * 0x01000193u; h = (h ^ g[4]) * 0x01000193u; h = (h ^ (uint32_t)sn) * 0x01000193u; h = (h ^ (uint32_t)(sn >> 32)) * 0x01000193u;
  h = fmix32(h);
  return h == SENT ? SENT - 1 : h;
}
__device__ __forceinline__ uint64_t writer_hash(const uint32_t g[KW]) {
  uint32_t a = 0x811c9dc5u, b = 0x9e3779b9u;
  for (int k = 0; k < KW; ++k) { a = (a ^ g[k]) * 0x01000193u; b = fmix32(b ^ g[k]) + 0x7f4a7c15u; }
  return (((uint64_t)fmix32(a) << 32) | fmix32(b)) | 1ull;
}
__device__ __forceinline__ bool same_key(const uint32_t a[KW], int64_t asn, const uint32_t b[KW], int64_t bsn) {
  return a[0] == b[0] && a[1] == b[1] && a[2] == b[2] && a[3] == b[3] && a[4] == b[4] && asn == bsn;
}
// workgroup-wide copy / zero fill of n bytes, 16 B per thread where possible
__device__ __forceinline__ void blk_copy(uint8_t* d, const uint8_t* s, uint64_t n) {
  uint64_t b = 16ull * threadIdx.x;
  for (; b + 16 <= n; b += 16ull * FT) {
    uint4 v;
    __builtin_memcpy(&v, s + b, 16);
    __builtin_memcpy(d + b, &v, 16);
  }
  for (uint64_t t = (n & ~15ull) + threadIdx.x; t < n; t += FT) d[t] = s[t];
}
__device__ __forceinline__ void blk_zero(uint8_t* d, uint64_t n) {
  const uint4 z = make_uint4(0, 0, 0, 0);
  uint64_t b = 16ull * threadIdx.x;
  for (; b + 16 <= n; b += 16ull * FT) __builtin_memcpy(d + b, &z, 16);
  for (uint64_t t = (n & ~15ull) + threadIdx.x; t < n; t += FT) d[t] = 0;
}
__device__ __forceinline__ uint32_t rl(uint32_t v, uint32_t l) { return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)l); }
__device__ __forceinline__ bool is_frag(const rtps_record* r) { return r->kind == RTPS_DATA_FRAG && (r->route & RTPS_ROUTE_PASS); }

__device__ __forceinline__ uint32_t wslot_find(const uint64_t* wkey, uint64_t h) {
  uint32_t s = (uint32_t)(h >> 7) & (WCAP - 1);
  for (uint32_t i = 0; i < WCAP; ++i, s = (s + 1) & (WCAP - 1)) {
    const uint64_t k = wkey[s];
    if (k == h) return s;
    if (k == 0) return NONE;
  }
  return NONE;
}

// Which DATA_FRAG records (that pass) the batch assembles, and their reader word (FragSel)
__device__ __forceinline__ bool frag_select(const FragSel& sel, const rtps_record* r, const uint4& ra, const uint4& rb,
                                            uint32_t& word) {
  word = 0;
  if (sel.mode == 0) return true;
  if (sel.mode == 2) { word = rb.z; return true; }  // an expanded copy: its reader_id
  // mode 1: the record's one target reader (Domain::handle_event, dp_event_loop.rs:266-327)
  const uint32_t route = (rb.w >> 16) & 0xffu;
  if (!(route & RTPS_ROUTE_TARGETED) || (route & RTPS_ROUTE_BUILTIN)) return false;
  uint32_t r2 = 0;
  const uint32_t set = rt_classify<false>(sel.rt, nullptr, ra.z, ra.w, rb.x, rb.y, r2);
  if (set == RTPS_NO_TARGET || sel.rt.set_first[set] == sel.rt.set_first[set + 1]) return false;
  const uint32_t slot = sel.rt.set_ent[sel.rt.set_first[set]].reader_slot;
  if (sel.any_life && (route & RTPS_ROUTE_TS_VALID)) {  // handle_datafrag_msg's Lifespan drop (reader.rs:578-589)
    const int64_t L = sel.life[slot];
    const uint64_t src = ((uint64_t)r->ts_sec << 32) | r->ts_frac;
    if (L != INT64_MAX && L < (int64_t)(sel.recv_ticks - src)) return false;
  }
  word = slot | 0x10000u;
  return true;
}

// ---- 1: sort keys ----
// Also collects the batch's writers (step 2's input): each wave dedupes its
// records' writers with ballots (one LDS insert per distinct writer, by its first
// lane: the smallest record index), each workgroup in LDS, and stages its first
// WST distinct writers with their first records (no global atomics: a thousand
// workgroups would all hit the same few writers' words).  writers_reg_wg merges
// the stages into the persistent table; a workgroup's writers past WST go there
// directly.
constexpr uint32_t WST = 8;       // staged writers per k_keys workgroup
constexpr uint32_t KGRID = 2048;  // k_keys workgroups at most
__device__ void writer_insert(uint64_t wh, uint32_t r, uint64_t* wkey, uint32_t* wfirst, const uint32_t* wF,
                              uint64_t* ctr) {
  uint32_t s = (uint32_t)(wh >> 7) & (WCAP - 1);
  uint32_t t = 0;
  for (; t < WCAP; ++t, s = (s + 1) & (WCAP - 1)) {
    // a plain probe first: slots only go from 0 to a writer
    const uint64_t cur = __atomic_load_n((const unsigned long long*)&wkey[s], __ATOMIC_RELAXED);
    if (cur == wh) break;
    if (cur != 0) continue;
    const uint64_t old = atomicCAS((unsigned long long*)&wkey[s], 0ull, (unsigned long long)wh);
    if (old == 0 || old == wh) break;
  }
  if (t == WCAP) { ctr[C_COUNT] = 1ull; return; }  // table full: reported by writers_fix_wg
  // wfirst only decreases: a plain read skips the atomic when an earlier record is in
  if (!(wF[s] & FIXED) && r < __atomic_load_n(&wfirst[s], __ATOMIC_RELAXED)) atomicMin(&wfirst[s], r);
}
constexpr uint32_t KPT = 4, KPASS = FT * KPT;  // records per thread / per workgroup pass
constexpr uint32_t KW_SLOTS = 2 * KPASS;       // >= 2 x records per workgroup pass
__global__ __launch_bounds__(FT) void k_keys(const rtps_record* recs, const uint64_t* n_rec, uint64_t max,
                                             uint32_t* keys, uint32_t* vals, uint32_t* rec_epoch, uint32_t* dmark,
                                             uint8_t* seen, uint64_t* ctr, uint32_t* new_ptable, uint64_t* wkey,
                                             uint32_t* wfirst, const uint32_t* wF, uint64_t* wst_key,
                                             uint32_t* wst_rec, FragSel sel, uint32_t* rword) {
  __shared__ unsigned long long s_wk[KW_SLOTS];
  __shared__ uint32_t s_wr[KW_SLOTS];
  __shared__ uint32_t s_nst;
  // the batch's counters and the next pending table start empty (instead of two memsets)
  if (blockIdx.x == 0 && threadIdx.x < C_COUNT - C_NEW_N) ctr[C_NEW_N + threadIdx.x] = 0ull;
  for (uint64_t t = (uint64_t)blockIdx.x * FT + threadIdx.x; t < PTCAP; t += (uint64_t)gridDim.x * FT)
    new_ptable[t] = NONE;
  for (uint32_t j = threadIdx.x; j < KW_SLOTS; j += FT) { s_wk[j] = 0ull; s_wr[j] = NONE; }
  if (threadIdx.x == 0) s_nst = 0u;
  __syncthreads();
  const uint64_t n = min(*n_rec, max);
  const uint32_t lane = threadIdx.x & 63u;
  for (uint64_t i0 = (uint64_t)blockIdx.x * KPASS; i0 < max; i0 += (uint64_t)gridDim.x * KPASS) {  // uniform trips
    // each thread's KPT records: bytes 0..39 (kind @6, GUID @8..23, route @30, sn @32)
    // loaded together, without a dependent second load for DATA_FRAG records
    uint4 ra[KPT], rb[KPT];
    uint64_t rs[KPT];
#pragma unroll
    for (uint32_t k = 0; k < KPT; ++k) {
      const uint64_t i = i0 + k * FT + threadIdx.x;
      ra[k] = rb[k] = make_uint4(0, 0, 0, 0);
      rs[k] = 0;
      if (i < n) {
        const uint4* q = reinterpret_cast<const uint4*>(recs + i);
        ra[k] = q[0];
        rb[k] = q[1];
        rs[k] = *reinterpret_cast<const uint64_t*>(q + 2);
      }
    }
#pragma unroll
    for (uint32_t kk = 0; kk < KPT; ++kk) {
      const uint64_t i = i0 + kk * FT + threadIdx.x;
      bool f = false;
      uint64_t wh = 0;
      if (i < max) {
        uint32_t k = SENT;
        const uint32_t kind = (ra[kk].y >> 16) & 0xffu, route = (rb[kk].w >> 16) & 0xffu;
        uint32_t word = 0;
        if (i < n && kind == RTPS_DATA_FRAG && (route & RTPS_ROUTE_PASS) &&
            frag_select(sel, recs + i, ra[kk], rb[kk], word)) {  // is_frag
          const uint32_t g[KW] = {ra[kk].z, ra[kk].w, rb[kk].x, rb[kk].y, word};  // guid_of
          k = key_hash(g, (int64_t)rs[kk]);
          wh = writer_hash(g);
          f = true;
        }
        keys[i] = k;
        rword[i] = word;
        if (vals) vals[i] = (uint32_t)i;  // the device sort's values (the bucket sort derives them)
        rec_epoch[i] = NONE;  // per-batch state, reset here instead of three memsets
        dmark[i] = NONE;
        seen[i] = 0;
      }
      // one LDS insert per distinct writer of the wave, by its lowest lane
      for (uint64_t todo = __ballot(f); todo;) {
        const uint32_t l = (uint32_t)__builtin_ctzll(todo);
        const uint64_t lh = ((uint64_t)rl((uint32_t)(wh >> 32), l) << 32) | rl((uint32_t)wh, l);
        todo &= ~__ballot(f && wh == lh);
        if (lane == l) {
          uint32_t h = (uint32_t)(lh >> 7) & (KW_SLOTS - 1);
          for (;;) {  // fewer distinct writers than slots: always ends
            const unsigned long long old = atomicCAS(&s_wk[h], 0ull, (unsigned long long)lh);
            if (old == 0ull || old == lh) break;
            h = (h + 1) & (KW_SLOTS - 1);
          }
          atomicMin(&s_wr[h], (uint32_t)i);
        }
      }
    }
    __syncthreads();
    // stage the pass's writers (or insert them directly past WST)
    for (uint32_t j = threadIdx.x; j < KW_SLOTS; j += FT) {
      const uint64_t wh = s_wk[j];
      if (!wh) continue;
      const uint32_t r = s_wr[j];
      s_wk[j] = 0ull;
      s_wr[j] = NONE;
      const uint32_t q = atomicAdd(&s_nst, 1u);
      if (q < WST) {
        wst_key[(uint64_t)blockIdx.x * WST + q] = wh;
        wst_rec[(uint64_t)blockIdx.x * WST + q] = r;
      } else {
        writer_insert(wh, r, wkey, wfirst, wF, ctr);
      }
    }
    __syncthreads();
  }
  for (uint32_t q = s_nst + threadIdx.x; q < WST; q += FT) wst_key[(uint64_t)blockIdx.x * WST + q] = 0ull;
}

// ---- 2: writers: the fragment size of a writer is its first DATA_FRAG's ever (registered by k_keys) ----
// The walk reads it through writer_F (the batch's first record of a new writer);
// after the walk, writers_fix_wg stores it for the next batches.
__device__ void writers_fix_wg(const rtps_record* recs, const uint64_t* wkey, uint32_t* wfirst, uint32_t* wF,
                               uint64_t* ctr, uint32_t bid) {
  const uint32_t s = bid * FT + threadIdx.x;
  if (s == 0 && ctr[C_COUNT]) {  // k_keys found the writer table full
    atomicOr((unsigned long long*)&ctr[C_OVERFLOW], 1ull);
    ctr[C_COUNT] = 0ull;
  }
  if (s >= WCAP || wkey[s] == 0 || (wF[s] & FIXED) || wfirst[s] == NONE) return;
  wF[s] = (uint32_t)recs[wfirst[s]].u.frag.frag_size | FIXED;
  wfirst[s] = NONE;
}

// merge k_keys' staged writers into the persistent table: WREG_WG workgroups take
// a range of the stages each (all loads in flight at once), dedupe it in LDS, and
// insert each distinct writer: a few workgroups per writer's words, not a thousand
constexpr uint32_t WREG_WG = 16, WR_SLOTS = 1024, WR_U = 4;
__device__ void writers_reg_wg(const uint64_t* wst_key, const uint32_t* wst_rec, uint32_t n_st, uint64_t* wkey,
                               uint32_t* wfirst, const uint32_t* wF, uint64_t* ctr, uint32_t part) {
  __shared__ unsigned long long s_k[WR_SLOTS];
  __shared__ uint32_t s_r[WR_SLOTS];
  for (uint32_t j = threadIdx.x; j < WR_SLOTS; j += FT) { s_k[j] = 0ull; s_r[j] = NONE; }
  __syncthreads();
  const uint32_t per = (n_st + WREG_WG - 1) / WREG_WG, lo = part * per, hi = min(lo + per, n_st);
  for (uint32_t e0 = lo; e0 < hi; e0 += FT * WR_U) {
    uint64_t k[WR_U];
    uint32_t r[WR_U];
#pragma unroll
    for (uint32_t u = 0; u < WR_U; ++u) {
      const uint32_t e = e0 + u * FT + threadIdx.x;
      k[u] = e < hi ? wst_key[e] : 0ull;
      r[u] = e < hi ? wst_rec[e] : NONE;
    }
#pragma unroll
    for (uint32_t u = 0; u < WR_U; ++u) {
      if (!k[u]) continue;
      uint32_t h = (uint32_t)(k[u] >> 23) & (WR_SLOTS - 1), t = 0;
      for (; t < WR_SLOTS; ++t, h = (h + 1) & (WR_SLOTS - 1)) {
        const unsigned long long old = atomicCAS(&s_k[h], 0ull, (unsigned long long)k[u]);
        if (old == 0ull || old == k[u]) break;
      }
      if (t < WR_SLOTS) atomicMin(&s_r[h], r[u]);
      else writer_insert(k[u], r[u], wkey, wfirst, wF, ctr);  // more writers than LDS slots
    }
  }
  __syncthreads();
  for (uint32_t j = threadIdx.x; j < WR_SLOTS; j += FT)
    if (s_k[j]) writer_insert(s_k[j], s_r[j], wkey, wfirst, wF, ctr);
}
__global__ __launch_bounds__(FT) void k_wreg(const uint64_t* wst_key, const uint32_t* wst_rec, uint32_t n_st,
                                             uint64_t* wkey, uint32_t* wfirst, const uint32_t* wF, uint64_t* ctr) {
  writers_reg_wg(wst_key, wst_rec, n_st, wkey, wfirst, wF, ctr, blockIdx.x);
}
// the same as the bucket sort's side job
struct WregSide {
  uint32_t wgs;
  const uint64_t* wst_key;
  const uint32_t* wst_rec;
  uint32_t n_st;
  uint64_t* wkey;
  uint32_t* wfirst;
  const uint32_t* wF;
  uint64_t* ctr;
  __device__ void operator()(uint32_t i) const { writers_reg_wg(wst_key, wst_rec, n_st, wkey, wfirst, wF, ctr, i); }
};

// ---- 3: walk ----
__device__ uint32_t pend_lookup(const uint32_t* ptable, const Pend* pend, uint32_t kh, const uint32_t g[KW],
                                int64_t sn) {
  uint32_t s = kh & (PTCAP - 1);
  for (uint32_t i = 0; i < PTCAP; ++i, s = (s + 1) & (PTCAP - 1)) {
    const uint32_t j = ptable[s];
    if (j == NONE) return NONE;
    if (same_key(pend[j].guid, pend[j].sn, g, sn)) return j;
  }
  return NONE;
}

struct WalkArgs {
  const rtps_record* recs;
  const uint32_t* skeys;
  const uint32_t* svals;
  uint64_t max;
  const uint64_t* wkey;
  const uint32_t* wF;
  const uint32_t* wfirst;
  Pend* old_pend;
  const uint32_t* old_ptable;
  const uint32_t* old_bits;
  Epoch* epochs;    // indexed by the sorted position of the epoch's first record
  uint32_t* special; // epochs needing more than their records' spans: continued, pending or irregular
  uint32_t* pool;
  uint64_t pool_words;
  uint32_t* rec_epoch;  // per record: its epoch (NONE: not assembled)
  uint32_t* dmark;
  uint8_t* seen;  // per position: consumed by a walk pass (collision runs)
  uint64_t* ctr;
  const uint32_t* rword;  // per position: the reader word of its assembly key (k_keys)
};
__device__ __forceinline__ void guid_at(const WalkArgs& A, uint32_t ri, uint32_t g[KW]) {
  guid_of(A.recs + ri, A.rword[ri], g);
}

// FragmentAssembler's fragment size of writer slot ws: fixed in an earlier batch, or
// its first DATA_FRAG in this one (k_keys' atomicMin), or 0 for no writer
__device__ __forceinline__ uint32_t writer_F(const WalkArgs& A, uint32_t ws) {
  if (ws == NONE) return 0u;
  const uint32_t f = A.wF[ws];
  if (f & FIXED) return f & 0xffffu;
  const uint32_t r = A.wfirst[ws];
  return r == NONE ? 0u : (uint32_t)A.recs[r].u.frag.frag_size;
}

// Epoch ids are the sorted position where the epoch starts (its first record,
// or the run's first position for a buffer carried over): distinct, no counter.
__device__ uint32_t new_epoch(const WalkArgs& A, const uint32_t g[KW], int64_t sn, uint32_t start, uint32_t p0,
                              uint32_t p1) {
  const uint32_t e = start;
  Epoch& E = A.epochs[e];
  for (int k = 0; k < KW; ++k) E.guid[k] = g[k];
  E.sn = sn; E.state = E_PENDING; E.eflags = 0; E.done_rec = NONE; E.old_pend = NONE; E.new_pend = NONE;
  E.p0 = p0; E.p1 = p1; E.nset = 0; E.rec_flags = 0; E.dst = 0; E.bits = 0;
  return e;
}
// after an epoch's last record: list it if the copy phase needs more than spans
__device__ void epoch_done(const WalkArgs& A, uint32_t e) {
  const Epoch& E = A.epochs[e];
  if (E.state == E_DEAD) return;
  if (E.old_pend != NONE || E.state == E_PENDING || (E.eflags & EF_IRREGULAR))
    A.special[atomicAdd((unsigned long long*)&A.ctr[C_SPECIAL], 1ull)] = e;
}
__device__ bool alloc_bits(const WalkArgs& A, Epoch& E) {
  const uint64_t words = ((uint64_t)E.count + 31) / 32;
  const uint64_t at = atomicAdd((unsigned long long*)&A.ctr[C_POOL], (unsigned long long)words);
  if (at + words > A.pool_words) {
    atomicOr((unsigned long long*)&A.ctr[C_OVERFLOW], 4ull);
    E.state = E_DEAD;
    E.eflags |= EF_SKIP;
    return false;
  }
  E.bits = at;
  return true;
}

// Sequential replay of one key run [p, p1) by one thread: the general case
// (hash collisions mixing several keys in one run, bitmaps larger than LDS).
__device__ void walk_run_serial(const WalkArgs& A, uint64_t p, uint64_t p1) {
  const uint32_t key = A.skeys[p];
  // one pass per distinct full key of the run (more than one only on a hash collision)
  for (uint64_t q0 = p; q0 < p1; ++q0) {
    if (A.seen[q0]) continue;
    uint32_t g[KW];
    const rtps_record* r0 = A.recs + A.svals[q0];
    guid_at(A, A.svals[q0], g);
    const int64_t sn = r0->sn;
    const uint64_t wh = writer_hash(g);
    const uint32_t ws = wslot_find(A.wkey, wh);
    const uint32_t F = writer_F(A, ws);
    // continue the buffer carried over from the previous batch
    uint32_t e = NONE;
    bool started = false;
    const uint32_t j = pend_lookup(A.old_ptable, A.old_pend, key, g, sn);
    if (j != NONE) {
      e = new_epoch(A, g, sn, (uint32_t)q0, (uint32_t)p, (uint32_t)p1);
      if (e != NONE) {
        Epoch& E = A.epochs[e];
        const Pend& P = A.old_pend[j];
        A.old_pend[j].consumed = 1;
        E.data_size = P.data_size; E.count = P.count; E.nset = P.nset; E.F = F; E.old_pend = j;
        if (alloc_bits(A, E)) {
          const uint64_t words = ((uint64_t)E.count + 31) / 32;
          for (uint64_t w = 0; w < words; ++w) A.pool[E.bits + w] = A.old_bits[P.bits + w];
          started = true;
        }
      }
    }
    for (uint64_t q = q0; q < p1; ++q) {
      if (A.seen[q]) continue;
      const uint32_t ri = A.svals[q];
      const rtps_record* r = A.recs + ri;
      uint32_t h[KW];
      guid_at(A, ri, h);
      if (!same_key(g, sn, h, r->sn)) continue;
      A.seen[q] = 1;
      const uint32_t ds = r->u.frag.data_size, fsz = r->u.frag.frag_size;
      if (!started) {  // AssemblyBuffer::new (fragment_assembler.rs:35-63)
        e = new_epoch(A, g, sn, (uint32_t)q, (uint32_t)p, (uint32_t)p1);
        Epoch& E = A.epochs[e];
        E.data_size = ds;
        E.count = ds / fsz + (ds % fsz > 0);
        E.F = F;
        if (!alloc_bits(A, E)) { A.rec_epoch[ri] = NONE; continue; }
        for (uint64_t w = 0; w < ((uint64_t)E.count + 31) / 32; ++w) A.pool[E.bits + w] = 0u;
        if (F != fsz) E.eflags |= EF_IRREGULAR;  // spans do not tile the buffer
        started = true;
      }
      Epoch& E = A.epochs[e];
      A.rec_epoch[ri] = e;
      // insert_frags (:65-140): byte range and fragment bits
      const uint64_t start0 = (uint64_t)r->u.frag.frag_start - 1, fis = r->u.frag.frags_in_sub;
      const uint64_t from = start0 * E.F;
      if (from > E.data_size) E.eflags |= EF_IRREGULAR;  // reference panics; clamped
      for (uint64_t k = 0; k < fis; ++k) {
        const uint64_t bit = start0 + k;
        if (bit >= E.count) { E.eflags |= EF_IRREGULAR; break; }  // reference panics; ignored
        uint32_t& word = A.pool[E.bits + bit / 32];
        const uint32_t m = 1u << (bit & 31);
        if (word & m) E.eflags |= EF_IRREGULAR;  // repeated fragment: copy order matters
        else { word |= m; E.nset++; }
      }
      if (E.nset == E.count) {  // is_complete -> emit, drop the buffer
        E.state = E_DONE;
        E.done_rec = ri;
        E.rec_flags = r->flags;
        A.dmark[ri] = e;
        started = false;
        epoch_done(A, e);
      }
    }
    if (started) epoch_done(A, e);  // still incomplete (bitmap already in the pool)
  }
}

constexpr uint32_t BMW = 1024;  // LDS bitmap words per wave: buffers of up to 32768 fragments


// The common run, decided without stepping: one new buffer (nothing carried
// over), at most 64 records, each a single fragment of the writer's size with
// the buffer's data size, all fragment numbers distinct and inside the
// buffer.  Every record then sets one new bit, so the buffer completes at the
// count-th record: with m <= count records it is complete iff m == count
// (is_complete at the last record), else pending with exactly these bits.
// The same outcome as walk_run_wave's replay below (which handles the rest);
// returns false, having written nothing but LDS, when the run is not of this
// form.
// one lane's record of a short run (position p0 + lane), loaded once
struct LaneRec {
  bool act;
  uint32_t ri, g[KW], fs, fis, fsz, dsz, fl;
  int64_t sn;
};
__device__ __forceinline__ LaneRec lane_rec(const WalkArgs& A, uint64_t p, uint64_t p1) {
  LaneRec L;
  L.act = p < p1;
  L.ri = 0; L.g[0] = L.g[1] = L.g[2] = L.g[3] = L.g[4] = 0; L.fs = 1; L.fis = 1; L.fsz = 0; L.dsz = 0; L.fl = 0; L.sn = 0;
  if (L.act) {
    L.ri = A.svals[p];
    const rtps_record* r = A.recs + L.ri;
    guid_at(A, L.ri, L.g);
    L.sn = r->sn;
    L.fs = r->u.frag.frag_start;
    L.fis = r->u.frag.frags_in_sub;
    L.fsz = r->u.frag.frag_size;
    L.dsz = r->u.frag.data_size;
    L.fl = r->flags;
  }
  return L;
}
__device__ bool walk_run_regular(const WalkArgs& A, uint64_t p0, uint64_t p1, uint32_t lane, uint32_t* bm,
                                 const uint32_t g[KW], int64_t sn, uint32_t F, const LaneRec& L) {
  const bool act = L.act;
  const uint32_t ri = L.ri, fs = L.fs, fis = L.fis, fsz = act ? L.fsz : F, dsz = L.dsz, fl = L.fl;
  const uint32_t ds0 = rl(dsz, 0);
  const uint32_t count = ds0 / F + (ds0 % F > 0);  // AssemblyBuffer::new with the first record (fsz == F)
  const uint32_t m = (uint32_t)(p1 - p0);
  const uint64_t bit = (uint64_t)fs - 1;
  const bool bad = act && (fis != 1 || fsz != F || dsz != ds0 || fs == 0 || bit >= count);
  if (__any(bad) || m > count || count > BMW * 32) return false;
  for (uint32_t w = lane; w < (count + 31) / 32; w += 64) bm[w] = 0u;
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  bool dup = false;
  if (act) dup = ((atomicOr(&bm[bit / 32], 1u << (bit & 31)) >> (bit & 31)) & 1u) != 0;
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  if (__any(dup)) return false;  // a repeated fragment: replay in order
  uint32_t e0 = NONE;
  if (lane == 0) e0 = new_epoch(A, g, sn, (uint32_t)p0, (uint32_t)p0, (uint32_t)p1);
  const uint32_t e = rl(e0, 0);
  if (act) A.rec_epoch[ri] = e;
  if (m == count) {  // is_complete at the last record -> emit
    const uint32_t rlast = rl(ri, m - 1), flast = rl(fl, m - 1);
    if (lane == 0) {
      Epoch& E = A.epochs[e];
      E.data_size = ds0; E.count = count; E.nset = m; E.F = F; E.eflags = 0; E.state = E_DONE;
      E.done_rec = rlast; E.rec_flags = flast; E.old_pend = NONE;
      A.dmark[rlast] = e;
      epoch_done(A, e);
    }
    return true;
  }
  // still incomplete: its bitmap goes to the pool for the pending store
  uint64_t bits = 0;
  bool got = true;
  if (lane == 0) {
    Epoch& E = A.epochs[e];
    E.count = count;
    got = alloc_bits(A, E);
    bits = E.bits;
  }
  got = rl(got ? 1u : 0u, 0) != 0;
  const uint64_t b = ((uint64_t)rl((uint32_t)(bits >> 32), 0) << 32) | rl((uint32_t)bits, 0);
  if (got) {
    for (uint32_t w = lane; w < (count + 31) / 32; w += 64) A.pool[b + w] = bm[w];
    if (lane == 0) {
      Epoch& E = A.epochs[e];
      E.data_size = ds0; E.count = count; E.nset = m; E.F = F; E.eflags = 0; E.state = E_PENDING;
      E.done_rec = NONE; E.rec_flags = 0; E.old_pend = NONE;
      epoch_done(A, e);
    }
  }
  return true;
}

// One key run replayed by a wave: each lane loads one record's fields, the
// wave steps through them in order with the fragment bitmap in LDS.  Runs that
// mix keys or need a bigger bitmap fall back to walk_run_serial on lane 0.
__device__ void walk_run_wave(const WalkArgs& A, uint64_t p0, uint64_t p1, uint32_t lane, uint32_t* bm,
                              uint32_t key) {
  if (p1 - p0 <= 64) {
    // a short run: every lane loads its record once; the run's key, the carried-over
    // buffer and the writer's fragment size are then looked up with independent loads
    const LaneRec L = lane_rec(A, p0 + lane, p1);
    uint32_t g[KW];
    for (int k = 0; k < KW; ++k) g[k] = rl(L.g[k], 0);
    const int64_t sn = (int64_t)(((uint64_t)rl((uint32_t)((uint64_t)L.sn >> 32), 0) << 32) | rl((uint32_t)L.sn, 0));
    const bool bad = L.act && (!same_key(g, sn, L.g, L.sn) ||
                               (uint64_t)(L.dsz / L.fsz + (L.dsz % L.fsz > 0)) > (uint64_t)BMW * 32);
    const uint64_t wh = writer_hash(g);
    const uint32_t ps = key & (PTCAP - 1), ws0 = (uint32_t)(wh >> 7) & (WCAP - 1);
    const uint32_t pj = A.old_ptable[ps];
    const uint64_t wk = A.wkey[ws0];
    if (!__any(bad) && pj == NONE) {  // nothing carried over (the first probe is empty)
      const uint32_t ws = wk == wh ? ws0 : (wk == 0 ? NONE : wslot_find(A.wkey, wh));
      const uint32_t F = writer_F(A, ws);
      if (F != 0 && walk_run_regular(A, p0, p1, lane, bm, g, sn, F, L)) return;
    }
  }
  const rtps_record* r0 = A.recs + A.svals[p0];
  uint32_t g[KW];
  guid_at(A, A.svals[p0], g);
  const int64_t sn = r0->sn;
  bool ok = true;
  for (uint64_t c = p0; c < p1 && ok; c += 64) {
    const uint64_t p = c + lane;
    bool bad = false;
    if (p < p1) {
      const rtps_record* r = A.recs + A.svals[p];
      uint32_t h[KW];
      guid_at(A, A.svals[p], h);
      const uint32_t ds = r->u.frag.data_size, fsz = r->u.frag.frag_size;
      bad = !same_key(g, sn, h, r->sn) || (uint64_t)(ds / fsz + (ds % fsz > 0)) > (uint64_t)BMW * 32;
    }
    ok = !__any(bad);
  }
  const uint32_t j = pend_lookup(A.old_ptable, A.old_pend, key, g, sn);
  if (ok && j != NONE && (uint64_t)A.old_pend[j].count > (uint64_t)BMW * 32) ok = false;
  if (!ok) {
    if (lane == 0) walk_run_serial(A, p0, p1);
    return;
  }
  const uint32_t ws = wslot_find(A.wkey, writer_hash(g));
  const uint32_t F = writer_F(A, ws);
  if (j == NONE && p1 - p0 <= 64 && F != 0 && walk_run_regular(A, p0, p1, lane, bm, g, sn, F, lane_rec(A, p0 + lane, p1)))
    return;
  uint32_t e = NONE, nset = 0, count = 0, ds = 0, eflags = 0, old_pend = NONE;
  bool started = false;
  if (j != NONE) {  // continue the buffer carried over from the previous batch
    uint32_t e0 = NONE;
    if (lane == 0) {
      e0 = new_epoch(A, g, sn, (uint32_t)p0, (uint32_t)p0, (uint32_t)p1);
      A.old_pend[j].consumed = 1;
    }
    e = rl(e0, 0);
    if (e != NONE) {
      const Pend& P = A.old_pend[j];
      ds = P.data_size; count = P.count; nset = P.nset; old_pend = j;
      for (uint32_t w = lane; w < (count + 31) / 32; w += 64) bm[w] = A.old_bits[P.bits + w];
      started = true;
    }
  }
  auto finish = [&](uint32_t state, uint32_t done_rec, uint32_t rec_flags) {
    if (lane == 0) {
      Epoch& E = A.epochs[e];
      E.data_size = ds; E.count = count; E.nset = nset; E.F = F; E.eflags = eflags; E.state = state;
      E.done_rec = done_rec; E.rec_flags = rec_flags; E.old_pend = old_pend;
      if (state == E_DONE) A.dmark[done_rec] = e;
      epoch_done(A, e);
    }
  };
  for (uint64_t c = p0; c < p1; c += 64) {
    const uint64_t p = c + lane;
    uint32_t ri = 0, fs = 0, fisz = 0, dsz = 0, fl = 0;
    if (p < p1) {
      ri = A.svals[p];
      const rtps_record* r = A.recs + ri;
      fs = r->u.frag.frag_start;
      fisz = (uint32_t)r->u.frag.frags_in_sub | ((uint32_t)r->u.frag.frag_size << 16);
      dsz = r->u.frag.data_size;
      fl = r->flags;
    }
    uint32_t my_e = NONE;
    uint32_t m = (uint32_t)min<uint64_t>(64, p1 - c);
    for (uint32_t jj = 0; jj < m; ++jj) {
      const uint32_t rj = rl(ri, jj), fsj = rl(fs, jj), fz = rl(fisz, jj), dj = rl(dsz, jj);
      const uint32_t fis = fz & 0xffffu, fsz = fz >> 16;
      if (!started) {  // AssemblyBuffer::new (fragment_assembler.rs:35-63)
        uint32_t e0 = NONE;
        if (lane == 0) e0 = new_epoch(A, g, sn, (uint32_t)(c + jj), (uint32_t)p0, (uint32_t)p1);
        e = rl(e0, 0);
        ds = dj;
        count = dj / fsz + (dj % fsz > 0);
        nset = 0;
        eflags = (F != fsz) ? EF_IRREGULAR : 0u;  // spans do not tile the buffer
        old_pend = NONE;
        for (uint32_t w = lane; w < (count + 31) / 32; w += 64) bm[w] = 0u;
        started = true;
      }
      if (lane == jj) my_e = e;
      // insert_frags (:65-140)
      const uint64_t start0 = (uint64_t)fsj - 1;
      if (start0 * F > ds) eflags |= EF_IRREGULAR;  // reference panics; clamped
      for (uint32_t k = 0; k < fis; ++k) {
        const uint64_t bit = start0 + k;
        if (bit >= count) { eflags |= EF_IRREGULAR; break; }  // reference panics; ignored
        const uint32_t w = bm[bit / 32], msk = 1u << (bit & 31);
        if (w & msk) {
          eflags |= EF_IRREGULAR;  // repeated fragment: copy order matters
        } else {
          if (lane == 0) bm[bit / 32] = w | msk;
          nset++;
        }
      }
      if (nset == count) {  // is_complete -> emit, drop the buffer
        finish(E_DONE, rj, rl(fl, jj));
        started = false;
      }
    }
    if (p < p1) A.rec_epoch[ri] = my_e;
  }
  if (started) {  // still incomplete: its bitmap goes to the pool for the pending store
    uint64_t bits = 0;
    bool got = true;
    if (lane == 0) {
      Epoch& E = A.epochs[e];
      E.count = count;
      got = alloc_bits(A, E);
      bits = E.bits;
    }
    got = rl(got ? 1u : 0u, 0) != 0;
    const uint64_t b = ((uint64_t)rl((uint32_t)(bits >> 32), 0) << 32) | rl((uint32_t)bits, 0);
    if (got) {
      for (uint32_t w = lane; w < (count + 31) / 32; w += 64) A.pool[b + w] = bm[w];
      finish(E_PENDING, NONE, 0);
    }
  }
}

// a wave takes 64 sorted positions and walks every run that starts there
__global__ __launch_bounds__(FT) void k_walk(WalkArgs A) {
  __shared__ uint32_t bms[FT / 64][BMW];
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  for (uint64_t c = ((uint64_t)blockIdx.x * (FT / 64) + wave) * 64; c < A.max; c += (uint64_t)gridDim.x * FT) {
    const uint64_t p = c + lane;
    const uint32_t key = p < A.max ? A.skeys[p] : SENT;
    const bool head = key != SENT && (p == 0 || A.skeys[p - 1] != key);
    uint64_t heads = __ballot(head);
    while (heads) {
      const uint32_t h = (uint32_t)__builtin_ctzll(heads);
      heads &= heads - 1;
      const uint64_t p0 = c + h;
      const uint32_t k0 = rl(key, h);
      uint64_t p1 = p0 + 1;
      for (;;) {  // run end: first position with another key
        const uint64_t q = p1 + lane;
        const bool other = q >= A.max || A.skeys[q] != k0;
        const uint64_t b = __ballot(other);
        if (b) { p1 += __builtin_ctzll(b); break; }
        p1 += 64;
      }
      walk_run_wave(A, p0, p1, lane, bms[wave], k0);
    }
  }
}

// ---- 4: place ----
// Completed samples are ranked by completing record, and their heap offsets are
// the exclusive sum of the preceding completions' 16-B-aligned sizes: a
// two-level scan over 4096-position tiles, 16 consecutive positions per thread.
constexpr uint32_t PPT = 16, PTILE = FT * PPT;
__device__ __forceinline__ void dmark16(const uint32_t* dmark, uint64_t base, uint64_t max, uint32_t d[PPT]) {
  if (base + PPT <= max) {
    const uint4* q = reinterpret_cast<const uint4*>(dmark + base);
#pragma unroll
    for (uint32_t k = 0; k < PPT / 4; ++k) {
      const uint4 v = q[k];
      d[4 * k] = v.x; d[4 * k + 1] = v.y; d[4 * k + 2] = v.z; d[4 * k + 3] = v.w;
    }
  } else {
#pragma unroll
    for (uint32_t k = 0; k < PPT; ++k) d[k] = base + k < max ? dmark[base + k] : NONE;
  }
}
__device__ __forceinline__ uint64_t sample_bytes(const Epoch* ep, uint32_t e) {
  return ((uint64_t)ep[e].data_size + 15) & ~15ull;
}
// workgroup-wide exclusive scan of (count, bytes); returns the totals too
__device__ __forceinline__ void blk_scan_cb(uint32_t c, uint64_t b, uint32_t& ce, uint64_t& be, uint32_t& ct,
                                            uint64_t& bt) {
  __shared__ uint32_t wc[FT / 64];
  __shared__ uint64_t wb[FT / 64];
  const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
  uint32_t xc = c;
  uint64_t xb = b;
  for (uint32_t d = 1; d < 64; d <<= 1) {
    const uint32_t yc = (uint32_t)__shfl_up((int)xc, d, 64);
    const uint32_t ylo = (uint32_t)__shfl_up((int)(uint32_t)xb, d, 64);
    const uint32_t yhi = (uint32_t)__shfl_up((int)(uint32_t)(xb >> 32), d, 64);
    if (lane >= d) { xc += yc; xb += ((uint64_t)yhi << 32) | ylo; }
  }
  if (lane == 63) { wc[w] = xc; wb[w] = xb; }
  __syncthreads();
  uint32_t pc = 0;
  uint64_t pb = 0;
  ct = 0; bt = 0;
  for (uint32_t k = 0; k < FT / 64; ++k) {
    if (k < w) { pc += wc[k]; pb += wb[k]; }
    ct += wc[k]; bt += wb[k];
  }
  ce = pc + xc - c;
  be = pb + xb - b;
  __syncthreads();
}
// per tile: completions and their bytes
__global__ __launch_bounds__(FT) void k_place_tiles(const uint32_t* dmark, const Epoch* ep, uint64_t max,
                                                    uint32_t* tc, uint64_t* tb) {
  const uint64_t base = (uint64_t)blockIdx.x * PTILE + (uint64_t)threadIdx.x * PPT;
  uint32_t d[PPT];
  dmark16(dmark, base, max, d);
  uint32_t c = 0;
  uint64_t b = 0;
#pragma unroll
  for (uint32_t k = 0; k < PPT; ++k)
    if (d[k] != NONE) { ++c; b += sample_bytes(ep, d[k]); }
  uint32_t ce, ct;
  uint64_t be, bt;
  blk_scan_cb(c, b, ce, be, ct, bt);
  if (threadIdx.x == 0) { tc[blockIdx.x] = ct; tb[blockIdx.x] = bt; }
}
// one workgroup: exclusive scan of the tile totals, and the batch's sample count and heap use
__global__ __launch_bounds__(FT) void k_place_scan(uint32_t* tc, uint64_t* tb, uint64_t T, rtps_frag_out out) {
  uint32_t cc = 0;
  uint64_t cb = 0;
  for (uint64_t t0 = 0; t0 < T; t0 += FT) {
    const uint64_t t = t0 + threadIdx.x;
    const uint32_t c = t < T ? tc[t] : 0u;
    const uint64_t b = t < T ? tb[t] : 0ull;
    uint32_t ce, ct;
    uint64_t be, bt;
    blk_scan_cb(c, b, ce, be, ct, bt);
    if (t < T) { tc[t] = cc + ce; tb[t] = cb + be; }
    cc += ct; cb += bt;
  }
  if (threadIdx.x == 0) { *out.n_samples = cc; *out.heap_used = cb; }
}
// tc / tb: the tiles' exclusive prefixes (k_place_scan), or with self_scan (up to
// SELF_SCAN tiles) their raw totals, which each workgroup then sums itself
constexpr uint64_t SELF_SCAN = 2048;
__device__ void samples_wg(const uint32_t* dmark, Epoch* ep, const uint32_t* tc, const uint64_t* tb, uint64_t max,
                           uint32_t self_scan, const rtps_frag_out& out, uint32_t bid, uint32_t ntiles,
                           const uint32_t* emap) {
  const uint64_t base = (uint64_t)bid * PTILE + (uint64_t)threadIdx.x * PPT;
  uint32_t d[PPT];
  dmark16(dmark, base, max, d);
  uint32_t c = 0;
  uint64_t b = 0;
#pragma unroll
  for (uint32_t k = 0; k < PPT; ++k)
    if (d[k] != NONE) { ++c; b += sample_bytes(ep, d[k]); }
  uint32_t ce, ct;
  uint64_t be, bt;
  blk_scan_cb(c, b, ce, be, ct, bt);
  uint64_t pc, pb;
  if (self_scan) {
    pc = 0; pb = 0;
    for (uint32_t t0 = 0; t0 < bid; t0 += FT) {
      const uint32_t t = t0 + threadIdx.x;
      uint32_t xe, xt;
      uint64_t ye, yt;
      blk_scan_cb(t < bid ? tc[t] : 0u, t < bid ? tb[t] : 0ull, xe, ye, xt, yt);
      pc += xt; pb += yt;
    }
    if (bid == ntiles - 1 && threadIdx.x == 0) { *out.n_samples = pc + ct; *out.heap_used = pb + bt; }
  } else {
    pc = tc[bid]; pb = tb[bid];
  }
  if (c == 0) return;
  uint64_t k_rank = pc + ce, hoff = pb + be;
  for (uint32_t k = 0; k < PPT; ++k) {
    const uint32_t e = d[k];
    if (e == NONE) continue;
    Epoch& E = ep[e];
    const uint64_t sz = ((uint64_t)E.data_size + 15) & ~15ull;
    E.dst = hoff;
    const uint64_t kk = k_rank;
    hoff += sz;
    ++k_rank;
    if (kk >= out.max_samples) { E.eflags |= EF_SKIP; continue; }
    rtps_frag_sample s;
    memset(&s, 0, sizeof(s));
    memcpy(s.writer_guid, E.guid, 16);
    s.sn = E.sn;
    s.heap_off = E.dst;
    s.data_size = E.data_size;
    // an expanded batch (one copy per target reader): the copy's record of the parse, and
    // the reader of the key's reader word (slot | 0x10000); else every reader of the record
    s.rec_idx = emap ? emap[base + k] : (uint32_t)(base + k);
    s.reader_slot = E.guid[4] ? (uint16_t)(E.guid[4] & 0xffffu) : (uint16_t)RTPS_NO_MATCH;
    s.flags = (uint8_t)E.rec_flags;
    s.status = E.data_size < 4 ? RTPS_FRAG_SHORT : RTPS_FRAG_OK;
    if (E.dst + E.data_size > out.heap_bytes) { s.status = RTPS_FRAG_NO_ROOM; E.eflags |= EF_SKIP; }
    out.samples[kk] = s;
  }
}

// pending epochs: room in the new pending store + carry their bitmaps
__device__ void pend_alloc_wg(Epoch* ep, const uint32_t* special, Pend* np, uint32_t* nbits, const uint32_t* pool,
                              uint64_t* ctr, uint64_t now, uint32_t bid, uint32_t nb) {
  const uint64_t ns = ctr[C_SPECIAL];
  for (uint64_t i = (uint64_t)bid * FT + threadIdx.x; i < ns; i += (uint64_t)nb * FT) {
    Epoch& E = ep[special[i]];
    if (E.state != E_PENDING) continue;
    const uint64_t words = ((uint64_t)E.count + 31) / 32;
    const uint64_t j = atomicAdd((unsigned long long*)&ctr[C_NEW_N], 1ull);
    const uint64_t b = atomicAdd((unsigned long long*)&ctr[C_NEW_BYTES], ((unsigned long long)E.data_size + 15) & ~15ull);
    const uint64_t w = atomicAdd((unsigned long long*)&ctr[C_NEW_WORDS], (unsigned long long)words);
    if (j >= PCAP || b + E.data_size > PBYTES || w + words > PWORDS) {
      atomicOr((unsigned long long*)&ctr[C_OVERFLOW], 8ull);
      E.eflags |= EF_SKIP;
      continue;
    }
    Pend& P = np[j];
    for (int k = 0; k < KW; ++k) P.guid[k] = E.guid[k];
    P.sn = E.sn; P.data_size = E.data_size; P.count = E.count; P.nset = E.nset; P.consumed = 0;
    P.bytes = b; P.bits = w;
    P.modified = now;  // a pending epoch had fragments in this batch (insert_frags :139)
    for (uint64_t t = 0; t < words; ++t) nbits[w + t] = pool[E.bits + t];
    E.new_pend = (uint32_t)j;
    E.dst = b;
  }
}

// old pending entries no record of this batch continued: move to the new store
__device__ void carry_wg(const Pend* op, const uint8_t* obytes, const uint32_t* obits, Pend* np, uint8_t* nbytes,
                         uint32_t* nbits, uint64_t* ctr, uint32_t bid, uint32_t nb) {
  const uint64_t n_old = ctr[C_OLD_N];
  __shared__ uint64_t sj, sb, sw;
  __shared__ int ok;
  for (uint64_t i = bid; i < n_old; i += nb) {
    const Pend& P = op[i];
    if (P.consumed) continue;
    const uint64_t words = ((uint64_t)P.count + 31) / 32;
    if (threadIdx.x == 0) {
      sj = atomicAdd((unsigned long long*)&ctr[C_NEW_N], 1ull);
      sb = atomicAdd((unsigned long long*)&ctr[C_NEW_BYTES], ((unsigned long long)P.data_size + 15) & ~15ull);
      sw = atomicAdd((unsigned long long*)&ctr[C_NEW_WORDS], (unsigned long long)words);
      ok = !(sj >= PCAP || sb + P.data_size > PBYTES || sw + words > PWORDS);
      if (!ok) atomicOr((unsigned long long*)&ctr[C_OVERFLOW], 8ull);
      else { Pend Q = P; Q.bytes = sb; Q.bits = sw; Q.consumed = 0; np[sj] = Q; }
    }
    __syncthreads();
    if (ok) {
      blk_copy(nbytes + sb, obytes + P.bytes, P.data_size);
      for (uint64_t t = threadIdx.x; t < words; t += FT) nbits[sw + t] = obits[P.bits + t];
    }
    __syncthreads();
  }
}

// after the walk, one launch: completed samples (one workgroup per position tile),
// pending epochs' room in the new store, old entries no record continued carried
// over, and the batch's new writers' fragment sizes stored
constexpr uint32_t PA_WG = 64, CARRY_WG = 1024, WFIX_WG = WCAP / FT;
struct PlaceArgs {
  const uint32_t* dmark;
  Epoch* ep;
  const uint32_t* tc;
  const uint64_t* tb;
  uint64_t max;
  uint32_t self_scan, ntiles;
  const uint32_t* special;
  const uint32_t* pool;
  uint64_t now;
  const Pend* op;
  const uint8_t* obytes;
  const uint32_t* obits;
  Pend* np;
  uint8_t* nbytes;
  uint32_t* nbits;
  uint64_t* ctr;
  const rtps_record* recs;
  const uint64_t* wkey;
  uint32_t* wfirst;
  uint32_t* wF;
  const uint32_t* emap;  // expanded batch: position -> record of the parse (nullptr: none)
};
__global__ __launch_bounds__(FT) void k_place(PlaceArgs P, rtps_frag_out out) {
  uint32_t b = blockIdx.x;
  if (b < P.ntiles) { samples_wg(P.dmark, P.ep, P.tc, P.tb, P.max, P.self_scan, out, b, P.ntiles, P.emap); return; }
  b -= P.ntiles;
  if (b < PA_WG) { pend_alloc_wg(P.ep, P.special, P.np, P.nbits, P.pool, P.ctr, P.now, b, PA_WG); return; }
  b -= PA_WG;
  if (b < CARRY_WG) { carry_wg(P.op, P.obytes, P.obits, P.np, P.nbytes, P.nbits, P.ctr, b, CARRY_WG); return; }
  writers_fix_wg(P.recs, P.wkey, P.wfirst, P.wF, P.ctr, b - CARRY_WG);
}

// ---- 5: copy ----
__device__ __forceinline__ uint8_t* epoch_dst(const Epoch& E, const rtps_frag_out& out, uint8_t* nbytes) {
  return E.state == E_DONE ? out.heap + E.dst : nbytes + E.dst;
}
// regular epochs: carried-over bytes (or zeros for a new pending buffer) first
__device__ void init_wg(const Epoch* ep, const uint32_t* special, const uint64_t* ctr, const Pend* op,
                        const uint8_t* obytes, uint8_t* nbytes, const rtps_frag_out& out, uint32_t bid, uint32_t nb) {
  const uint64_t ns = ctr[C_SPECIAL];
  for (uint64_t i = bid; i < ns; i += nb) {
    const Epoch& E = ep[special[i]];
    if (E.eflags & (EF_IRREGULAR | EF_SKIP)) continue;
    if (E.state == E_DONE && E.old_pend == NONE) continue;  // its spans cover every byte
    uint8_t* d = epoch_dst(E, out, nbytes);
    if (E.old_pend != NONE) {
      const uint8_t* s = obytes + op[E.old_pend].bytes;
      blk_copy(d, s, E.data_size);
    } else {
      blk_zero(d, E.data_size);
    }
  }
}

__device__ __forceinline__ uint4 ld16(const uint8_t* p) { uint4 v; __builtin_memcpy(&v, p, 16); return v; }
__device__ __forceinline__ void st16(uint8_t* p, uint4 v) { __builtin_memcpy(p, &v, 16); }
// the same store through a global (not flat) address: heap and pending store are device memory
typedef __attribute__((address_space(1))) uint4 g_u4 __attribute__((aligned(1)));
__device__ __forceinline__ void gst16(uint8_t* p, uint4 v) {
#if defined(__HIP_DEVICE_COMPILE__)  // the host pass only type-checks device functions
  *(g_u4*)(uintptr_t)p = v;
#else
  __builtin_memcpy(p, &v, 16);
#endif
}

// regular epochs: every record writes its fragments' span (payload, then zeros
// for a short payload).  k_fill resolves each record's span into a descriptor in
// record order; k_span then copies them one wave per record, the waves striding
// over the records, so that the waves resident at any time read and write two
// narrow windows of the arena and the heap (consecutive records are mostly
// consecutive fragments of one sample, and samples are placed in completion
// order).  Copying 64 records per wave in sorted order instead touched samples
// all over both: 619 us on C4 against the same-shape copy ceiling's 524 us
// (scripts/diag_frag_copy.py), and 603 us in record order with 64 per wave.
#ifndef RTPS_SPAN_NT
#define RTPS_SPAN_NT 1      // non-temporal heap stores
#endif
#ifndef RTPS_SPAN_U
#define RTPS_SPAN_U 3       // 16-B loads in flight per lane (3 KiB per wave per step: two C4 records)
#endif
#ifndef SPAN_GRID
#define SPAN_GRID 16384  // span-copy workgroups at most: 16384 0.687-0.688 ms per C4 step, 8192 0.692-0.694, 4096 0.697-0.699
#endif
constexpr uint32_t SPAN_U = RTPS_SPAN_U;
struct SpanDesc {  // 32 B: arena offset of the payload, heap / pending-store address, bytes
  uint64_t src, dst;
  uint32_t nv, n, _r[2];
};
typedef uint32_t nt_u4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) nt_u4 g_nt_u4 __attribute__((aligned(16)));
__device__ __forceinline__ void span_st16(uint8_t* p, uint4 v) {
#if RTPS_SPAN_NT  // non-temporal heap stores (written once, read by the host side later)
  nt_u4 w = {v.x, v.y, v.z, v.w};
#if defined(__HIP_DEVICE_COMPILE__)  // a global (not flat) store: heap and pending store are device memory
  __builtin_nontemporal_store(w, (g_nt_u4*)(uintptr_t)p);
#else
  __builtin_memcpy(p, &w, 16);
#endif
#else
  gst16(p, v);
#endif
}
__device__ void desc_wg(const rtps_record* recs, const uint64_t* dgram_off, const uint32_t* rec_epoch, uint64_t max,
                        const Epoch* ep, uint8_t* nbytes, const rtps_frag_out& out, SpanDesc* desc, uint32_t bid,
                        uint32_t nb) {
  for (uint64_t p = (uint64_t)bid * FT + threadIdx.x; p < max; p += (uint64_t)nb * FT) {
    uint64_t src = 0, dst = 0;
    uint32_t nv = 0, n = 0;
    const uint32_t e = rec_epoch[p];
    if (e != NONE) {
      const Epoch& E = ep[e];
      if (!(E.eflags & (EF_IRREGULAR | EF_SKIP)) && E.state != E_DEAD) {
        const rtps_record* r = recs + p;
        const uint64_t from = (uint64_t)(r->u.frag.frag_start - 1) * E.F;
        const uint64_t fisF = (uint64_t)r->u.frag.frags_in_sub * E.F;
        const uint64_t span_end = min<uint64_t>(from + fisF, E.data_size);
        const uint64_t to = min<uint64_t>(from + min<uint64_t>(fisF, r->u.frag.pl_len), E.data_size);
        if (span_end > from) {
          src = dgram_off[r->dgram_idx] + r->u.frag.pl_off;
          dst = (uint64_t)(uintptr_t)(epoch_dst(E, out, nbytes) + from);
          nv = (uint32_t)(to - from);
          n = (uint32_t)(span_end - from);
        }
      }
    }
    uint4* q = reinterpret_cast<uint4*>(desc + p);
    q[0] = make_uint4((uint32_t)src, (uint32_t)(src >> 32), (uint32_t)dst, (uint32_t)(dst >> 32));
    q[1] = make_uint4(nv, n, 0u, 0u);
  }
}
// SPAN_R consecutive records per wave step, copied as one flat list of 16-B
// chunks (lane l takes chunks l, l + 64, ...): the loads of both records are in
// flight together and no lane idles on a record's tail (C4: 84 chunks per
// record, 20 of them in a second, mostly idle, pass with one record per wave).
// The copy ceiling of this shape (scripts/diag_frag_group.py): 515 us with one
// record per wave, 505 us with two, 515 / 553 us with three / four.
#ifndef RTPS_SPAN_R
#define RTPS_SPAN_R 2
#endif
constexpr uint32_t SPAN_R = RTPS_SPAN_R;
static_assert(SPAN_R >= 1 && SPAN_R <= 4, "records per wave step");
template <class T>
__device__ __forceinline__ T span_pick(const T (&a)[SPAN_R], uint32_t j) {
  T v = a[0];
#pragma unroll
  for (uint32_t t = 1; t < SPAN_R; ++t) v = j == t ? a[t] : v;
  return v;
}
__global__ __launch_bounds__(FT) void k_span(const uint8_t* arena, const SpanDesc* desc, uint64_t max) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t nw = (uint64_t)gridDim.x * (FT / 64);
  const uint32_t w0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)(blockIdx.x * (FT / 64) + (threadIdx.x >> 6)));
  for (uint64_t g = w0; g * SPAN_R < max; g += nw) {
    const uint8_t* sp[SPAN_R];
    uint8_t* dp[SPAN_R];
    uint32_t nv[SPAN_R], nn[SPAN_R], cb[SPAN_R];  // cb: first chunk of record t in the flat list
    uint32_t tot = 0;
#pragma unroll
    for (uint32_t t = 0; t < SPAN_R; ++t) {
      const uint64_t r = g * SPAN_R + t;
      uint4 a = make_uint4(0, 0, 0, 0), b = a;
      if (r < max) {
        const uint4* q = reinterpret_cast<const uint4*>(desc + r);
        a = q[0]; b = q[1];
      }
      sp[t] = arena + (((uint64_t)a.y << 32) | a.x);
      dp[t] = (uint8_t*)(uintptr_t)(((uint64_t)a.w << 32) | a.z);
      nv[t] = b.x; nn[t] = b.y;
      cb[t] = tot;
      tot += (b.y + 15u) >> 4;
    }
    for (uint32_t c0 = lane; c0 < tot; c0 += 64u * SPAN_U) {
      uint4 v[SPAN_U];
#pragma unroll
      for (uint32_t k = 0; k < SPAN_U; ++k) {
        const uint32_t c = c0 + 64u * k;
        uint32_t j = 0;
#pragma unroll
        for (uint32_t t = 1; t < SPAN_R; ++t) j += c >= cb[t] ? 1u : 0u;
        const uint32_t bb = 16u * (c - span_pick(cb, j));
        v[k] = make_uint4(0, 0, 0, 0);
        if (c < tot && bb + 16 <= span_pick(nv, j)) v[k] = ld16(span_pick(sp, j) + bb);
      }
#pragma unroll
      for (uint32_t k = 0; k < SPAN_U; ++k) {
        const uint32_t c = c0 + 64u * k;
        if (c >= tot) continue;
        uint32_t j = 0;
#pragma unroll
        for (uint32_t t = 1; t < SPAN_R; ++t) j += c >= cb[t] ? 1u : 0u;
        const uint32_t bb = 16u * (c - span_pick(cb, j)), n = span_pick(nn, j), vn = span_pick(nv, j);
        uint8_t* d = span_pick(dp, j);
        if (bb + 16 <= n && (bb + 16 <= vn || bb >= vn)) {
          span_st16(d + bb, v[k]);  // payload, or zeros past a short payload
        } else {
          const uint8_t* s = span_pick(sp, j);
          for (uint32_t t = bb; t < bb + 16 && t < n; ++t) d[t] = t < vn ? s[t] : (uint8_t)0;
        }
      }
    }
  }
}

// irregular epochs: the sequential replay (zero buffer, carried bytes, then every
// record's clamped copy in record order), one workgroup each
__device__ void serial_wg(const rtps_record* recs, const uint8_t* arena, const uint64_t* dgram_off,
                          const uint32_t* svals, const uint32_t* rec_epoch, const Epoch* ep, const uint32_t* special,
                          const uint64_t* ctr, const Pend* op, const uint8_t* obytes, uint8_t* nbytes,
                          const rtps_frag_out& out, uint32_t bid, uint32_t nb) {
  const uint64_t ns = ctr[C_SPECIAL];
  for (uint64_t i = bid; i < ns; i += nb) {
    const uint32_t e = special[i];
    const Epoch& E = ep[e];
    if (!(E.eflags & EF_IRREGULAR) || (E.eflags & EF_SKIP)) continue;
    uint8_t* d = epoch_dst(E, out, nbytes);
    if (E.old_pend != NONE) {
      const uint8_t* s = obytes + op[E.old_pend].bytes;
      blk_copy(d, s, E.data_size);
    } else {
      blk_zero(d, E.data_size);
    }
    __threadfence();
    __syncthreads();
    for (uint64_t p = E.p0; p < E.p1; ++p) {
      const uint32_t ri = svals[p];
      if (rec_epoch[ri] != e) continue;
      const rtps_record* r = recs + ri;
      const uint64_t from = (uint64_t)(r->u.frag.frag_start - 1) * E.F;
      const uint64_t to = min<uint64_t>(from + min<uint64_t>((uint64_t)r->u.frag.frags_in_sub * E.F, r->u.frag.pl_len),
                                        E.data_size);
      if (to > from) {
        const uint8_t* src = arena + dgram_off[r->dgram_idx] + r->u.frag.pl_off;
        for (uint64_t b = threadIdx.x; b < to - from; b += FT) d[from + b] = src[b];
      }
      __threadfence();
      __syncthreads();
    }
  }
}

// new pending hash table (for the next batch's walk); block 0 also finishes the batch
// (k_finish's work: n_pending, and the pending count the next batch starts from)
__device__ void ptable_wg(const Pend* np, uint64_t* ctr, uint32_t* ptable, uint64_t* n_pending, uint32_t bid,
                          uint32_t nb) {
  const uint64_t n = min<uint64_t>(ctr[C_NEW_N], PCAP);
  if (bid == 0 && threadIdx.x == 0) {
    *n_pending = n | (ctr[C_OVERFLOW] ? (1ull << 63) : 0ull);
    ctr[C_OLD_N] = n;
  }
  for (uint64_t j = (uint64_t)bid * FT + threadIdx.x; j < n; j += (uint64_t)nb * FT) {
    uint32_t g[KW] = {np[j].guid[0], np[j].guid[1], np[j].guid[2], np[j].guid[3], np[j].guid[4]};
    uint32_t s = key_hash(g, np[j].sn) & (PTCAP - 1);
    while (atomicCAS(&ptable[s], NONE, (uint32_t)j) != NONE) s = (s + 1) & (PTCAP - 1);
  }
}

// before the span copy, one launch: carried-over bytes / zeros of regular epochs
// (k_span then writes their spans), the irregular epochs' serial replays (their
// own bytes, disjoint from every span), and the next batch's pending table
constexpr uint32_t INIT_WG = 1024, SERIAL_WG = 1024, PTAB_WG = PCAP / FT, DESC_WG = 2048;
__global__ __launch_bounds__(FT) void k_fill(const rtps_record* recs, const uint8_t* arena, const uint64_t* dgram_off,
                                             const uint32_t* svals, const uint32_t* rec_epoch, const Epoch* ep,
                                             const uint32_t* special, uint64_t* ctr, const Pend* op,
                                             const uint8_t* obytes, uint8_t* nbytes, const Pend* np,
                                             uint32_t* ptable, uint64_t* n_pending, uint64_t max, SpanDesc* desc,
                                             rtps_frag_out out) {
  const uint32_t b = blockIdx.x;
  if (b >= INIT_WG + SERIAL_WG + PTAB_WG) {
    desc_wg(recs, dgram_off, rec_epoch, max, ep, nbytes, out, desc, b - INIT_WG - SERIAL_WG - PTAB_WG, DESC_WG);
    return;
  }
  if (b < INIT_WG) init_wg(ep, special, ctr, op, obytes, nbytes, out, b, INIT_WG);
  else if (b < INIT_WG + SERIAL_WG)
    serial_wg(recs, arena, dgram_off, svals, rec_epoch, ep, special, ctr, op, obytes, nbytes, out, b - INIT_WG,
              SERIAL_WG);
  else ptable_wg(np, ctr, ptable, n_pending, b - INIT_WG - SERIAL_WG, PTAB_WG);
}
// garbage_collect_before (fragment_assembler.rs:216-224): the carried buffers last
// modified before `expire` are marked consumed (the next batch neither finds nor
// carries them) and the lookup table is rebuilt over the live ones
__global__ __launch_bounds__(FT) void k_gc_mark(Pend* op, uint64_t* ctr, uint64_t expire) {
  const uint64_t n = min<uint64_t>(ctr[C_OLD_N], PCAP);
  uint32_t live = 0;
  for (uint64_t j = (uint64_t)blockIdx.x * FT + threadIdx.x; j < n; j += (uint64_t)gridDim.x * FT) {
    if (op[j].consumed) continue;
    if (op[j].modified < expire) op[j].consumed = 1u;
    else live++;
  }
#pragma unroll
  for (uint32_t d = 32; d >= 1; d >>= 1) live += __shfl_xor(live, d, 64);
  if ((threadIdx.x & 63u) == 0 && live) atomicAdd((unsigned long long*)&ctr[C_LIVE], (unsigned long long)live);
}
__global__ __launch_bounds__(FT) void k_ptable_live(const Pend* op, const uint64_t* ctr, uint32_t* ptable) {
  const uint64_t n = min<uint64_t>(ctr[C_OLD_N], PCAP);
  for (uint64_t j = (uint64_t)blockIdx.x * FT + threadIdx.x; j < n; j += (uint64_t)gridDim.x * FT) {
    if (op[j].consumed) continue;
    uint32_t g[KW] = {op[j].guid[0], op[j].guid[1], op[j].guid[2], op[j].guid[3], op[j].guid[4]};
    uint32_t s = key_hash(g, op[j].sn) & (PTCAP - 1);
    while (atomicCAS(&ptable[s], NONE, (uint32_t)j) != NONE) s = (s + 1) & (PTCAP - 1);
  }
}
__global__ void k_gc_finish(const uint64_t* ctr, uint64_t* n_pending) { *n_pending = ctr[C_LIVE]; }


}  // namespace

static inline uint64_t hmin(uint64_t a, uint64_t b) { return a < b ? a : b; }

struct FragState {
  int device = 0;
  int cur = 0;  // pending side holding the previous batch's buffers
  uint64_t now = 0;  // clock stamped on the buffers the next batches create or extend
  uint64_t* wkey = nullptr;
  uint32_t* wfirst = nullptr;
  uint32_t* wF = nullptr;
  uint64_t* wst_key = nullptr;  // k_keys' staged writers (KGRID x WST)
  uint32_t* wst_rec = nullptr;
  Pend* pend[2] = {nullptr, nullptr};
  uint8_t* pbytes[2] = {nullptr, nullptr};
  uint32_t* pbits[2] = {nullptr, nullptr};
  uint32_t* ptable[2] = {nullptr, nullptr};
  uint64_t* ctr = nullptr;
  // per-batch scratch (grown on demand)
  uint64_t cap = 0;
  uint32_t *keys = nullptr, *vals = nullptr, *skeys = nullptr, *svals = nullptr;
  uint32_t *rec_epoch = nullptr, *dmark = nullptr, *special = nullptr, *rword = nullptr;
  uint32_t* tcnt = nullptr;   // per 4096-position tile: completions, then their exclusive scan
  uint64_t* tbytes = nullptr; // per tile: heap bytes, then their exclusive scan
  uint8_t* seen = nullptr;
  uint64_t *dsz = nullptr, *hoff = nullptr;
  Epoch* epochs = nullptr;
  uint32_t* pool = nullptr;
  uint64_t pool_words = 0;
  void* tmp = nullptr;
  size_t tmp_bytes = 0;
  // the key sort (rtps_bsort.h) for batches of up to rtps_bsort::MAX_N records
  uint32_t* bh = nullptr;
  uint64_t *bk = nullptr, *bk2 = nullptr;
  SpanDesc* desc = nullptr;  // per record: its span copy
  int sort_mode = 0;  // 0: rtps_bsort where it applies, 1: rocprim's device sort always (tests)
};

static void free_scratch(FragState* s) {
  void* ptrs[] = {s->keys, s->vals, s->skeys, s->svals, s->rec_epoch, s->dmark, s->tcnt, s->special,
                  s->seen, s->tbytes, s->epochs, s->pool, s->tmp, s->bh, s->bk, s->bk2, s->desc, s->rword};
  for (void* p : ptrs) if (p) (void)hipFree(p);
  s->keys = s->vals = s->skeys = s->svals = s->rec_epoch = s->dmark = s->tcnt = s->special = s->rword = nullptr;
  s->seen = nullptr; s->tbytes = nullptr; s->epochs = nullptr; s->pool = nullptr; s->tmp = nullptr;
  s->bh = nullptr; s->bk = s->bk2 = nullptr; s->desc = nullptr;
  s->cap = 0; s->tmp_bytes = 0;
}

static bool grow(FragState* s, uint64_t max, hipStream_t st) {
  if (max <= s->cap) return true;
  (void)hipStreamSynchronize(st);
  free_scratch(s);
  const uint64_t n = max;
  bool ok = hipMalloc(&s->keys, n * 4) == hipSuccess && hipMalloc(&s->vals, n * 4) == hipSuccess &&
            hipMalloc(&s->skeys, n * 4) == hipSuccess && hipMalloc(&s->svals, n * 4) == hipSuccess &&
            hipMalloc(&s->rec_epoch, n * 4) == hipSuccess && hipMalloc(&s->dmark, n * 4) == hipSuccess &&
            hipMalloc(&s->rword, n * 4) == hipSuccess &&
            hipMalloc(&s->tcnt, (n / PTILE + 1) * 4) == hipSuccess && hipMalloc(&s->special, n * 4) == hipSuccess &&
            hipMalloc(&s->seen, n) == hipSuccess && hipMalloc(&s->tbytes, (n / PTILE + 1) * 8) == hipSuccess;
  s->pool_words = 4 * n + PWORDS;
  const uint64_t nb = n < rtps_bsort::MAX_N ? n : rtps_bsort::MAX_N;
  ok = ok && hipMalloc(&s->bh, rtps_bsort::hist_words(nb) * 4) == hipSuccess &&
       hipMalloc(&s->bk, nb * 8) == hipSuccess && hipMalloc(&s->bk2, nb * 8) == hipSuccess;
  ok = ok && hipMalloc(&s->desc, n * sizeof(SpanDesc)) == hipSuccess;
  ok = ok && hipMalloc(&s->epochs, n * sizeof(Epoch)) == hipSuccess &&
       hipMalloc(&s->pool, s->pool_words * 4) == hipSuccess;
  size_t b1 = 0;
  ok = ok && rtps_sort_pairs(nullptr, b1, s->keys, s->skeys, s->vals, s->svals, (uint32_t)n, (int)32, st) == hipSuccess;
  s->tmp_bytes = b1;
  ok = ok && hipMalloc(&s->tmp, s->tmp_bytes) == hipSuccess;
  if (!ok) { free_scratch(s); return false; }
  s->cap = n;
  return true;
}

FragState* rtps_frag_state_new(int device) {
  FragState* s = new (std::nothrow) FragState();
  if (!s) return nullptr;
  s->device = device;
  bool ok = hipMalloc(&s->wkey, WCAP * 8) == hipSuccess && hipMalloc(&s->wfirst, WCAP * 4) == hipSuccess &&
            hipMalloc(&s->wF, WCAP * 4) == hipSuccess && hipMalloc(&s->ctr, (C_COUNT + 1) * 8) == hipSuccess &&
            hipMalloc(&s->wst_key, KGRID * WST * 8) == hipSuccess && hipMalloc(&s->wst_rec, KGRID * WST * 4) == hipSuccess;  // + the writer-table-full word
  for (int k = 0; k < 2 && ok; ++k)
    ok = hipMalloc(&s->pend[k], PCAP * sizeof(Pend)) == hipSuccess && hipMalloc(&s->pbytes[k], PBYTES) == hipSuccess &&
         hipMalloc(&s->pbits[k], PWORDS * 4) == hipSuccess && hipMalloc(&s->ptable[k], PTCAP * 4) == hipSuccess;
  if (!ok) { rtps_frag_state_free(s); return nullptr; }
  if (rtps_frag_state_reset(s, nullptr) != RTPS_RX_OK || hipDeviceSynchronize() != hipSuccess) {
    rtps_frag_state_free(s);
    return nullptr;
  }
  return s;
}

void rtps_frag_state_free(FragState* s) {
  if (!s) return;
  free_scratch(s);
  void* ptrs[] = {s->wkey, s->wfirst, s->wF, s->ctr, s->wst_key, s->wst_rec, s->pend[0], s->pend[1], s->pbytes[0], s->pbytes[1],
                  s->pbits[0], s->pbits[1], s->ptable[0], s->ptable[1]};
  for (void* p : ptrs) if (p) (void)hipFree(p);
  delete s;
}

int rtps_frag_state_reset(FragState* s, hipStream_t st) {
  bool ok = hipMemsetAsync(s->wkey, 0, WCAP * 8, st) == hipSuccess &&
            hipMemsetAsync(s->wfirst, 0xff, WCAP * 4, st) == hipSuccess &&
            hipMemsetAsync(s->wF, 0, WCAP * 4, st) == hipSuccess &&
            hipMemsetAsync(s->ctr, 0, (C_COUNT + 1) * 8, st) == hipSuccess &&
            hipMemsetAsync(s->ptable[0], 0xff, PTCAP * 4, st) == hipSuccess &&
            hipMemsetAsync(s->ptable[1], 0xff, PTCAP * 4, st) == hipSuccess;
  s->cur = 0;
  return ok ? RTPS_RX_OK : RTPS_RX_EHIP;
}

int rtps_frag_assemble(FragState* s, hipStream_t st, const uint8_t* arena, uint64_t arena_len,
                       const uint64_t* dgram_off, const rtps_record* records, const uint64_t* n_records,
                       uint64_t max_records, const rtps_frag_out* out, const FragSel& sel, const uint32_t* emap) {
  if (max_records > 0x7fffffffull) return RTPS_RX_ETOOBIG;
  const uint64_t max = max_records ? max_records : 1;
  if (!grow(s, max, st)) return RTPS_RX_ENOMEM;
  const int o = s->cur, nw = s->cur ^ 1;
  const uint32_t gk = (uint32_t)hmin((max + KPASS - 1) / KPASS, KGRID);
  if (max_records == 0) {
    (void)hipMemsetAsync(out->n_samples, 0, 8, st);
    (void)hipMemsetAsync(out->heap_used, 0, 8, st);
  }
  const bool bsort = s->sort_mode == 0 && max <= rtps_bsort::MAX_N;
  hipLaunchKernelGGL(k_keys, dim3(gk), dim3(FT), 0, st, records, n_records, max, s->keys, bsort ? nullptr : s->vals,
                     s->rec_epoch, s->dmark, s->seen, s->ctr, s->ptable[nw], s->wkey, s->wfirst, s->wF, s->wst_key,
                     s->wst_rec, sel, s->rword);
  size_t tb = s->tmp_bytes;
  const WregSide wreg{WREG_WG, s->wst_key, s->wst_rec, gk * WST, s->wkey, s->wfirst, s->wF, s->ctr};
  if (bsort) {  // the writers' merge rides on the sort's column-scan launch
    if (rtps_bsort::sort_pairs(s->keys, (uint32_t)max, s->bh, s->bk, s->bk2, s->skeys, s->svals, st, wreg) !=
        hipSuccess)
      return RTPS_RX_EHIP;
  } else {
    if (rtps_sort_pairs(s->tmp, tb, s->keys, s->skeys, s->vals, s->svals, (uint32_t)max, (int)32, st) != hipSuccess)
      return RTPS_RX_EHIP;
    hipLaunchKernelGGL(k_wreg, dim3(WREG_WG), dim3(FT), 0, st, s->wst_key, s->wst_rec, gk * WST, s->wkey, s->wfirst,
                       s->wF, s->ctr);
  }
  WalkArgs A{records, s->skeys, s->svals, max, s->wkey, s->wF, s->wfirst, s->pend[o], s->ptable[o], s->pbits[o], s->epochs,
             s->special, s->pool, s->pool_words, s->rec_epoch, s->dmark, s->seen, s->ctr, s->rword};
  hipLaunchKernelGGL(k_walk, dim3((uint32_t)hmin((max + FT - 1) / FT, 8192)), dim3(FT), 0, st, A);
  const uint64_t tiles = (max + PTILE - 1) / PTILE;
  hipLaunchKernelGGL(k_place_tiles, dim3((uint32_t)tiles), dim3(FT), 0, st, s->dmark, s->epochs, max, s->tcnt,
                     s->tbytes);
  const uint32_t self_scan = tiles <= SELF_SCAN;
  if (!self_scan) hipLaunchKernelGGL(k_place_scan, dim3(1), dim3(FT), 0, st, s->tcnt, s->tbytes, tiles, *out);
  const PlaceArgs P{s->dmark, s->epochs, s->tcnt, s->tbytes, max, self_scan, (uint32_t)tiles, s->special, s->pool,
                    s->now, s->pend[o], s->pbytes[o], s->pbits[o], s->pend[nw], s->pbytes[nw], s->pbits[nw], s->ctr,
                    records, s->wkey, s->wfirst, s->wF, emap};
  hipLaunchKernelGGL(k_place, dim3((uint32_t)tiles + PA_WG + CARRY_WG + WFIX_WG), dim3(FT), 0, st, P, *out);
  hipLaunchKernelGGL(k_fill, dim3(INIT_WG + SERIAL_WG + PTAB_WG + DESC_WG), dim3(FT), 0, st, records, arena,
                     dgram_off, s->svals, s->rec_epoch, s->epochs, s->special, s->ctr, s->pend[o], s->pbytes[o],
                     s->pbytes[nw], s->pend[nw], s->ptable[nw], out->n_pending, max, s->desc, *out);
  hipLaunchKernelGGL(k_span, dim3((uint32_t)hmin((max + FT / 64 - 1) / (FT / 64), SPAN_GRID)), dim3(FT), 0, st, arena,
                     s->desc, max);
  if (hipGetLastError() != hipSuccess) return RTPS_RX_EHIP;
  s->cur = nw;
  return RTPS_RX_OK;
}

void rtps_frag_set_clock(FragState* s, uint64_t now) { s->now = now; }
void rtps_frag_set_sort(FragState* s, int mode) { s->sort_mode = mode; }

int rtps_frag_gc(FragState* s, hipStream_t st, uint64_t expire_before, uint64_t* n_pending) {
  const int o = s->cur;
  if (hipMemsetAsync(s->ctr + C_LIVE, 0, 8, st) != hipSuccess ||
      hipMemsetAsync(s->ptable[o], 0xff, PTCAP * 4, st) != hipSuccess)
    return RTPS_RX_EHIP;
  hipLaunchKernelGGL(k_gc_mark, dim3(PCAP / FT), dim3(FT), 0, st, s->pend[o], s->ctr, expire_before);
  hipLaunchKernelGGL(k_ptable_live, dim3(PCAP / FT), dim3(FT), 0, st, s->pend[o], s->ctr, s->ptable[o]);
  hipLaunchKernelGGL(k_gc_finish, dim3(1), dim3(1), 0, st, s->ctr, n_pending);
  return hipGetLastError() == hipSuccess ? RTPS_RX_OK : RTPS_RX_EHIP;
}
