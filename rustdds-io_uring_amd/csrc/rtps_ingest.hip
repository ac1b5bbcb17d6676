// rtps_ingest.hip — history-cache ingest on the device.
//
// Replaces the stateful readers' per-writer bookkeeping that decides which
// samples enter which history cache (RtpsWriterProxy, rtps/rtps_writer_proxy.rs;
// Reader::handle_data_msg / handle_datafrag_msg / handle_heartbeat_msg /
// handle_gap_msg, io_uring/rtps/reader.rs:514-1116; TopicCache::add_change's
// duplicate check, structure/dds_cache.rs:210-262), for every target reader of
// every routed record (Domain::handle_event, io_uring/rtps/dp_event_loop.rs:266-327).
// The reference applies the submessages one by one, reader by reader; a whole
// parsed batch is decided at once here.
//
// Events.  A record of the batch reaches every reader of its target set
// (rtps_readers.h); each (record, reader) pair that can change something is an
// EVENT: a sample (DATA / completed DATA_FRAG) with the reader's proxy of the
// writer, or without one for a writer whose entity kind is not user-defined
// (accepted unchecked, reader.rs:734-739); a HEARTBEAT with a proxy for a
// reliable reader; a valid GAP with a proxy.  When no target set has more
// than one reader, event i is record i ("identity" batches: the common case);
// otherwise the events are laid out by a scan over the per-record counts, in
// (record, set order) order.  Writer-proxy state is per PROXY.
//
// Why the batch can be decided in parallel.  Call a sequence number s of a
// proxy "covered" once a sample with sn s has been processed for it, a valid
// GAP listed s or had s in [gapStart, gapList.base), or an accepted HEARTBEAT
// had firstSN > s.  The proxy's all_ackable_before (ack_base) is then always
// the smallest s >= 1 that is not covered (every transition of
// rtps_writer_proxy.rs:202-355 keeps that invariant), so
// should_ignore_change(s) = s < ack_base || changes.contains(s) is exactly
// "s < 1 or s covered by an earlier event".  Only HEARTBEAT acceptance is
// order-dependent (count > every earlier accepted count, reader.rs:902-905,
// i.e. a strict prefix maximum), and it needs per-proxy order only among the
// HEARTBEATs.  So:
//   1 classify  lane per record: target set, event count (identity: the event);
//   1b expand   (non-identity batches) scan of the counts, lane per record
//               writes its events;
//   2 heartbeats stable radix sort of the HEARTBEAT events by proxy, scans by
//               key: accepted = count > max(state count, earlier counts);
//               running max of accepted firstSN (the coverage threshold);
//   3 marks     lane per sample / GAP event: atomicMin(first covering event)
//               over a per-proxy window of RTPS_INGEST_WINDOW sequence numbers;
//   4 decide    lane per sample event: s >= 1, s >= ack_base, s >= threshold of
//               the HEARTBEATs before it, not in the carried change set, and it
//               is its sn's first covering event;
//   5 select    accepted events -> deliveries (record, reader slot), ascending;
//   6 merge     the batch's coverage into the persistent change-set bitmap;
//   7 state     workgroup per proxy: new ack_base = first uncovered s from
//               max(ack_base, threshold), window re-anchored there, count.
// The CPU restatement the tests hold this to (oracle/, test-only) is the
// reference's sequential algorithm, so tests/ check this derivation too.
//
// Roofline: HBM / L2-bound integer work (64-B record read + a few bytes of
// state per event); no MFMA.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include "rtps_sort.h"
#include <string.h>

#include <atomic>
#include <chrono>
#include <new>
#include <vector>

#include "rtps_ingest.h"

namespace {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr uint32_t IT = 256;
constexpr uint32_t NONE = 0xffffffffu;
constexpr uint32_t W = RTPS_INGEST_WINDOW;  // sequence numbers tracked per proxy
constexpr uint32_t WW = W / 32;             // bitmap words per proxy
constexpr uint32_t ECAP_MAX = 1u << 14;     // writer proxies
enum : uint8_t { EV_NONE = 0, EV_SAMPLE = 1, EV_HB = 2, EV_GAP = 3 };
// counters: window overflow, selected HEARTBEATs, selected deliveries, records of the batch, then
// the HEARTBEAT / GAP / event / proxy-less sample counts in 64 slot quads (one atomic per block, spread: no hot address)
// (C_FARC: classify's far-SN candidates, the host's cue for k_far; C_NFAR: far items appended)
// (C_MODE: k_signal's verdict on an identity batch, read by the kernels queued before the host saw it)
// (C_TGAP: GAPs whose range starts at or below their proxy's all_ackable_before and reaches past its
//  window: irrelevant_changes_range then only moves all_ackable_before, a threshold the per-proxy
//  path applies as such; the host sends such batches there)
enum { C_OVF = 0, C_NSEL, C_NDEL, C_NREC, C_FARC, C_NFAR, C_MODE, C_TGAP, C_FDEF, C_PAD, C_SPREAD,
       C_COUNT = C_SPREAD + 4 * 64 };
static_assert(C_SPREAD % 2 == 0, "the spread counters are loaded as 16-B pairs");
// the batch's counts as k_signal writes them to pinned host memory:
// [0] = the batch's tag (written last), HEARTBEAT / GAP / event / proxy-less sample counts,
// records, far-item candidates, the verdict, the far-set pool's slots in use (as the earlier
// batches left it), threshold GAPs (C_TGAP)
enum { SIG_TAG = 0, SIG_HB, SIG_GAP, SIG_EV, SIG_FREE, SIG_NREC, SIG_FARC, SIG_MODE, SIG_FUSED, SIG_TGAP, SIG_WORDS = 10 };
// event metadata: reader slot | flags << 16 (EVF_*)
constexpr uint32_t EVF_DUP_OK = 1u << 16;  // RTPS_TARGET_DUPLICATES_OK reader
constexpr uint32_t EVF_FREE = 1u << 17;    // sample without a proxy (writer kind not user-defined)

// atomicOr(*addr, m) for the active lanes, the bits of a word shared by several lanes
// combined first.  A writer's sequential SNs share bitmap words (T: a few distinct
// words per wave), while mixed traffic has mostly distinct words (C3), where combining
// gains nothing.  So: up to WOR_ROUNDS rounds of "the first pending lane's word: OR of
// every lane on it, one atomic", then a plain atomic per lane still pending.  A round
// is a ballot, a read-lane and a 6-step OR reduction.  Every lane of the wave must call it.
constexpr uint32_t WOR_ROUNDS = 4;
__device__ __forceinline__ void wave_or(uint32_t* base, uint32_t* addr, uint32_t m, bool active) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t key = (uint32_t)(addr - base);
  bool todo = active && m != 0u;
#pragma unroll
  for (uint32_t r = 0; r < WOR_ROUNDS; ++r) {
    const uint64_t t = __ballot(todo);
    if (t == 0) return;
    const uint32_t leader = (uint32_t)__builtin_ctzll(t);
    const uint32_t k = (uint32_t)__builtin_amdgcn_readlane((int)key, (int)leader);
    const bool mine = todo && key == k;
    uint32_t v = mine ? m : 0u;
#pragma unroll
    for (uint32_t d = 1; d < 64; d <<= 1) v |= (uint32_t)__shfl_xor((int)v, d, 64);
    if (lane == leader) atomicOr(base + k, v);
    todo = todo && !mine;
  }
  if (todo) atomicOr(addr, m);
}
// first-cover key of event k in batch `epoch`: no reset between batches is needed
__device__ __forceinline__ unsigned long long ekey(uint32_t epoch, uint32_t k) {
  return ((unsigned long long)(0xffffffffu - epoch) << 32) | k;
}
typedef uint32_t u32u __attribute__((aligned(1)));
// one unaligned dword load (gfx950 global loads need no alignment), not four byte loads
__device__ __forceinline__ uint32_t rd32(const uint8_t* p, bool le) {
  const uint32_t x = *reinterpret_cast<const u32u*>(p);
  return le ? x : __builtin_bswap32(x);
}

struct Scratch {
  // per record
  uint32_t* fidx;   // completed DataFrag sample of a record, or NONE
  uint64_t* fmask;  // the target-set entries (bit k: entry k) whose assembler completed it at the record
  uint8_t* fall;    // a writer-keyed sample (every entry) completed at the record
  const rtps_frag_sample* frag;  // this batch's completed samples (entries past 64: their readers)
  const uint64_t* n_frag;
  uint64_t max_frag;
  uint32_t* rcnt;   // events of the record (non-identity batches), then their exclusive scan (roff)
  uint32_t* roff;
  uint32_t* rset;   // target set, record event kind, sample / event sn
  uint8_t* rkind;
  int64_t* rsn;
  // per event
  uint8_t* evt;     // event kind
  uint32_t* ent;    // proxy, or NONE (a free sample)
  int64_t* esn;     // sample sn
  uint32_t* erec;   // record of the event
  uint32_t* emeta;  // reader slot | EVF_* flags
  uint8_t* eacc;    // accepted (non-identity batches; identity batches decide into accept[] directly)
  uint32_t* sel;    // accepted event indices
  uint32_t *hkey, *hval, *skey, *sval;  // HEARTBEAT sort (hkey: HB flag per event, then the keys)
  int32_t *hcnt, *hexcl;
  int64_t *hf, *hpre;
};
struct FarItem;
struct State {
  int64_t* base;    // all_ackable_before
  int64_t* lo;      // first sequence number of the window (multiple of 32, <= base)
  int32_t* hbc;     // received_heartbeat_count
  uint32_t* bits;   // change set: bit (s - lo) of proxy e at bits[e * WW + ...]
  uint64_t* fc;     // first covering event of (e, s - lo): (~epoch << 32 | event); older epochs compare larger
  uint32_t* dbits;  // this batch's samples, same layout as bits (cleared by k_merge)
  uint32_t* seg_b;  // HEARTBEAT segment of each proxy in sorted order
  uint32_t* seg_e;
  uint64_t* ctr;
  // far sets (see "far sequence numbers" below): proxy e's hash table is the pool slots
  // [far_off[e], + far_cap[e]) of fsn / fkey (far_cap 0: none)
  uint64_t* far_off;
  uint32_t* far_cap;
  uint32_t* far_n;    // occupied slots
  int64_t* far_min;   // least SN of the set at or above the window's end (INT64_MAX: none)
  uint64_t* fneed;    // k_far_need: SNs the batch's items of proxy e cover (cleared by k_far_grow)
  uint32_t* fstat;    // k_far_grow: 1 = the pool could not grow proxy e's table this batch
  int64_t* fsn;       // pool: SN per slot (FEMPTY: free)
  uint64_t* fkey;     // pool: the first event that covered the slot's SN, epoch << 32 | event
  uint64_t* fused;    // pool slots handed out (device counter; may pass fpcap when the pool is out)
  uint64_t fpcap;     // pool slots
  FarItem* fl;        // this batch's far items (global paths), C_NFAR of them, at most fl_cap
  uint64_t fl_cap;
  uint32_t epoch;     // this batch's (first-cover keys)
  // far sets of more than FT_BIG slots: the state pass leaves their far_extend / far_pull to the
  // grid-wide k_fx_* launches (fdefer: the host launches them after this batch's state pass)
  uint32_t fdefer;
  uint32_t* fdl;      // the deferred proxies (C_FDEF of them)
  int64_t* fext;      // per proxy: all_ackable_before through the far set (k_fx_ext's minimum)
  uint32_t* fkeep;    // per proxy: the far SNs left past the new window (k_fx_pull; 0 between batches)
  int64_t* fkmin;     // per proxy: their least (INT64_MAX between batches)
};

// ---- 1 classify ----
// A per-reader sample (reader_slot != RTPS_NO_MATCH) goes to that reader only: its
// entry of the completing record's target set (handle_datafrag_msg runs per reader,
// reader.rs:563-636; entries 0..63 of a set: the mask's bits); a writer-keyed sample to
// every entry (fall).
__global__ __launch_bounds__(IT) void k_fidx(const rtps_frag_sample* frag, const uint64_t* n_frag, uint64_t max_frag,
                                             uint64_t max, uint32_t* fidx, uint64_t* fmask, uint8_t* fall, ReaderDev t,
                                             const rtps_record* recs) {
  const uint64_t nf = n_frag ? (*n_frag < max_frag ? *n_frag : max_frag) : 0;
  for (uint64_t s = (uint64_t)blockIdx.x * IT + threadIdx.x; s < nf; s += (uint64_t)gridDim.x * IT) {
    const rtps_frag_sample& f = frag[s];
    if (f.status == RTPS_FRAG_SHORT || f.rec_idx >= max) continue;
    // the record's first sample (samples of one record share the writer and SN, and are
    // adjacent: completing-record order)
    atomicMin(&fidx[f.rec_idx], (uint32_t)s);
    uint64_t bit = ~0ull;
    if (f.reader_slot == RTPS_NO_MATCH) fall[f.rec_idx] = 1u;
    if (f.reader_slot != RTPS_NO_MATCH) {
      const uint32_t* d = reinterpret_cast<const uint32_t*>(recs + f.rec_idx);
      uint32_t r2 = 0;
      const uint32_t set = rt_classify<false>(t, nullptr, d[2], d[3], d[4], d[5], r2);
      bit = 0;
      if (set != NONE)
        for (uint32_t k = t.set_first[set], e = t.set_first[set + 1]; k < e; ++k)
          if (t.set_ent[k].reader_slot == f.reader_slot && k - t.set_first[set] < 64u) bit = 1ull << (k - t.set_first[set]);
    }
    atomicOr(reinterpret_cast<unsigned long long*>(fmask + f.rec_idx), (unsigned long long)bit);
  }
}

// k_fidx's tables cleared for the batch's record slots in one launch (three memsets before):
// four slots per thread, 16-B / 32-B / 4-B stores (the arrays are hipMalloc-aligned)
__global__ __launch_bounds__(IT) void k_fclear(uint64_t max, uint32_t* fidx, uint64_t* fmask, uint8_t* fall) {
  const uint64_t n4 = max / 4u;
  for (uint64_t q = (uint64_t)blockIdx.x * IT + threadIdx.x; q < n4; q += (uint64_t)gridDim.x * IT) {
    reinterpret_cast<uint4*>(fidx)[q] = make_uint4(NONE, NONE, NONE, NONE);
    reinterpret_cast<ulonglong2*>(fmask)[2u * q] = make_ulonglong2(0ull, 0ull);
    reinterpret_cast<ulonglong2*>(fmask)[2u * q + 1u] = make_ulonglong2(0ull, 0ull);
    reinterpret_cast<uint32_t*>(fall)[q] = 0u;
  }
  if (blockIdx.x == 0 && threadIdx.x < (max & 3u)) {
    const uint64_t i = 4u * n4 + threadIdx.x;
    fidx[i] = NONE;
    fmask[i] = 0ull;
    fall[i] = 0u;
  }
}

// Does entry `pos` (reader `slot`) of record i's target set take its completed DataFrag
// sample?  fm: the entries whose assembler completed it (bits 0..63), all: a writer-keyed
// sample (every entry); a record without one: fm = ~0, all.  Entries past 64 look for
// their reader among the record's samples (adjacent, from its first, fidx).
__device__ __forceinline__ bool frag_takes(uint64_t fm, bool all, uint32_t pos, const Scratch& x, uint64_t i,
                                           uint16_t slot) {
  if (pos < 64u) return ((fm >> pos) & 1ull) != 0ull;
  if (all || !x.frag || !x.n_frag) return all;
  const uint64_t nf = *x.n_frag < x.max_frag ? *x.n_frag : x.max_frag;
  for (uint64_t f = x.fidx[i]; f < nf && x.frag[f].rec_idx == i; ++f)
    if (x.frag[f].status != RTPS_FRAG_SHORT && x.frag[f].reader_slot == slot) return true;
  return false;
}

// Does (record event kind, target x) make an event?  Sets ent / meta.
__device__ __forceinline__ bool ev_of(uint8_t ev, const rtps_target& x, bool user_kind, bool reliable, uint32_t& ent,
                                      uint32_t& meta) {
  ent = x.proxy;
  meta = x.reader_slot | ((x.reader_flags & RTPS_TARGET_DUPLICATES_OK) ? EVF_DUP_OK : 0u);
  if (ev == EV_SAMPLE) {
    if (x.proxy != RTPS_NO_PROXY) return true;
    meta |= EVF_FREE;
    return !user_kind;  // no proxy: dropped for user-defined writers, accepted otherwise (reader.rs:734-739)
  }
  if (x.proxy == RTPS_NO_PROXY) return false;  // HEARTBEAT / GAP need the proxy (reader.rs:885-891, 1076-1086)
  if (ev == EV_HB) return reliable && !(x.reader_flags & RTPS_READER_BEST_EFFORT);  // (reader.rs:871-881)
  return true;
}

constexpr uint32_t PM_DUP = 4u, PM_LE = 8u, PM_INL = 16u;
// One proxied event as the proxy's workgroup reads it (the sort's value): the
// fields it needs gathered in event order, so that the per-proxy pass reads its
// events contiguously.  m = kind (2 bits) | DUP_OK << 2 | little-endian << 3 |
// inline bitmap << 4 | GAP numBits << 8; a = HEARTBEAT count or GAP list base;
// bw = a GAP's bitmap words (host order, numBits <= 64) or its arena offset.
struct PEv {
  int64_t sn;
  int64_t a;
  uint64_t bw;
  uint32_t m;
  uint32_t k;  // event index (accept[] slot)
};
static_assert(sizeof(PEv) == 32, "PEv layout");

// ---- far sequence numbers: the change set beyond the window ----
// The window [lo, lo + W) holds the change set as bits; the reference's BTreeMap has no
// bound (rtps_writer_proxy.rs:62), so the SNs a proxy has covered at or above lo + W (a
// writer that jumped ahead, a GAP reaching past the window) are kept per proxy in a FAR
// SET: an open-addressing hash set of SNs in a device pool (load <= 1/2; grown by rehashing
// into a larger table), each slot with the first event that covered its SN, epoch-tagged
// (epoch << 32 | event: the SNs of earlier batches compare smaller).  A batch's events
// beyond the window, FAR ITEMS (samples past it, DUPLICATES_OK samples there, GAPs whose
// coverage reaches past it), are decided provisionally (samples accepted), then every SN an
// item covers is inserted with an atomicMin of the item's key, and a far sample is accepted
// iff its own key is its SN's minimum: no earlier event of the batch and no earlier batch
// covered it -- the window's first-cover rule (k_marks_d) over the hash, so no replay in
// event order is needed.  k_far (global paths: every proxy's items from the batch list) and
// the chunk loop of k_proxy (per-proxy path: each chunk's items right after they are
// decided) share it.  The state pass continues all_ackable_before through the set when the
// window is covered up to its end (far_extend), re-anchors, and sets the bits of the set's
// SNs the new window spans (far_pull, which also drops what lies below the new window's end
// once that is most of the table).
// Capacity: tables come from the pool by a device bump counter; the host keeps the pool's
// free part at >= 4 x (the batch's record capacity + the live far slots) between batches
// (far_pool_ensure: grown and compacted there), which holds every table a batch's samples
// can need.  Only GAPs covering more SNs past the window than that can find the pool out:
// those samples are accepted unchecked and counted in *n_window_overflow (the reference
// inserts such ranges one SN at a time too, rtps_writer_proxy.rs:284-291).
// a free slot: all ones (far SNs are >= W > 0), like its key ~0, so that a byte fill clears the
// pool; the slots at and above the pool's counter are always free (fresh tables need no clearing)
// A GAP whose range reaches more than FAR_BIG sequence numbers past its proxy's window would
// fill the far set SN by SN.  It is a threshold instead (irrelevant_changes_range's jump,
// rtps_writer_proxy.rs:241-292) whenever its gapStart is at or below all_ackable_before when it
// arrives, which this batch's earlier events may have moved: classify sends every such GAP to
// the per-proxy path (C_TGAP), whose k_proxy decides it against the running value.
constexpr int64_t FAR_BIG = 256;
__host__ __device__ __forceinline__ bool gap_far_big(int64_t start, int64_t list_base, int64_t lim) {
  return start <= list_base && list_base - (start > lim ? start : lim) > FAR_BIG;
}
constexpr int64_t FEMPTY = -1;
constexpr uint32_t FT_MIN = 64;         // smallest table
enum : uint32_t { FI_SAMPLE = 1, FI_DUP = 2, FI_GAP = 3 };
struct FarItem {
  PEv p;        // the event as the per-proxy pass packs it (p.k: its accept slot)
  int64_t lim;  // lo + W when it was decided: the SNs at or above it are the far part
  uint32_t e, kind;
};
static_assert(sizeof(FarItem) == 48, "FarItem layout");
// its list position, or NONE: the list is full (sized by the host to the batch's events: not
// reached).  The lanes of the wave that push at the same call reserve their places with one
// atomic (the active mask; one counter for the whole batch, so no hot-address queue).
__device__ __forceinline__ uint32_t far_push(const State& s, const FarItem& it) {
  const uint64_t act = __ballot(1);
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t rank = (uint32_t)__popcll(act & ((1ull << lane) - 1ull));
  unsigned long long b = 0;
  if (rank == 0) b = atomicAdd(reinterpret_cast<unsigned long long*>(s.ctr + C_NFAR), (unsigned long long)__popcll(act));
  const uint32_t lo32 = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)b);
  const uint32_t hi32 = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(b >> 32));
  const uint64_t pos = (((uint64_t)hi32 << 32) | lo32) + rank;
  if (pos >= s.fl_cap) return NONE;
  s.fl[pos] = it;
  return (uint32_t)pos;
}

// What the per-proxy path of an identity batch needs from classify (FAST): the
// packed events at their record slots, the sort pairs (proxy or n_proxies, slot),
// accept[] initialised (proxy-less samples accepted) and the proxy segments cleared.
struct FastOut {
  PEv* pev;
  uint8_t* acc;
  const uint8_t* arena;
  const uint64_t* dgram_off;
  uint32_t* seg_b;
  uint32_t* seg_e;
  uint32_t n_seg;
  uint32_t* bk_cl;   // BUCKET: per (workgroup, proxy), workgroup-major [block * n_proxies + proxy]: the
                     //   proxy's events in the workgroup's region | their first position there << 16
  uint32_t sets_lds; // classify: set_first / set_ent staged in LDS behind the hash tables
};
// bytes of the target sets' LDS image (set_first words, then 8-B entries)
__host__ __device__ inline uint32_t sets_lds_bytes(const ReaderDev& t) { return (t.n_sets + 1u) * 4u + t.n_ent * 8u; }

// Proxy bucketing (BUCKET: identity batches over at most PB_MAX proxies and
// BK_MAX workgroups).  Classify takes CHR consecutive record slots per
// workgroup (wave w the w-th quarter, 64 slots per step) and keeps every
// proxied event's packed form in registers; after a workgroup-wide count per
// proxy it writes the packed events into the workgroup's own region of pev[]
// (CHR entries), grouped by proxy with slot order kept (a bitonic sort of
// (proxy << 6 | lane) ranks each step's 64 slots; each wave's running offset
// per proxy advances by its runs), plus the (workgroup, proxy) counts and
// first positions.  k_proxy<true> then walks its proxy's pieces of every
// workgroup's region in workgroup order (a scan of the counts in LDS): the
// proxy's events in slot order, with no sort of the record slots and no
// separate scatter pass (the radix sort it replaces takes two 8-bit Onesweep
// passes over every slot at 256 proxies).
constexpr uint32_t PB_MAX = 1024;  // proxies of the bucketing path (LDS counters: 4 x PB_MAX words)
constexpr uint32_t BK_MAX = 4096;  // classify workgroups of the bucketing path (k_proxy's LDS tables)
constexpr uint32_t BK_IDX = 4096;  // k_proxy's sampled piece index: proxies of up to 4 x BK_IDX events
#ifndef RTPS_PB_CHR
#define RTPS_PB_CHR 2048  // measured on C3: 1024 -> 2048 classify +2 us, k_proxy -8 (half the pieces)
#endif
#ifndef RTPS_CL_PRELOAD
#define RTPS_CL_PRELOAD 0  // measured: classify 139 -> 145 us on C3 (VGPRs 77 -> 94)
#endif
#ifndef RTPS_CL_GAP_INLINE
#define RTPS_CL_GAP_INLINE 0  // 1: classify reads short GAP bitmaps inline (a second dependent load)
#endif
#ifndef RTPS_CL_FULLREC
#define RTPS_CL_FULLREC 1  // the whole record in one round trip
#endif
constexpr uint32_t CHR = RTPS_PB_CHR;         // record slots per classify workgroup
constexpr uint32_t PB_SUB = CHR / (IT / 64);  // slots per wave
constexpr uint32_t PB_STEPS = PB_SUB / 64;
static_assert(PB_SUB % 64 == 0 && PB_MAX <= (1u << 20) && PB_MAX % IT == 0 && CHR < 65536u,
              "bucketing steps, sort words, packed piece counts");

__device__ __forceinline__ uint32_t wave_incl_sum(uint32_t x, uint32_t lane) {
#pragma unroll
  for (uint32_t d = 1; d < 64; d <<= 1) {
    const uint32_t y = (uint32_t)__shfl_up((int)x, d, 64);
    if (lane >= d) x += y;
  }
  return x;
}

// IDENT: no target set has more than one reader, so event i = record i.
// FAST (IDENT only): also the per-proxy path's inputs (FastOut), so that an identity
// batch on that path needs no host read-back of the counts.
// BUCKET (FAST only): CHR consecutive slots per workgroup and the per-proxy counts
// (the proxy bucketing above) instead of the radix sort's (key, slot) pairs.
// MARK (IDENT, not FAST): also the samples' first-cover keys (the marks of the global path,
// k_marks_d's atomicMin), so that the global path needs no separate marks pass.
#if defined(RTPS_PROXY_STAMPS) || defined(RTPS_CLS_STAMPS)  // tuning builds: phase timestamps
__device__ unsigned long long g_proxy_stamps[16384 * 16];
#endif
#ifdef RTPS_CLS_STAMPS  // bucketing classify: wave 0's absolute times at its phase ends, per workgroup
#define CST(k) do { if (BUCKET && threadIdx.x == 0) g_proxy_stamps[blockIdx.x * 16u + (k)] = __builtin_amdgcn_s_memrealtime(); } while (0)
// inside a record step: wait for everything outstanding, then add the time since the last mark
// to phase sum k (slots 8.. of the workgroup's 16)
#define CSS(k) do { if (BUCKET) { asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory"); \
  const uint64_t t_ = __builtin_amdgcn_s_memrealtime(); css[k] += t_ - css_t; css_t = t_; } } while (0)
#define CSS_DECL uint64_t css[4] = {0, 0, 0, 0}, css_t = __builtin_amdgcn_s_memrealtime()
#define CSS_FLUSH() do { if (BUCKET && threadIdx.x == 0) for (uint32_t k_ = 0; k_ < 4; ++k_) g_proxy_stamps[blockIdx.x * 16u + 8u + k_] = css[k_]; } while (0)
#else
#define CST(k) do {} while (0)
#define CSS(k) do {} while (0)
#define CSS_DECL do {} while (0)
#define CSS_FLUSH() do {} while (0)
#endif
template <bool IDENT, bool FAST, bool BUCKET = false, bool MARK = false>
__global__ __launch_bounds__(IT) void k_classify(ReaderDev t, const rtps_record* recs, const uint64_t* n_rec,
                                                 uint64_t max, const rtps_frag_sample* frag, uint32_t flags,
                                                 Scratch x, uint64_t* ctr, FastOut fo, uint64_t* ctr_next, State st,
                                                 uint32_t epoch) {
  extern __shared__ __attribute__((aligned(16))) uint32_t s_rt[];  // (rt_writer_set reads 16-B keys)
  __shared__ uint32_t s_cnt[BUCKET ? IT / 64 : 1][BUCKET ? PB_MAX : 1];  // per (wave, proxy)
  CST(0);
  if (blockIdx.x == gridDim.x - 1u)  // the next batch's counters start at zero (no memset launch)
    for (uint32_t c = threadIdx.x; c < C_COUNT; c += IT) ctr_next[c] = 0ull;
  __shared__ uint32_t s_part[IT / 64];
  const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const uint64_t n = *n_rec < max ? *n_rec : max;
  if (blockIdx.x == 0 && tid == 0) ctr[C_NREC] = n;
  if (FAST && !BUCKET)
    for (uint32_t e = blockIdx.x * IT + tid; e < fo.n_seg; e += gridDim.x * IT) { fo.seg_b[e] = 0u; fo.seg_e[e] = 0u; }
  if (BUCKET)
    for (uint32_t e = lane; e < t.n_proxies; e += 64) s_cnt[wave][e] = 0u;
  const bool lds = rt_fits_lds(t);
  // the tables, and the target sets behind them when the host sized the LDS for them (a
  // record's set entries then cost two LDS reads instead of two dependent global loads): one
  // flat copy of the device image
  uint32_t* const s_sf = s_rt + rt_lds_bytes(t.gmask + 1u, t.emask + 1u) / 4u;
  const rtps_target* const s_se = reinterpret_cast<const rtps_target*>(s_sf + t.n_sets + 1u);
  if (lds) rt_copy(s_rt, t.gkeys, fo.sets_lds ? rt_image_words(t) : rt_lds_words(t));
  const uint32_t* const sfirst = fo.sets_lds ? s_sf : t.set_first;
  const rtps_target* const sent = fo.sets_lds ? s_se : t.set_ent;
  if (lds || BUCKET) __syncthreads();
  CST(1);
  const bool reliable = !(flags & RTPS_INGEST_BEST_EFFORT);
  uint32_t nh = 0, ng = 0, ne = 0, nf = 0, nfar = 0, ntg = 0;
  CSS_DECL;
  // record slot i: its events; FAST: *key = the proxy of its proxied event (NONE: none)
  // and *P its packed form, stored at pev[i] unless BUCKET (which places it itself)
  // rq: the record's four 16-B quads (global memory, or registers the caller filled ahead)
  auto body = [&](uint64_t i, uint32_t& key, PEv& P, const u32x4* rq) {
    uint8_t ev = EV_NONE;
    uint32_t set = NONE;
    int64_t sn = 0;
    bool user_kind = true;
    key = NONE;
    u32x4 q0 = {0u, 0u, 0u, 0u}, q2 = q0, q3 = q0;  // FAST: the record's fields for the packed event
    if (i < n) {
      // bytes 0..31 of the record (kind @6, prefix||writer_id @8, route @30,
      // payload_kind @31), then 32..47 (sn, gap.list_base) for the candidates:
      // three of the record's four 16-B quads at most
      const u32x4* q = rq;
      CSS(3);
      q0 = q[0];
      const u32x4 q1 = q[1];
#if RTPS_CL_FULLREC
      // the rest of the record in the same round trip (same 64-B line), not after the kind test
      const u32x4 f2 = q[2], f3 = q[3];
#endif
      CSS(0);
      const uint32_t kind = (q0[1] >> 16) & 0xffu, route = (q1[3] >> 16) & 0xffu, pk = q1[3] >> 24;
      const uint32_t f = frag ? x.fidx[i] : NONE;
      // records the receiver passes to the user readers (not a builtin pair: discovery's)
      if ((route & RTPS_ROUTE_PASS) && (route & RTPS_ROUTE_TARGETED) && !(route & RTPS_ROUTE_BUILTIN)) {
        if (f != NONE) {  // completed DataFrag sample, processed at its completing record (reader.rs:614-626)
          ev = EV_SAMPLE;
          sn = frag[f].sn;
        } else if (kind == RTPS_DATA || kind == RTPS_HEARTBEAT || kind == RTPS_GAP) {
#if RTPS_CL_FULLREC
          q2 = f2;
          q3 = f3;
#else
          q2 = q[2];
          if ((FAST && kind != RTPS_DATA) || ((MARK || !IDENT) && kind == RTPS_GAP)) q3 = q[3];
#endif
          const int64_t rsn = (int64_t)(((uint64_t)q2[1] << 32) | q2[0]);
          if (kind == RTPS_DATA) {
            // data_to_dds_data must succeed (reader.rs:552-558)
            if (pk == RTPS_PK_DATA || pk == RTPS_PK_KEY || pk == RTPS_PK_KEY_HASH) ev = EV_SAMPLE;
          } else if (kind == RTPS_HEARTBEAT) {
            ev = EV_HB;
          } else {
            const int64_t list_base = (int64_t)(((uint64_t)q2[3] << 32) | q2[2]);
            if (rsn > 0 && list_base > 0) ev = EV_GAP;  // validity (reader.rs:1087-1102)
          }
          sn = rsn;
        }
        if (ev != EV_NONE) {
          uint32_t r2 = 0;
          set = lds ? rt_classify<true>(t, s_rt, q0[2], q0[3], q1[0], q1[1], r2)
                    : rt_classify<false>(t, s_rt, q0[2], q0[3], q1[0], q1[1], r2);
          if (set == NONE) ev = EV_NONE;
          user_kind = (q1[1] >> 24 & 0xf0u) == 0u;  // EntityKind::is_user_defined (guid.rs:168-170)
        }
      }
    }
    CSS(1);
    // the record's events: one per target reader that the event concerns (a completed
    // DataFrag sample: the readers whose assembler completed it)
    uint32_t cnt = 0;
    uint32_t ent = NONE, meta = 0;
    if (ev != EV_NONE) {
      const uint32_t b = sfirst[set], e = sfirst[set + 1];
      const bool fs = frag && x.fidx[i] != NONE;
      const uint64_t fm = fs ? x.fmask[i] : ~0ull;
      const bool fa = !fs || x.fall[i] != 0u;
      for (uint32_t k = b; k < e; ++k) {
        uint32_t en, me;
        if (frag_takes(fm, fa, k - b, x, i, sent[k].reader_slot) && ev_of(ev, sent[k], user_kind, reliable, en, me)) {
          ++cnt;
          ent = en;
          meta = me;
          nh += ev == EV_HB;
          ng += ev == EV_GAP;
          nf += en == NONE;
          if (!IDENT && en != NONE && ev != EV_HB) {  // far-item candidates of expanded batches (see below)
            const int64_t lim = st.lo[en] + (int64_t)W;
            if (ev == EV_SAMPLE ? sn >= lim : (int64_t)(((uint64_t)q2[3] << 32) | q2[2]) + (int64_t)q3[0] > lim) {
              ++nfar;
              if (ev == EV_GAP && (sn <= st.base[en] || gap_far_big(sn, (int64_t)(((uint64_t)q2[3] << 32) | q2[2]), lim)))
                ++ntg;
            }
          }
        }
      }
    }
    ne += cnt;
    CSS(2);
    if (IDENT) {  // at most one event: write it at index i
      const uint8_t evi = cnt ? ev : EV_NONE;
      x.emeta[i] = meta;
      if (!FAST) x.erec[i] = (uint32_t)i;  // (the per-proxy identity path reads no event -> record map)
      if (!FAST) {  // (the per-proxy identity path reads the packed events instead)
        x.evt[i] = evi;
        x.ent[i] = ent;
        x.esn[i] = sn;
        if (MARK && evi == EV_SAMPLE && ent != NONE) {  // k_marks_d's first-cover key
          const int64_t lo = st.lo[ent];
          if (sn >= lo && sn < lo + (int64_t)W)
            atomicMin(reinterpret_cast<unsigned long long*>(st.fc + (uint64_t)ent * W) + (uint64_t)(sn - lo),
                      ekey(epoch, (uint32_t)i));
          else if (sn >= lo + (int64_t)W)
            ++nfar;  // a far-item candidate: the host launches k_far
        } else if (MARK && evi == EV_GAP) {
          const int64_t list_base = (int64_t)(((uint64_t)q2[3] << 32) | q2[2]);
          if (list_base + (int64_t)q3[0] > st.lo[ent] + (int64_t)W) {  // coverage past the window
            ++nfar;
            if (sn <= st.base[ent] || gap_far_big(sn, list_base, st.lo[ent] + (int64_t)W)) ++ntg;
          }
        }
      }
      if (!FAST) {
        x.hkey[i] = evi == EV_HB ? 1u : 0u;  // selection flag of the HEARTBEAT compaction
      } else {
        const bool px = evi != EV_NONE && ent != NONE;
        if (!BUCKET) {
          x.hkey[i] = px ? ent : t.n_proxies;  // sort pairs: (proxy, slot); n_proxies sorts last
          x.sval[i] = (uint32_t)i;
        }
        fo.acc[i] = (evi == EV_SAMPLE && ent == NONE) ? 1 : 0;  // proxy-less samples (reader.rs:734-739)
        if (px) {
          key = ent;
          P.sn = sn;
          P.a = 0;
          P.bw = 0;
          P.k = (uint32_t)i;
          P.m = evi | ((meta & EVF_DUP_OK) ? PM_DUP : 0u);
          if (evi == EV_HB) {
            P.a = (int32_t)q3[0];  // u.hb.count
          } else if (evi == EV_GAP) {
            P.a = (int64_t)(((uint64_t)q2[3] << 32) | q2[2]);  // u.gap.list_base
            const uint32_t nbits = q3[0], fl = q0[1] >> 24;
            const bool le = (fl & 1u) != 0u;
            P.m |= (le ? PM_LE : 0u) | (nbits << 8);
            P.bw = fo.dgram_off[q0[0]] + (q3[1] & 0xffffu);  // dgram_idx, u.gap.bitmap_off
            // (RTPS_CL_GAP_INLINE: short bitmaps read here, a dependent load that holds the wave;
            // measured: classify -15 us, k_proxy +6 on C3 without it)
            if (RTPS_CL_GAP_INLINE && nbits <= 64u) {
              const uint8_t* bp = fo.arena + P.bw;
              const uint32_t w0 = nbits ? rd32(bp, le) : 0u, w1 = nbits > 32u ? rd32(bp + 4, le) : 0u;
              P.bw = (uint64_t)w0 | ((uint64_t)w1 << 32);
              P.m |= PM_INL;
            }
          }
          if (!BUCKET) fo.pev[i] = P;
        }
      }
    } else {
      x.rcnt[i] = cnt;
      x.rset[i] = set;
      x.rkind[i] = cnt ? (uint8_t)(ev | (user_kind ? 0x80u : 0u)) : EV_NONE;
      x.rsn[i] = sn;
    }
  };
  if (!BUCKET) {
    for (uint64_t i = (uint64_t)blockIdx.x * IT + tid; i < max; i += (uint64_t)gridDim.x * IT) {
      uint32_t key;
      PEv P;
      body(i, key, P, reinterpret_cast<const u32x4*>(recs + i));
    }
  } else {
    // wave w: slots [c0, c0 + PB_SUB) in PB_STEPS steps of 64; the proxied events stay in registers
    const uint64_t c0 = (uint64_t)blockIdx.x * CHR + (uint64_t)wave * PB_SUB;
    uint32_t key[PB_STEPS];
    PEv P[PB_STEPS];
#if RTPS_CL_PRELOAD
    // every step's record loaded ahead (whole 64-B records: the same lines), so that the steps'
    // loads are in flight together instead of one step's dependent chain at a time
    u32x4 rq[PB_STEPS][4];
#pragma unroll
    for (uint32_t j = 0; j < PB_STEPS; ++j) {
      const uint64_t i = c0 + j * 64u + lane;
      const u32x4* q = reinterpret_cast<const u32x4*>(recs + i);
#pragma unroll
      for (uint32_t k = 0; k < 4; ++k) rq[j][k] = i < n ? q[k] : u32x4{0u, 0u, 0u, 0u};
    }
#endif
#pragma unroll
    for (uint32_t j = 0; j < PB_STEPS; ++j) {
      const uint64_t i = c0 + j * 64u + lane;
      key[j] = NONE;
#if RTPS_CL_PRELOAD
      if (i < max) body(i, key[j], P[j], rq[j]);
#else
      if (i < max) body(i, key[j], P[j], reinterpret_cast<const u32x4*>(recs + i));
#endif
      if (key[j] != NONE) atomicAdd(&s_cnt[wave][key[j]], 1u);
    }
    CSS(3);
    CSS_FLUSH();
    CST(2);
    __syncthreads();
    CST(3);
    // the workgroup's region: proxies in order, each proxy's events in slot order (waves in
    // order); thread t owns proxies [t * PPB, t * PPB + PPB)
    constexpr uint32_t PPB = PB_MAX / IT;
    const uint32_t np = t.n_proxies;
    uint32_t tot[PPB], sum = 0;
#pragma unroll
    for (uint32_t r = 0; r < PPB; ++r) {
      const uint32_t e = tid * PPB + r;
      tot[r] = 0;
      if (e < np)
        for (uint32_t w = 0; w < IT / 64; ++w) tot[r] += s_cnt[w][e];
      sum += tot[r];
    }
    const uint32_t incl = wave_incl_sum(sum, lane);
    if (lane == 63u) s_part[wave] = incl;
    __syncthreads();
    uint32_t run = incl - sum;
    for (uint32_t w = 0; w < wave; ++w) run += s_part[w];
    const uint64_t tb = (uint64_t)blockIdx.x * np;
#pragma unroll
    for (uint32_t r = 0; r < PPB; ++r) {
      const uint32_t e = tid * PPB + r;
      if (e >= np) break;
      fo.bk_cl[tb + e] = tot[r] | run << 16;  // (both <= CHR < 2^16)
      for (uint32_t w = 0; w < IT / 64; ++w) {
        const uint32_t c = s_cnt[w][e];
        s_cnt[w][e] = run;
        run += c;
      }
    }
    __syncthreads();
    CST(4);
    PEv* region = fo.pev + (uint64_t)blockIdx.x * CHR;
#pragma unroll
    for (uint32_t j = 0; j < PB_STEPS; ++j) {
      // stable rank among the step's equal proxies: bitonic sort of (proxy << 6 | lane)
      uint32_t v = ((key[j] != NONE ? key[j] : PB_MAX) << 6) | lane;
#pragma unroll
      for (uint32_t kk = 2; kk <= 64; kk <<= 1) {
#pragma unroll
        for (uint32_t d = kk >> 1; d > 0; d >>= 1) {
          const uint32_t p = (uint32_t)__shfl_xor((int)v, d, 64);
          const bool up = (lane & kk) == 0, lower = (lane & d) == 0;
          v = (lower == up) ? (p < v ? p : v) : (p > v ? p : v);
        }
      }
      const uint32_t sk = v >> 6, sl = v & 63u;
      const uint32_t prev = (uint32_t)__shfl_up((int)sk, 1, 64);
      uint32_t start = (lane == 0 || prev != sk) ? lane : 0u;  // first lane of this lane's run
#pragma unroll
      for (uint32_t d = 1; d < 64; d <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)start, d, 64);
        if (lane >= d && y > start) start = y;
      }
      const uint32_t next = (uint32_t)__shfl_down((int)sk, 1, 64);
      const bool tail = lane == 63u || next != sk;
      uint32_t pos = 0;
      if (sk < PB_MAX) {
        const uint32_t base = s_cnt[wave][sk];  // read by every lane of the run before its tail advances it
        pos = base + (lane - start);
        if (tail) s_cnt[wave][sk] = pos + 1u;
      }
      // the position back to the slot's own lane (forward permute: lane sl receives it)
      pos = (uint32_t)__builtin_amdgcn_ds_permute((int)(sl << 2), (int)pos);
      if (key[j] != NONE) region[pos] = P[j];
    }
    CST(5);
  }
  __shared__ uint32_t s_n[4];
  if (tid < 4) s_n[tid] = 0;
  __syncthreads();
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    nh += __shfl_xor(nh, d, 64); ng += __shfl_xor(ng, d, 64); ne += __shfl_xor(ne, d, 64);
    nf += __shfl_xor(nf, d, 64);
  }
  if (lane == 0) {
    atomicAdd(&s_n[0], nh); atomicAdd(&s_n[1], ng); atomicAdd(&s_n[2], ne); atomicAdd(&s_n[3], nf);
  }
  __syncthreads();
  if (tid < 4 && s_n[tid])
    atomicAdd(reinterpret_cast<unsigned long long*>(ctr + C_SPREAD + 4u * (blockIdx.x & 63u) + tid),
              (unsigned long long)s_n[tid]);
  if ((MARK || !IDENT) && nfar) atomicAdd(reinterpret_cast<unsigned long long*>(ctr + C_FARC), (unsigned long long)nfar);
  if ((MARK || !IDENT) && ntg) atomicAdd(reinterpret_cast<unsigned long long*>(ctr + C_TGAP), (unsigned long long)ntg);
  CST(6);
}

// The batch's counts to pinned host memory (one wave, after classify): the sums, then the tag
// last, written through (system scope) after the sums' stores have completed.  The host
// spins on the tag instead of a copy and an interrupt-driven stream sync.
// ident: also the verdict on an identity batch (SIG_MODE): 0 = the host decides, 1 / 2 =
// the plain global path (no HEARTBEAT that counts, no GAP, no far item, not per proxy), merged by
// the samples' wave_or / from the first-cover keys; the guarded decide and state launches queued
// behind this kernel then run it without waiting for the host (the host's rule, on the device).
struct SigCfg {
  uint32_t ident, n_proxies, path, reliable;
  const uint64_t* fused;  // the far-set pool's counter
};
// the verdict from the batch's counts (the host's path rule, on the device)
__device__ __forceinline__ uint64_t plain_mode(uint64_t n_hb, uint64_t n_gap, uint64_t n_ev, uint64_t nev,
                                               uint64_t farc, const SigCfg& cf) {
  if (!cf.ident || !nev) return 0;
  const bool have_hb = cf.reliable && n_hb > 0;
  const bool per_proxy = cf.n_proxies > 0 && (cf.path == 2 || cf.path == 4 ||
                                              (cf.path == 0 && cf.n_proxies >= 64 &&
                                               n_ev <= (uint64_t)cf.n_proxies * 32768u));
  if (have_hb || n_gap != 0 || farc != 0 || per_proxy) return 0;
  return (cf.path == 3 || (cf.path != 1 && (uint64_t)cf.n_proxies * W <= 4ull * nev)) ? 2u : 1u;
}
// The batch's counts by one wave: lane k loads spread slot k's four counters, a wave reduction
// sums them (every lane gets the sums)
struct Counts {
  uint64_t n_hb, n_gap, n_ev, n_free, nrec, farc, tgap;
};
__device__ __forceinline__ Counts wave_counts(const uint64_t* ctr, uint32_t lane) {
  const ulonglong2 a = *reinterpret_cast<const ulonglong2*>(ctr + C_SPREAD + 4u * lane);
  const ulonglong2 b = *reinterpret_cast<const ulonglong2*>(ctr + C_SPREAD + 4u * lane + 2u);
  Counts c{a.x, a.y, b.x, b.y, ctr[C_NREC], ctr[C_FARC], ctr[C_TGAP]};
#pragma unroll
  for (uint32_t d = 32; d >= 1; d >>= 1) {
    c.n_hb += __shfl_xor(c.n_hb, d, 64); c.n_gap += __shfl_xor(c.n_gap, d, 64);
    c.n_ev += __shfl_xor(c.n_ev, d, 64); c.n_free += __shfl_xor(c.n_free, d, 64);
  }
  return c;
}
// the counts (and the verdict) to pinned host memory, the tag last, written through after the
// rest completed (one wave: lane k writes word k)
__device__ __forceinline__ void signal_host(const Counts& c, uint64_t mode, uint64_t* hsig, uint64_t tag,
                                            uint32_t lane, const SigCfg& cf) {
  const uint64_t v = lane == 0 ? c.n_hb : lane == 1 ? c.n_gap : lane == 2 ? c.n_ev : lane == 3 ? c.n_free
                   : lane == 4 ? c.nrec : lane == 5 ? c.farc : lane == 6 ? mode : lane == 7 ? (cf.fused ? *cf.fused : 0)
                   : c.tgap;
  if (lane < 9) __hip_atomic_store(hsig + SIG_HB + lane, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (lane == 0) __hip_atomic_store(hsig + SIG_TAG, tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
// one wave: lane k loads spread slot k's four counters, a wave reduction sums them; then the
// sums, the record / far counts and the verdict go out (C_MODE for the queued kernels, the pinned
// words for the host, the tag last, written through after the rest completed)
__global__ void k_signal(uint64_t* ctr, uint64_t* hsig, uint64_t tag, SigCfg cf) {
  const uint32_t lane = threadIdx.x;
  const Counts c = wave_counts(ctr, lane);
  const uint64_t mode = plain_mode(c.n_hb, c.n_gap, c.n_ev, c.nrec, c.farc, cf);
  if (lane == 0) ctr[C_MODE] = mode;
  signal_host(c, mode, hsig, tag, lane, cf);
}

// 1b: lane per record writes its events at roff[i] (set order = EntityId order of the readers)
__global__ __launch_bounds__(IT) void k_expand(ReaderDev t, uint64_t n, uint32_t flags, Scratch x, bool with_frag) {
  const bool reliable = !(flags & RTPS_INGEST_BEST_EFFORT);
  for (uint64_t i = (uint64_t)blockIdx.x * IT + threadIdx.x; i < n; i += (uint64_t)gridDim.x * IT) {
    const uint8_t rk = x.rkind[i];
    if (rk == EV_NONE) continue;
    const uint8_t ev = rk & 0x7fu;
    const bool user_kind = (rk & 0x80u) != 0u;
    const uint32_t set = x.rset[i];
    uint32_t k = x.roff[i];
    const int64_t sn = x.rsn[i];
    const bool fs = with_frag && x.fidx[i] != NONE;
    const uint64_t fm = fs ? x.fmask[i] : ~0ull;
    const bool fa = !fs || x.fall[i] != 0u;
    for (uint32_t j = t.set_first[set], b = j, e = t.set_first[set + 1]; j < e; ++j) {
      uint32_t en, me;
      if (!frag_takes(fm, fa, j - b, x, i, t.set_ent[j].reader_slot)) continue;
      if (!ev_of(ev, t.set_ent[j], user_kind, reliable, en, me)) continue;
      x.evt[k] = ev;
      x.ent[k] = en;
      x.esn[k] = sn;
      x.erec[k] = (uint32_t)i;
      x.emeta[k] = me;
      x.hkey[k] = ev == EV_HB ? 1u : 0u;
      ++k;
    }
  }
}

// the compacted HEARTBEAT event indices (hval, event order) -> their proxies (hkey)
__global__ __launch_bounds__(IT) void k_hkeys(uint64_t n_hb, Scratch x) {
  for (uint64_t q = (uint64_t)blockIdx.x * IT + threadIdx.x; q < n_hb; q += (uint64_t)gridDim.x * IT)
    x.hkey[q] = x.ent[x.hval[q]];
}

// ---- 2 heartbeats ----
__global__ __launch_bounds__(IT) void k_hvals(const rtps_record* recs, uint64_t n_hb, Scratch x, State s) {
  for (uint64_t q = (uint64_t)blockIdx.x * IT + threadIdx.x; q < n_hb; q += (uint64_t)gridDim.x * IT) {
    const uint32_t k = x.skey[q];
    x.hcnt[q] = recs[x.erec[x.sval[q]]].u.hb.count;
    if (q == 0 || x.skey[q - 1] != k) s.seg_b[k] = (uint32_t)q;
    if (q + 1 == n_hb || x.skey[q + 1] != k) s.seg_e[k] = (uint32_t)q + 1u;
  }
}
// accepted iff count > max(state count, every earlier count of the proxy) (reader.rs:902-905);
// an accepted HEARTBEAT covers [0, firstSN) (irrelevant_changes_up_to)
__global__ __launch_bounds__(IT) void k_hacc(const rtps_record* recs, uint64_t n_hb, Scratch x, State s) {
  for (uint64_t q = (uint64_t)blockIdx.x * IT + threadIdx.x; q < n_hb; q += (uint64_t)gridDim.x * IT) {
    const uint32_t k = x.skey[q];
    const int32_t before = x.hexcl[q] > s.hbc[k] ? x.hexcl[q] : s.hbc[k];
    x.hf[q] = x.hcnt[q] > before ? recs[x.erec[x.sval[q]]].sn : INT64_MIN;
  }
}

// ---- 3 marks ----
// The sequence numbers a valid GAP covers, as (window word, bit mask) pairs:
// irrelevant_changes_range(gapStart, gapList.base) (a negative range changes
// nothing) and set_irrelevant_change per listed SN (NumberSetIter,
// sequence_number.rs:543-557), clipped to the proxy's window [lo, lo + W).
// The window words a valid GAP covers, (word, bits) pairs to f: the range
// [gapStart, gapList.base) (irrelevant_changes_range; a negative range changes
// nothing) and the listed SNs (set_irrelevant_change per NumberSetIter element,
// sequence_number.rs:543-557), clipped to the window [lo, lo + W).  word(w): the
// bitmap's w-th u32 in host order (MSB first = SN base + 32 w).
template <typename WF, typename F>
__device__ __forceinline__ void gap_cover_w(int64_t start, int64_t base, uint32_t num_bits, WF&& word_of, int64_t lo,
                                            F&& f) {
  if (start <= base) {
    const int64_t a = (start > lo ? start : lo) - lo, b = (base < lo + (int64_t)W ? base : lo + (int64_t)W) - lo;
    for (int64_t w = a >> 5; a < b && (w << 5) < b; ++w) {
      const int64_t lb = a > (w << 5) ? a - (w << 5) : 0, hb = b < ((w + 1) << 5) ? b - (w << 5) : 32;
      const uint32_t m = (uint32_t)((hb == 32 ? 0xffffffffull : ((1ull << hb) - 1ull)) & ~((1ull << lb) - 1ull));
      if (m) f((uint64_t)w, m);
    }
  }
  for (uint32_t w = 0; w * 32u < num_bits; ++w) {
    uint32_t word = word_of(w);
    const uint32_t valid = num_bits - w * 32u;
    if (valid < 32u) word &= ~(0xffffffffu >> valid);
    uint64_t src = __builtin_bitreverse32(word);  // bit j = SN base + 32 w + j
    int64_t off = base + (int64_t)(w * 32u) - lo;
    if (off < 0) { if (off <= -32) continue; src >>= (uint32_t)(-off); off = 0; }
    if (!src || off >= (int64_t)W) continue;
    const uint64_t sh = (uint64_t)off & 31u, dw = (uint64_t)off >> 5;
    const uint64_t v2 = src << sh;
    if ((uint32_t)v2) f(dw, (uint32_t)v2);
    if ((uint32_t)(v2 >> 32) && dw + 1u < WW) f(dw + 1u, (uint32_t)(v2 >> 32));
  }
}
template <typename F>
__device__ __forceinline__ void gap_cover(int64_t start, int64_t base, const uint8_t* bm, uint32_t num_bits, bool le,
                                          int64_t lo, F&& f) {
  gap_cover_w(start, base, num_bits, [&](uint32_t w) { return rd32(bm + 4u * w, le); }, lo, f);
}
template <typename F>
__device__ __forceinline__ void gap_words(const rtps_record& r, const uint8_t* arena, const uint64_t* dgram_off,
                                          int64_t lo, F&& f) {
  gap_cover(r.sn, r.u.gap.list_base, arena + dgram_off[r.dgram_idx] + r.u.gap.bitmap_off, r.u.gap.num_bits,
            (r.flags & 1u) != 0u, lo, f);
}

__device__ __forceinline__ bool proxied_sample(const Scratch& x, uint64_t k) {
  return x.evt[k] == EV_SAMPLE && x.ent[k] != NONE;
}

// samples first: their sequence numbers (dbits) and first-cover keys
__global__ __launch_bounds__(IT) void k_marks_d(uint64_t n, Scratch x, State s, uint32_t epoch, bool gaps,
                                                bool keys = true) {
  for (uint64_t i0 = (uint64_t)blockIdx.x * IT; i0 < n; i0 += (uint64_t)gridDim.x * IT) {  // wave-uniform trip count
    const uint64_t i = i0 + threadIdx.x;
    bool act = i < n && proxied_sample(x, i);
    uint32_t* word = s.dbits;
    uint32_t bit = 0;
    if (act) {
      const uint32_t e = x.ent[i];
      const int64_t v = x.esn[i], lo = s.lo[e];
      act = v >= lo && v < lo + (int64_t)W;
      if (act) {
        const uint64_t off = (uint64_t)(v - lo);
        word = s.dbits + (uint64_t)e * WW + (off >> 5);
        bit = 1u << (off & 31u);
        if (keys) atomicMin(reinterpret_cast<unsigned long long*>(s.fc + (uint64_t)e * W) + off, ekey(epoch, (uint32_t)i));
      }
    }
    if (gaps) wave_or(s.dbits, word, bit, act);  // the sample bitmap only serves k_marks_g
  }
}
// then GAPs: a GAP's first-cover key matters only where a sample of the batch
// has the same sequence number, so only those are marked (32 at a time)
__global__ __launch_bounds__(IT) void k_marks_g(const rtps_record* recs, const uint8_t* arena, const uint64_t* dgram_off,
                                                uint64_t n, Scratch x, State s, uint32_t epoch) {
  for (uint64_t i = (uint64_t)blockIdx.x * IT + threadIdx.x; i < n; i += (uint64_t)gridDim.x * IT) {
    if (x.evt[i] != EV_GAP) continue;
    const uint32_t e = x.ent[i];
    const int64_t lo = s.lo[e];
    const uint32_t* db = s.dbits + (uint64_t)e * WW;
    unsigned long long* fc = reinterpret_cast<unsigned long long*>(s.fc + (uint64_t)e * W);
    const unsigned long long key = ekey(epoch, (uint32_t)i);
    auto mark_word = [&](uint64_t w, uint32_t m) {  // window word w, covered bits m
      m &= db[w];
      while (m) {
        const uint32_t b = (uint32_t)__builtin_ctz(m);
        m &= m - 1u;
        atomicMin(fc + (w << 5) + b, key);
      }
    };
    gap_words(recs[x.erec[i]], arena, dgram_off, lo, mark_word);
  }
}

// ---- 4 decide ----
// one sample event: accepted?  pe / poff / merge: the proxy and window offset of a sample
// whose position the change-set merge sets (an accepted sample in the window, or any sample
// of a DUPLICATES_OK reader's proxy in it: received_changes_add runs for those too)
// Far items go to the batch's list (recs / dgram_off: a GAP's fields; the bitmap stays in the arena).
struct FarSrc {
  const rtps_record* recs;
  const uint64_t* dgram_off;
};
__device__ __forceinline__ void gap_far_item(uint64_t i, const Scratch& x, const State& s, const FarSrc& fs) {
  const uint32_t e = x.ent[i];
  const rtps_record& r = fs.recs[x.erec[i]];
  const int64_t lim = s.lo[e] + (int64_t)W;
  if (r.u.gap.list_base + (int64_t)r.u.gap.num_bits > lim)
    far_push(s,
             FarItem{PEv{r.sn, r.u.gap.list_base, fs.dgram_off[r.dgram_idx] + r.u.gap.bitmap_off,
                         EV_GAP | ((r.flags & 1u) ? PM_LE : 0u) | (r.u.gap.num_bits << 8), (uint32_t)i},
                     lim, e, FI_GAP});
}
// a sample's accepting HEARTBEAT threshold at event i (the binary search over the proxy's sorted
// HEARTBEATs, only when the proxy's final threshold lies above v)
__device__ __forceinline__ int64_t hb_thr(uint64_t i, int64_t v, int64_t thr, uint32_t sb, uint32_t se,
                                          const Scratch& x, bool reliable) {
  if (reliable && se > sb && x.hpre[se - 1u] > v && v >= thr) {
    uint32_t a = sb, b = se;
    while (a < b) {  // first sorted position whose event is >= i
      const uint32_t m = (a + b) >> 1;
      if (x.sval[m] < (uint32_t)i) a = m + 1u; else b = m;
    }
    if (a > sb && x.hpre[a - 1u] > thr) thr = x.hpre[a - 1u];
  }
  return thr;
}
__device__ __forceinline__ uint8_t decide_one(uint64_t i, uint64_t n, const Scratch& x, const State& s, bool reliable,
                                              uint32_t epoch, const FarSrc& fs, uint32_t& pe, uint64_t& poff,
                                              bool& merge) {
  merge = false;
  if (i >= n) return 0;
  const uint8_t ev = x.evt[i];
  if (ev == EV_GAP) {  // its coverage past the window is the far replay's
    gap_far_item(i, x, s, fs);
    return 0;
  }
  if (ev != EV_SAMPLE) return 0;
  const uint32_t e = x.ent[i], meta = x.emeta[i];
  if (e == NONE) return 1;  // no proxy: the writer kind is not user-defined (reader.rs:734-739)
  const int64_t v = x.esn[i], lo = s.lo[e];
  const bool in_win = v >= lo && v < lo + (int64_t)W;
  pe = e;
  poff = (uint64_t)(v - lo);
  if (meta & EVF_DUP_OK) {  // the participant reader's duplicates (reader.rs:712-722)
    merge = in_win;
    if (v >= lo + (int64_t)W) far_push(s, FarItem{PEv{v, 0, 0, EV_SAMPLE, (uint32_t)i}, lo + (int64_t)W, e, FI_DUP});
    return 1;
  }
  const int64_t thr = hb_thr(i, v, s.base[e], s.seg_b[e], s.seg_e[e], x, reliable);
  if (v < 1 || v < thr) return 0;
  if (v >= lo + (int64_t)W) {  // beyond the window: accepted until the far replay (k_far) decides
    far_push(s, FarItem{PEv{v, 0, 0, EV_SAMPLE, (uint32_t)i}, lo + (int64_t)W, e, FI_SAMPLE});
    return 1;
  }
  const bool known = (s.bits[(uint64_t)e * WW + (poff >> 5)] >> (poff & 31u)) & 1u;
  const uint8_t acc = (!known && s.fc[(uint64_t)e * W + poff] == ekey(epoch, (uint32_t)i)) ? 1 : 0;
  merge = acc != 0;
  return acc;
}
// (acc[0, cap): entries past n are cleared)
__global__ __launch_bounds__(IT) void k_decide(uint64_t n, uint64_t cap, Scratch x, State s, uint8_t* acc_out,
                                               bool reliable, uint32_t epoch, FarSrc fs) {
  for (uint64_t i = (uint64_t)blockIdx.x * IT + threadIdx.x; i < cap; i += (uint64_t)gridDim.x * IT) {
    uint32_t e;
    uint64_t off;
    bool w;
    acc_out[i] = decide_one(i, n, x, s, reliable, epoch, fs, e, off, w);
  }
}

// ---- 5 deliveries: selected events -> (record, reader slot); per-record accept counts ----
// The flagged events in order, as deliveries, in two launches (instead of a device
// select of the indices and a gather): k_dcount counts each tile of DT flags;
// k_dwrite sums the earlier tiles' counts again per workgroup (from L2: a few KB),
// ranks its tile's flags with a block scan and writes the deliveries.
#ifndef RTPS_DPT
#define RTPS_DPT 8
#endif
constexpr uint32_t DPT = RTPS_DPT, DT = IT * DPT;  // flags per thread / per tile
static_assert(DPT % 8 == 0 && DPT <= 32, "whole 8-B flag groups per thread");
// nonzero bytes of a word
__device__ __forceinline__ uint32_t nz_bytes(uint32_t v) {
  const uint32_t t = ~(((v & 0x7f7f7f7fu) + 0x7f7f7f7fu) | v | 0x7f7f7f7fu);  // 0x80 in the zero bytes
  return 4u - (uint32_t)__builtin_popcount(t);
}
__device__ __forceinline__ void dflags(const uint8_t* flag, uint64_t n, uint64_t b0, uint32_t (&w)[DPT / 4]) {
  if (b0 + DPT <= n) {
#pragma unroll
    for (uint32_t q = 0; q < DPT / 8; ++q) {  // any alignment of the caller's flag array
      uint2 a;
      __builtin_memcpy(&a, flag + b0 + 8u * q, 8);
      w[2 * q] = a.x; w[2 * q + 1] = a.y;
    }
  } else {
#pragma unroll
    for (uint32_t q = 0; q < DPT / 4; ++q) w[q] = 0u;
    for (uint64_t i = b0; i < n; ++i) w[(i - b0) >> 2] |= (flag[i] ? 1u : 0u) << (8u * ((i - b0) & 3u));
  }
}
__device__ __forceinline__ uint64_t block_sum64(uint64_t v, uint64_t* s_w) {
#pragma unroll
  for (uint32_t d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
  __syncthreads();
  if ((threadIdx.x & 63u) == 0) s_w[threadIdx.x >> 6] = v;
  __syncthreads();
  uint64_t t = 0;
#pragma unroll
  for (uint32_t w = 0; w < IT / 64; ++w) t += s_w[w];
  return t;
}
// Global identity path: decide + the delivery tile counts (k_dcount's) in one pass, DPT
// consecutive events per thread (tiles of DT, the tiling k_dwrite reads), and for GAP-free
// batches (MERGE) the change-set merge: a window position is set by its accepted first
// cover (or by a DUPLICATES_OK reader's samples, whose proxy's decisions read no bits), so
// no decision of the pass reads a bit the pass sets for another event; the positions of
// the other samples lie below the new ack_base (v < 1 or below a HEARTBEAT threshold) or
// are set already, so k_merge's extra bits there change nothing k_state reads.
// MERGE 2 (GAP-free batches whose proxies' windows are few against their events, T): the
// merge is the first-cover keys instead: workgroups [ntiles, grid) scan every proxy's window
// of keys and write each word's positions that carry this batch's epoch into dbits (every
// word written, zeros too), which state_proxy ORs into the window and clears.  The decisions
// read `bits` only, so the scan runs beside them; it replaces k_merge's per-sample wave_or.
constexpr uint32_t FCM_POS = 8192;  // window positions per scanning workgroup
static_assert(FCM_POS % (IT * 2) == 0 && W % FCM_POS == 0, "whole wave steps of 128 positions");
struct SigOut {
  uint64_t* hsig;
  uint64_t tag;
  SigCfg cf;
};
// The workgroup's far samples (per thread: bit j of fpm = event b0 + j, fpd: DUPLICATES_OK) into
// the far list: a block scan of the counts, one atomic on the list counter, then each thread
// writes its items (their fields re-read: the event's sn and proxy, the proxy's window).
// Every thread calls it.
__device__ void far_push_block(const State& s, const Scratch& x, uint64_t b0, uint32_t fpm, uint32_t fpd) {
  __shared__ uint32_t s_fw[IT / 64];
  __shared__ unsigned long long s_fbase;
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  const uint32_t cnt = (uint32_t)__builtin_popcount(fpm);
  const uint32_t incl = wave_incl_sum(cnt, lane);
  if (lane == 63u) s_fw[wave] = incl;
  __syncthreads();
  uint32_t off = incl - cnt, tot = 0;
#pragma unroll
  for (uint32_t v = 0; v < IT / 64; ++v) {
    off += v < wave ? s_fw[v] : 0u;
    tot += s_fw[v];
  }
  if (tot == 0) return;  // (uniform)
  if (threadIdx.x == 0) s_fbase = atomicAdd(reinterpret_cast<unsigned long long*>(s.ctr + C_NFAR), (unsigned long long)tot);
  __syncthreads();
  uint64_t pos = s_fbase + off;
  while (fpm) {
    const uint32_t j = (uint32_t)__builtin_ctz(fpm);
    fpm &= fpm - 1u;
    const uint64_t i = b0 + j;
    const uint32_t e = x.ent[i];
    const int64_t v = x.esn[i], lim = s.lo[e] + (int64_t)W;
    if (pos < s.fl_cap)
      s.fl[pos] = FarItem{PEv{v, 0, 0, EV_SAMPLE, (uint32_t)i}, lim, e, ((fpd >> j) & 1u) ? (uint32_t)FI_DUP : (uint32_t)FI_SAMPLE};
    ++pos;
  }
}
template <int MERGE>
__global__ __launch_bounds__(IT) void k_decide_t(uint64_t n, uint64_t cap, Scratch x, State s, uint8_t* acc_out,
                                                 bool reliable, uint32_t epoch, uint32_t* tcnt, FarSrc fs,
                                                 uint32_t ntiles, SigOut so) {
  __shared__ uint64_t s_w[IT / 64];
  __shared__ uint32_t s_mode;
  // MERGE 3: launched before the host has the counts.  Every workgroup's first wave sums them and
  // applies the host's path rule (plain_mode); workgroup 0 also hands the counts and the verdict
  // to the host (and to the state launch, C_MODE).  Not plain: every workgroup returns.
  int mm = MERGE;
  if (MERGE == 3) {
    if (threadIdx.x < 64) {
      const Counts c = wave_counts(s.ctr, threadIdx.x);
      const uint64_t mode = plain_mode(c.n_hb, c.n_gap, c.n_ev, c.nrec, c.farc, so.cf);
      if (threadIdx.x == 0) s_mode = (uint32_t)mode;
      if (blockIdx.x == 0) {
        if (threadIdx.x == 0) s.ctr[C_MODE] = mode;
        signal_host(c, mode, so.hsig, so.tag, threadIdx.x, so.cf);
      }
    }
    __syncthreads();
    mm = (int)s_mode;
    if (mm == 0) return;
  }
  // (MERGE 2: the key-scanning workgroups come first, so that they run beside the decisions)
  const uint32_t nfcm = (MERGE == 2 || MERGE == 3) ? gridDim.x - ntiles : 0u;
  if ((MERGE == 2 || MERGE == 3) && blockIdx.x < nfcm) {
    if (mm != 2) return;
    // two positions per lane (one 16-B load), 128 per wave step: the even and the odd
    // positions' ballots interleave into the step's four words (lanes 0..3 store them)
    const uint64_t p0 = (uint64_t)blockIdx.x * FCM_POS;  // a multiple of W / FCM_POS per proxy
    const uint32_t tag = 0xffffffffu - epoch, lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    auto spread = [](uint32_t x) {  // bit i -> bit 2i (16 bits)
      x = (x | (x << 8)) & 0x00ff00ffu;
      x = (x | (x << 4)) & 0x0f0f0f0fu;
      x = (x | (x << 2)) & 0x33333333u;
      return (x | (x << 1)) & 0x55555555u;
    };
#pragma unroll 4
    for (uint32_t r = 0; r < FCM_POS / (IT * 2); ++r) {
      const uint64_t g = p0 + (uint64_t)(r * (IT / 64) + wave) * 128u;  // the wave's 128 positions
      const ulonglong2 k = *reinterpret_cast<const ulonglong2*>(s.fc + g + 2u * lane);
      const uint64_t me = __ballot((uint32_t)(k.x >> 32) == tag), mo = __ballot((uint32_t)(k.y >> 32) == tag);
      if (lane < 4u) {
        const uint32_t sh = 16u * lane;
        s.dbits[(g >> 5) + lane] = spread((uint32_t)(me >> sh) & 0xffffu) | (spread((uint32_t)(mo >> sh) & 0xffffu) << 1);
      }
    }
    return;
  }
  const uint32_t blk = blockIdx.x - nfcm;  // the delivery tile
  const uint64_t b0 = (uint64_t)blk * DT + threadIdx.x * DPT;
  uint32_t w[DPT / 4];
#pragma unroll
  for (uint32_t q = 0; q < DPT / 4; ++q) w[q] = 0u;
  uint32_t c = 0;
  // far samples: bit j of fpm = event b0 + j goes to the far list, fpd: as a DUPLICATES_OK one;
  // the workgroup reserves their places with ONE atomic at the end (far_push's per-wave atomic
  // on the list counter serialises at the memory side when most samples are far: SPDP)
  uint32_t fpm = 0, fpd = 0;
  // the thread's DPT events in groups of HG, decide_one's rule in phases so that each phase's
  // loads are in flight together: the event fields (vector loads), the proxies' state, the
  // window words (HG = 4: 8 would hold 130 VGPRs, 3 waves per SIMD)
  constexpr uint32_t HG = 4;
#pragma unroll
  for (uint32_t h = 0; h < DPT; h += HG) {
  const uint64_t g0 = b0 + h;
  uint32_t evw, ent[HG], meta[HG];
  int64_t sn[HG];
  if (g0 + HG <= n) {
    evw = *reinterpret_cast<const uint32_t*>(x.evt + g0);
    const uint4 a = *reinterpret_cast<const uint4*>(x.ent + g0);
    const uint4 b = *reinterpret_cast<const uint4*>(x.emeta + g0);
    ent[0] = a.x; ent[1] = a.y; ent[2] = a.z; ent[3] = a.w;
    meta[0] = b.x; meta[1] = b.y; meta[2] = b.z; meta[3] = b.w;
#pragma unroll
    for (uint32_t q = 0; q < HG / 2; ++q) {
      const longlong2 c2 = *reinterpret_cast<const longlong2*>(x.esn + g0 + 2u * q);
      sn[2 * q] = c2.x; sn[2 * q + 1] = c2.y;
    }
  } else {
    evw = 0u;
#pragma unroll
    for (uint32_t j = 0; j < HG; ++j) {
      const bool in = g0 + j < n;
      if (in) evw |= (uint32_t)x.evt[g0 + j] << (8u * j);
      ent[j] = in ? x.ent[g0 + j] : NONE;
      meta[j] = in ? x.emeta[g0 + j] : 0u;
      sn[j] = in ? x.esn[g0 + j] : 0;
    }
  }
  int64_t lo[HG], base[HG];
#pragma unroll
  for (uint32_t j = 0; j < HG; ++j) {
    const uint32_t ev = (evw >> (8u * j)) & 0xffu;
    const uint32_t e = (ev == EV_SAMPLE && ent[j] != NONE) ? ent[j] : 0u;
    lo[j] = s.lo[e];
    base[j] = s.base[e];
  }
  uint32_t bw[HG];
  uint64_t fk[HG];
#pragma unroll
  for (uint32_t j = 0; j < HG; ++j) {
    const uint32_t ev = (evw >> (8u * j)) & 0xffu;
    const bool win = ev == EV_SAMPLE && ent[j] != NONE && sn[j] >= lo[j] && sn[j] < lo[j] + (int64_t)W;
    const uint64_t off = win ? (uint64_t)(sn[j] - lo[j]) : 0u;
    const uint32_t e = win ? ent[j] : 0u;
    bw[j] = s.bits[(uint64_t)e * WW + (off >> 5)];
    fk[j] = s.fc[(uint64_t)e * W + off];
  }
#pragma unroll
  for (uint32_t jj = 0; jj < HG; ++jj) {
    const uint32_t j = h + jj;
    const uint64_t i = b0 + j;
    const uint32_t ev = (evw >> (8u * jj)) & 0xffu, e = ent[jj];
    const int64_t v = sn[jj];
    uint8_t a = 0;
    bool merge = false;
    uint64_t off = 0;
    if (ev == EV_GAP) {
      gap_far_item(i, x, s, fs);
    } else if (ev == EV_SAMPLE) {
      if (e == NONE) {
        a = 1;  // no proxy: the writer kind is not user-defined (reader.rs:734-739)
      } else {
        const bool in_win = v >= lo[jj] && v < lo[jj] + (int64_t)W;
        off = (uint64_t)(v - lo[jj]);
        if (meta[jj] & EVF_DUP_OK) {  // the participant reader's duplicates (reader.rs:712-722)
          a = 1;
          merge = in_win;
          if (v >= lo[jj] + (int64_t)W) { fpm |= 1u << j; fpd |= 1u << j; }
        } else {
          const int64_t thr = hb_thr(i, v, base[jj], reliable ? s.seg_b[e] : 0u, reliable ? s.seg_e[e] : 0u, x,
                                     reliable);
          if (v >= 1 && v >= thr) {
            if (v >= lo[jj] + (int64_t)W) {  // beyond the window: accepted until the far replay decides
              fpm |= 1u << j;
              a = 1;
            } else {
              const bool known = (bw[jj] >> (off & 31u)) & 1u;
              a = (!known && fk[jj] == ekey(epoch, (uint32_t)i)) ? 1 : 0;
              merge = a != 0;
            }
          }
        }
      }
    }
    w[j >> 2] |= (uint32_t)a << (8u * (j & 3u));
    c += a;
    if (mm == 1)
      wave_or(s.bits, merge ? s.bits + (uint64_t)e * WW + (off >> 5) : s.bits, 1u << (off & 31u), merge);
  }
  }
  if (b0 + DPT <= cap) {
#pragma unroll
    for (uint32_t q = 0; q < DPT / 8; ++q) {
      uint2 v = make_uint2(w[2 * q], w[2 * q + 1]);
      __builtin_memcpy(acc_out + b0 + 8u * q, &v, 8);
    }
  } else {
    for (uint64_t i = b0; i < cap; ++i) acc_out[i] = (uint8_t)(w[(i - b0) >> 2] >> (8u * ((i - b0) & 3u)));
  }
  const uint64_t t = block_sum64(c, s_w);
  if (threadIdx.x == 0) tcnt[blk] = (uint32_t)t;
  far_push_block(s, x, b0, fpm, fpd);
}

__global__ __launch_bounds__(IT) void k_dcount(const uint8_t* flag, uint64_t n, uint32_t* tcnt) {
  __shared__ uint64_t s_w[IT / 64];
  uint32_t w[DPT / 4];
  const uint64_t b0 = (uint64_t)blockIdx.x * DT + threadIdx.x * DPT;
  uint32_t c = 0;
  if (b0 < n) {
    dflags(flag, n, b0, w);
#pragma unroll
    for (uint32_t q = 0; q < DPT / 4; ++q) c += nz_bytes(w[q]);
  }
  const uint64_t t = block_sum64(c, s_w);
  if (threadIdx.x == 0) tcnt[blockIdx.x] = (uint32_t)t;
}
__device__ __forceinline__ void dwrite_tile(uint32_t blk, const uint8_t* flag, uint64_t n, const uint32_t* tcnt,
                                            uint32_t ntiles, const Scratch& x, bool ident, uint64_t max_out,
                                            rtps_delivery* out, uint64_t* n_out, const uint64_t* ctr, uint64_t* ovf_out,
                                            uint64_t* hev, const uint64_t* fused, uint64_t* s_w, uint32_t* s_c) {
  const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  uint64_t pre = 0;
  for (uint32_t t = tid; t < blk; t += IT) pre += tcnt[t];
  pre = block_sum64(pre, s_w);
  uint32_t w[DPT / 4];
  const uint64_t b0 = (uint64_t)blk * DT + tid * DPT;
  uint32_t c = 0;
  if (b0 < n) {
    dflags(flag, n, b0, w);
#pragma unroll
    for (uint32_t q = 0; q < DPT / 4; ++q) c += nz_bytes(w[q]);
  }
  uint32_t incl = c;  // block-wide inclusive scan of the per-thread counts
#pragma unroll
  for (uint32_t d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(incl, d, 64);
    if (lane >= d) incl += y;
  }
  if (lane == 63) s_c[wave] = incl;
  __syncthreads();
  uint32_t woff = 0, tot = 0;
#pragma unroll
  for (uint32_t v = 0; v < IT / 64; ++v) {
    if (v < wave) woff += s_c[v];
    tot += s_c[v];
  }
  uint64_t o = pre + woff + incl - c;
  if (c) {
#pragma unroll
    for (uint32_t q = 0; q < DPT / 4; ++q) {
      for (uint32_t j = 0; j < 4; ++j) {
        if (!((w[q] >> (8u * j)) & 0xffu)) continue;
        const uint64_t k = b0 + 4u * q + j;
        if (o < max_out) {
          rtps_delivery d;
          d.rec_idx = ident ? (uint32_t)k : x.erec[k];
          d.reader_slot = (uint16_t)(x.emeta[k] & 0xffffu);
          d.flags = 0;
          out[o] = d;
        }
        ++o;
      }
    }
  }
  if (blk + 1 == ntiles && tid == 0) {
    *n_out = pre + tot;
    if (ovf_out) *ovf_out = ctr[C_OVF];  // the batch's window overflows (counted before the select)
    if (hev) {  // the batch's events, for the next batch's path choice (pinned host memory, read without a sync)
      uint64_t ne = 0;
      for (uint32_t k = 0; k < 64; ++k) ne += ctr[C_SPREAD + 4 * k + 2];
      hev[0] = ne;
      hev[1] = ctr[C_NFAR];  // (per-proxy path: its far items and the pool's use, for the far-set room)
      hev[2] = fused ? *fused : 0;
    }
  }
}
__global__ __launch_bounds__(IT) void k_dwrite(const uint8_t* flag, uint64_t n, const uint32_t* tcnt, uint32_t ntiles,
                                               Scratch x, bool ident, uint64_t max_out, rtps_delivery* out,
                                               uint64_t* n_out, const uint64_t* ctr, uint64_t* ovf_out,
                                               uint64_t* hev, const uint64_t* fused) {
  __shared__ uint64_t s_w[IT / 64];
  __shared__ uint32_t s_c[IT / 64];
  dwrite_tile(blockIdx.x, flag, n, tcnt, ntiles, x, ident, max_out, out, n_out, ctr, ovf_out, hev, fused, s_w, s_c);
}
__global__ __launch_bounds__(IT) void k_accept_counts(uint64_t n, uint64_t cap, Scratch x, uint8_t* accept) {
  for (uint64_t i = (uint64_t)blockIdx.x * IT + threadIdx.x; i < cap; i += (uint64_t)gridDim.x * IT) {
    uint32_t c = 0;
    if (i < n && x.rkind[i] != EV_NONE)
      for (uint32_t k = x.roff[i], e = k + x.rcnt[i]; k < e; ++k) c += x.eacc[k];
    accept[i] = (uint8_t)(c < 255u ? c : 255u);
  }
}

// ---- far sets (see "far sequence numbers" above) ----
// Table words are read with device-coherent loads: other workgroups' (k_far, the pool
// compaction) and other waves' atomics land in the L2, past this CU's L1.
__device__ __forceinline__ int64_t fld(const int64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t fldk(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t fld32(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t fslot(int64_t v, uint32_t mask) {
  return (uint32_t)(((uint64_t)v * 0x9e3779b97f4a7c15ull) >> 32) & mask;
}
// v into the table (sn, key; mask + 1 slots) with first-cover key k; 1 when it took a free slot
__device__ uint32_t fset_add(int64_t* sn, uint64_t* key, uint32_t mask, int64_t v, uint64_t k) {
  for (uint32_t j = fslot(v, mask);; j = (j + 1u) & mask) {
    int64_t cur = fld(sn + j);
    if (cur == FEMPTY) {
      cur = (int64_t)atomicCAS(reinterpret_cast<unsigned long long*>(sn + j), (unsigned long long)FEMPTY,
                               (unsigned long long)v);
      if (cur == FEMPTY) {
        atomicMin(reinterpret_cast<unsigned long long*>(key + j), (unsigned long long)k);
        return 1u;
      }
    }
    if (cur == v) {
      atomicMin(reinterpret_cast<unsigned long long*>(key + j), (unsigned long long)k);
      return 0u;
    }
  }
}
__device__ uint32_t fset_find(const int64_t* sn, uint32_t mask, int64_t v) {
  for (uint32_t j = fslot(v, mask);; j = (j + 1u) & mask) {
    const int64_t cur = fld(sn + j);
    if (cur == v) return j;
    if (cur == FEMPTY) return NONE;
  }
}
// The SNs >= lim a GAP covers (what gap_cover_w clips at the window's end): the range
// [gapStart, gapList.base) when not negative, then the listed SNs.  range(a, b) for
// [a, b) (non-empty), point(v) for each listed one.
template <typename WF, typename RF, typename PF>
__device__ void gap_far(int64_t start, int64_t base, uint32_t num_bits, WF&& word_of, int64_t lim, RF&& range,
                        PF&& point) {
  if (start <= base) {
    const int64_t a = start > lim ? start : lim;
    if (a < base) range(a, base);
  }
  for (uint32_t w = 0; w * 32u < num_bits; ++w) {
    uint32_t word = word_of(w);
    const uint32_t valid = num_bits - w * 32u;
    if (valid < 32u) word &= ~(0xffffffffu >> valid);
    while (word) {
      const uint32_t b = (uint32_t)__builtin_clz(word);  // MSB first: SN base + 32 w + b
      word &= ~(0x80000000u >> b);
      const int64_t v = base + (int64_t)(w * 32u + b);
      if (v >= lim) point(v);
    }
  }
}
// every SN a far item covers: f(v)
template <typename F>
__device__ void far_sns(const PEv& P, uint32_t kind, int64_t lim, const uint8_t* arena, F&& f) {
  if (kind != FI_GAP) {
    f(P.sn);
    return;
  }
  auto range = [&](int64_t a, int64_t b) { for (int64_t v = a; v < b; ++v) f(v); };
  if (P.m & PM_INL)
    gap_far(P.sn, P.a, P.m >> 8, [&](uint32_t w) { return (uint32_t)(P.bw >> (32u * w)); }, lim, range, f);
  else
    gap_far(P.sn, P.a, P.m >> 8, [&](uint32_t w) { return rd32(arena + P.bw + 4u * w, (P.m & PM_LE) != 0u); }, lim,
            range, f);
}
// how many (an upper bound: a GAP's listed SNs inside its own range count twice), at most
// FAR_COUNT_MAX: no table can hold more (ftab_reserve), and sums of counts cannot wrap
constexpr uint64_t FAR_COUNT_MAX = 1ull << 32;  // (x 2^31 items per batch: no u64 sum wraps)
__device__ uint64_t far_count(const PEv& P, uint32_t kind, int64_t lim, const uint8_t* arena) {
  if (kind != FI_GAP) return 1;
  uint64_t c = 0;
  auto range = [&](int64_t a, int64_t b) {
    const uint64_t r = (uint64_t)b - (uint64_t)a;
    c += r < FAR_COUNT_MAX ? r : FAR_COUNT_MAX;
  };
  auto point = [&](int64_t) { ++c; };
  if (P.m & PM_INL)
    gap_far(P.sn, P.a, P.m >> 8, [&](uint32_t w) { return (uint32_t)(P.bw >> (32u * w)); }, lim, range, point);
  else
    gap_far(P.sn, P.a, P.m >> 8, [&](uint32_t w) { return rd32(arena + P.bw + 4u * w, (P.m & PM_LE) != 0u); }, lim,
            range, point);
  return c < FAR_COUNT_MAX ? c : FAR_COUNT_MAX;
}
// One proxy's far set as a workgroup works on it (LDS; loaded / stored by thread 0) and the
// workgroup's scratch for the block-wide operations below.
struct FTab {
  uint64_t off;
  uint32_t cap, n;
  int64_t min;
};
struct FarSh {
  FTab t;
  unsigned long long x;  // reductions
  uint64_t off;
  uint32_t nc, k;
};
__device__ __forceinline__ void ftab_load(const State& s, uint32_t e, FTab& t) {
  t = FTab{s.far_off[e], s.far_cap[e], s.far_n[e], s.far_min[e]};
}
__device__ __forceinline__ void ftab_store(const State& s, uint32_t e, const FTab& t) {
  s.far_off[e] = t.off;
  s.far_cap[e] = t.cap;
  s.far_n[e] = t.n;
  s.far_min[e] = t.min;
}
// t's SNs >= keep_from rehashed (keys kept) into a fresh pool table of nc slots.  Every thread
// of the block calls it (nt threads), t read by all before; false: the pool is out (t unchanged).
__device__ bool ftab_rehash(const State& s, FarSh& f, uint64_t nc, int64_t keep_from, uint32_t nt) {
  const uint32_t tid = threadIdx.x;
  __syncthreads();  // every thread has read f.t
  if (tid == 0) {
    f.nc = 0;
    if (nc <= (1ull << 31)) {
      const uint64_t off = atomicAdd(reinterpret_cast<unsigned long long*>(s.fused), (unsigned long long)nc);
      if (off + nc <= s.fpcap) {
        f.off = off;
        f.nc = (uint32_t)nc;
      }
    }
    f.k = 0;
  }
  __syncthreads();
  const uint32_t c = f.nc;
  if (c == 0) return false;
  int64_t* nsn = s.fsn + f.off;  // (free: taken from above the counter)
  uint64_t* nkey = s.fkey + f.off;
  uint32_t moved = 0;
  const int64_t* osn = s.fsn + f.t.off;
  const uint64_t* okey = s.fkey + f.t.off;
  for (uint32_t j = tid; j < f.t.cap; j += nt) {
    const int64_t v = fld(osn + j);
    if (v != FEMPTY && v >= keep_from) moved += fset_add(nsn, nkey, c - 1u, v, fldk(okey + j));
  }
  if (moved) atomicAdd(&f.k, moved);
  __threadfence();
  __syncthreads();
  if (tid == 0) {
    f.t.off = f.off;
    f.t.cap = c;
    f.t.n = f.k;
  }
  __syncthreads();
  return true;
}
// t made to take `need` more SNs at load <= 1/2 (a table of >= 4 x (n + need) slots when it
// must grow).  Every thread calls it with the same need; false: the pool is out.
__device__ bool ftab_reserve(const State& s, FarSh& f, uint64_t need, uint32_t nt) {
  if (need > (1ull << 31)) return false;  // (no table that large: the pool is out for it)
  const uint64_t want = 2ull * ((uint64_t)f.t.n + need);
  if (want <= f.t.cap) return true;
  uint64_t nc = FT_MIN;
  while (nc < 2ull * want) nc <<= 1;
  return ftab_rehash(s, f, nc, 0, nt);
}
// the SNs each thread holds (f_of(j) for j < cnt) into t with key k_of(j); returns this thread's
// least inserted SN (INT64_MAX: none).  Every thread calls it after ftab_reserve succeeded.
template <typename F>
__device__ void ftab_insert(const State& s, FarSh& f, F&& each) {
  int64_t* sn = s.fsn + f.t.off;
  uint64_t* key = s.fkey + f.t.off;
  const uint32_t mask = f.t.cap - 1u;
  uint32_t claimed = 0;
  int64_t mn = INT64_MAX;
  each([&](int64_t v, uint64_t k) {
    claimed += fset_add(sn, key, mask, v, k);
    if (v < mn) mn = v;
  });
  if (claimed) atomicAdd(&f.t.n, claimed);
  if (mn != INT64_MAX) atomicMin(reinterpret_cast<unsigned long long*>(&f.t.min), (unsigned long long)mn);
}
// is sample key k its SN's first cover in t? (after every insert of the batch is visible)
__device__ __forceinline__ bool ftab_first(const State& s, const FTab& t, int64_t v, uint64_t k) {
  const uint32_t j = fset_find(s.fsn + t.off, t.cap - 1u, v);
  return j != NONE && fldk(s.fkey + t.off + j) == k;
}
__device__ __forceinline__ uint64_t fkey_of(uint32_t epoch, uint32_t event) {
  return ((uint64_t)epoch << 32) | event;
}

// op(base[key], v) for the active lanes of the wave, the lanes sharing a key combined first
// (red): up to 4 rounds of "the first pending lane's key: every lane on it reduced, one
// atomic", then one atomic per lane still pending.  Every lane of the wave calls it.
template <typename T, typename RED, typename OP>
__device__ __forceinline__ void wave_atomic(uint32_t key, T v, bool active, T ident, RED&& red, OP&& op) {
  const uint32_t lane = threadIdx.x & 63u;
  bool todo = active;
#pragma unroll
  for (uint32_t r = 0; r < 4u; ++r) {
    const uint64_t t = __ballot(todo);
    if (t == 0) return;
    const uint32_t leader = (uint32_t)__builtin_ctzll(t);
    const uint32_t k = (uint32_t)__builtin_amdgcn_readlane((int)key, (int)leader);
    const bool mine = todo && key == k;
    T a = mine ? v : ident;  // (the other lanes add the identity: every lane ends with the group's total)
    for (uint32_t d = 1; d < 64; d <<= 1) a = red(a, (T)__shfl_xor(a, d, 64));
    if (lane == leader) op(k, a);
    todo = todo && !mine;
  }
  if (todo) op(key, v);
}

// The global paths' far items (after decide, before the deliveries), in four launches over
// the batch list (its length on the device, the grid from classify's candidate count):
//   k_far_need  each item's far SNs summed per proxy (fneed);
//   k_far_grow  one workgroup per proxy: its table grown for them (fstat: 1 = the pool was out);
//   k_far_ins   every SN of every item inserted with its key;
//   k_far_dec   the samples decided (rejected: acc 0; tcnt: its delivery tile's count).
constexpr uint32_t KF = 256;
// The proxy of a workgroup's first item (its "hot" proxy: one proxy's backlog fills the list,
// SPDP) is reduced in LDS and added to global memory once per workgroup; the rest per wave.
__device__ __forceinline__ uint32_t far_hot(const State& s, uint64_t nf) {
  __shared__ uint32_t s_hk;
  if (threadIdx.x == 0) s_hk = (uint64_t)blockIdx.x * KF < nf ? s.fl[(uint64_t)blockIdx.x * KF].e : NONE;
  __syncthreads();
  return s_hk;
}
__global__ __launch_bounds__(KF) void k_far_need(State s, const uint8_t* arena) {
  __shared__ unsigned long long s_need;
  const uint64_t nf0 = s.ctr[C_NFAR], nf = nf0 < s.fl_cap ? nf0 : s.fl_cap;
  const uint64_t span = (uint64_t)gridDim.x * KF;
  if (threadIdx.x == 0) s_need = 0;
  const uint32_t hk = far_hot(s, nf);
  for (uint64_t b = (uint64_t)blockIdx.x * KF; b < nf; b += span) {  // (whole waves: wave_atomic)
    const uint64_t k = b + threadIdx.x;
    FarItem it{};
    if (k < nf) it = s.fl[k];
    const uint64_t c = k < nf ? far_count(it.p, it.kind, it.lim, arena) : 0;
    wave_atomic<uint64_t>(it.e, c, k < nf, 0ull, [](uint64_t a, uint64_t o) { return a + o; },
                          [&](uint32_t e, uint64_t a) {
                            if (e == hk) atomicAdd(&s_need, (unsigned long long)a);
                            else atomicAdd(reinterpret_cast<unsigned long long*>(s.fneed + e), (unsigned long long)a);
                          });
  }
  __syncthreads();
  if (threadIdx.x == 0 && s_need) atomicAdd(reinterpret_cast<unsigned long long*>(s.fneed + hk), s_need);
}
constexpr uint32_t KG = 1024;  // k_far_grow: a new table's slots initialised and the old one rehashed by 16 waves
__global__ __launch_bounds__(KG) void k_far_grow(State s, uint32_t n_proxies) {
  __shared__ FarSh f;
  const uint32_t e = blockIdx.x;
  if (e >= n_proxies) return;
  const uint64_t need = s.fneed[e];
  if (need == 0) {
    if (threadIdx.x == 0) s.fstat[e] = 0u;
    return;
  }
  if (threadIdx.x == 0) ftab_load(s, e, f.t);
  __syncthreads();
  const bool ok = ftab_reserve(s, f, need, KG);
  if (threadIdx.x == 0) {
    if (ok) ftab_store(s, e, f.t);
    s.fstat[e] = ok ? 0u : 1u;
    s.fneed[e] = 0;
  }
}
__global__ __launch_bounds__(KF) void k_far_ins(State s, const uint8_t* arena) {
  __shared__ uint32_t s_n;
  __shared__ unsigned long long s_min;
  const uint64_t nf0 = s.ctr[C_NFAR], nf = nf0 < s.fl_cap ? nf0 : s.fl_cap;
  const uint64_t span = (uint64_t)gridDim.x * KF;
  if (threadIdx.x == 0) { s_n = 0; s_min = ~0ull; }
  const uint32_t hk = far_hot(s, nf);
  for (uint64_t b = (uint64_t)blockIdx.x * KF; b < nf; b += span) {
    const uint64_t k = b + threadIdx.x;
    FarItem it{};
    bool act = k < nf;
    if (act) {
      it = s.fl[k];
      act = s.fstat[it.e] == 0u;
    }
    uint32_t claimed = 0;
    int64_t mn = INT64_MAX;
    if (act) {
      const uint64_t toff = s.far_off[it.e];
      const uint32_t mask = s.far_cap[it.e] - 1u;
      const uint64_t key = fkey_of(s.epoch, it.p.k);
      far_sns(it.p, it.kind, it.lim, arena, [&](int64_t v) {
        claimed += fset_add(s.fsn + toff, s.fkey + toff, mask, v, key);
        if (v < mn) mn = v;
      });
    }
    wave_atomic<uint32_t>(it.e, claimed, act && claimed, 0u, [](uint32_t a, uint32_t o) { return a + o; },
                          [&](uint32_t e, uint32_t a) {
                            if (e == hk) atomicAdd(&s_n, a);
                            else atomicAdd(s.far_n + e, a);
                          });
    wave_atomic<uint64_t>(it.e, (uint64_t)mn, act && mn != INT64_MAX, ~0ull,
                          [](uint64_t a, uint64_t o) { return a < o ? a : o; },
                          [&](uint32_t e, uint64_t a) {
                            if (e == hk) atomicMin(&s_min, (unsigned long long)a);
                            else atomicMin(reinterpret_cast<unsigned long long*>(s.far_min + e), (unsigned long long)a);
                          });
  }
  __syncthreads();
  if (threadIdx.x == 0 && hk != NONE) {
    if (s_n) atomicAdd(s.far_n + hk, s_n);
    if (s_min != ~0ull) atomicMin(reinterpret_cast<unsigned long long*>(s.far_min + hk), s_min);
  }
}
__global__ __launch_bounds__(KF) void k_far_dec(State s, uint8_t* acc, uint32_t* tcnt) {
  const uint64_t nf0 = s.ctr[C_NFAR], nf = nf0 < s.fl_cap ? nf0 : s.fl_cap;
  uint64_t miss = (blockIdx.x == 0 && threadIdx.x == 0) ? nf0 - nf : 0;  // (past the list: not reached)
  for (uint64_t k = (uint64_t)blockIdx.x * KF + threadIdx.x; k < nf; k += (uint64_t)gridDim.x * KF) {
    const FarItem it = s.fl[k];
    if (it.kind != FI_SAMPLE) continue;
    if (s.fstat[it.e] != 0u) {
      ++miss;  // the pool was out: accepted unchecked
      continue;
    }
    const FTab t{s.far_off[it.e], s.far_cap[it.e], 0u, 0};
    if (!ftab_first(s, t, it.p.sn, fkey_of(s.epoch, it.p.k))) {
      acc[it.p.k] = 0;
      if (tcnt) atomicSub(&tcnt[it.p.k / DT], 1u);
    }
  }
  if (miss) atomicAdd(reinterpret_cast<unsigned long long*>(s.ctr + C_OVF), (unsigned long long)miss);
}

// State, after the window pass found nb (the first uncovered SN >= the threshold inside the
// window, or >= lo + W: every position covered, or the threshold past the window): nb
// continues through the far set t, 8 nt SNs looked up at a time.  Every thread; returns to all.
__device__ int64_t far_extend(const State& s, FarSh& f, int64_t lo, int64_t nb, uint32_t nt) {
  if (f.t.cap == 0 || nb < lo + (int64_t)W || nb < f.t.min) return nb;
  const int64_t* sn = s.fsn + f.t.off;
  const uint32_t mask = f.t.cap - 1u;
  for (int64_t b = nb;; b += 8 * (int64_t)nt) {  // ends: the set holds at most n SNs
    __syncthreads();
    if (threadIdx.x == 0) f.x = ~0ull;
    __syncthreads();
    // the 8 SNs' first probes issued together (independent loads), then each resolved
    int64_t cur[8];
#pragma unroll
    for (uint32_t r = 0; r < 8u; ++r) cur[r] = fld(sn + fslot(b + (int64_t)(r * nt + threadIdx.x), mask));
#pragma unroll
    for (uint32_t r = 0; r < 8u; ++r) {
      const int64_t v = b + (int64_t)(r * nt + threadIdx.x);
      const bool miss = cur[r] == FEMPTY || (cur[r] != v && fset_find(sn, mask, v) == NONE);
      if (miss) {
        atomicMin(&f.x, (unsigned long long)v);
        break;
      }
    }
    __syncthreads();
    if (f.x != ~0ull) return (int64_t)f.x;
  }
}
// ...and after the window was re-anchored at nlo (its bits written to `bits`): the far SNs
// the new window spans set their bits there; t.min becomes the least SN at or above its end.
// When the SNs at or above it are under a quarter of the table's, they move to a smaller
// one (the old table is left to the pool's compaction); none: the set is emptied.
__device__ void far_pull(const State& s, FarSh& f, uint32_t* bits, int64_t nlo, uint32_t nt) {
  const int64_t hi = nlo + (int64_t)W;
  if (f.t.cap == 0 || f.t.min >= hi) return;
  const uint32_t tid = threadIdx.x;
  __syncthreads();  // the window's bits are written; every thread has read f.t
  if (tid == 0) {
    f.x = ~0ull;
    f.k = 0;
  }
  __syncthreads();
  __threadfence();  // (the table's inserts of this kernel, by other waves, are seen by the plain loads below)
  const int64_t* sn = s.fsn + f.t.off;
  uint32_t keep = 0;
  int64_t mn = INT64_MAX;
  auto one = [&](int64_t v) {
    if (v == FEMPTY || v < nlo) return;
    if (v >= hi) {
      ++keep;
      if (v < mn) mn = v;
    } else {
      atomicOr(bits + ((uint64_t)(v - nlo) >> 5), 1u << ((uint64_t)(v - nlo) & 31u));
    }
  };
  const longlong2* sn2 = reinterpret_cast<const longlong2*>(sn);  // (tables: >= 64 slots, 16-B aligned)
  for (uint32_t j = tid; j < f.t.cap / 2u; j += nt) {
    const longlong2 p = sn2[j];
    one(p.x);
    one(p.y);
  }
  if (keep) atomicAdd(&f.k, keep);
  if (mn != INT64_MAX) atomicMin(&f.x, (unsigned long long)mn);
  __syncthreads();
  const uint32_t k = f.k;
  const bool shrink = k != 0 && 4u * k < f.t.n && f.t.cap > FT_MIN;
  uint64_t nc = FT_MIN;
  while (nc < 4ull * k) nc <<= 1;
  if (shrink) (void)ftab_rehash(s, f, nc, hi, nt);  // (the pool out: the table stays as it is)
  if (tid == 0) {
    if (k == 0) f.t = FTab{0, 0u, 0u, INT64_MAX};
    else f.t.min = (int64_t)f.x;
  }
  __syncthreads();
}

// ---- far sets past FT_BIG slots: far_extend / far_pull by the whole grid ----
// far_extend probes the set one SN after another from all_ackable_before, and far_pull scans the
// whole table: one workgroup does that for a large set in milliseconds (one writer a million SNs
// ahead of its window: the SPDP reader's repeats).  With S.fdefer the state pass leaves such a
// proxy at its window's answer (base = nb, the window unshifted in dbits, its table stored) and
// lists it; four launches then finish it with every workgroup:
//   k_fx_ext    the first SN >= nb the set lacks: the candidates [nb, nb + n] in chunks, one
//               probe per thread, an atomicMin; chunks past the minimum found are skipped;
//   k_fx_shift  the window re-anchored at the new all_ackable_before (from dbits);
//   k_fx_pull   the table's SNs the new window spans set their bits, the rest past it counted;
//   k_fx_fin    base / lo / the far set's min (emptied when nothing lies past the window).
constexpr uint32_t FT_BIG = 1u << 14;
// does the state pass need the far set (far_extend, far_pull) after finding nb in the window?
__device__ __forceinline__ bool far_touch(const FTab& t, int64_t lo, int64_t nb) {
  if (t.cap == 0) return false;
  if (nb >= lo + (int64_t)W && nb >= t.min) return true;  // extend
  return t.min < (nb & ~(int64_t)31) + (int64_t)W;      // pull
}
// the deferral (every thread of the state workgroup): the window `win` (LDS, unshifted) to
// dbits, the table and the window's answer stored, the proxy listed
__device__ void far_defer(const State& s, uint32_t e, const FTab& t, const uint32_t* win, int64_t nb, int32_t hbc,
                          uint32_t nt) {
  uint32_t* db = s.dbits + (uint64_t)e * WW;
  for (uint32_t w = threadIdx.x; w < WW; w += nt) db[w] = win[w];
  if (threadIdx.x == 0) {
    ftab_store(s, e, t);
    s.base[e] = nb;
    s.hbc[e] = hbc;
    s.fext[e] = nb + (int64_t)t.n;  // (at most n SNs of the set lie at or above nb)
    const uint64_t i = atomicAdd(reinterpret_cast<unsigned long long*>(s.ctr + C_FDEF), 1ull);
    s.fdl[i] = e;
  }
}
constexpr uint32_t FX = 256, FX_PER = 16;  // threads, SNs per thread per k_fx_ext chunk
__global__ __launch_bounds__(FX) void k_fx_ext(State s) {
  const uint32_t nd = (uint32_t)s.ctr[C_FDEF];
  for (uint32_t i = 0; i < nd; ++i) {
    const uint32_t e = s.fdl[i];
    const int64_t lo = s.lo[e], nb = s.base[e], mn = s.far_min[e];
    const uint32_t cap = s.far_cap[e];
    if (cap == 0 || nb < lo + (int64_t)W || nb < mn) continue;  // no extension (far_extend's test)
    const int64_t* sn = s.fsn + s.far_off[e];
    const uint32_t mask = cap - 1u;
    const uint64_t span = (uint64_t)s.far_n[e] + 1u, chunk = (uint64_t)FX * FX_PER;
    for (uint64_t c = blockIdx.x; c * chunk < span; c += gridDim.x) {
      const int64_t c0 = nb + (int64_t)(c * chunk);
      if (__hip_atomic_load(&s.fext[e], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < c0) break;  // (uniform)
      int64_t cur[FX_PER];
#pragma unroll
      for (uint32_t r = 0; r < FX_PER; ++r) cur[r] = fld(sn + fslot(c0 + (int64_t)(r * FX + threadIdx.x), mask));
#pragma unroll
      for (uint32_t r = 0; r < FX_PER; ++r) {
        const int64_t v = c0 + (int64_t)(r * FX + threadIdx.x);
        if (cur[r] == FEMPTY || (cur[r] != v && fset_find(sn, mask, v) == NONE)) {
          atomicMin(reinterpret_cast<long long*>(&s.fext[e]), (long long)v);
          break;
        }
      }
    }
  }
}
// the window re-anchored at the new all_ackable_before: bits from dbits (the state pass's window
// at lo), dbits' words read only (k_fx_pull clears them)
__global__ __launch_bounds__(FX) void k_fx_shift(State s) {
  const uint32_t nd = (uint32_t)s.ctr[C_FDEF];
  for (uint64_t k = (uint64_t)blockIdx.x * FX + threadIdx.x; k < (uint64_t)nd * WW; k += (uint64_t)gridDim.x * FX) {
    const uint32_t e = s.fdl[k / WW], w = (uint32_t)(k % WW);
    const int64_t lo = s.lo[e], nb = s.base[e], mn = s.far_min[e];
    const int64_t fnb = (s.far_cap[e] && nb >= lo + (int64_t)W && nb >= mn) ? s.fext[e] : nb;
    const uint64_t shift = (uint64_t)((fnb & ~(int64_t)31) - lo) >> 5;
    s.bits[(uint64_t)e * WW + w] = (w + shift < WW) ? s.dbits[(uint64_t)e * WW + w + shift] : 0u;
  }
}
__global__ __launch_bounds__(FX) void k_fx_pull(State s) {
  __shared__ uint32_t s_keep;
  __shared__ unsigned long long s_min;
  const uint32_t nd = (uint32_t)s.ctr[C_FDEF];
  for (uint64_t k = (uint64_t)blockIdx.x * FX + threadIdx.x; k < (uint64_t)nd * WW; k += (uint64_t)gridDim.x * FX)
    s.dbits[(uint64_t)s.fdl[k / WW] * WW + k % WW] = 0u;  // (k_fx_shift has read them)
  for (uint32_t i = 0; i < nd; ++i) {
    const uint32_t e = s.fdl[i];
    const int64_t lo = s.lo[e], nb = s.base[e], mn = s.far_min[e];
    const uint32_t cap = s.far_cap[e];
    const int64_t fnb = (cap && nb >= lo + (int64_t)W && nb >= mn) ? s.fext[e] : nb;
    const int64_t nlo = fnb & ~(int64_t)31, hi = nlo + (int64_t)W;
    if (cap == 0 || mn >= hi) continue;  // (far_pull's test)
    if (threadIdx.x == 0) { s_keep = 0; s_min = ~0ull; }
    __syncthreads();
    const int64_t* sn = s.fsn + s.far_off[e];
    uint32_t* bits = s.bits + (uint64_t)e * WW;
    uint32_t keep = 0;
    int64_t kmin = INT64_MAX;
    for (uint64_t j = (uint64_t)blockIdx.x * FX + threadIdx.x; j < cap; j += (uint64_t)gridDim.x * FX) {
      const int64_t v = fld(sn + j);
      if (v == FEMPTY || v < nlo) continue;
      if (v >= hi) {
        ++keep;
        if (v < kmin) kmin = v;
      } else {
        atomicOr(bits + ((uint64_t)(v - nlo) >> 5), 1u << ((uint64_t)(v - nlo) & 31u));
      }
    }
    if (keep) atomicAdd(&s_keep, keep);
    if (kmin != INT64_MAX) atomicMin(&s_min, (unsigned long long)kmin);
    __syncthreads();
    if (threadIdx.x == 0 && s_keep) {
      atomicAdd(&s.fkeep[e], s_keep);
      atomicMin(reinterpret_cast<long long*>(&s.fkmin[e]), (long long)s_min);
    }
    __syncthreads();
  }
}
__global__ __launch_bounds__(FX) void k_fx_fin(State s, int64_t* ack_out) {
  const uint32_t nd = (uint32_t)s.ctr[C_FDEF];
  for (uint32_t i = threadIdx.x; i < nd; i += FX) {
    const uint32_t e = s.fdl[i];
    const int64_t lo = s.lo[e], nb = s.base[e], mn = s.far_min[e];
    const uint32_t cap = s.far_cap[e];
    const int64_t fnb = (cap && nb >= lo + (int64_t)W && nb >= mn) ? s.fext[e] : nb;
    const int64_t nlo = fnb & ~(int64_t)31, hi = nlo + (int64_t)W;
    if (cap && mn < hi) {  // far_pull ran: the set's least SN past the window, or the set emptied
      if (s.fkeep[e] == 0) {
        s.far_off[e] = 0; s.far_cap[e] = 0; s.far_n[e] = 0; s.far_min[e] = INT64_MAX;
      } else {
        s.far_min[e] = s.fkmin[e];
      }
    }
    s.fkeep[e] = 0;
    s.fkmin[e] = INT64_MAX;
    s.base[e] = fnb;
    s.lo[e] = nlo;
    if (ack_out) ack_out[e] = fnb;
  }
  __syncthreads();
  if (threadIdx.x == 0) s.ctr[C_FDEF] = 0;  // (a later state pass of this batch's counters may list again)
}

// ---- 6 merge ----
// Batches without GAPs whose proxies' windows are few against their events (T:
// 16 proxies x 2^17 positions for 1M samples): the batch's sample coverage is
// exactly the window positions whose first-cover key (k_marks_d) carries this
// batch's epoch, so a pass over the keys ORs it into the change sets as whole
// words, one ballot per 64 positions and no atomics (each word has one owner),
// instead of k_merge's per-sample wave sort and atomics (T: 48 us).
__global__ __launch_bounds__(IT) void k_fcmerge(uint32_t n_proxies, State s, uint32_t epoch) {
  const uint64_t total = (uint64_t)n_proxies * W;  // a multiple of IT: every lane of a wave takes part
  const uint32_t tag = 0xffffffffu - epoch, lane = threadIdx.x & 63u;
  for (uint64_t p = (uint64_t)blockIdx.x * IT + threadIdx.x; p < total; p += (uint64_t)gridDim.x * IT) {
    const uint64_t m = __ballot((uint32_t)(s.fc[p] >> 32) == tag);
    const uint32_t half = lane == 0 ? (uint32_t)m : (uint32_t)(m >> 32);
    if ((lane == 0 || lane == 32) && half) s.bits[p >> 5] |= half;  // window offset p - e * W -> word e * WW + off / 32
  }
}
static_assert(W % IT == 0, "k_fcmerge: whole waves per proxy window");

__global__ __launch_bounds__(IT) void k_merge(const rtps_record* recs, const uint8_t* arena, const uint64_t* dgram_off,
                                              uint64_t n, Scratch x, State s, bool gaps) {
  for (uint64_t i0 = (uint64_t)blockIdx.x * IT; i0 < n; i0 += (uint64_t)gridDim.x * IT) {  // wave-uniform trip count
    const uint64_t i = i0 + threadIdx.x;
    uint8_t ev = i < n ? x.evt[i] : EV_NONE;
    const uint32_t e0 = ev != EV_NONE ? x.ent[i] : NONE;
    if (e0 == NONE) ev = EV_NONE;  // free samples touch no proxy
    const uint32_t e = (ev == EV_SAMPLE || ev == EV_GAP) ? e0 : 0u;
    const int64_t lo = (ev == EV_SAMPLE || ev == EV_GAP) ? s.lo[e] : 0;
    uint32_t* bits = s.bits + (uint64_t)e * WW;
    bool act = false;
    uint32_t* word = s.bits;
    uint32_t bit = 0;
    if (ev == EV_SAMPLE) {
      const int64_t v = x.esn[i];
      if (v >= lo && v < lo + (int64_t)W) {
        const uint64_t w = (uint64_t)(v - lo) >> 5;
        act = true;
        word = bits + w;
        bit = 1u << ((v - lo) & 31);
        if (gaps) s.dbits[(uint64_t)e * WW + w] = 0u;  // every mark of the batch is done (k_marks_g read them)
      }
    } else if (ev == EV_GAP) {
      gap_words(recs[x.erec[i]], arena, dgram_off, lo, [&](uint64_t w, uint32_t m) { atomicOr(bits + w, m); });
    }
    wave_or(s.bits, word, bit, act);
  }
}

// ---- 7 state: one workgroup per proxy ----
// The proxy's window is read once into LDS (16 words per thread, all loads in flight), the
// first uncovered sequence number at or above the threshold found with one block-wide
// minimum, and the window re-anchored at the new ack_base from the LDS copy.
// fcm: the batch's coverage is in dbits (k_decide_t<2>): OR it into the window, clear it
__device__ __forceinline__ void state_proxy(uint32_t e, const Scratch& x, const State& s, bool reliable,
                                            int64_t* ack_out, uint32_t* sh, uint32_t& s_first, FarSh& f,
                                            bool fcm = false) {
  const uint32_t tid = threadIdx.x;
  if (tid == 0) ftab_load(s, e, f.t);
  const int64_t lo = s.lo[e];
  int64_t thr = s.base[e];
  int32_t hbc = s.hbc[e];
  const uint32_t b0 = s.seg_b[e], b1 = s.seg_e[e];
  if (reliable && b1 > b0) {
    const int64_t f = x.hpre[b1 - 1u];
    if (f > thr) thr = f;
    const int32_t c = x.hexcl[b1 - 1u] > x.hcnt[b1 - 1u] ? x.hexcl[b1 - 1u] : x.hcnt[b1 - 1u];
    if (c > hbc) hbc = c;
  }
  uint32_t* bits = s.bits + (uint64_t)e * WW;
  const u32x4* b4 = reinterpret_cast<const u32x4*>(bits);
  u32x4* sh4 = reinterpret_cast<u32x4*>(sh);
  if (fcm) {
    u32x4* d4 = reinterpret_cast<u32x4*>(s.dbits + (uint64_t)e * WW);
    for (uint32_t q = tid; q < WW / 4; q += IT) {
      sh4[q] = b4[q] | d4[q];
      d4[q] = u32x4{0u, 0u, 0u, 0u};
    }
  } else {
    for (uint32_t q = tid; q < WW / 4; q += IT) sh4[q] = b4[q];
  }
  if (tid == 0) s_first = NONE;
  __syncthreads();
  // advance_ack_base: the first sequence number >= thr outside the change set
  int64_t nb = thr;
  if (thr < lo + (int64_t)W) {
    const uint32_t off0 = (uint32_t)(thr - lo), w0 = off0 >> 5;
    for (uint32_t w = w0 + tid; w < WW; w += IT) {  // a thread's words ascend: its first hit is its least
      uint32_t word = sh[w];
      if (w == w0) word |= (1u << (off0 & 31u)) - 1u;  // below thr: covered
      if (word != 0xffffffffu) {
        atomicMin(&s_first, w * 32u + (uint32_t)__builtin_ctz(~word));
        break;
      }
    }
    __syncthreads();
    nb = lo + (int64_t)(s_first != NONE ? s_first : W);
  }
  if (s.fdefer && f.t.cap > FT_BIG && far_touch(f.t, lo, nb)) {  // (uniform: f is shared)
    far_defer(s, e, f.t, sh, nb, hbc, IT);  // the k_fx_* launches finish it
    return;
  }
  nb = far_extend(s, f, lo, nb, IT);
  // re-anchor the window at the new ack_base (bits below it are no longer needed)
  const int64_t nlo = nb & ~(int64_t)31;
  if (nlo != lo) {
    const uint64_t shift = (uint64_t)(nlo - lo) >> 5;
    for (uint32_t w = tid; w < WW; w += IT) bits[w] = (w + shift < WW) ? sh[w + shift] : 0u;
  }
  far_pull(s, f, bits, nlo, IT);
  if (tid == 0) {
    ftab_store(s, e, f.t);
    s.base[e] = nb;
    s.lo[e] = nlo;
    s.hbc[e] = hbc;
    if (ack_out) ack_out[e] = nb;
  }
}
// (workgroup 0 also reports the window-overflow count: every decision is made by now)
__global__ __launch_bounds__(IT) void k_state(uint32_t n_entries, Scratch x, State s, bool reliable, int64_t* ack_out,
                                              uint64_t* ovf_out) {
  __shared__ __attribute__((aligned(16))) uint32_t sh[WW];
  __shared__ uint32_t s_first;
  __shared__ FarSh f;
  const uint32_t e = blockIdx.x;
  if (e >= n_entries) return;
  state_proxy(e, x, s, reliable, ack_out, sh, s_first, f);
  if (threadIdx.x == 0 && e == 0 && ovf_out) *ovf_out = s.ctr[C_OVF];
}
// Global identity path, last launch: workgroups [0, ntiles) write the deliveries (k_dwrite;
// the last one also the overflow count), the next n_entries one proxy's state each.
__global__ __launch_bounds__(IT) void k_dstate(const uint8_t* flag, uint64_t n, const uint32_t* tcnt, uint32_t ntiles,
                                               Scratch x, uint64_t max_out, rtps_delivery* out, uint64_t* n_out,
                                               const uint64_t* ctr, uint64_t* ovf_out, uint32_t n_entries, State s,
                                               bool reliable, int64_t* ack_out, bool fcm, bool guarded) {
  __shared__ uint64_t s_w[IT / 64];
  __shared__ uint32_t s_c[IT / 64];
  __shared__ __attribute__((aligned(16))) uint32_t sh[WW];
  __shared__ uint32_t s_first;
  __shared__ FarSh f;
  if (guarded) {  // queued before the host had the counts: only k_signal's plain batches
    const uint64_t mode = ctr[C_MODE];
    if (mode == 0) return;
    fcm = mode == 2;
  }
  if (blockIdx.x < ntiles) {
    dwrite_tile(blockIdx.x, flag, n, tcnt, ntiles, x, true, max_out, out, n_out, ctr, ovf_out, nullptr, nullptr, s_w,
                s_c);
  } else if (blockIdx.x - ntiles < n_entries) {
    state_proxy(blockIdx.x - ntiles, x, s, reliable, ack_out, sh, s_first, f, fcm);
  }
}

// ---- per-proxy path (batches over many proxies) ----
// Global atomics execute at the memory side (about 20 G scattered atomics/s for
// the whole chip), so marks / merge over a few million events of hundreds of
// writers cost ~130 us each.  When the events spread over many proxies, they are
// instead grouped by proxy in event order (identity batches: the proxy bucketing
// in classify; otherwise a stable radix sort) and ONE workgroup per proxy replays its events
// in order, 256 at a time, against the proxy's change-set window held in LDS:
// HEARTBEAT acceptance and thresholds by block scans, a sample's coverage by the
// window (earlier chunks and carried state), an LDS hash (earlier samples of the
// chunk) and the chunk's earlier GAPs; then the chunk's coverage is ORed into the
// window.  The same decisions as marks / decide / merge / state, with no global
// atomics; a proxy with very many events would serialise on one workgroup, so the
// host picks this path only when the mean load per proxy is small.
#ifdef RTPS_PROXY_STAMPS  // tuning builds: per-phase time sums of k_proxy, per proxy
constexpr uint32_t PST_N = 8;
#define PST_DECL uint64_t pst_t = __builtin_amdgcn_s_memrealtime(), pst_t0 = pst_t, pst_acc[PST_N] = {0, 0, 0, 0, 0, 0, 0, 0}
#define PST(k) do { const uint64_t t_ = __builtin_amdgcn_s_memrealtime(); pst_acc[k] += t_ - pst_t; pst_t = t_; } while (0)
#define PST_FLUSH(e) do { if (threadIdx.x == 0) { for (uint32_t k_ = 0; k_ < PST_N; ++k_) g_proxy_stamps[(e) * PST_N + k_] = pst_acc[k_]; \
  g_proxy_stamps[16384u * 8u + 2u * (e)] = pst_t0; g_proxy_stamps[16384u * 8u + 2u * (e) + 1u] = pst_t; } } while (0)
#else
#define PST_DECL do {} while (0)
#define PST(k) do {} while (0)
#define PST_FLUSH(e) do {} while (0)
#endif
#ifndef RTPS_PROXY_PT
#define RTPS_PROXY_PT 512
#endif
constexpr uint32_t PT = RTPS_PROXY_PT;   // threads of the per-proxy workgroup (one per CU)
#ifndef RTPS_PROXY_PPT
#define RTPS_PROXY_PPT 4
#endif
constexpr uint32_t PPT = RTPS_PROXY_PPT;  // consecutive events per thread
constexpr uint32_t PCH = PT * PPT;       // events per chunk
constexpr uint32_t PH = 2 * PCH;         // chunk hash slots (>= 2 x events per chunk)
constexpr uint32_t PH_BITS = PH == 2048 ? 11 : PH == 4096 ? 12 : PH == 8192 ? 13 : 0;
static_assert((1u << PH_BITS) == PH, "hash width");
constexpr uint32_t PWAVES = PT / 64;

// selection flags: events that touch proxy state
__global__ __launch_bounds__(IT) void k_pflag(uint64_t n, Scratch x) {
  uint8_t* flag = reinterpret_cast<uint8_t*>(x.hkey);
  for (uint64_t k = (uint64_t)blockIdx.x * IT + threadIdx.x; k < n; k += (uint64_t)gridDim.x * IT)
    flag[k] = (x.evt[k] != EV_NONE && x.ent[k] != NONE) ? 1 : 0;
}
// the selected events (x.hval[0, n), ascending) -> sort keys (proxy) and PEv values
__global__ __launch_bounds__(IT) void k_pack(const rtps_record* recs, const uint8_t* arena, const uint64_t* dgram_off,
                                             uint64_t n, Scratch x, PEv* out) {
  for (uint64_t i = (uint64_t)blockIdx.x * IT + threadIdx.x; i < n; i += (uint64_t)gridDim.x * IT) {
    const uint32_t k = x.hval[i];
    const uint8_t ev = x.evt[k];
    PEv P;
    P.sn = x.esn[k];
    P.a = 0;
    P.bw = 0;
    P.k = k;
    P.m = ev | ((x.emeta[k] & EVF_DUP_OK) ? PM_DUP : 0u);
    if (ev == EV_HB) {
      P.a = recs[x.erec[k]].u.hb.count;
    } else if (ev == EV_GAP) {
      const rtps_record& r = recs[x.erec[k]];
      P.a = r.u.gap.list_base;
      const bool le = (r.flags & 1u) != 0u;
      P.m |= (le ? PM_LE : 0u) | (r.u.gap.num_bits << 8);
      P.bw = dgram_off[r.dgram_idx] + r.u.gap.bitmap_off;
      if (r.u.gap.num_bits <= 64u) {  // the bitmap itself: the proxy's pass reads no arena
        const uint8_t* p = arena + P.bw;
        const uint32_t w0 = r.u.gap.num_bits ? rd32(p, le) : 0u, w1 = r.u.gap.num_bits > 32u ? rd32(p + 4, le) : 0u;
        P.bw = (uint64_t)w0 | ((uint64_t)w1 << 32);
        P.m |= PM_INL;
      }
    }
    x.hkey[i] = x.ent[k];
    x.sval[i] = (uint32_t)i;  // sort value: the packed event's position
    out[i] = P;
  }
}
// sorted keys -> each proxy's segment [seg_b, seg_e) (seg_* zeroed before; keys >= n_proxies: none)
__global__ __launch_bounds__(IT) void k_pseg(uint64_t n, uint32_t n_proxies, Scratch x, State s) {
  for (uint64_t q = (uint64_t)blockIdx.x * IT + threadIdx.x; q < n; q += (uint64_t)gridDim.x * IT) {
    const uint32_t key = x.skey[q];
    if (key >= n_proxies) continue;
    if (q == 0 || x.skey[q - 1] != key) s.seg_b[key] = (uint32_t)q;
    if (q + 1 == n || x.skey[q + 1] != key) s.seg_e[key] = (uint32_t)q + 1u;
  }
}
// accept[] for the events no proxy decides: samples without a proxy (writer kind
// not user-defined, reader.rs:734-739) are accepted; everything else starts at 0
__global__ __launch_bounds__(IT) void k_decide_free(uint64_t n, uint64_t cap, Scratch x, uint8_t* acc_out) {
  for (uint64_t i = (uint64_t)blockIdx.x * IT + threadIdx.x; i < cap; i += (uint64_t)gridDim.x * IT)
    acc_out[i] = (i < n && x.evt[i] == EV_SAMPLE && x.ent[i] == NONE) ? 1 : 0;
}

// block-wide EXCLUSIVE scan of max (int64) over threads; `carry` joins from the left;
// *total = the block's max (with the carry)
__device__ __forceinline__ int64_t block_max_excl(int64_t v, int64_t carry, int64_t* s_w, int64_t& total) {
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  int64_t inc = v;
#pragma unroll
  for (uint32_t d = 1; d < 64; d <<= 1) {
    const int64_t y = __shfl_up(inc, d, 64);
    if (lane >= d && y > inc) inc = y;
  }
  int64_t ex = __shfl_up(inc, 1, 64);
  if (lane == 0) ex = INT64_MIN;
  if (lane == 63) s_w[wave] = inc;
  __syncthreads();
  int64_t pre = carry;
  total = carry;
  for (uint32_t w = 0; w < PWAVES; ++w) {
    if (w < wave) pre = s_w[w] > pre ? s_w[w] : pre;
    total = s_w[w] > total ? s_w[w] : total;
  }
  __syncthreads();
  return ex > pre ? ex : pre;
}
__device__ __forceinline__ uint32_t ph_hash(uint32_t off) { return (off * 0x9e3779b1u) >> (32 - PH_BITS); }
__device__ __forceinline__ uint32_t ph_find(const uint32_t* h_key, uint32_t off) {
  for (uint32_t h = ph_hash(off);; h = (h + 1) & (PH - 1)) {
    const uint32_t k = h_key[h];
    if (k == off) return h;
    if (k == NONE) return NONE;
  }
}

// the proxy bucketing's tables (k_classify<.., true>): per (classify workgroup, proxy)
// event counts and first positions in the workgroup's region of pev, nb workgroups
struct BkIn {
  const uint32_t* cl;  // FastOut::bk_cl
  uint32_t nb;
};
// block-wide EXCLUSIVE sum over the PT threads; *total = the block's sum
__device__ __forceinline__ uint32_t block_sum_excl(uint32_t v, uint32_t* s_w, uint32_t& total) {
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  uint32_t inc = v;
#pragma unroll
  for (uint32_t d = 1; d < 64; d <<= 1) {
    const uint32_t y = (uint32_t)__shfl_up((int)inc, d, 64);
    if (lane >= d) inc += y;
  }
  if (lane == 63) s_w[wave] = inc;
  __syncthreads();
  uint32_t pre = 0;
  total = 0;
  for (uint32_t w = 0; w < PWAVES; ++w) {
    if (w < wave) pre += s_w[w];
    total += s_w[w];
  }
  __syncthreads();
  return pre + inc - v;
}

// a GAP of the chunk as the GAP phases read it from LDS (the event's own registers are its thread's)
struct GapE {
  int64_t v, a;  // gapStart, gapList.base
  uint64_t bw;   // inline bitmap words or the bitmap's arena offset
  uint32_t m, q; // PEv.m, the event's position
};
constexpr uint32_t GCAP = 512;  // GAPs per chunk spread one per thread; the rest stay with their threads

// One workgroup per proxy: its events in slot order replayed in chunks of PCH
// against the proxy's change-set window in LDS.  The events: BK = false, sorted by
// proxy (`order` holds positions in the packed events `pev`, the proxy's segment
// [seg_b, seg_e)); BK = true, the proxy's pieces of every classify workgroup's
// region of pev, in workgroup order (the bucketing's tables, scanned into LDS).
template <bool BK>
__global__ __launch_bounds__(PT) void k_proxy(const uint8_t* arena, const PEv* pev, const uint32_t* order,
                                              uint32_t n_proxies, State s, uint8_t* acc_out, int64_t* ack_out,
                                              BkIn bk) {
  __shared__ uint32_t sb[WW];                           // the change set window [lo, lo + W)
  __shared__ __attribute__((aligned(16))) uint32_t pres[WW];  // window offsets of the chunk's samples
  // window offset -> first sample / GAP position (h_key / h_min: the far replay's hash and keys at the end)
  __shared__ __attribute__((aligned(16))) uint32_t h_key[PH], h_min[PH], h_gap[PH];
  __shared__ int64_t s_w[PWAVES];
  __shared__ uint32_t s_w32[PWAVES];
  __shared__ uint32_t s_pre[BK ? BK_MAX + 1 : 1];  // BK: the proxy's events before workgroup b's piece
  __shared__ uint32_t s_base[BK ? BK_MAX : 1];     // BK: pev index of the proxy's event q in piece b = s_base[b] + q
  __shared__ uint32_t s_idx[BK ? BK_IDX : 1];      // BK: the piece holding event 4m (when the proxy has <= 4 BK_IDX)
  __shared__ uint32_t s_first, s_split;
  __shared__ GapE s_gap[GCAP];  // the chunk's GAPs (the first GCAP), one per thread in the GAP phases
  __shared__ uint32_t s_ngap;
  __shared__ FarSh fsh;                // the proxy's far set
  __shared__ unsigned long long s_fp;  // SNs the chunk's far items cover
  __shared__ uint32_t s_anyfar;        // some thread holds a far item of the chunk
  const uint32_t e = blockIdx.x, tid = threadIdx.x;
  if (e >= n_proxies) return;
  PST_DECL;  // (setup: the window, the hash and the piece tables)
  if (tid == 0) {
    s_ngap = 0u;
    s_fp = 0ull;
    s_anyfar = 0u;
    ftab_load(s, e, fsh.t);
  }
  const int64_t lo = s.lo[e], base = s.base[e];
  uint32_t* gbits = s.bits + (uint64_t)e * WW;
  for (uint32_t w = tid; w < WW; w += PT) { sb[w] = gbits[w]; pres[w] = 0u; }
  for (uint32_t h = tid; h < PH; h += PT) { h_key[h] = NONE; h_min[h] = NONE; h_gap[h] = NONE; }
  uint32_t qb = 0, qe = 0;
  bool idx = false;
  if (BK) {
    // thread t: pieces [t K, t K + K), every table load issued before the one block scan
    constexpr uint32_t K = BK_MAX / PT;
    const uint32_t kp = (bk.nb + PT - 1) / PT;
    uint32_t c[K], l[K], sum = 0;
#pragma unroll
    for (uint32_t k = 0; k < K; ++k) {
      const uint32_t b = tid * kp + k;
      const uint32_t cl = (k < kp && b < bk.nb) ? bk.cl[(uint64_t)b * n_proxies + e] : 0u;
      c[k] = cl & 0xffffu;
      l[k] = cl >> 16;
      sum += c[k];
    }
    uint32_t ex = block_sum_excl(sum, s_w32, qe);
#pragma unroll
    for (uint32_t k = 0; k < K; ++k) {
      const uint32_t b = tid * kp + k;
      if (k < kp && b < bk.nb) {
        s_pre[b] = ex;
        s_base[b] = b * CHR + l[k] - ex;
      }
      ex += c[k];
    }
    if (tid == 0) s_pre[bk.nb] = qe;
    // the sampled index: each piece names itself at the multiples of PPT it holds
    idx = qe <= PPT * BK_IDX;
    if (idx) {
      __syncthreads();
      for (uint32_t b = tid; b < bk.nb; b += PT)
        for (uint32_t m = (s_pre[b] + PPT - 1) / PPT; m * PPT < s_pre[b + 1]; ++m) s_idx[m] = b;
    }
  } else {
    qb = s.seg_b[e];
    qe = s.seg_e[e];
  }
  int64_t run_cnt = s.hbc[e], run_thr = base;  // max HEARTBEAT count so far; max accepted firstSN (>= base)
  int64_t abc = base;  // a lower bound of all_ackable_before at the chunk's start (exact where a far GAP asked)
  uint64_t n_ovf = 0;
  // the first sequence number >= from that the window leaves uncovered (lo + W: none; from < lo + W)
  auto first_open = [&](int64_t from) -> int64_t {
    const uint32_t off0 = (uint32_t)(from - lo);
    if (tid == 0) s_first = NONE;
    __syncthreads();
    for (uint32_t w0 = (off0 >> 5); w0 < WW; w0 += PT) {  // rounds of PT words, stop at the first hit
      const uint32_t w = w0 + tid;
      uint32_t word = w < WW ? sb[w] : 0xffffffffu;
      if (w == (off0 >> 5)) word |= (1u << (off0 & 31u)) - 1u;
      const uint64_t open = __ballot(word != 0xffffffffu);  // lowest lane first: one LDS atomic per wave
      if (open && (tid & 63u) == (uint32_t)__builtin_ctzll(open))
        atomicMin(&s_first, w * 32u + (uint32_t)__builtin_ctz(~word));
      __syncthreads();
      if (s_first != NONE) break;
    }
    const int64_t r = lo + (int64_t)(s_first != NONE ? s_first : W);
    __syncthreads();  // (s_first read by every thread before it is reused)
    return r;
  };
  __syncthreads();
  PST(0);
  // the chunk at c0's events of this thread (BK: found through the piece tables)
  auto load_chunk = [&](uint32_t c0, PEv (&dst)[PPT]) {
    uint32_t pb = 0;  // BK: the piece of the thread's first event (the largest b with s_pre[b] <= q)
    if (BK && c0 + tid * PPT < qe) {
      const uint32_t q = c0 + tid * PPT;  // a multiple of PPT
      if (idx) {
        pb = s_idx[q / PPT];
      } else {
        for (uint32_t hi = bk.nb; hi - pb > 1u;) {
          const uint32_t mid = (pb + hi) >> 1;
          if (s_pre[mid] <= q) pb = mid; else hi = mid;
        }
      }
    }
#pragma unroll
    for (uint32_t j = 0; j < PPT; ++j) {
      const uint32_t q = c0 + tid * PPT + j;
      dst[j] = PEv{0, 0, 0, 0, 0};
      if (BK) {
        if (q < qe) {
          while (s_pre[pb + 1u] <= q) ++pb;  // (s_pre[nb] = the proxy's events > q)
          dst[j] = pev[s_base[pb] + q];
        }
      } else if (q < qe) {
        dst[j] = pev[order[q]];
      }
    }
  };
  // the events are loaded one chunk ahead: the next chunk's loads are in flight while
  // this chunk is decided (its barriers are LDS-only: plain loads survive them)
  PEv nx[PPT];
  if (qb < qe) load_chunk(qb, nx);
  for (uint32_t q0 = qb, q1; q0 < qe; q0 = q1) {
    uint32_t m[PPT], slot[PPT], kk[PPT];
    int64_t v[PPT], a[PPT];
    uint64_t bwj[PPT];
    int64_t cmax = INT64_MIN;
#pragma unroll
    for (uint32_t j = 0; j < PPT; ++j) {
      m[j] = nx[j].m;
      v[j] = nx[j].sn;
      a[j] = nx[j].a;
      bwj[j] = nx[j].bw;
      kk[j] = nx[j].k;
    }
    q1 = q0 + PCH < qe ? q0 + PCH : qe;
    if (q0 + PCH < qe) load_chunk(q0 + PCH, nx);
    // A GAP reaching far past the window (gap_far_big) that the chunk-start bound abc does not
    // show at or below all_ackable_before may still be (the chunk's earlier events can move it):
    // abc is made exact for the window, and the chunk ends before the first such GAP after its
    // start, so that the next chunk starts at that GAP with the exact running value
    {
      const int64_t lim0 = lo + (int64_t)W;
      bool big = false;
#pragma unroll
      for (uint32_t j = 0; j < PPT; ++j) big |= (m[j] & 3u) == EV_GAP && v[j] > abc && gap_far_big(v[j], a[j], lim0);
      if (__syncthreads_or(big)) {
        const int64_t from = run_thr > abc ? run_thr : abc;
        abc = from < lim0 ? first_open(from) : from;
        if (tid == 0) s_split = NONE;
        __syncthreads();
#pragma unroll
        for (uint32_t j = 0; j < PPT; ++j) {
          const uint32_t q = q0 + tid * PPT + j;
          if (q > q0 && (m[j] & 3u) == EV_GAP && v[j] > abc && gap_far_big(v[j], a[j], lim0)) atomicMin(&s_split, q);
        }
        __syncthreads();
        if (s_split != NONE) {
          q1 = s_split;
#pragma unroll
          for (uint32_t j = 0; j < PPT; ++j)
            if (q0 + tid * PPT + j >= q1) m[j] = EV_NONE;  // (the next chunk, which starts at q1, takes them)
        }
        __syncthreads();  // (s_split read by every thread)
      }
    }
#pragma unroll
    for (uint32_t j = 0; j < PPT; ++j)
      if ((m[j] & 3u) == EV_HB && a[j] > cmax) cmax = a[j];
    // HEARTBEATs: accepted iff count > every earlier count and the state's (reader.rs:902-905);
    // an accepted one covers [0, firstSN) (irrelevant_changes_up_to)
    PST(1);
    int64_t cnt_total;
    int64_t c_ex = run_cnt;
    cnt_total = run_cnt;
    c_ex = block_max_excl(cmax, run_cnt, s_w, cnt_total);
    int64_t fmax = INT64_MIN, f[PPT];
#pragma unroll
    for (uint32_t j = 0; j < PPT; ++j) {
      const bool hb = (m[j] & 3u) == EV_HB;
      f[j] = (hb && a[j] > c_ex) ? v[j] : INT64_MIN;
      if (hb && a[j] > c_ex) c_ex = a[j];
      // a GAP whose range starts at or below all_ackable_before (abc bounds it from below: it only
      // grows) moves it to gapList.base (irrelevant_changes_range, rtps_writer_proxy.rs:241-292): a
      // threshold like an accepted HEARTBEAT's, with no SN to record past the window
      if ((m[j] & 3u) == EV_GAP && v[j] <= abc && v[j] <= a[j] && a[j] > f[j]) f[j] = a[j];
      if (f[j] > fmax) fmax = f[j];
    }
    int64_t thr_total;
    int64_t thr = run_thr;
    thr_total = run_thr;
    thr = block_max_excl(fmax, run_thr, s_w, thr_total);
    run_cnt = cnt_total;
    run_thr = thr_total;
    PST(2);
    // samples in the window -> the chunk hash (first position per sequence number)
#pragma unroll
    for (uint32_t j = 0; j < PPT; ++j) {
      slot[j] = NONE;
      const int64_t vj = v[j];
      if ((m[j] & 3u) == EV_SAMPLE && vj >= lo && vj < lo + (int64_t)W) {
        const uint32_t off = (uint32_t)(vj - lo);
        uint32_t h = ph_hash(off);
        for (;;) {
          const uint32_t prev = atomicCAS(&h_key[h], NONE, off);
          if (prev == NONE || prev == off) break;
          h = (h + 1) & (PH - 1);
        }
        slot[j] = h;
        atomicMin(&h_min[h], q0 + tid * PPT + j);
        atomicOr(&pres[off >> 5], 1u << (off & 31u));
      }
    }
    // the thread's GAPs into the chunk's GAP list: their coverage walks (a dependent chain of
    // LDS probes each) then run one GAP per thread instead of PPT in a row per thread
    uint32_t listed = 0;
    {
      uint32_t ngj = 0;
#pragma unroll
      for (uint32_t j = 0; j < PPT; ++j) ngj += (m[j] & 3u) == EV_GAP;
      if (ngj) {
        uint32_t g = atomicAdd(&s_ngap, ngj);
#pragma unroll
        for (uint32_t j = 0; j < PPT; ++j) {
          if ((m[j] & 3u) != EV_GAP) continue;
          if (g < GCAP) {
            s_gap[g] = GapE{v[j], a[j], bwj[j], m[j], q0 + tid * PPT + j};
            listed |= 1u << j;
          }
          ++g;
        }
      }
    }
    __syncthreads();
    PST(3);
    const uint32_t ngap = s_ngap < GCAP ? s_ngap : GCAP;
    // GAPs: their first covering position for the chunk's sample sequence numbers (only
    // window words holding a sample of the chunk are looked up: the presence bitmap)
    auto gap_mark = [&](int64_t gv, int64_t ga, uint64_t bw, uint32_t gm, uint32_t q) {
      auto mark = [&](uint64_t w, uint32_t bits) {
        bits &= pres[w];
        while (bits) {
          const uint32_t b = (uint32_t)__builtin_ctz(bits);
          bits &= bits - 1u;
          const uint32_t h = ph_find(h_key, (uint32_t)(w * 32u + b));
          if (h != NONE) atomicMin(&h_gap[h], q);
        }
      };
      if (gm & PM_INL)
        gap_cover_w(gv, ga, gm >> 8, [&](uint32_t w) { return (uint32_t)(bw >> (32u * w)); }, lo, mark);
      else
        gap_cover(gv, ga, arena + bw, gm >> 8, (gm & PM_LE) != 0u, lo, mark);
    };
    for (uint32_t g = tid; g < ngap; g += PT) {
      const GapE ge = s_gap[g];
      gap_mark(ge.v, ge.a, ge.bw, ge.m, ge.q);
    }
#pragma unroll
    for (uint32_t j = 0; j < PPT; ++j)
      if ((m[j] & 3u) == EV_GAP && !((listed >> j) & 1u)) gap_mark(v[j], a[j], bwj[j], m[j], q0 + tid * PPT + j);
    __syncthreads();
    PST(4);
    if (tid == 0) s_ngap = 0u;  // (every thread read it before the barrier above; the next list is built after barriers)
    // decide (should_ignore_change: rtps_writer_proxy.rs:202-230, reader.rs:693-758)
    int64_t t_run = thr;
    const int64_t lim = lo + (int64_t)W;
    uint32_t fkind = 0;  // far items (rare) of the thread's events: kind << 2 j, into the far set below
    auto far = [&](uint32_t j, uint32_t kind) { fkind |= kind << (2u * j); };
    // a far item's first SN: a threshold GAP's range is the threshold's (above), only its list is recorded
    auto fsn0 = [&](uint32_t kind, int64_t gv, int64_t ga) { return (kind == FI_GAP && gv <= abc) ? ga + 1 : gv; };
#pragma unroll
    for (uint32_t j = 0; j < PPT; ++j) {
      if (f[j] > t_run) t_run = f[j];
      if ((m[j] & 3u) == EV_GAP && a[j] + (int64_t)(m[j] >> 8) > lim) far(j, FI_GAP);
      if ((m[j] & 3u) != EV_SAMPLE) continue;
      const uint32_t q = q0 + tid * PPT + j;
      uint8_t acc = 0;
      const int64_t vj = v[j];
      if (m[j] & PM_DUP) {
        acc = 1;  // the participant reader's duplicates (reader.rs:712-722)
        if (vj >= lim) far(j, FI_DUP);
      } else if (vj >= 1 && vj >= t_run) {
        if (slot[j] == NONE) {
          acc = 1;  // beyond the window (vj >= t_run >= lo): the far replay decides
          far(j, FI_SAMPLE);
        } else {
          const uint32_t off = (uint32_t)(vj - lo);
          acc = (((sb[off >> 5] >> (off & 31u)) & 1u) == 0u && h_min[slot[j]] == q && h_gap[slot[j]] > q) ? 1 : 0;
        }
      }
      acc_out[kk[j]] = acc;
    }
    if (__ballot(fkind != 0u) && (tid & 63u) == 0u) s_anyfar = 1u;  // (rare: one LDS store per wave)
    __syncthreads();
    if (s_anyfar) {
      // the chunk's far items: every SN they cover into the far set (the table grown first for
      // all of them), then their samples decided by first cover (see "far sequence numbers")
      uint64_t pc = 0;
#pragma unroll
      for (uint32_t j = 0; j < PPT; ++j) {
        const uint32_t kind = (fkind >> (2u * j)) & 3u;
        if (kind) pc += far_count(PEv{fsn0(kind, v[j], a[j]), a[j], bwj[j], m[j], kk[j]}, kind, lim, arena);
      }
      if (pc) atomicAdd(&s_fp, (unsigned long long)pc);
      uint32_t nfi = 0;
#pragma unroll
      for (uint32_t j = 0; j < PPT; ++j) nfi += ((fkind >> (2u * j)) & 3u) != 0u;
      if (nfi) atomicAdd(reinterpret_cast<unsigned long long*>(s.ctr + C_NFAR), (unsigned long long)nfi);
      __syncthreads();
      if (ftab_reserve(s, fsh, s_fp, PT)) {
        ftab_insert(s, fsh, [&](auto&& add) {
#pragma unroll
          for (uint32_t j = 0; j < PPT; ++j) {
            const uint32_t kind = (fkind >> (2u * j)) & 3u;
            if (kind)
              far_sns(PEv{fsn0(kind, v[j], a[j]), a[j], bwj[j], m[j], kk[j]}, kind, lim, arena,
                      [&](int64_t sn) { add(sn, fkey_of(s.epoch, kk[j])); });
          }
        });
        __threadfence();
        __syncthreads();
#pragma unroll
        for (uint32_t j = 0; j < PPT; ++j)
          if (((fkind >> (2u * j)) & 3u) == FI_SAMPLE && !ftab_first(s, fsh.t, v[j], fkey_of(s.epoch, kk[j])))
            acc_out[kk[j]] = 0;
      } else {
#pragma unroll
        for (uint32_t j = 0; j < PPT; ++j) n_ovf += ((fkind >> (2u * j)) & 3u) == FI_SAMPLE;  // the pool was out: unchecked
      }
      __syncthreads();
      if (tid == 0) {
        s_fp = 0ull;
        s_anyfar = 0u;
      }
    }
    PST(5);
    // merge the chunk's coverage into the window, clear the hash and the presence bits
    auto gap_or = [&](int64_t gv, int64_t ga, uint64_t bw, uint32_t gm) {
      auto orw = [&](uint64_t w, uint32_t bits) { atomicOr(&sb[w], bits); };
      if (gm & PM_INL)
        gap_cover_w(gv, ga, gm >> 8, [&](uint32_t w) { return (uint32_t)(bw >> (32u * w)); }, lo, orw);
      else
        gap_cover(gv, ga, arena + bw, gm >> 8, (gm & PM_LE) != 0u, lo, orw);
    };
#pragma unroll
    for (uint32_t j = 0; j < PPT; ++j) {
      if (slot[j] != NONE) {
        const uint32_t off = (uint32_t)(v[j] - lo);
        atomicOr(&sb[off >> 5], 1u << (off & 31u));
        pres[off >> 5] = 0u;
        h_key[slot[j]] = NONE; h_min[slot[j]] = NONE; h_gap[slot[j]] = NONE;
      } else if ((m[j] & 3u) == EV_GAP && !((listed >> j) & 1u)) {
        gap_or(v[j], a[j], bwj[j], m[j]);
      }
    }
    for (uint32_t g = tid; g < ngap; g += PT) {
      const GapE ge = s_gap[g];
      gap_or(ge.v, ge.a, ge.bw, ge.m);
    }
    __syncthreads();
    PST(6);
    if (q1 < q0 + PCH && q1 < qe) load_chunk(q1, nx);  // the chunk ended at a far GAP: the next starts there
  }
  if (n_ovf) atomicAdd(reinterpret_cast<unsigned long long*>(s.ctr + C_OVF), (unsigned long long)n_ovf);
  // state (as k_state): ack_base = first sequence number >= threshold outside the change set
  int64_t nb = run_thr < lo + (int64_t)W ? first_open(run_thr) : run_thr;
  __syncthreads();  // (fsh.t final for every thread)
  if (s.fdefer && fsh.t.cap > FT_BIG && far_touch(fsh.t, lo, nb)) {
    far_defer(s, e, fsh.t, sb, nb, (int32_t)run_cnt, PT);  // the k_fx_* launches finish it
    return;
  }
  nb = far_extend(s, fsh, lo, nb, PT);
  const int64_t nlo = nb & ~(int64_t)31;
  const uint64_t shift = (uint64_t)(nlo - lo) >> 5;
  for (uint32_t w = tid; w < WW; w += PT) gbits[w] = (w + shift < WW) ? sb[w + shift] : 0u;
  far_pull(s, fsh, gbits, nlo, PT);
  if (tid == 0) {
    ftab_store(s, e, fsh.t);
    s.base[e] = nb;
    s.lo[e] = nlo;
    s.hbc[e] = (int32_t)run_cnt;
    if (ack_out) ack_out[e] = nb;
  }
  PST(7);
  PST_FLUSH(e);
}

__global__ void k_init_state(uint32_t n, State s) {
  for (uint32_t e = blockIdx.x * IT + threadIdx.x; e < n; e += gridDim.x * IT) {
    s.base[e] = 1;  // RtpsWriterProxy::new: ack_base = SequenceNumber::new(1)
    s.lo[e] = 0;
    s.hbc[e] = 0;
    s.far_off[e] = 0;
    s.far_cap[e] = 0;
    s.far_n[e] = 0;
    s.far_min[e] = INT64_MAX;
    s.fneed[e] = 0;
    s.fstat[e] = 0;
    s.fkeep[e] = 0;
    s.fkmin[e] = INT64_MAX;
  }
}
// the far-set pool compacted: proxy e's table [far_off[e], + far_cap[e]) to noff[e] of the new pool
__global__ void k_far_move(uint32_t n, State s, int64_t* nsn, uint64_t* nkey, const uint64_t* noff) {
  const uint32_t e = blockIdx.x;
  if (e >= n || s.far_cap[e] == 0) return;
  const uint64_t o = s.far_off[e], d = noff[e];
  for (uint32_t j = threadIdx.x; j < s.far_cap[e]; j += blockDim.x) {
    nsn[d + j] = s.fsn[o + j];
    nkey[d + j] = s.fkey[o + j];
  }
  __syncthreads();
  if (threadIdx.x == 0) s.far_off[e] = d;
}
// the epoch counter wrapped: every far SN held becomes "covered before" (key 0)
__global__ void k_far_rekey(uint64_t n, int64_t* sn, uint64_t* key) {
  for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += (uint64_t)gridDim.x * blockDim.x)
    key[j] = sn[j] == FEMPTY ? ~0ull : 0ull;
}
__global__ void k_finish(const uint64_t* ctr, uint64_t* ovf) { if (ovf) *ovf = ctr[C_OVF]; }
__global__ void k_hev(const uint64_t* ctr, uint64_t* hev, const uint64_t* fused) {
  uint64_t ne = 0;
  for (uint32_t k = 0; k < 64; ++k) ne += ctr[C_SPREAD + 4 * k + 2];
  hev[0] = ne;
  hev[1] = ctr[C_NFAR];
  hev[2] = *fused;
}

static inline uint64_t hmin(uint64_t a, uint64_t b) { return a < b ? a : b; }

// the global paths' far items (at most farc of them, see k_far_need)
static void far_launch(const State& S, const uint8_t* arena, uint8_t* acc, uint32_t* tcnt, uint32_t n_proxies,
                       uint64_t farc, hipStream_t st) {
  const uint32_t g = (uint32_t)hmin((farc + KF - 1) / KF, 2048);
  hipLaunchKernelGGL(k_far_need, dim3(g), dim3(KF), 0, st, S, arena);
  hipLaunchKernelGGL(k_far_grow, dim3(n_proxies), dim3(KG), 0, st, S, n_proxies);
  hipLaunchKernelGGL(k_far_ins, dim3(g), dim3(KF), 0, st, S, arena);
  hipLaunchKernelGGL(k_far_dec, dim3(g), dim3(KF), 0, st, S, acc, tcnt);
}

// accepted flags[0, n) -> deliveries (k_dcount + k_dwrite; x.sel holds the tile counts)
// ovf: also copy the batch's window-overflow count out (the paths whose last kernel this is)
// hev: also write the batch's event count there (pinned host memory)
static void deliver(const uint8_t* flag, uint64_t n, const Scratch& x, bool ident, const rtps_ingest_out* out,
                    hipStream_t st, const uint64_t* ctr = nullptr, bool ovf = false, uint64_t* hev = nullptr,
                    const uint64_t* fused = nullptr) {
  const uint32_t ntiles = (uint32_t)((n + DT - 1) / DT);
  if (ntiles == 0) {
    (void)hipMemsetAsync(out->n_accepted, 0, sizeof(uint64_t), st);
    if (ovf && out->n_window_overflow) hipLaunchKernelGGL(k_finish, dim3(1), dim3(1), 0, st, ctr, out->n_window_overflow);
    if (hev) hipLaunchKernelGGL(k_hev, dim3(1), dim3(1), 0, st, ctr, hev, fused);
    return;
  }
  hipLaunchKernelGGL(k_dcount, dim3(ntiles), dim3(IT), 0, st, flag, n, x.sel);
  hipLaunchKernelGGL(k_dwrite, dim3(ntiles), dim3(IT), 0, st, flag, n, x.sel, ntiles, x, ident, out->max_accepted,
                     out->accepted, out->n_accepted, ctr, ovf ? out->n_window_overflow : nullptr, hev, fused);
}

}  // namespace

struct IngestState {
  int device = 0;
  uint32_t ecap = 0;  // proxies with state
  State st{};
  uint64_t rcap = 0;  // records of the per-record scratch
  uint64_t vcap = 0;  // events of the per-event scratch
  Scratch x{};
  void* tmp = nullptr;
  size_t tmp_bytes = 0;
  uint32_t epoch = 0;  // batches since the first-cover table was last cleared
  uint64_t* hctr = nullptr;  // pinned host copy of the event counters
  uint32_t path = 0;         // 0: chosen per batch, 1: global marks / merge, 2: per-proxy workgroups,
                             // 3: global, merged by k_fcmerge whenever the batch has no GAPs (tests)
  PEv* pev = nullptr;  // per-proxy path: the proxied events, packed (event order, or record slots)
  uint64_t pcap = 0;
  uint64_t* hctr2 = nullptr;  // pinned: [0] = the last per-proxy identity batch's events (no sync)
  uint64_t* ctr_base = nullptr;  // two counter sets: a batch uses ctr_base[cpar], its classify zeroes the other
  uint32_t cpar = 0;
  hipEvent_t hnev_ev = nullptr;
  bool hnev_ready = false;
  uint64_t last_nev = 0;      // events of the last batch whose counts were read
  uint64_t last_far = 0;      // ...and its far items (per-proxy path)
  uint64_t last_farc = 0;     // the last signalled batch's far candidates (its tables may have grown)
  uint64_t* hsig = nullptr;    // pinned, coherent: classify's count signal (SIG_*)
  uint64_t sig_tag = 0;
  uint32_t* bk_cl = nullptr;  // proxy bucketing: per (classify workgroup, proxy) events | first position << 16
  uint64_t bkcap = 0;
  // far-set pool (st.fsn / fkey / fused / fpcap; see "far sequence numbers"): the device counter
  // as last seen -- exact after a sync or from the count signal (every earlier batch done), else
  // from the last per-proxy batch's pinned words (hctr2[2])
  uint64_t fp_used = 0;
};

static void free_bk(IngestState* s) {
  if (s->bk_cl) (void)hipFree(s->bk_cl);
  s->bk_cl = nullptr;
  s->bkcap = 0;
}
static bool grow_bk(IngestState* s, uint64_t n, hipStream_t st) {
  if (n <= s->bkcap) return true;
  (void)hipStreamSynchronize(st);
  free_bk(s);
  if (hipMalloc(&s->bk_cl, n * 4) != hipSuccess) {
    free_bk(s);
    return false;
  }
  s->bkcap = n;
  return true;
}

static void free_pscratch(IngestState* s) {
  if (s->pev) (void)hipFree(s->pev);
  s->pev = nullptr;
  s->pcap = 0;
}
// packed events for n proxied events (sort keys / values in the HEARTBEAT scratch: vcap >= n)
static bool grow_pscratch(IngestState* s, uint64_t n, hipStream_t st) {
  if (n <= s->pcap) return true;
  (void)hipStreamSynchronize(st);
  free_pscratch(s);
  if (hipMalloc(&s->pev, n * sizeof(PEv)) != hipSuccess) return false;
  s->pcap = n;
  return true;
}

void rtps_ingest_set_path(IngestState* s, uint32_t path) { s->path = path; }

// tuning builds (RTPS_PROXY_STAMPS): k_proxy's per-proxy phase sums (100 MHz ticks), PST_N per proxy
int rtps_ingest_proxy_stamps(uint64_t* host, uint64_t n) {
#if defined(RTPS_PROXY_STAMPS) || defined(RTPS_CLS_STAMPS)
  if (n > 16384ull * 16) n = 16384ull * 16;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_proxy_stamps), n * 8, 0, hipMemcpyDeviceToHost) == hipSuccess
             ? RTPS_RX_OK : RTPS_RX_EHIP;
#else
  (void)host; (void)n;
  return RTPS_RX_EINVAL;
#endif
}

// the fields of State that are not per proxy (kept when the per-proxy arrays are rebuilt)
static void keep_shared(State& m, const State& o) {
  m.ctr = o.ctr;
  m.fsn = o.fsn;
  m.fkey = o.fkey;
  m.fused = o.fused;
  m.fpcap = o.fpcap;
  m.fl = o.fl;
  m.fl_cap = o.fl_cap;
  m.epoch = o.epoch;
}
static void free_state(IngestState* s) {
  void* p[] = {s->st.base, s->st.lo, s->st.hbc, s->st.bits, s->st.fc, s->st.dbits, s->st.seg_b, s->st.seg_e,
               s->st.far_off, s->st.far_cap, s->st.far_n, s->st.far_min, s->st.fneed, s->st.fstat,
               s->st.fdl, s->st.fext, s->st.fkeep, s->st.fkmin};
  for (void* q : p) if (q) (void)hipFree(q);
  State k{};
  keep_shared(k, s->st);
  s->st = k;
  s->ecap = 0;
}
static void free_far(IngestState* s) {
  void* p[] = {s->st.fsn, s->st.fkey, s->st.fl};
  for (void* q : p) if (q) (void)hipFree(q);
  s->st.fsn = nullptr;
  s->st.fkey = nullptr;
  s->st.fpcap = 0;
  s->st.fl = nullptr;
  s->st.fl_cap = 0;
}
// the batch's far-item list (global paths): one entry per event at most
static bool grow_fl(IngestState* s, uint64_t n, hipStream_t st) {
  if (n <= s->st.fl_cap) return true;
  (void)hipStreamSynchronize(st);
  if (s->st.fl) (void)hipFree(s->st.fl);
  s->st.fl = nullptr;
  s->st.fl_cap = 0;
  uint64_t c = 1024;
  while (c < n) c <<= 1;
  if (hipMalloc(&s->st.fl, c * sizeof(FarItem)) != hipSuccess) {
    s->st.fl = nullptr;
    return false;
  }
  s->st.fl_cap = c;
  return true;
}
// Before the far items of a batch that can cover up to F far SNs are decided: the far-set pool
// keeps >= 8 (F + 2^16) + 2 x used slots free -- what the batch's tables can take (a table
// grows to <= 4 x its SNs, the proxy's old entries included, and a chain of growths in the
// per-proxy pass sums to <= twice its last table).  When the last seen count says it may
// not, the stream is synchronised and the count read; still short: the live tables are
// packed at the front of a larger pool (k_far_move) and the abandoned ones dropped.
static bool far_pool_ensure(IngestState* s, uint64_t F, hipStream_t st) {
  auto room = [&](uint64_t used) { return 8 * (F + 65536) + 2 * used; };
  if (s->st.fpcap && s->fp_used + room(s->fp_used) <= s->st.fpcap) return true;
  if (hipStreamSynchronize(st) != hipSuccess) return false;
  uint64_t used = 0;
  if (hipMemcpy(&used, s->st.fused, 8, hipMemcpyDeviceToHost) != hipSuccess) return false;
  s->fp_used = used;
  if (s->st.fpcap && used + room(used) <= s->st.fpcap) return true;
  // compaction: the live tables' new offsets (packed in proxy order)
  const uint32_t ne = s->ecap;
  std::vector<uint32_t> cap(ne);
  std::vector<uint64_t> noff(ne);
  if (ne && hipMemcpy(cap.data(), s->st.far_cap, ne * 4ull, hipMemcpyDeviceToHost) != hipSuccess) return false;
  uint64_t live = 0;
  for (uint32_t e = 0; e < ne; ++e) {
    noff[e] = live;
    live += cap[e];
  }
  const uint64_t nc = (live + room(live)) * 3 / 2;
  int64_t* nsn = nullptr;
  uint64_t* nkey = nullptr;
  uint64_t* dnoff = nullptr;
  bool ok = hipMalloc(&nsn, nc * 8) == hipSuccess && hipMalloc(&nkey, nc * 8) == hipSuccess &&
            hipMemsetAsync(nsn, 0xff, nc * 8, st) == hipSuccess && hipMemsetAsync(nkey, 0xff, nc * 8, st) == hipSuccess;
  if (ok && live) {
    ok = hipMalloc(&dnoff, ne * 8ull) == hipSuccess &&
         hipMemcpy(dnoff, noff.data(), ne * 8ull, hipMemcpyHostToDevice) == hipSuccess;
    if (ok) hipLaunchKernelGGL(k_far_move, dim3(ne), dim3(256), 0, st, ne, s->st, nsn, nkey, dnoff);
    ok = ok && hipStreamSynchronize(st) == hipSuccess;
  }
  ok = ok && hipMemcpy(s->st.fused, &live, 8, hipMemcpyHostToDevice) == hipSuccess;
  if (dnoff) (void)hipFree(dnoff);
  if (!ok) {
    if (nsn) (void)hipFree(nsn);
    if (nkey) (void)hipFree(nkey);
    return false;
  }
  if (s->st.fsn) (void)hipFree(s->st.fsn);
  if (s->st.fkey) (void)hipFree(s->st.fkey);
  s->st.fsn = nsn;
  s->st.fkey = nkey;
  s->st.fpcap = nc;
  s->fp_used = live;
  return true;
}
static void free_rscratch(IngestState* s) {
  void* p[] = {s->x.fidx, s->x.fmask, s->x.fall, s->x.rcnt, s->x.roff, s->x.rset, s->x.rkind, s->x.rsn};
  for (void* q : p) if (q) (void)hipFree(q);
  s->x.fmask = nullptr;
  s->x.fall = nullptr;
  s->x.fidx = nullptr; s->x.rcnt = nullptr; s->x.roff = nullptr; s->x.rset = nullptr; s->x.rkind = nullptr;
  s->x.rsn = nullptr;
  s->rcap = 0;
}
static void free_vscratch(IngestState* s) {
  void* p[] = {s->x.evt, s->x.ent, s->x.esn, s->x.erec, s->x.emeta, s->x.eacc, s->x.sel, s->x.hkey, s->x.hval,
               s->x.skey, s->x.sval, s->x.hcnt, s->x.hexcl, s->x.hf, s->x.hpre, s->tmp};
  for (void* q : p) if (q) (void)hipFree(q);
  Scratch keep = s->x;
  s->x = Scratch{};
  s->x.fidx = keep.fidx; s->x.fmask = keep.fmask; s->x.fall = keep.fall; s->x.rcnt = keep.rcnt; s->x.roff = keep.roff; s->x.rset = keep.rset;
  s->x.rkind = keep.rkind; s->x.rsn = keep.rsn;
  s->x.frag = keep.frag; s->x.n_frag = keep.n_frag; s->x.max_frag = keep.max_frag;  // (this batch's, set before the events are sized)
  s->tmp = nullptr;
  s->tmp_bytes = 0;
  s->vcap = 0;
}

// per-proxy state for n proxies; existing proxies keep theirs
static bool grow_state(IngestState* s, uint32_t n, hipStream_t st) {
  if (n <= s->ecap) return true;
  uint32_t ncap = s->ecap ? s->ecap : 16;
  while (ncap < n) ncap <<= 1;
  (void)hipStreamSynchronize(st);
  State o = s->st;
  State m{};
  keep_shared(m, o);
  bool ok = hipMalloc(&m.base, ncap * 8ull) == hipSuccess && hipMalloc(&m.lo, ncap * 8ull) == hipSuccess &&
            hipMalloc(&m.hbc, ncap * 4ull) == hipSuccess && hipMalloc(&m.bits, (uint64_t)ncap * WW * 4) == hipSuccess &&
            hipMalloc(&m.fc, (uint64_t)ncap * W * 8) == hipSuccess && hipMalloc(&m.seg_b, ncap * 4ull) == hipSuccess &&
            hipMalloc(&m.dbits, (uint64_t)ncap * WW * 4) == hipSuccess &&
            hipMalloc(&m.seg_e, ncap * 4ull) == hipSuccess && hipMalloc(&m.far_off, ncap * 8ull) == hipSuccess &&
            hipMalloc(&m.far_cap, ncap * 4ull) == hipSuccess && hipMalloc(&m.far_n, ncap * 4ull) == hipSuccess &&
            hipMalloc(&m.far_min, ncap * 8ull) == hipSuccess && hipMalloc(&m.fneed, ncap * 8ull) == hipSuccess &&
            hipMalloc(&m.fstat, ncap * 4ull) == hipSuccess && hipMalloc(&m.fdl, ncap * 4ull) == hipSuccess &&
            hipMalloc(&m.fext, ncap * 8ull) == hipSuccess && hipMalloc(&m.fkeep, ncap * 4ull) == hipSuccess &&
            hipMalloc(&m.fkmin, ncap * 8ull) == hipSuccess;
  ok = ok && hipMemsetAsync(m.bits, 0, (uint64_t)ncap * WW * 4, st) == hipSuccess &&
       hipMemsetAsync(m.dbits, 0, (uint64_t)ncap * WW * 4, st) == hipSuccess &&
       hipMemsetAsync(m.fc, 0xff, (uint64_t)ncap * W * 8, st) == hipSuccess;
  if (ok) hipLaunchKernelGGL(k_init_state, dim3((ncap + IT - 1) / IT), dim3(IT), 0, st, ncap, m);
  if (ok && s->ecap) {  // carry the existing proxies' state
    const uint64_t e = s->ecap;
    ok = hipMemcpyAsync(m.base, o.base, e * 8, hipMemcpyDeviceToDevice, st) == hipSuccess &&
         hipMemcpyAsync(m.lo, o.lo, e * 8, hipMemcpyDeviceToDevice, st) == hipSuccess &&
         hipMemcpyAsync(m.hbc, o.hbc, e * 4, hipMemcpyDeviceToDevice, st) == hipSuccess &&
         hipMemcpyAsync(m.bits, o.bits, e * WW * 4, hipMemcpyDeviceToDevice, st) == hipSuccess &&
         hipMemcpyAsync(m.far_off, o.far_off, e * 8, hipMemcpyDeviceToDevice, st) == hipSuccess &&
         hipMemcpyAsync(m.far_cap, o.far_cap, e * 4, hipMemcpyDeviceToDevice, st) == hipSuccess &&
         hipMemcpyAsync(m.far_n, o.far_n, e * 4, hipMemcpyDeviceToDevice, st) == hipSuccess &&
         hipMemcpyAsync(m.far_min, o.far_min, e * 8, hipMemcpyDeviceToDevice, st) == hipSuccess;
  }
  ok = ok && hipStreamSynchronize(st) == hipSuccess;
  s->st = m;
  s->ecap = ncap;
  State dead = o;
  void* p[] = {dead.base, dead.lo, dead.hbc, dead.bits, dead.fc, dead.dbits, dead.seg_b, dead.seg_e,
               dead.far_off, dead.far_cap, dead.far_n, dead.far_min, dead.fneed, dead.fstat,
               dead.fdl, dead.fext, dead.fkeep, dead.fkmin};
  for (void* q : p) if (q) (void)hipFree(q);
  if (!ok) { free_state(s); return false; }
  return true;
}

static bool grow_rscratch(IngestState* s, uint64_t max, hipStream_t st) {
  if (max <= s->rcap) return true;
  (void)hipStreamSynchronize(st);
  free_rscratch(s);
  Scratch& x = s->x;
  const uint64_t n = max;
  bool ok = hipMalloc(&x.fidx, n * 4) == hipSuccess && hipMalloc(&x.fmask, n * 8) == hipSuccess &&
            hipMalloc(&x.fall, n) == hipSuccess &&
            hipMalloc(&x.rcnt, n * 4) == hipSuccess &&
            hipMalloc(&x.roff, n * 4) == hipSuccess && hipMalloc(&x.rset, n * 4) == hipSuccess &&
            hipMalloc(&x.rkind, n) == hipSuccess && hipMalloc(&x.rsn, n * 8) == hipSuccess;
  if (!ok) { free_rscratch(s); return false; }
  s->rcap = n;
  return true;
}

// event scratch + hipcub temporary storage for n events (the per-record scan needs rcap)
static bool grow_vscratch(IngestState* s, uint64_t n, hipStream_t st) {
  if (n <= s->vcap) return true;
  (void)hipStreamSynchronize(st);
  free_vscratch(s);
  Scratch& x = s->x;
  bool ok = hipMalloc(&x.evt, n) == hipSuccess && hipMalloc(&x.ent, n * 4) == hipSuccess &&
            hipMalloc(&x.esn, n * 8) == hipSuccess && hipMalloc(&x.erec, n * 4) == hipSuccess &&
            hipMalloc(&x.emeta, n * 4) == hipSuccess && hipMalloc(&x.eacc, n) == hipSuccess &&
            hipMalloc(&x.sel, n * 4) == hipSuccess &&
            hipMalloc(&x.hkey, n * 4) == hipSuccess && hipMalloc(&x.hval, n * 4) == hipSuccess &&
            hipMalloc(&x.skey, n * 4) == hipSuccess && hipMalloc(&x.sval, n * 4) == hipSuccess &&
            hipMalloc(&x.hcnt, n * 4) == hipSuccess && hipMalloc(&x.hexcl, n * 4) == hipSuccess &&
            hipMalloc(&x.hf, n * 8) == hipSuccess && hipMalloc(&x.hpre, n * 8) == hipSuccess;
  const uint64_t nr = s->rcap > n ? s->rcap : n;
  size_t b1 = 0, b2 = 0, b3 = 0, b4 = 0, b5 = 0, b6 = 0;
  ok = ok && rtps_sort_pairs(nullptr, b1, x.hkey, x.skey, x.hval, x.sval, (uint32_t)n, (int)32, st) == hipSuccess;
  ok = ok && hipcub::DeviceScan::ExclusiveScanByKey(nullptr, b2, x.skey, x.hcnt, x.hexcl, hipcub::Max(), INT32_MIN,
                                                    (uint32_t)n, hipcub::Equality(), st) == hipSuccess;
  ok = ok && hipcub::DeviceScan::InclusiveScanByKey(nullptr, b3, x.skey, x.hf, x.hpre, hipcub::Max(), (uint32_t)n,
                                                    hipcub::Equality(), st) == hipSuccess;
  ok = ok && hipcub::DeviceSelect::Flagged(nullptr, b4, hipcub::CountingInputIterator<uint32_t>(0), (uint8_t*)nullptr,
                                           (uint32_t*)nullptr, (uint64_t*)nullptr, (int64_t)n, st) == hipSuccess;
  ok = ok && hipcub::DeviceSelect::Flagged(nullptr, b5, hipcub::CountingInputIterator<uint32_t>(0), x.hkey, x.hval,
                                           (uint64_t*)nullptr, (int64_t)n, st) == hipSuccess;
  ok = ok && hipcub::DeviceScan::ExclusiveSum(nullptr, b6, x.rcnt, x.roff, (uint32_t)nr, st) == hipSuccess;
  size_t tb = b1;
  for (size_t b : {b2, b3, b4, b5, b6}) tb = b > tb ? b : tb;
  s->tmp_bytes = tb;
  ok = ok && hipMalloc(&s->tmp, tb) == hipSuccess;
  if (!ok) { free_vscratch(s); return false; }
  s->vcap = n;
  return true;
}

IngestState* rtps_ingest_state_new(int device) {
  IngestState* s = new (std::nothrow) IngestState();
  if (!s) return nullptr;
  s->device = device;
  if (hipMalloc(&s->ctr_base, 2 * C_COUNT * 8) != hipSuccess) { delete s; return nullptr; }
  if (hipMalloc(&s->st.fused, 8) != hipSuccess || hipMemset(s->st.fused, 0, 8) != hipSuccess) {
    rtps_ingest_state_free(s);
    return nullptr;
  }
  if (hipMemset(s->ctr_base, 0, 2 * C_COUNT * 8) != hipSuccess) {
    (void)hipFree(s->ctr_base);
    delete s;
    return nullptr;
  }
  s->st.ctr = s->ctr_base;
  if (hipHostMalloc(&s->hctr, C_COUNT * 8, hipHostMallocDefault) != hipSuccess ||
      hipHostMalloc(&s->hctr2, C_COUNT * 8, hipHostMallocDefault) != hipSuccess ||
      hipHostMalloc(&s->hsig, SIG_WORDS * 8, hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess ||
      hipEventCreateWithFlags(&s->hnev_ev, hipEventDisableTiming) != hipSuccess) {
    rtps_ingest_state_free(s);
    return nullptr;
  }
  return s;
}

void rtps_ingest_state_free(IngestState* s) {
  if (!s) return;
  free_bk(s);
  free_pscratch(s);
  free_vscratch(s);
  free_rscratch(s);
  free_state(s);
  free_far(s);
  if (s->st.fused) (void)hipFree(s->st.fused);
  if (s->ctr_base) (void)hipFree(s->ctr_base);
  if (s->hctr) (void)hipHostFree(s->hctr);
  if (s->hctr2) (void)hipHostFree(s->hctr2);
  if (s->hsig) (void)hipHostFree(s->hsig);
  if (s->hnev_ev) (void)hipEventDestroy(s->hnev_ev);
  delete s;
}

int rtps_ingest_state_reset(IngestState* s, hipStream_t st) {
  if (!s->ecap) return RTPS_RX_OK;
  bool ok = hipMemsetAsync(s->st.bits, 0, (uint64_t)s->ecap * WW * 4, st) == hipSuccess &&  // fc: epoch-tagged
            hipMemsetAsync(s->st.dbits, 0, (uint64_t)s->ecap * WW * 4, st) == hipSuccess;
  if (ok) hipLaunchKernelGGL(k_init_state, dim3((s->ecap + IT - 1) / IT), dim3(IT), 0, st, s->ecap, s->st);
  // every far set emptied: the pool's tables are all free again
  ok = ok && hipMemsetAsync(s->st.fused, 0, 8, st) == hipSuccess;
  if (s->st.fpcap)  // the whole pool free again (all ones)
    ok = ok && hipMemsetAsync(s->st.fsn, 0xff, s->st.fpcap * 8, st) == hipSuccess &&
         hipMemsetAsync(s->st.fkey, 0xff, s->st.fpcap * 8, st) == hipSuccess;
  s->fp_used = 0;
  return ok && hipGetLastError() == hipSuccess ? RTPS_RX_OK : RTPS_RX_EHIP;
}

// the k_fx_* launches that finish the far sets a state pass deferred (S.fdefer: that pass may
// have listed some; none listed: each returns at once)
static void far_finish(const State& S, int64_t* ack_out, hipStream_t st) {
  if (!S.fdefer) return;
  hipLaunchKernelGGL(k_fx_ext, dim3(1024), dim3(FX), 0, st, S);
  hipLaunchKernelGGL(k_fx_shift, dim3(512), dim3(FX), 0, st, S);
  hipLaunchKernelGGL(k_fx_pull, dim3(1024), dim3(FX), 0, st, S);
  hipLaunchKernelGGL(k_fx_fin, dim3(1), dim3(FX), 0, st, S, ack_out);
}

static int ingest_batch(IngestState* s, hipStream_t st, const ReaderDev& t, const uint8_t* arena, uint64_t arena_len,
                      const uint64_t* dgram_off, const rtps_record* records, const uint64_t* n_records,
                      uint64_t max_records, const rtps_frag_sample* frag, const uint64_t* n_frag, uint64_t max_frag,
                      uint32_t flags, const rtps_ingest_out* out, const IngestTail* tail, bool& tail_queued) {
  (void)arena_len;
  tail_queued = false;
  if (t.n_proxies > ECAP_MAX) return RTPS_RX_ETOOBIG;
  if (max_records > 0x7fffffffull) return RTPS_RX_ETOOBIG;
  if (!grow_state(s, t.n_proxies ? t.n_proxies : 1, st)) return RTPS_RX_ENOMEM;
  const uint64_t max = max_records ? max_records : 1;
  if (!grow_rscratch(s, max, st)) return RTPS_RX_ENOMEM;
  const bool ident = t.max_set <= 1u;
  if (ident && !grow_vscratch(s, max, st)) return RTPS_RX_ENOMEM;
  if (!ident && s->vcap == 0 && !grow_vscratch(s, 1, st)) return RTPS_RX_ENOMEM;
  const bool reliable = !(flags & RTPS_INGEST_BEST_EFFORT);
  const FarSrc fs{records, dgram_off};
  const SigCfg cfg{ident ? 1u : 0u, t.n_proxies, s->path, reliable ? 1u : 0u, s->st.fused};
  if (++s->epoch == 0xffffffffu) {  // keys would wrap: clear the first-cover table, age the far sets' keys
    if (hipMemsetAsync(s->st.fc, 0xff, (uint64_t)s->ecap * W * 8, st) != hipSuccess) return RTPS_RX_EHIP;
    uint64_t used = 0;
    if (hipStreamSynchronize(st) != hipSuccess || hipMemcpy(&used, s->st.fused, 8, hipMemcpyDeviceToHost) != hipSuccess)
      return RTPS_RX_EHIP;
    used = used < s->st.fpcap ? used : s->st.fpcap;
    if (used)
      hipLaunchKernelGGL(k_far_rekey, dim3((uint32_t)hmin((used + 255) / 256, 4096)), dim3(256), 0, st, used, s->st.fsn,
                         s->st.fkey);
    s->epoch = 1;
  }
  s->st.epoch = s->epoch;
  uint32_t ebits = 1;
  while ((1u << ebits) < t.n_proxies) ++ebits;  // sort key width: proxies < 2^ebits
  const uint32_t gb = (uint32_t)hmin((max + IT - 1) / IT, 8192);
  Scratch& x = s->x;
  State& S = s->st;
  // counters: this batch's set is zero (the previous classify zeroed it); this classify zeroes the other
  S.ctr = s->ctr_base + (uint64_t)s->cpar * C_COUNT;
  uint64_t* const ctr_next = s->ctr_base + (uint64_t)(s->cpar ^ 1u) * C_COUNT;
  bool ok = true;
  const bool with_frag = frag && n_frag && max_frag;
  x.frag = frag;
  x.n_frag = n_frag;
  x.max_frag = max_frag;
  if (with_frag) {
    hipLaunchKernelGGL(k_fclear, dim3((uint32_t)hmin((max / 4u + IT - 1) / IT + 1u, 4096)), dim3(IT), 0, st, max,
                       x.fidx, x.fmask, x.fall);
    hipLaunchKernelGGL(k_fidx, dim3((uint32_t)hmin((max_frag + IT - 1) / IT, 4096)), dim3(IT), 0, st, frag, n_frag,
                       max_frag, max, x.fidx, x.fmask, x.fall, t, records);
  }
  uint32_t lds = rt_fits_lds(t) ? rt_lds_bytes(t.gmask + 1u, t.emask + 1u) : 0u;
  // the target sets join the hash tables in LDS when both fit the tables' own limit
  const bool sets_lds = lds && lds + sets_lds_bytes(t) <= RT_LDS_MAX;
  if (sets_lds) lds += sets_lds_bytes(t);
  // Identity batches over many proxies take the per-proxy path with no host read-back:
  // classify writes the path's inputs, the sort runs over every record slot. The choice
  // uses the previous batch's counts (mean events per proxy), read without a sync.
  if (s->hnev_ready && hipEventQuery(s->hnev_ev) == hipSuccess) {
    s->last_nev = s->hctr2[0];
    s->last_far = s->hctr2[1];
    s->fp_used = s->fp_used > s->hctr2[2] ? s->fp_used : s->hctr2[2];  // (a compaction since lowered it: exact then)
    s->hnev_ready = false;
  }
  // (after a batch with far items the next takes the signalled path, which sizes the far-set
  // pool from its own counts; the fast path sizes it from the last one's far items)
  const bool fast = ident && t.n_proxies > 0 &&
                    (s->path == 2 || s->path == 4 || (s->path == 0 && t.n_proxies >= 64 && s->last_far == 0 &&
                                                      s->last_nev <= (uint64_t)t.n_proxies * 32768u));
  // the proxy bucketing (k_classify<.., BUCKET>, k_proxy<true>) unless the proxies or the
  // classify workgroups exceed its LDS tables (or path 4: the radix sort, tests)
  const uint64_t nblk = (max + CHR - 1) / CHR;
  const bool bucket = fast && t.n_proxies <= PB_MAX && nblk <= BK_MAX && s->path != 4;
  FastOut fo{nullptr, nullptr, arena, dgram_off, S.seg_b, S.seg_e, s->ecap, nullptr, sets_lds ? 1u : 0u};
  if (fast) {
    if (!far_pool_ensure(s, 2 * s->last_far, st)) return RTPS_RX_ENOMEM;
    if (!grow_pscratch(s, bucket ? nblk * CHR : max, st)) return RTPS_RX_ENOMEM;
    fo.pev = s->pev;
    fo.acc = out->accept;
  }
  if (bucket) {
    if (!grow_bk(s, (uint64_t)t.n_proxies * nblk, st)) return RTPS_RX_ENOMEM;
    fo.bk_cl = s->bk_cl;
    hipLaunchKernelGGL((k_classify<true, true, true>), dim3((uint32_t)nblk), dim3(IT), lds, st, t, records,
                       n_records, max, with_frag ? frag : nullptr, flags, x, S.ctr, fo, ctr_next, S, s->epoch);
  } else if (ident && fast)
    hipLaunchKernelGGL((k_classify<true, true>), dim3(gb), dim3(IT), lds, st, t, records, n_records, max,
                       with_frag ? frag : nullptr, flags, x, S.ctr, fo, ctr_next, S, s->epoch);
  else if (ident)  // the global path's marks ride along (harmless keys of this epoch if the batch goes per proxy)
    hipLaunchKernelGGL((k_classify<true, false, false, true>), dim3(gb), dim3(IT), lds, st, t, records, n_records,
                       max, with_frag ? frag : nullptr, flags, x, S.ctr, fo, ctr_next, S, s->epoch);
  else
    hipLaunchKernelGGL((k_classify<false, false>), dim3(gb), dim3(IT), lds, st, t, records, n_records, max,
                       with_frag ? frag : nullptr, flags, x, S.ctr, fo, ctr_next, S, s->epoch);
  s->cpar ^= 1u;  // the next batch uses the set this classify zeroes
  // a far set past FT_BIG slots exists only where the pool holds that many, or grows in a batch
  // with far items (the signalled path's farc; the fast path is not taken after one)
  S.fdefer = s->fp_used > FT_BIG ? 1u : 0u;
  if (bucket) {
    hipLaunchKernelGGL(k_proxy<true>, dim3(t.n_proxies), dim3(PT), 0, st, arena, s->pev, x.hval, t.n_proxies, S,
                       out->accept, out->ack_base, BkIn{s->bk_cl, (uint32_t)nblk});
    far_finish(S, out->ack_base, st);
  } else if (fast) {
    uint32_t kb = 1;
    while ((1u << kb) <= t.n_proxies) ++kb;  // keys 0..n_proxies (n_proxies: no proxy, sorts last)
    size_t tb = s->tmp_bytes;
    if (rtps_sort_pairs(s->tmp, tb, x.hkey, x.skey, x.sval, x.hval, (uint32_t)max, (int)kb, st) != hipSuccess)
      return RTPS_RX_EHIP;
    const uint32_t gm = (uint32_t)hmin((max + IT - 1) / IT, 8192);
    hipLaunchKernelGGL(k_pseg, dim3(gm), dim3(IT), 0, st, max, t.n_proxies, x, S);
    hipLaunchKernelGGL(k_proxy<false>, dim3(t.n_proxies), dim3(PT), 0, st, arena, s->pev, x.hval, t.n_proxies, S,
                       out->accept, out->ack_base, BkIn{});
    far_finish(S, out->ack_base, st);
  }
  if (fast) {
    // the select also writes this batch's event count for the next batch's choice (pinned, read
    // without a sync once the event has passed)
    deliver(out->accept, max, x, true, out, st, S.ctr, true, s->hctr2, S.fused);
    if (hipEventRecord(s->hnev_ev, st) != hipSuccess) return RTPS_RX_EHIP;
    s->hnev_ready = true;
    return hipGetLastError() == hipSuccess ? RTPS_RX_OK : RTPS_RX_EHIP;
  }
  // the batch's record / HEARTBEAT / GAP / event counts size the rest: k_signal writes them to
  // pinned memory, the host spins on the tag (no copy, no interrupt-driven wait); a wait past
  // the limit falls back to a stream sync (a failed launch surfaces there)
  const uint64_t tag = ++s->sig_tag;
  if (ident) {
    // the plain global path's two launches, queued now: they run at once if the batch's counts
    // make it plain and return otherwise (the host then launches the batch's path below); the
    // decide launch signals the counts and its verdict to the host
    const uint32_t ntiles = (uint32_t)((max + DT - 1) / DT);
    const uint32_t nfcm = (uint32_t)((uint64_t)t.n_proxies * W / FCM_POS);
    hipLaunchKernelGGL(k_decide_t<3>, dim3(ntiles + nfcm), dim3(IT), 0, st, max, max, x, S, out->accept, false,
                       s->epoch, x.sel, fs, ntiles, SigOut{s->hsig, tag, cfg});
    S.fdefer = (s->fp_used > FT_BIG || s->last_farc) ? 1u : 0u;  // (the pool as the last batch left it)
    hipLaunchKernelGGL(k_dstate, dim3(ntiles + t.n_proxies), dim3(IT), 0, st, out->accept, max, x.sel, ntiles, x,
                       out->max_accepted, out->accepted, out->n_accepted, S.ctr, out->n_window_overflow, t.n_proxies,
                       S, false, out->ack_base, false, true);
    far_finish(S, out->ack_base, st);
    if (tail) {  // behind the plain path, gated by its verdict (C_MODE, written by k_decide_t<3>)
      const int rc = tail->run(tail->ctx, S.ctr + C_MODE);
      if (rc) return rc;
    }
  } else {
    hipLaunchKernelGGL(k_signal, dim3(1), dim3(64), 0, st, S.ctr, s->hsig, tag, cfg);
  }
  if (hipGetLastError() != hipSuccess) return RTPS_RX_EHIP;
  {
    volatile uint64_t* hs = s->hsig;
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t spin = 0; hs[SIG_TAG] != tag; ++spin) {
      if ((spin & 1023u) == 1023u && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(200)) {
        if (hipStreamSynchronize(st) != hipSuccess || hs[SIG_TAG] != tag) return RTPS_RX_EHIP;
        break;
      }
      __builtin_ia32_pause();
    }
    std::atomic_thread_fence(std::memory_order_acquire);
  }
  const uint64_t n_hb = s->hsig[SIG_HB], n_gap = s->hsig[SIG_GAP], n_ev = s->hsig[SIG_EV], n_free = s->hsig[SIG_FREE];
  const uint64_t n_rec = s->hsig[SIG_NREC], farc = s->hsig[SIG_FARC];
  s->fp_used = s->hsig[SIG_FUSED];  // (exact: every earlier batch has finished)
  if (ident && s->hsig[SIG_MODE] != 0) {  // the queued plain path runs it (and the gated tail)
    tail_queued = true;
    return RTPS_RX_OK;
  }
  // events live at [0, nev): record slots in identity batches, the expanded list otherwise
  uint64_t nev = ident ? n_rec : n_ev;
  // far items: at most classify's candidates (every path but the fast one counts them); their far SNs
  // (a GAP's listed ones included) bound the far-set tables this batch can grow
  const uint64_t nfi = farc;
  if (nfi && (!grow_fl(s, nfi, st) || !far_pool_ensure(s, nfi + 256 * n_gap, st))) return RTPS_RX_ENOMEM;
  s->last_farc = farc;
  S.fdefer = (farc || s->fp_used > FT_BIG) ? 1u : 0u;  // (this batch's state pass may defer large far sets)
  if (!ident) {
    if (n_ev > 0x7fffffffull) return RTPS_RX_ETOOBIG;
    if (!grow_vscratch(s, n_ev ? n_ev : 1, st)) return RTPS_RX_ENOMEM;
    size_t tb = s->tmp_bytes;
    if (n_rec && hipcub::DeviceScan::ExclusiveSum(s->tmp, tb, x.rcnt, x.roff, (uint32_t)n_rec, st) != hipSuccess)
      return RTPS_RX_EHIP;
    if (n_rec)
      hipLaunchKernelGGL(k_expand, dim3((uint32_t)hmin((n_rec + IT - 1) / IT, 8192)), dim3(IT), 0, st, t, n_rec, flags, x, with_frag);
  }
  const uint32_t gv = (uint32_t)hmin((nev + IT - 1) / IT, 8192) ? (uint32_t)hmin((nev + IT - 1) / IT, 8192) : 1u;
  // per-proxy workgroups when the events spread over many proxies (mean load bounded:
  // one workgroup replays a proxy's events in order); global marks / merge otherwise
  // (threshold GAPs past a window: the per-proxy path applies them as thresholds, whatever the path)
  const uint64_t tgap = s->hsig[SIG_TGAP];
  const bool per_proxy = t.n_proxies > 0 && nev > 0 &&
                         (tgap != 0 || s->path == 2 || s->path == 4 ||
                          (s->path == 0 && t.n_proxies >= 64 && n_ev <= (uint64_t)t.n_proxies * 32768u));
  uint8_t* acc = ident ? out->accept : x.eacc;
  const uint64_t acc_cap = ident ? max : nev;
  if (per_proxy) {
    // the proxied events, in event order (order-preserving select), packed, sorted by proxy (stable)
    const uint64_t n_px = n_ev - n_free;
    if (!grow_pscratch(s, n_px ? n_px : 1, st)) return RTPS_RX_ENOMEM;
    uint32_t kb = 1;
    while ((1u << kb) < t.n_proxies) ++kb;  // keys 0..n_proxies-1
    ok = hipMemsetAsync(S.seg_b, 0, (uint64_t)s->ecap * 4, st) == hipSuccess &&
         hipMemsetAsync(S.seg_e, 0, (uint64_t)s->ecap * 4, st) == hipSuccess;
    if (!ok) return RTPS_RX_EHIP;
    if (n_px) {
      hipLaunchKernelGGL(k_pflag, dim3(gv), dim3(IT), 0, st, nev, x);
      size_t tb = s->tmp_bytes;
      if (hipcub::DeviceSelect::Flagged(s->tmp, tb, hipcub::CountingInputIterator<uint32_t>(0),
                                        reinterpret_cast<uint8_t*>(x.hkey), x.hval, S.ctr + C_NSEL, (int64_t)nev,
                                        st) != hipSuccess)
        return RTPS_RX_EHIP;
      const uint32_t gp = (uint32_t)hmin((n_px + IT - 1) / IT, 8192);
      hipLaunchKernelGGL(k_pack, dim3(gp), dim3(IT), 0, st, records, arena, dgram_off, n_px, x, s->pev);
      tb = s->tmp_bytes;  // (proxy, packed position) pairs: 8 B per event per pass, not the 32-B events
      if (rtps_sort_pairs(s->tmp, tb, x.hkey, x.skey, x.sval, x.hval, (uint32_t)n_px, (int)kb, st) != hipSuccess)
        return RTPS_RX_EHIP;
      hipLaunchKernelGGL(k_pseg, dim3(gp), dim3(IT), 0, st, n_px, t.n_proxies, x, S);
    }
    hipLaunchKernelGGL(k_decide_free, dim3((uint32_t)hmin((acc_cap + IT - 1) / IT, 8192)), dim3(IT), 0, st, nev,
                       acc_cap, x, acc);
    hipLaunchKernelGGL(k_proxy<false>, dim3(t.n_proxies), dim3(PT), 0, st, arena, s->pev, x.hval, t.n_proxies, S,
                       acc, out->ack_base, BkIn{});
    far_finish(S, out->ack_base, st);
  }
  const bool have_hb = reliable && n_hb > 0 && !per_proxy;
  if (have_hb) {  // stable compaction of the HEARTBEAT events, sort by proxy, scans by key
    const uint32_t hb_blocks = (uint32_t)hmin((n_hb + IT - 1) / IT, 8192);
    ok = hipMemsetAsync(S.seg_b, 0, (uint64_t)s->ecap * 4, st) == hipSuccess &&
         hipMemsetAsync(S.seg_e, 0, (uint64_t)s->ecap * 4, st) == hipSuccess;
    if (!ok) return RTPS_RX_EHIP;
    size_t tb = s->tmp_bytes;
    if (hipcub::DeviceSelect::Flagged(s->tmp, tb, hipcub::CountingInputIterator<uint32_t>(0), x.hkey, x.hval,
                                      S.ctr + C_NSEL, (int64_t)nev, st) != hipSuccess)
      return RTPS_RX_EHIP;
    hipLaunchKernelGGL(k_hkeys, dim3(hb_blocks), dim3(IT), 0, st, n_hb, x);
    tb = s->tmp_bytes;
    if (rtps_sort_pairs(s->tmp, tb, x.hkey, x.skey, x.hval, x.sval, (uint32_t)n_hb, (int)ebits, st) !=
        hipSuccess)
      return RTPS_RX_EHIP;
    hipLaunchKernelGGL(k_hvals, dim3(hb_blocks), dim3(IT), 0, st, records, n_hb, x, S);
    tb = s->tmp_bytes;
    if (hipcub::DeviceScan::ExclusiveScanByKey(s->tmp, tb, x.skey, x.hcnt, x.hexcl, hipcub::Max(), INT32_MIN,
                                               (uint32_t)n_hb, hipcub::Equality(), st) != hipSuccess)
      return RTPS_RX_EHIP;
    hipLaunchKernelGGL(k_hacc, dim3(hb_blocks), dim3(IT), 0, st, records, n_hb, x, S);
    tb = s->tmp_bytes;
    if (hipcub::DeviceScan::InclusiveScanByKey(s->tmp, tb, x.skey, x.hf, x.hpre, hipcub::Max(), (uint32_t)n_hb,
                                               hipcub::Equality(), st) != hipSuccess)
      return RTPS_RX_EHIP;
  }
  if (ident && !per_proxy && nev) {
    // identity batches, global path: the marks ran in classify; decide + tile counts (+ the
    // merge for GAP-free batches), then the deliveries and every proxy's state in one launch
    if (n_gap) {  // the samples' bitmap for the GAP marks (the keys are set)
      hipLaunchKernelGGL(k_marks_d, dim3(gv), dim3(IT), 0, st, nev, x, S, s->epoch, true, false);
      hipLaunchKernelGGL(k_marks_g, dim3(gv), dim3(IT), 0, st, records, arena, dgram_off, nev, x, S, s->epoch);
    }
    const uint32_t ntiles = (uint32_t)((acc_cap + DT - 1) / DT);
    // GAP-free batches merge in decide: from the first-cover keys when the proxies' windows are
    // few against the events (T; path 3 forces it), else by the samples' wave_or
    const bool fc_merge = n_gap == 0 && (s->path == 3 || (s->path != 1 && (uint64_t)t.n_proxies * W <= 4ull * nev));
    const uint32_t nfcm = fc_merge ? (uint32_t)((uint64_t)t.n_proxies * W / FCM_POS) : 0u;
    if (fc_merge)
      hipLaunchKernelGGL(k_decide_t<2>, dim3(ntiles + nfcm), dim3(IT), 0, st, nev, acc_cap, x, S, acc, have_hb,
                         s->epoch, x.sel, fs, ntiles, SigOut{});
    else if (n_gap == 0)
      hipLaunchKernelGGL(k_decide_t<1>, dim3(ntiles), dim3(IT), 0, st, nev, acc_cap, x, S, acc, have_hb, s->epoch,
                         x.sel, fs, ntiles, SigOut{});
    else
      hipLaunchKernelGGL(k_decide_t<0>, dim3(ntiles), dim3(IT), 0, st, nev, acc_cap, x, S, acc, have_hb, s->epoch,
                         x.sel, fs, ntiles, SigOut{});
    if (farc)  // samples / GAPs past some window: their first covers (fixes accept[] and the tile counts)
      far_launch(S, arena, acc, x.sel, t.n_proxies, farc, st);
    if (n_gap)
      hipLaunchKernelGGL(k_merge, dim3(gv), dim3(IT), 0, st, records, arena, dgram_off, nev, x, S, true);
    hipLaunchKernelGGL(k_dstate, dim3(ntiles + t.n_proxies), dim3(IT), 0, st, acc, acc_cap, x.sel, ntiles, x,
                       out->max_accepted, out->accepted, out->n_accepted, S.ctr, out->n_window_overflow, t.n_proxies,
                       S, have_hb, out->ack_base, fc_merge, false);
    far_finish(S, out->ack_base, st);
    return hipGetLastError() == hipSuccess ? RTPS_RX_OK : RTPS_RX_EHIP;
  }
  if (nev && !per_proxy) {
    hipLaunchKernelGGL(k_marks_d, dim3(gv), dim3(IT), 0, st, nev, x, S, s->epoch, n_gap > 0);
    if (n_gap)
      hipLaunchKernelGGL(k_marks_g, dim3(gv), dim3(IT), 0, st, records, arena, dgram_off, nev, x, S, s->epoch);
  }
  // identity batches decide straight into accept[] (event i = record i: max slots, cleared past n)
  if (acc_cap && !per_proxy) {
    hipLaunchKernelGGL(k_decide, dim3((uint32_t)hmin((acc_cap + IT - 1) / IT, 8192)), dim3(IT), 0, st, nev, acc_cap,
                       x, S, acc, have_hb, s->epoch, fs);
    if (farc)  // the far items' first covers (fixes accept[])
      far_launch(S, arena, acc, nullptr, t.n_proxies, farc, st);
  }
  const bool state_pass = t.n_proxies && !per_proxy;  // k_state copies the overflow count out, else the select does
  deliver(acc, acc_cap, x, ident, out, st, S.ctr, !state_pass);
  if (!ident)
    hipLaunchKernelGGL(k_accept_counts, dim3(gb), dim3(IT), 0, st, n_rec, max, x, out->accept);
  if (nev && !per_proxy && n_gap == 0 && (s->path == 3 || (uint64_t)t.n_proxies * W <= 4ull * nev))
    hipLaunchKernelGGL(k_fcmerge, dim3((uint32_t)hmin((uint64_t)t.n_proxies * W / IT, 8192)), dim3(IT), 0, st,
                       t.n_proxies, S, s->epoch);
  else if (nev && !per_proxy)
    hipLaunchKernelGGL(k_merge, dim3(gv), dim3(IT), 0, st, records, arena, dgram_off, nev, x, S, n_gap > 0);
  if (state_pass) {
    hipLaunchKernelGGL(k_state, dim3(t.n_proxies), dim3(IT), 0, st, t.n_proxies, x, S, have_hb, out->ack_base,
                       out->n_window_overflow);
    far_finish(S, out->ack_base, st);
  }
  return hipGetLastError() == hipSuccess ? RTPS_RX_OK : RTPS_RX_EHIP;
}

int rtps_ingest_batch(IngestState* s, hipStream_t st, const ReaderDev& t, const uint8_t* arena, uint64_t arena_len,
                      const uint64_t* dgram_off, const rtps_record* records, const uint64_t* n_records,
                      uint64_t max_records, const rtps_frag_sample* frag, const uint64_t* n_frag, uint64_t max_frag,
                      uint32_t flags, const rtps_ingest_out* out, const IngestTail* tail) {
  bool queued = false;
  const int rc = ingest_batch(s, st, t, arena, arena_len, dgram_off, records, n_records, max_records, frag, n_frag,
                              max_frag, flags, out, tail, queued);
  if (rc || !tail || queued) return rc;
  return tail->run(tail->ctx, nullptr);
}
