// rtps_shard.hip — the owner-side exchange for >= 2 GPUs (include/rtps_rx.h,
// rtps_rx_shard_*): pack on the source, unpack on the owner.  The RCCL rounds
// between them are in rtps_exchange.cpp.
//
// Why it exists: the reference keeps per-writer state — one FragmentAssembler
// and one RtpsWriterProxy per matched writer (io_uring/rtps/reader.rs:563-758,
// rtps/rtps_writer_proxy.rs:202-355) — and it is only right where every
// submessage of that writer is seen, in order.  With the stream split over N
// GPUs by datagram, that place is the writer's owner GPU.
//
// What crosses per writer record is a 16-B item (rtps_shard_item): a DATA of a writer in the
// owner table's writer list holds everything the owner's ingest reads of it (the writer's list
// index, SN, kind, flags, route, payload kind: "compact"), so it costs 16 B instead of its 64-B
// record; another DATA adds a 32-B blob (GUID, SN); any other kind sends its 64-B record in its
// blob, ahead of the bytes its consumers read.
// Pack (source rank), three launches over the parse output:
//   1. shard_hist    per 256-record tile and destination: items and blob bytes;
//   2. shard_scan    per destination, exclusive scans of both over the tiles
//                    (its records' positions and blob offsets) and the totals;
//   3. shard_scatter every item to its destination's fixed slot when it fits
//                    (position < cap and blob end <= bcap: a prefix of the
//                    destination's items, since both grow with position), else
//                    to the spill at its exact-layout position; the first item
//                    that does not fit sets the cut.  The blobs go
//                    with their records: small ones copied by their lane, long
//                    DATA_FRAG payloads by whole waves (16 B per lane).
// Unpack (owner), with the counts on the host:
//   1. shard_segments one flat copy of the received slots and spills into the
//                    owner's contiguous items and arena (≤ 4 segments / source);
//   2. shard_fix      per item: origin, blob size;
//   3. exclusive sum of the blob sizes (hipCUB) = each blob's arena offset;
//   4. shard_expand   the owner's 64-B records: a DATA's from its item, any other
//                    from the copy in its blob; dgram_idx := record index; dgram_off =
//                    LEAD + blob offset + 64 - the bytes' offset in their datagram, so
//                    the consumers' arena + dgram_off[dgram_idx] + pl_off / bitmap_off
//                    lands on them.
// Blob streams are concatenated in source order, the same order as the
// records, so one global scan gives every blob's place.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <string.h>

#include <algorithm>
#include <new>
#include <vector>

#include "../../include/rtps_rx.h"
#include "rtps_ctx.h"
#include "rtps_readers.h"
#include "rtps_shard.h"

namespace {

constexpr uint32_t ST = 256;   // threads per workgroup, one record each
constexpr uint32_t SW = ST / 64;
constexpr uint32_t SMALL_BLOB = 64;  // blobs up to this many bytes are copied by their own lane
constexpr uint32_t NONE = 0xffffffffu;

__device__ __forceinline__ uint32_t owner_hash(uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
  uint32_t h = 0x811c9dc5u;  // FNV-1a over the writer GUID's four words, then fmix32 (rtps_rx.hip owner_hash)
  h = (h ^ a) * 0x01000193u; h = (h ^ b) * 0x01000193u;
  h = (h ^ c) * 0x01000193u; h = (h ^ d) * 0x01000193u;
  h ^= h >> 16; h *= 0x85ebca6bu;
  h ^= h >> 13; h *= 0xc2b2ae35u;
  return h ^ (h >> 16);
}

// What the owner's consumers read of a record in the arena: (offset in its datagram, bytes)
struct Blob {
  uint32_t rel, len;
};
__device__ __forceinline__ Blob blob_of(const uint32_t* w) {  // w: the record's 16 words
  const uint32_t kind = (w[1] >> 16) & 0xffu;
  if (kind == RTPS_GAP) {  // u.gap: list_base (w10, w11), num_bits (w12), bitmap_off (w13 low)
    const uint32_t nb = w[12];
    return Blob{w[13] & 0xffffu, nb ? 4u * ((nb + 31u) >> 5) : 0u};
  }
  if (kind == RTPS_DATA_FRAG) return Blob{w[10] & 0xffffu, w[10] >> 16};  // u.frag.pl_off, pl_len
  return Blob{0u, 0u};
}
__device__ __forceinline__ uint32_t round16(uint32_t x) { return (x + 15u) & ~15u; }
// blob bytes of an item: none for a compact DATA, 32 for another DATA (GUID, SN), else its record +
// its consumers' bytes
__device__ __forceinline__ uint32_t item_bytes(uint32_t kind, bool compact, const Blob& b) {
  return kind == RTPS_DATA ? (compact ? 0u : 32u) : 64u + round16(b.len);
}

// The writer -> owner table (rtps_rx_shard_set_owners): a writer in it goes to its owner,
// any other by the GUID hash.
// RTPS_OWNER_TOPIC adds entity keys (OWNER_EKEY_PREFIX x 12 || entity id): a writer without a
// proxy whose entity id some reader contains (its records reach that reader's topic cache,
// rt_classify's entity sets) goes to the owner of that entity set's group.
struct OwnerDev {
  const uint32_t* keys;  // nullptr: no table
  const uint32_t* val;   // owner | (writer-list index + 1) << 8
  uint32_t mask;
  uint32_t ent;          // the table has entity keys
};
constexpr uint32_t EKEY_WORD = 0x01010101u * OWNER_EKEY_PREFIX;
__device__ __forceinline__ uint32_t owner_probe(const OwnerDev& t, uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
  uint32_t i = rt_hash16(a, b, c, d) & t.mask;
  for (uint32_t probe = 0; probe <= t.mask; ++probe) {
    const uint32_t v = t.val[i];
    if (v == NONE) break;
    const uint4 k = *reinterpret_cast<const uint4*>(t.keys + 4u * i);
    if (k.x == a && k.y == b && k.z == c && k.w == d) return v;
    i = (i + 1u) & t.mask;
  }
  return NONE;
}
// a writer's owner and its writer-list index (NONE: not in the list)
__device__ __forceinline__ uint32_t owner_of_writer(const OwnerDev& t, uint32_t a, uint32_t b, uint32_t c, uint32_t d,
                                                    uint32_t n_dest, uint32_t& widx) {
  widx = NONE;
  if (t.keys) {
    uint32_t v = owner_probe(t, a, b, c, d);
    if (v != NONE) {
      if (v >> 8) widx = (v >> 8) - 1u;
      return v & 0xffu;
    }
    if (t.ent) v = owner_probe(t, EKEY_WORD, EKEY_WORD, EKEY_WORD, d);
    if (v != NONE) return v & 0xffu;
  }
  return owner_hash(a, b, c, d) % n_dest;
}

// Destination of a record (NONE: not an item), its blob, and whether it crosses as a compact item
// (a DATA of a listed writer whose SN's high word is 0..255)
__device__ __forceinline__ uint32_t item_of(const uint32_t* w, const OwnerDev& ot, uint32_t n_dest, Blob& b,
                                            bool& compact, uint32_t& widx) {
  const uint32_t kind = (w[1] >> 16) & 0xffu;
  const uint32_t route = (w[7] >> 16) & 0xffu;
  const bool writer = kind == RTPS_DATA || kind == RTPS_DATA_FRAG || kind == RTPS_HEARTBEAT || kind == RTPS_GAP ||
                      kind == RTPS_HEARTBEAT_FRAG;
  b = Blob{0u, 0u};
  compact = false;
  widx = NONE;
  if (!writer || !(route & RTPS_ROUTE_PASS)) return NONE;
  b = blob_of(w);
  const uint32_t o = owner_of_writer(ot, w[2], w[3], w[4], w[5], n_dest, widx);
  compact = kind == RTPS_DATA && widx < SHARD_WLIST_MAX && w[9] <= 0xffu;  // (w[9]: the SN's high word)
  return o;
}

__device__ __forceinline__ void load_record(const rtps_record* r, uint32_t* w) {
  const uint4* q = reinterpret_cast<const uint4*>(r);
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint4 v = q[k];
    w[4 * k] = v.x; w[4 * k + 1] = v.y; w[4 * k + 2] = v.z; w[4 * k + 3] = v.w;
  }
}
__device__ __forceinline__ void store_record(rtps_record* r, const uint32_t* w) {
  uint4* q = reinterpret_cast<uint4*>(r);
#pragma unroll
  for (int k = 0; k < 4; ++k) q[k] = make_uint4(w[4 * k], w[4 * k + 1], w[4 * k + 2], w[4 * k + 3]);
}

__device__ __forceinline__ uint4 ld16u(const uint8_t* p) {  // any alignment (one unaligned dwordx4 on gfx950)
  uint4 v;
  __builtin_memcpy(&v, p, 16);
  return v;
}
// chunk [c, c + 16) of a blob of len bytes at src into aligned dst (zero past len); the
// bytes past len are never read, so a blob that ends at the arena's end cannot fault
__device__ __forceinline__ void copy_chunk(const uint8_t* src, uint8_t* dst, uint32_t c, uint32_t len) {
  uint4 v = make_uint4(0, 0, 0, 0);
  if (c + 16u <= len) {
    v = ld16u(src + c);
  } else {
    uint32_t t[4] = {0, 0, 0, 0};
    for (uint32_t k = c; k < len; ++k) t[(k - c) >> 2] |= (uint32_t)src[k] << (8u * ((k - c) & 3u));
    v = make_uint4(t[0], t[1], t[2], t[3]);
  }
  *reinterpret_cast<uint4*>(dst + c) = v;
}

__device__ __forceinline__ uint32_t wave_incl(uint32_t x, uint32_t lane) {
#pragma unroll
  for (uint32_t d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(x, d, 64);
    if (lane >= d) x += y;
  }
  return x;
}
__device__ __forceinline__ uint64_t wave_incl64(uint64_t x, uint32_t lane) {
#pragma unroll
  for (uint32_t d = 1; d < 64; d <<= 1) {
    const uint64_t y = __shfl_up(x, d, 64);
    if (lane >= d) x += y;
  }
  return x;
}

// 1. per tile t and destination d: hist[2 (t n + d)] = items, [+1] = blob bytes
__global__ __launch_bounds__(ST) void shard_hist(const rtps_record* recs, const uint64_t* n_rec, OwnerDev ot,
                                                 uint32_t n_dest, uint32_t* hist) {
  __shared__ uint32_t h[2 * SHARD_MAX_RANKS];
  if (threadIdx.x < 2 * n_dest) h[threadIdx.x] = 0;
  __syncthreads();
  const uint64_t i = (uint64_t)blockIdx.x * ST + threadIdx.x;
  if (i < *n_rec) {
    uint32_t w[16];
    load_record(recs + i, w);
    Blob b;
    bool compact;
    uint32_t widx;
    const uint32_t o = item_of(w, ot, n_dest, b, compact, widx);
    if (o != NONE) {
      atomicAdd(&h[2 * o], 1u);
      const uint32_t ib = item_bytes((w[1] >> 16) & 0xffu, compact, b);
      if (ib) atomicAdd(&h[2 * o + 1], ib);
    }
  }
  __syncthreads();
  if (threadIdx.x < 2 * n_dest) hist[(uint64_t)blockIdx.x * 2 * n_dest + threadIdx.x] = h[threadIdx.x];
}

// 2. one workgroup per destination d: exclusive scans over the tiles -> hscan[2 (t n + d)] =
//    {first position, first blob offset} of tile t's items for d; counts[d] = totals, cut = totals
__global__ __launch_bounds__(ST) void shard_scan(const uint32_t* hist, uint64_t tiles, uint32_t n_dest,
                                                 uint64_t* hscan, rtps_shard_counts* counts) {
  __shared__ uint64_t wsum[2][SW];
  const uint32_t d = blockIdx.x, tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
  uint64_t carry_n = 0, carry_b = 0;
  for (uint64_t t0 = 0; t0 < tiles; t0 += ST) {
    const uint64_t t = t0 + tid;
    const uint64_t vn = t < tiles ? hist[2 * (t * n_dest + d)] : 0u;
    const uint64_t vb = t < tiles ? hist[2 * (t * n_dest + d) + 1] : 0u;
    const uint64_t in = wave_incl64(vn, lane), ib = wave_incl64(vb, lane);
    if (lane == 63) { wsum[0][wave] = in; wsum[1][wave] = ib; }
    __syncthreads();
    uint64_t bn = carry_n, bb = carry_b, tn = carry_n, tb = carry_b;
    for (uint32_t w = 0; w < SW; ++w) {
      if (w < wave) { bn += wsum[0][w]; bb += wsum[1][w]; }
      tn += wsum[0][w]; tb += wsum[1][w];
    }
    if (t < tiles) {
      hscan[2 * (t * n_dest + d)] = bn + in - vn;
      hscan[2 * (t * n_dest + d) + 1] = bb + ib - vb;
    }
    carry_n = tn; carry_b = tb;
    __syncthreads();
  }
  if (tid == 0) counts[d] = rtps_shard_counts{carry_n, carry_b, carry_n, carry_b};
}

struct PackArgs {
  const uint8_t* arena;
  uint64_t arena_len;
  const uint64_t* dgram_off;
  const rtps_record* recs;
  const uint64_t* n_rec;
  OwnerDev ot;
  uint32_t n_dest;
  uint64_t cap, bcap;
  const uint64_t* hscan;
  rtps_shard_counts* counts;
  shard_item* slots;
  uint8_t* blob;
  shard_item* spill;
  uint8_t* bspill;
};

// 3. items to their slots or the spill, with their blobs
__global__ __launch_bounds__(ST) void shard_scatter(PackArgs a) {
  __shared__ uint32_t wcnt[SW][SHARD_MAX_RANKS], wbyt[SW][SHARD_MAX_RANKS];
  __shared__ uint64_t sbase[SHARD_MAX_RANKS], bsbase[SHARD_MAX_RANKS];
  __shared__ uint64_t big_src[ST], big_dst[ST];
  __shared__ uint32_t big_len[ST], n_big;
  const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6, n = a.n_dest;
  if (tid == 0) {
    uint64_t rn = 0, rb = 0;
    for (uint32_t d = 0; d < n; ++d) {
      sbase[d] = rn; bsbase[d] = rb;
      rn += a.counts[d].n; rb += a.counts[d].bytes;
    }
    n_big = 0;
  }
  const uint64_t i = (uint64_t)blockIdx.x * ST + tid;
  uint32_t w[16];
  uint32_t o = NONE, widx = NONE;
  bool compact = false;
  Blob b{0u, 0u};
  if (i < *a.n_rec) {
    load_record(a.recs + i, w);
    o = item_of(w, a.ot, n, b, compact, widx);
  }
  const uint32_t kind = o != NONE ? (w[1] >> 16) & 0xffu : 0u;
  const uint32_t size = o != NONE ? item_bytes(kind, compact, b) : 0u;
  uint32_t rank = 0, bex = 0;
  const uint64_t lt = lane ? (~0ull >> (64u - lane)) : 0ull;
  for (uint32_t d = 0; d < n; ++d) {
    const uint64_t m = __ballot(o == d);
    if (m == 0) {
      if (lane == 0) { wcnt[wave][d] = 0; wbyt[wave][d] = 0; }
      continue;
    }
    const uint32_t v = o == d ? size : 0u;
    const uint32_t incl = wave_incl(v, lane);
    if (o == d) { rank = (uint32_t)__popcll(m & lt); bex = incl - v; }
    if (lane == 63) { wcnt[wave][d] = (uint32_t)__popcll(m); wbyt[wave][d] = incl; }
  }
  __syncthreads();
  uint64_t pos = 0, boff = 0;
  bool slot = true;
  if (o != NONE) {
    pos = a.hscan[2 * ((uint64_t)blockIdx.x * n + o)] + rank;
    boff = a.hscan[2 * ((uint64_t)blockIdx.x * n + o) + 1] + bex;
    for (uint32_t v = 0; v < wave; ++v) { pos += wcnt[v][o]; boff += wbyt[v][o]; }
    slot = pos < a.cap && boff + size <= a.bcap;
  }
  // each destination's cut: its first item that does not fit (both position and blob end grow
  // with the position, so the items that fit are a prefix).  That item is the one whose
  // predecessor fit (position - 1 < cap, its blob ending at this one's start <= bcap): a single
  // writer per destination, no atomics (the scan set cut = n for a destination that all fits)
  if (o != NONE && !slot && (pos == 0 || (pos - 1u < a.cap && boff <= a.bcap))) {
    a.counts[o].cut = pos;
    a.counts[o].cut_bytes = boff;
  }
  if (o != NONE) {
    shard_item* it = slot ? a.slots + (uint64_t)o * a.cap + pos : a.spill + sbase[o] + pos;
    uint8_t* bd = slot ? a.blob + (uint64_t)o * a.bcap + boff : a.bspill + bsbase[o] + boff;
    const uint32_t tail = kind | (w[1] & 0xff000000u) >> 16 | (w[7] & 0xffff0000u);  // kind, flags, route, pk
    uint4* q = reinterpret_cast<uint4*>(it);
    if (compact) {
      *q = make_uint4(RTPS_SHARD_COMPACT | widx << 4 | w[9] << 24, (uint32_t)i, w[8], tail);
    } else if (kind == RTPS_DATA) {  // its GUID and SN in a 32-B blob
      *q = make_uint4(size, (uint32_t)i, 0u, tail);
      uint4* bq = reinterpret_cast<uint4*>(bd);
      bq[0] = make_uint4(w[2], w[3], w[4], w[5]);
      bq[1] = make_uint4(w[8], w[9], 0u, 0u);
    } else {
      *q = make_uint4(size, (uint32_t)i, 0u, tail);
      const uint32_t didx = w[0];
      w[0] = (uint32_t)i;  // the record's copy names its source record
      store_record(reinterpret_cast<rtps_record*>(bd), w);
      bd += 64;
      if (b.len) {
        const uint8_t* src = a.arena + a.dgram_off[didx] + b.rel;
        if (round16(b.len) <= SMALL_BLOB) {
          for (uint32_t c = 0; c < round16(b.len); c += 16u) copy_chunk(src, bd, c, b.len);
        } else {
          const uint32_t k = atomicAdd(&n_big, 1u);
          big_src[k] = (uint64_t)(uintptr_t)src;
          big_dst[k] = (uint64_t)(uintptr_t)bd;
          big_len[k] = b.len;
        }
      }
    }
  }
  __syncthreads();
  // long blobs (DATA_FRAG payloads): one wave per blob, 16 B per lane per step
  for (uint32_t k = wave; k < n_big; k += SW) {
    const uint8_t* src = (const uint8_t*)(uintptr_t)big_src[k];
    uint8_t* dst = (uint8_t*)(uintptr_t)big_dst[k];
    const uint32_t len = big_len[k], sz = round16(len);
    for (uint32_t c = 16u * lane; c < sz; c += 1024u) copy_chunk(src, dst, c, len);
  }
}

// ---- unpack ----
struct Seg {  // one contiguous copy: 16-B chunks [c0, c0 + nc) of the flat chunk space
  uint64_t src, dst, c0, nc;
};
struct SegArgs {
  const rtps_shard_counts* counts;  // [n_src] received counts (device)
  uint32_t n_src;
  uint64_t cap, bcap;
  const shard_item* r_slots;
  const uint8_t* r_blob;
  const shard_item* r_spill;
  const uint8_t* r_bspill;
  shard_item* o_item;
  uint8_t* o_blob;  // owner arena + RTPS_SHARD_LEAD
};
// Per source: its slot records, its spilled records, its slot blob bytes, its spilled
// bytes, each one contiguous copy.  Every workgroup builds the (<= 4 x 64 entry)
// table from the device counts, so no host staging is involved.
__global__ __launch_bounds__(ST) void shard_segments(SegArgs a) {
  __shared__ Seg seg[4 * SHARD_MAX_RANKS];
  __shared__ uint32_t n_seg;
  __shared__ uint64_t total;
  if (threadIdx.x == 0) {
    uint32_t ns = 0;
    uint64_t chunks = 0, rpos = 0, bpos = 0, rsp = 0, bsp = 0;
    auto add = [&](const void* src, void* dst, uint64_t nbytes) {
      if (!nbytes) return;
      seg[ns++] = Seg{(uint64_t)(uintptr_t)src, (uint64_t)(uintptr_t)dst, chunks, nbytes / 16};
      chunks += nbytes / 16;
    };
    for (uint32_t k = 0; k < a.n_src; ++k) {
      const rtps_shard_counts c = a.counts[k];
      add(a.r_slots + (uint64_t)k * a.cap, a.o_item + rpos, c.cut * sizeof(shard_item));
      add(a.r_spill + rsp, a.o_item + rpos + c.cut, (c.n - c.cut) * sizeof(shard_item));
      add(a.r_blob + (uint64_t)k * a.bcap, a.o_blob + bpos, c.cut_bytes);
      add(a.r_bspill + bsp, a.o_blob + bpos + c.cut_bytes, c.bytes - c.cut_bytes);
      rpos += c.n;
      bpos += c.bytes;
      rsp += c.n - c.cut;
      bsp += c.bytes - c.cut_bytes;
    }
    n_seg = ns;
    total = chunks;
  }
  __syncthreads();
  const uint64_t stride = (uint64_t)gridDim.x * ST;
  for (uint64_t c = (uint64_t)blockIdx.x * ST + threadIdx.x; c < total; c += stride) {
    uint32_t lo = 0, hi = n_seg;  // last segment with c0 <= c
    while (hi - lo > 1) {
      const uint32_t mid = (lo + hi) >> 1;
      if (seg[mid].c0 <= c) lo = mid; else hi = mid;
    }
    const Seg sg = seg[lo];
    const uint64_t k = c - sg.c0;
    const uint4* src = reinterpret_cast<const uint4*>((uintptr_t)sg.src) + k;
    uint4* dst = reinterpret_cast<uint4*>((uintptr_t)sg.dst) + k;
    *dst = *src;
  }
}

struct FixArgs {
  const shard_item* item;
  uint64_t* origin;
  uint64_t* size;
  uint64_t n;
  uint32_t n_src;
  uint64_t first[SHARD_MAX_RANKS + 1];  // owner record index of source s's first record
};
__global__ __launch_bounds__(ST) void shard_fix(FixArgs a) {
  const uint64_t j = (uint64_t)blockIdx.x * ST + threadIdx.x;
  if (j >= a.n) return;
  uint32_t s = 0;
  while (s + 1 < a.n_src && a.first[s + 1] <= j) ++s;
  const uint4 q = *reinterpret_cast<const uint4*>(a.item + j);
  a.origin[j] = ((uint64_t)s << 32) | q.y;                        // src_rec
  a.size[j] = (q.x & 0xfu) == RTPS_SHARD_COMPACT ? 0u : q.x;  // the blob bytes (none for a compact DATA)
}
// the owner's records: a DATA's from its item, the others' from the copy in their blob
__global__ __launch_bounds__(ST) void shard_expand(const shard_item* item, const uint8_t* arena, const uint64_t* boff,
                                                   const uint32_t* wlist, rtps_record* rec, uint64_t* off, uint64_t n) {
  const uint64_t j = (uint64_t)blockIdx.x * ST + threadIdx.x;
  if (j >= n) return;
  const uint4 q = *reinterpret_cast<const uint4*>(item + j);
  const uint32_t kind = q.w & 0xffu;
  uint32_t w[16];
  if (kind == RTPS_DATA) {
    for (int k = 0; k < 16; ++k) w[k] = 0u;
    w[1] = (kind << 16) | ((q.w >> 8) & 0xffu) << 24;  // sub_off 0, kind, flags
    w[7] = q.w & 0xffff0000u;                          // route, payload_kind
    if ((q.x & 0xfu) == RTPS_SHARD_COMPACT) {          // the writer from the list
      const uint4 g = *reinterpret_cast<const uint4*>(wlist + 4u * ((q.x >> 4) & (SHARD_WLIST_MAX - 1u)));
      w[2] = g.x; w[3] = g.y; w[4] = g.z; w[5] = g.w;
      w[8] = q.z; w[9] = q.x >> 24;                    // sn
    } else {                                           // from its blob
      const uint4* bq = reinterpret_cast<const uint4*>(arena + RTPS_SHARD_LEAD + boff[j]);
      const uint4 g = bq[0], sn = bq[1];
      w[2] = g.x; w[3] = g.y; w[4] = g.z; w[5] = g.w;
      w[8] = sn.x; w[9] = sn.y;
    }
    off[j] = RTPS_SHARD_LEAD;                          // (no payload bytes in the owner arena)
  } else {
    load_record(reinterpret_cast<const rtps_record*>(arena + RTPS_SHARD_LEAD + boff[j]), w);
    off[j] = RTPS_SHARD_LEAD + boff[j] + 64u - blob_of(w).rel;
  }
  w[0] = (uint32_t)j;
  store_record(rec + j, w);
}

__global__ void shard_set_n(uint64_t* p, uint64_t v) { *p = v; }

int hip_rc(hipError_t e) { return e == hipSuccess ? RTPS_RX_OK : RTPS_RX_EHIP; }

}  // namespace

bool shard_reserve(void** p, uint64_t* cap, uint64_t need) {
  if (*p && need <= *cap) return true;
  if (*p) (void)hipFree(*p);
  *p = nullptr;
  *cap = 0;
  if (hipMalloc(p, need ? need : 16) != hipSuccess) {
    *p = nullptr;
    return false;
  }
  *cap = need;
  return true;
}

extern "C" {

int rtps_rx_shard_create(rtps_rx_ctx* ctx, uint32_t n_ranks, uint64_t cap, uint64_t bcap, rtps_shard** out) {
  if (!ctx || !out || n_ranks < 1 || n_ranks > SHARD_MAX_RANKS || cap == 0 || (bcap & 15u)) return RTPS_RX_EINVAL;
  rtps_shard* s = new (std::nothrow) rtps_shard();
  if (!s) return RTPS_RX_ENOMEM;
  s->ctx = ctx;
  s->device = rtps_ctx_device(ctx);
  s->n_ranks = n_ranks;
  s->cap = cap;
  s->bcap = bcap;
  (void)hipSetDevice(s->device);
  const size_t slots = (size_t)n_ranks * cap * sizeof(shard_item), blobs = (size_t)n_ranks * bcap;
  bool ok = hipMalloc(&s->s_slots, slots) == hipSuccess && hipMalloc(&s->r_slots, slots) == hipSuccess &&
            hipMalloc(&s->s_blob, blobs ? blobs : 16) == hipSuccess &&
            hipMalloc(&s->r_blob, blobs ? blobs : 16) == hipSuccess &&
            hipMalloc(&s->s_counts, n_ranks * sizeof(rtps_shard_counts)) == hipSuccess &&
            hipMalloc(&s->r_counts, n_ranks * sizeof(rtps_shard_counts)) == hipSuccess &&
            hipMemset(s->r_counts, 0, n_ranks * sizeof(rtps_shard_counts)) == hipSuccess &&
            hipMemset(s->s_counts, 0, n_ranks * sizeof(rtps_shard_counts)) == hipSuccess &&
            hipHostMalloc(&s->h_send, n_ranks * sizeof(rtps_shard_counts), hipHostMallocDefault) == hipSuccess &&
            hipHostMalloc(&s->h_recv, n_ranks * sizeof(rtps_shard_counts), hipHostMallocDefault) == hipSuccess &&
            hipMalloc(&s->o_n, sizeof(uint64_t)) == hipSuccess &&
            hipMemset(s->o_n, 0, sizeof(uint64_t)) == hipSuccess &&
            hipEventCreateWithFlags(&s->packed, hipEventDisableTiming) == hipSuccess &&
            hipEventCreateWithFlags(&s->counts_ev, hipEventDisableTiming) == hipSuccess &&
            hipEventCreateWithFlags(&s->done, hipEventDisableTiming) == hipSuccess;
  if (!ok) {
    rtps_rx_shard_destroy(s);
    return RTPS_RX_ENOMEM;
  }
  rtps_ctx_shard_attach(ctx, s, true);
  *out = s;
  return RTPS_RX_OK;
}

int rtps_rx_shard_destroy(rtps_shard* s) {
  if (!s) return RTPS_RX_EINVAL;
  rtps_ctx_shard_attach(s->ctx, s, false);
  (void)hipSetDevice(s->device);
  (void)hipDeviceSynchronize();
  void* dev[] = {s->s_slots, s->s_blob, s->s_counts, s->s_spill, s->s_bspill, s->hist, s->hscan, s->r_slots,
                 s->r_blob, s->r_counts, s->r_spill, s->r_bspill, s->o_rec, s->o_off, s->o_origin, s->o_size,
                 s->o_boff, s->o_arena, s->o_n, s->cub_tmp, s->o_item, s->d_okeys, s->d_oval, s->d_wlist};
  for (void* p : dev)
    if (p) (void)hipFree(p);
  if (s->h_send) (void)hipHostFree(s->h_send);
  if (s->h_recv) (void)hipHostFree(s->h_recv);
  hipEvent_t ev[] = {s->packed, s->counts_ev, s->done};
  for (hipEvent_t e : ev)
    if (e) (void)hipEventDestroy(e);
  delete s;
  return RTPS_RX_OK;
}

int rtps_rx_owner_assign_sticky(const uint8_t* writers, const uint64_t* weights, const uint32_t* groups, uint32_t n,
                                uint32_t n_ranks, const int32_t* prev, uint32_t* owners) {
  if ((n && (!writers || !owners)) || n_ranks < 1) return RTPS_RX_EINVAL;
  for (uint32_t w = 0; w < n; ++w)
    if ((groups && groups[w] >= n) || (prev && prev[w] >= (int32_t)n_ranks)) return RTPS_RX_EINVAL;
  // groups: total weight, smallest member GUID (the tie-break that makes the deal order-free)
  std::vector<uint32_t> gid(n), rep;  // writer -> dense group, group -> its smallest-GUID writer
  std::vector<uint64_t> gw;
  std::vector<uint32_t> dense(n, NONE);
  for (uint32_t w = 0; w < n; ++w) {
    const uint32_t g = groups ? groups[w] : w;
    if (dense[g] == NONE) { dense[g] = (uint32_t)rep.size(); rep.push_back(w); gw.push_back(0); }
    const uint32_t k = dense[g];
    gid[w] = k;
    gw[k] += weights ? weights[w] : 1u;
    if (memcmp(writers + 16ull * w, writers + 16ull * rep[k], 16) < 0) rep[k] = w;
  }
  std::vector<uint64_t> load(n_ranks, 0);
  std::vector<uint32_t> owner_of(rep.size(), NONE);
  if (prev) {  // sticky: a group with owned members stays where most of its weight is (ties: lowest rank)
    std::vector<uint64_t> held((size_t)rep.size() * n_ranks, 0);
    std::vector<uint8_t> any(rep.size(), 0);
    for (uint32_t w = 0; w < n; ++w)
      if (prev[w] >= 0) {
        held[(size_t)gid[w] * n_ranks + (uint32_t)prev[w]] += (weights ? weights[w] : 1u) + 1u;
        any[gid[w]] = 1;
      }
    for (uint32_t k = 0; k < rep.size(); ++k) {
      if (!any[k]) continue;
      uint32_t best = 0;
      for (uint32_t r = 1; r < n_ranks; ++r)
        if (held[(size_t)k * n_ranks + r] > held[(size_t)k * n_ranks + best]) best = r;
      owner_of[k] = best;
      load[best] += gw[k];
    }
  }
  std::vector<uint32_t> order;
  for (uint32_t k = 0; k < rep.size(); ++k)
    if (owner_of[k] == NONE) order.push_back(k);
  std::sort(order.begin(), order.end(), [&](uint32_t x, uint32_t y) {
    if (gw[x] != gw[y]) return gw[x] > gw[y];
    return memcmp(writers + 16ull * rep[x], writers + 16ull * rep[y], 16) < 0;
  });
  // the new groups: largest first, each to the least-loaded owner (ties: the lowest rank)
  for (uint32_t k : order) {
    uint32_t best = 0;
    for (uint32_t r = 1; r < n_ranks; ++r)
      if (load[r] < load[best]) best = r;
    owner_of[k] = best;
    load[best] += gw[k];
  }
  for (uint32_t w = 0; w < n; ++w) owners[w] = owner_of[gid[w]];
  return RTPS_RX_OK;
}

int rtps_rx_owner_assign(const uint8_t* writers, const uint64_t* weights, const uint32_t* groups, uint32_t n,
                         uint32_t n_ranks, uint32_t* owners) {
  return rtps_rx_owner_assign_sticky(writers, weights, groups, n, n_ranks, nullptr, owners);
}

}  // extern "C"

// the mode the table follows: the caller's, else RTPS_OWNER_TOPIC once the context has topics
// (the topic caches' GC needs every writer of a topic on one owner), else RTPS_OWNER_BALANCED
static uint32_t effective_mode(const rtps_shard* s) {
  if (s->mode_explicit) return s->owner_mode;
  return rtps_ctx_topics_configured(s->ctx) ? RTPS_OWNER_TOPIC : RTPS_OWNER_BALANCED;
}
static bool owner_stale(const rtps_shard* s) {
  const uint32_t m = effective_mode(s);
  return m != s->t_mode || (m != RTPS_OWNER_HASH && s->owner_version != rtps_ctx_readers_version(s->ctx));
}
bool rtps_shard_splits_topics(const rtps_shard* s) { return s->n_ranks > 1 && effective_mode(s) != RTPS_OWNER_TOPIC; }

// The owner table for the context's current readers (and topics) and the caller's writers.
// Sticky: a key the previous table (same mode) held keeps its owner, so that its writer
// proxy, far set, DataFrag assemblies and topic-cache changes stay where they are; new keys
// are dealt onto the ranks' loads.  Only a group that joins keys of different owners (a topic
// linking them, RTPS_OWNER_TOPIC) moves some, to where most of its weight already is.
static int owner_table_compute(const rtps_shard* s, bool fresh, std::vector<uint8_t>& g, std::vector<uint32_t>& own,
                               bool& ent) {
  const uint32_t mode = effective_mode(s);
  g.clear();
  own.clear();
  ent = false;
  if (mode == RTPS_OWNER_HASH) return RTPS_RX_OK;
  std::vector<uint32_t> grp;
  rtps_ctx_owner_keys(s->ctx, mode == RTPS_OWNER_TOPIC, g, grp);
  ent = mode == RTPS_OWNER_TOPIC;
  std::vector<uint64_t> wt(grp.size(), 1u);
  for (size_t x = 0; x < s->x_weight.size(); ++x) {  // the caller's writers: weight known ones, add the rest
    const uint8_t* q = s->x_guid.data() + 16 * x;
    size_t w = 0;
    while (w < grp.size() && memcmp(g.data() + 16 * w, q, 16) != 0) ++w;
    if (w == grp.size()) {
      g.insert(g.end(), q, q + 16);
      grp.push_back((uint32_t)w);
      wt.push_back(0);
    }
    wt[w] = s->x_weight[x];
  }
  std::vector<int32_t> prev(grp.size(), -1);
  if (!fresh && mode == s->t_mode)
    for (size_t w = 0; w < grp.size(); ++w)
      for (size_t k = 0; k < s->t_owner.size(); ++k)
        if (memcmp(g.data() + 16 * w, s->t_guid.data() + 16 * k, 16) == 0) { prev[w] = (int32_t)s->t_owner[k]; break; }
  own.resize(grp.size());
  return rtps_rx_owner_assign_sticky(g.data(), wt.data(), grp.data(), (uint32_t)grp.size(), s->n_ranks, prev.data(),
                                     own.data());
}

// (re)build the owner table and upload it
static int owner_table_build(rtps_shard* s, bool fresh) {
  std::vector<uint8_t> g;
  std::vector<uint32_t> own;
  bool ent = false;
  const int rc = owner_table_compute(s, fresh, g, own, ent);
  if (rc) return rc;
  s->owner_version = rtps_ctx_readers_version(s->ctx);
  s->t_mode = effective_mode(s);
  s->t_guid.swap(g);
  s->t_owner.swap(own);
  s->t_ent = ent;
  const uint32_t n = (uint32_t)s->t_owner.size();
  uint32_t cap = 0;
  if (n) {
    cap = 16;
    while (cap < 4ull * n) cap <<= 1;
  }
  // the writer list (compact DATA items name their writer by its index): the table's writer GUIDs
  // (not the entity keys) in ascending byte order, the same on every rank that builds this table
  std::vector<uint32_t> wl;
  for (uint32_t w = 0; w < n; ++w) {
    const uint8_t* g = s->t_guid.data() + 16ull * w;
    bool ekey = true;
    for (int b = 0; b < 12; ++b) ekey = ekey && g[b] == OWNER_EKEY_PREFIX;
    if (!ekey) wl.push_back(w);
  }
  std::sort(wl.begin(), wl.end(), [&](uint32_t x, uint32_t y) {
    return memcmp(s->t_guid.data() + 16ull * x, s->t_guid.data() + 16ull * y, 16) < 0;
  });
  std::vector<uint32_t> widx(n, NONE), wlist(4ull * wl.size());
  for (size_t r = 0; r < wl.size(); ++r) {
    widx[wl[r]] = (uint32_t)r;
    memcpy(&wlist[4 * r], s->t_guid.data() + 16ull * wl[r], 16);
  }
  std::vector<uint32_t> keys(4ull * cap, 0u), val(cap, NONE);
  for (uint32_t w = 0; w < n; ++w) {
    uint32_t k[4];
    memcpy(k, s->t_guid.data() + 16ull * w, 16);
    uint32_t i = rt_hash16(k[0], k[1], k[2], k[3]) & (cap - 1);
    while (val[i] != NONE) i = (i + 1) & (cap - 1);
    memcpy(&keys[4ull * i], k, 16);
    // owner | (list index + 1) << 8; writers past the compact items' reach keep 0 (never compact)
    val[i] = s->t_owner[w] | (widx[w] < SHARD_WLIST_MAX ? (widx[w] + 1u) << 8 : 0u);
  }
  hipStream_t st = rtps_ctx_stream(s->ctx);
  if (hipStreamSynchronize(st) != hipSuccess) return RTPS_RX_EHIP;  // an earlier pack may read the old table
  if (cap > s->ocap) {
    (void)hipFree(s->d_okeys);
    (void)hipFree(s->d_oval);
    s->d_okeys = nullptr;
    s->d_oval = nullptr;
    s->ocap = 0;
    if (hipMalloc(&s->d_okeys, 16ull * cap) != hipSuccess || hipMalloc(&s->d_oval, 4ull * cap) != hipSuccess)
      return RTPS_RX_ENOMEM;
  }
  s->ocap = cap;
  if (cap && (hipMemcpy(s->d_okeys, keys.data(), 16ull * cap, hipMemcpyHostToDevice) != hipSuccess ||
              hipMemcpy(s->d_oval, val.data(), 4ull * cap, hipMemcpyHostToDevice) != hipSuccess))
    return RTPS_RX_EHIP;
  const uint32_t nw = (uint32_t)wl.size();
  if (nw > s->wlist_cap) {
    (void)hipFree(s->d_wlist);
    s->d_wlist = nullptr;
    s->wlist_cap = 0;
    if (hipMalloc(&s->d_wlist, 16ull * nw) != hipSuccess) return RTPS_RX_ENOMEM;
    s->wlist_cap = nw;
  }
  s->n_wlist = nw;
  if (nw && hipMemcpy(s->d_wlist, wlist.data(), 16ull * nw, hipMemcpyHostToDevice) != hipSuccess) return RTPS_RX_EHIP;
  return RTPS_RX_OK;
}

extern "C" {

int rtps_rx_shard_set_owners(rtps_shard* s, uint32_t mode, const uint8_t* guids, const uint64_t* weights,
                             uint32_t n) {
  if (!s || mode > RTPS_OWNER_TOPIC || (n && (!guids || !weights))) return RTPS_RX_EINVAL;
  (void)hipSetDevice(s->device);
  s->owner_mode = mode;
  s->mode_explicit = true;
  s->x_guid.assign(guids, guids + 16ull * n);
  s->x_weight.assign(weights, weights + n);
  return owner_table_build(s, true);  // an explicit deal starts afresh (documented: moved writers' state stays behind)
}

int rtps_rx_shard_owner(rtps_shard* s, const uint8_t guid[16]) {
  if (!s || !guid) return RTPS_RX_EINVAL;
  // a stale table is answered from the table the next pack will build, without committing it,
  // so that a query never changes the deal's history (every rank must build the same tables)
  std::vector<uint8_t> tg;
  std::vector<uint32_t> to;
  bool ent = s->t_ent;
  const std::vector<uint8_t>* g = &s->t_guid;
  const std::vector<uint32_t>* o = &s->t_owner;
  if (owner_stale(s)) {
    const int rc = owner_table_compute(s, false, tg, to, ent);
    if (rc) return rc;
    g = &tg;
    o = &to;
  }
  for (int pass = 0; pass < (ent ? 2 : 1); ++pass) {
    uint8_t key[16];
    memcpy(key, guid, 16);
    if (pass) memset(key, OWNER_EKEY_PREFIX, 12);
    for (size_t w = 0; w < o->size(); ++w)
      if (memcmp(g->data() + 16 * w, key, 16) == 0) return (int)(*o)[w];
  }
  uint32_t k[4];
  memcpy(k, guid, 16);
  uint32_t h = 0x811c9dc5u;  // owner_hash on the host
  for (int j = 0; j < 4; ++j) h = (h ^ k[j]) * 0x01000193u;
  h ^= h >> 16; h *= 0x85ebca6bu;
  h ^= h >> 13; h *= 0xc2b2ae35u;
  h ^= h >> 16;
  return (int)(h % s->n_ranks);
}

int rtps_rx_shard_pack(rtps_shard* s, const uint8_t* arena, uint64_t arena_len, const uint64_t* dgram_off,
                       const rtps_record* records, const uint64_t* n_records, uint64_t max_records) {
  if (!s || !records || !n_records || (max_records && (!arena || !dgram_off))) return RTPS_RX_EINVAL;
  (void)hipSetDevice(s->device);
  hipStream_t st = rtps_ctx_stream(s->ctx);
  if (owner_stale(s)) {
    const int rc = owner_table_build(s, false);  // the readers (or topics) changed: the table follows them
    if (rc) return rc;
  }
  const OwnerDev ot{s->ocap ? s->d_okeys : nullptr, s->d_oval, s->ocap ? s->ocap - 1u : 0u, s->t_ent ? 1u : 0u};
  const uint32_t n = s->n_ranks;
  const uint64_t tiles = (max_records + ST - 1) / ST;
  if (tiles > 0xffffffffull) return RTPS_RX_ETOOBIG;
  if (tiles > s->hist_tiles) {
    if (hipStreamSynchronize(st) != hipSuccess) return RTPS_RX_EHIP;  // the last pack may still use them
    uint64_t c1 = 0, c2 = 0;
    (void)hipFree(s->hist); (void)hipFree(s->hscan);
    s->hist = nullptr; s->hscan = nullptr; s->hist_tiles = 0;
    if (!shard_reserve((void**)&s->hist, &c1, tiles * n * 2 * sizeof(uint32_t)) ||
        !shard_reserve((void**)&s->hscan, &c2, tiles * n * 2 * sizeof(uint64_t)))
      return RTPS_RX_ENOMEM;
    s->hist_tiles = tiles;
  }
  // the spill holds every item in the worst case: all records, and blobs that are a
  // record copy plus disjoint byte ranges of the arena plus < 16 B of rounding each
  const uint64_t need_rec = max_records * sizeof(shard_item), need_b = arena_len + 80ull * max_records;
  if (need_rec > s->s_spill_cap * sizeof(shard_item) || need_b > s->s_bspill_cap) {
    if (hipStreamSynchronize(st) != hipSuccess) return RTPS_RX_EHIP;
    uint64_t cap_bytes = s->s_spill_cap * sizeof(shard_item);
    if (!shard_reserve((void**)&s->s_spill, &cap_bytes, need_rec)) return RTPS_RX_ENOMEM;
    s->s_spill_cap = cap_bytes / sizeof(shard_item);
    if (!shard_reserve((void**)&s->s_bspill, &s->s_bspill_cap, need_b)) return RTPS_RX_ENOMEM;
  }
  if (tiles == 0) {
    if (hipMemsetAsync(s->s_counts, 0, n * sizeof(rtps_shard_counts), st) != hipSuccess) return RTPS_RX_EHIP;
  } else {
    hipLaunchKernelGGL(shard_hist, dim3((uint32_t)tiles), dim3(ST), 0, st, records, n_records, ot, n, s->hist);
    hipLaunchKernelGGL(shard_scan, dim3(n), dim3(ST), 0, st, s->hist, tiles, n, s->hscan, s->s_counts);
    PackArgs a{arena, arena_len, dgram_off, records, n_records, ot, n, s->cap, s->bcap, s->hscan, s->s_counts,
               s->s_slots, s->s_blob, s->s_spill, s->s_bspill};
    hipLaunchKernelGGL(shard_scatter, dim3((uint32_t)tiles), dim3(ST), 0, st, a);
  }
  if (hipGetLastError() != hipSuccess) return RTPS_RX_EHIP;
  s->exchanged = false;
  s->finished = false;
  return hip_rc(hipEventRecord(s->packed, st));
}

int rtps_rx_shard_buffers(rtps_shard* s, rtps_shard_buffers* o) {
  if (!s || !o) return RTPS_RX_EINVAL;
  o->send_slots = s->s_slots; o->send_blob = s->s_blob; o->send_counts = s->s_counts;
  o->recv_slots = s->r_slots; o->recv_blob = s->r_blob; o->recv_counts = s->r_counts;
  o->send_spill = s->s_spill; o->send_blob_spill = s->s_bspill;
  o->recv_spill = s->r_spill; o->recv_blob_spill = s->r_bspill;
  o->recv_spill_cap = s->r_spill_cap;
  o->recv_blob_spill_cap = s->r_bspill_cap;
  return RTPS_RX_OK;
}

int rtps_rx_shard_reserve_spill(rtps_shard* s, uint64_t records, uint64_t bytes) {
  if (!s) return RTPS_RX_EINVAL;
  (void)hipSetDevice(s->device);
  if (records > s->r_spill_cap || bytes > s->r_bspill_cap) {
    if (hipDeviceSynchronize() != hipSuccess) return RTPS_RX_EHIP;  // an unpack may still read the old ones
    uint64_t cap_bytes = s->r_spill_cap * sizeof(shard_item);
    if (records > s->r_spill_cap) {
      if (!shard_reserve((void**)&s->r_spill, &cap_bytes, records * sizeof(shard_item))) return RTPS_RX_ENOMEM;
      s->r_spill_cap = cap_bytes / sizeof(shard_item);
    }
    if (bytes > s->r_bspill_cap && !shard_reserve((void**)&s->r_bspill, &s->r_bspill_cap, bytes))
      return RTPS_RX_ENOMEM;
  }
  return RTPS_RX_OK;
}

int rtps_rx_shard_unpack(rtps_shard* s, rtps_owner_batch* out) {
  if (!s || !out) return RTPS_RX_EINVAL;
  (void)hipSetDevice(s->device);
  hipStream_t st = rtps_ctx_stream(s->ctx);
  const uint32_t n = s->n_ranks;
  // the received counts: the RCCL rounds left them in pinned memory (no sync beyond
  // round 0's counts); after a host-driven transport they are read from the device
  if (s->exchanged) {
    if (hipEventSynchronize(s->counts_ev) != hipSuccess || hipStreamWaitEvent(st, s->done, 0) != hipSuccess)
      return RTPS_RX_EHIP;
  } else if (hipMemcpyAsync(s->h_recv, s->r_counts, n * sizeof(rtps_shard_counts), hipMemcpyDeviceToHost, st) !=
                 hipSuccess ||
             hipStreamSynchronize(st) != hipSuccess) {
    return RTPS_RX_EHIP;
  }
  uint64_t total = 0, bytes = 0, sp = 0, bsp = 0;
  FixArgs fa;
  memset(&fa, 0, sizeof fa);
  for (uint32_t k = 0; k < n; ++k) {
    const rtps_shard_counts& c = s->h_recv[k];
    if (c.cut > c.n || c.cut_bytes > c.bytes || c.cut > s->cap || c.cut_bytes > s->bcap || (c.bytes & 15u))
      return RTPS_RX_EINVAL;  // not counts this protocol wrote
    fa.first[k] = total;
    total += c.n;
    bytes += c.bytes;
    sp += c.n - c.cut;
    bsp += c.bytes - c.cut_bytes;
  }
  fa.first[n] = total;
  if (sp > s->r_spill_cap || bsp > s->r_bspill_cap) return RTPS_RX_ETOOBIG;  // spill not received
  // after RCCL round 0, a spill is in the spill buffers only once rtps_rx_shard_finish moved it
  // (otherwise they may still hold an earlier batch's)
  if (s->exchanged && !s->finished && (sp || bsp)) return RTPS_RX_EINVAL;
  if (total > s->o_cap) {
    uint64_t c[6] = {0, 0, 0, 0, 0, 0};
    void** p[6] = {(void**)&s->o_rec, (void**)&s->o_off, (void**)&s->o_origin, (void**)&s->o_size,
                   (void**)&s->o_boff, (void**)&s->o_item};
    const size_t b[6] = {sizeof(rtps_record), 8, 8, 8, 8, sizeof(shard_item)};
    for (int k = 0; k < 6; ++k) {
      (void)hipFree(*p[k]);
      *p[k] = nullptr;
    }
    s->o_cap = 0;
    for (int k = 0; k < 6; ++k)
      if (!shard_reserve(p[k], &c[k], total * b[k])) return RTPS_RX_ENOMEM;
    s->o_cap = total;
  }
  const uint64_t arena_need = RTPS_SHARD_LEAD + bytes;
  if (arena_need > s->o_arena_cap) {
    if (!shard_reserve((void**)&s->o_arena, &s->o_arena_cap, arena_need) ||
        hipMemset(s->o_arena, 0, RTPS_SHARD_LEAD) != hipSuccess)
      return RTPS_RX_ENOMEM;
  }
  {
    SegArgs sa{s->r_counts, n, s->cap, s->bcap, s->r_slots, s->r_blob, s->r_spill, s->r_bspill, s->o_item,
               s->o_arena + RTPS_SHARD_LEAD};
    const uint64_t chunks = (total * sizeof(shard_item) + bytes) / 16;
    const uint64_t blocks = (chunks + ST - 1) / ST;
    if (chunks)
      hipLaunchKernelGGL(shard_segments, dim3((uint32_t)(blocks < 16384 ? blocks : 16384)), dim3(ST), 0, st, sa);
  }
  if (total) {
    fa.item = s->o_item; fa.origin = s->o_origin; fa.size = s->o_size; fa.n = total; fa.n_src = n;
    const uint32_t g = (uint32_t)((total + ST - 1) / ST);
    hipLaunchKernelGGL(shard_fix, dim3(g), dim3(ST), 0, st, fa);
    size_t tb = 0;
    if (hipcub::DeviceScan::ExclusiveSum(nullptr, tb, s->o_size, s->o_boff, (int64_t)total, st) != hipSuccess)
      return RTPS_RX_EHIP;
    if (tb > s->cub_bytes) {
      uint64_t cb = s->cub_bytes;
      if (!shard_reserve(&s->cub_tmp, &cb, tb)) return RTPS_RX_ENOMEM;
      s->cub_bytes = cb;
    }
    if (hipcub::DeviceScan::ExclusiveSum(s->cub_tmp, tb, s->o_size, s->o_boff, (int64_t)total, st) != hipSuccess)
      return RTPS_RX_EHIP;
    hipLaunchKernelGGL(shard_expand, dim3(g), dim3(ST), 0, st, s->o_item, s->o_arena, s->o_boff, s->d_wlist, s->o_rec,
                       s->o_off, total);
  }
  hipLaunchKernelGGL(shard_set_n, dim3(1), dim3(1), 0, st, s->o_n, total);
  if (hipGetLastError() != hipSuccess) return RTPS_RX_EHIP;
  out->arena = s->o_arena;
  out->arena_len = arena_need;
  out->dgram_off = s->o_off;
  out->records = s->o_rec;
  out->origin = s->o_origin;
  out->n_records_dev = s->o_n;
  out->n_records = total;
  s->exchanged = false;
  s->finished = false;
  return RTPS_RX_OK;
}

}  // extern "C"
