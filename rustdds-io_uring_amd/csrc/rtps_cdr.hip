// rtps_cdr.hip — batch CDR primitive decode of DATA payloads.
//
// Replaces, for fixed-layout sample types, the per-sample decode chain
//   SimpleDataReader::deserialize_with      io_uring/dds/with_key/simpledatareader.rs:137-160
//   -> CDRDeserializerAdapter (REPR_IDS)     serialization/cdr_adapters.rs:96-100
//   -> deserialize_from_cdr_with_decoder_and_rep_id   cdr_adapters.rs:246-275
//   -> cdr_encoding::CdrDeserializer         (external crate cdr-encoding 0.10)
// The sample type is a program of ops (rtps_cdr_op), wave-uniform (a kernel
// argument).  Flat programs (cdr_decode_kernel): a wave takes 64 records, each
// lane validates one record and leaves its per-op data offsets in LDS, then the
// whole wave writes the 64 rows slot by slot, one 4-byte word per lane, so row
// stores are coalesced and every row byte is written once (failed rows as
// zeros).  Composite programs (SEQ_BEGIN / ARRAY_BEGIN ... END, whose element
// offsets differ per record: cdr_nested_kernel): lane = row, the values staged in
// LDS by the wave, the open elements as LDS frames.
//
// Roofline: HBM-bound.  Algorithmic bytes per record = 40 B of the record +
// the value bytes a decoded row consumes + row_bytes + 1 status byte written.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/rtps_rx.h"
#include "rtps_cdr.h"

namespace {

typedef uint16_t u16u __attribute__((aligned(1)));
typedef uint32_t u32u __attribute__((aligned(1)));
typedef uint64_t u64u __attribute__((aligned(1)));

__device__ __forceinline__ uint32_t pad_to(uint32_t pos, uint32_t a) { return (0u - pos) & (a - 1u); }

// One primitive of `size` bytes at v (unaligned), converted to host order.
__device__ __forceinline__ uint64_t load_prim(const uint8_t* v, uint32_t size, bool le) {
  uint64_t x;
  switch (size) {
    case 1: return v[0];
    case 2: x = *(const u16u*)v; return le ? x : __builtin_bswap16((uint16_t)x);
    case 4: x = *(const u32u*)v; return le ? x : __builtin_bswap32((uint32_t)x);
    default: x = *(const u64u*)v; return le ? x : __builtin_bswap64(x);
  }
}
__device__ __forceinline__ void store_prim(uint8_t* d, uint64_t x, uint32_t size) {
  switch (size) {
    case 1: d[0] = (uint8_t)x; break;
    case 2: *(u16u*)d = (uint16_t)x; break;
    case 4: *(u32u*)d = (uint32_t)x; break;
    default: *(u64u*)d = x; break;
  }
}

// 16-byte loads / stores at any byte alignment (gfx950 runs them as single
// unaligned dwordx4 accesses)
__device__ __forceinline__ uint4 ld16u(const uint8_t* p) {
  uint4 v;
  __builtin_memcpy(&v, p, 16);
  return v;
}
__device__ __forceinline__ void st16u(uint8_t* p, uint4 v) { __builtin_memcpy(p, &v, 16); }

// std::str::from_utf8 acceptance over m bytes.  A multi-byte character is
// checked with selects (its lead's class and the allowed range of its first
// continuation byte), not a branch per lead class: lanes that validate different
// characters then run the same instructions.
__device__ bool utf8_ok(const uint8_t* s, uint32_t m) {
  uint32_t i = 0;
  while (i < m) {
    // ASCII fast path: 4 bytes at a time
    if (i + 4 <= m) {
      uint32_t w = *(const u32u*)(s + i);
      if ((w & 0x80808080u) == 0) { i += 4; continue; }
    }
    const uint32_t c = s[i];
    if (c < 0x80) { i++; continue; }
    // C2..DF: 1 continuation, E0..EF: 2, F0..F4: 3; E0 / ED / F0 / F4 narrow the first one
    const uint32_t need = c >= 0xF0 ? 3u : (c >= 0xE0 ? 2u : 1u);
    const uint32_t lo = c == 0xE0 ? 0xA0u : (c == 0xF0 ? 0x90u : 0x80u);
    const uint32_t hi = c == 0xED ? 0x9Fu : (c == 0xF4 ? 0x8Fu : 0xBFu);
    if (c < 0xC2 || c > 0xF4 || i + need >= m) return false;
    const uint32_t b1 = s[i + 1];
    const uint32_t b2 = s[i + (need >= 2 ? 2u : 1u)], b3 = s[i + need];  // (re-read b1 / b2 when shorter)
    const bool cont = ((b2 & 0xC0u) == 0x80u) & ((b3 & 0xC0u) == 0x80u);
    if (b1 < lo || b1 > hi || !cont) return false;
    i += need + 1;
  }
  return true;
}

// Phase A (one lane per record): walk the program, return the status and
// record each op's data start (pos) and run-time length (string chars /
// sequence elements) in the wave's LDS table.  Reads only lengths, bools and
// string bytes.
// the bytes [b, b + 4) of a word that lie below m, as a mask
__device__ __forceinline__ uint32_t byte_mask(uint32_t m, uint32_t b) {
  const uint32_t n = m > b ? m - b : 0u;
  return n >= 4u ? 0xffffffffu : (1u << (8u * n)) - 1u;
}

// avail: the arena bytes readable from v (at least len)
__device__ uint8_t cdr_validate(const CdrProg& P, const uint8_t* v, uint32_t len, uint64_t avail, bool le,
                                uint32_t* posT, uint32_t* lenT, uint32_t lane) {
  uint32_t pos = 0;
  for (uint32_t k = 0; k < P.n_ops; ++k) {
    const rtps_cdr_op op = P.ops[k];
    const uint32_t size = op.size;
    uint32_t dpos = pos, dlen = 0;
    switch (op.kind) {
      case RTPS_CDR_PRIM:
      case RTPS_CDR_ARRAY: {
        const uint32_t cnt = op.kind == RTPS_CDR_PRIM ? 1u : op.count;
        if (cnt == 0) break;
        const uint32_t pad = pad_to(pos, size);
        if ((uint64_t)pos + pad + (uint64_t)cnt * size > len) return RTPS_CDR_EOF;
        dpos = pos + pad;
        pos = dpos + cnt * size;
        break;
      }
      case RTPS_CDR_BOOL:
        if (pos + 1 > len) return RTPS_CDR_EOF;
        if (v[pos] > 1) return RTPS_CDR_BAD_BOOL;
        pos += 1;
        break;
      case RTPS_CDR_STRING: {
        pos += pad_to(pos, 4);
        if ((uint64_t)pos + 4 > len) return RTPS_CDR_EOF;
        // the length and the first 12 characters in one 16-B load when the arena has the bytes:
        // a short ASCII string is then checked without the byte loop's dependent loads
        const bool q16 = (uint64_t)pos + 16 <= avail;
        const uint4 h = ld16u(v + (q16 ? pos : 0u));
        const uint32_t l = q16 ? (le ? h.x : __builtin_bswap32(h.x)) : (uint32_t)load_prim(v + pos, 4, le);
        pos += 4;
        if ((uint64_t)pos + l > len) return RTPS_CDR_EOF;
        const uint32_t m = l ? l - 1 : 0;
        const bool ascii12 = q16 && m <= 12u &&
                             (((h.y & byte_mask(m, 0)) | (h.z & byte_mask(m, 4)) | (h.w & byte_mask(m, 8))) &
                              0x80808080u) == 0u;
        if (!ascii12 && !utf8_ok(v + pos, m)) return RTPS_CDR_BAD_UTF8;
        if (m > op.count) return RTPS_CDR_TOO_LONG;
        dpos = pos;
        dlen = m;
        pos += l;
        break;
      }
      case RTPS_CDR_SEQ: {
        pos += pad_to(pos, 4);
        if ((uint64_t)pos + 4 > len) return RTPS_CDR_EOF;
        const uint32_t n = (uint32_t)load_prim(v + pos, 4, le);
        pos += 4;
        dpos = pos;
        if (n) {
          const uint32_t pe = pad_to(pos, size);
          if ((uint64_t)pos + pe + (uint64_t)n * size > len) return RTPS_CDR_EOF;
          if (n > op.count) return RTPS_CDR_TOO_LONG;
          dpos = pos + pe;
          pos = dpos + n * size;
        }
        dlen = n;
        break;
      }
      default:
        return RTPS_CDR_TOO_LONG;
    }
    posT[k * 64 + lane] = dpos;
    lenT[k * 64 + lane] = dlen;
  }
  return RTPS_CDR_OK;
}

#ifndef CDR_UNROLL_N
#define CDR_UNROLL_N 6  // narrow-slot words per lane per round: 6 keeps 6 waves / SIMD without scratch
#endif
#ifndef CDR_RUN_N
#define CDR_RUN_N 2
#endif
#ifndef CDR_GRID_MULT
#define CDR_GRID_MULT 1  // grid cap = resident blocks x this
#endif
#ifndef CDR_PROBE
#define CDR_PROBE 0  // diagnosis builds only: 1 phase A only, 2 no wide slots, 3 no narrow slots, 4 loads of phase A only
#endif
#ifndef CDR_WAVES_PER_EU
#define CDR_WAVES_PER_EU 6  // 80 VGPRs: C2 162 -> 135 us, C3 211 -> 200 us, T unchanged (scripts/gpu_cdr_ab.sh)
#endif
constexpr uint32_t CDR_UNROLL = CDR_UNROLL_N;
constexpr uint32_t CDR_WIDE_DWORDS = 8;   // slots at least this long take the 16-B-per-lane path
constexpr uint32_t CDR_RUN = CDR_RUN_N;   // record groups per round of the wide path


// Host-order fix of one loaded word (mask the bytes at or past nb, swap big-endian elements)
__device__ __forceinline__ uint32_t fix_word(uint32_t x, uint32_t bb, uint32_t nb, uint32_t size, bool le) {
  if (bb >= nb) return 0u;
  const uint32_t rem = nb - bb;
  if (rem < 4) x &= (1u << (8u * rem)) - 1u;
  if (!le) {
    if (size == 2) x = ((x & 0xff00ff00u) >> 8) | ((x & 0x00ff00ffu) << 8);
    else if (size >= 4) x = __builtin_bswap32(x);
  }
  return x;
}

// Wide slot: lane (lr, lq) handles data quad lq (16 bytes, aligned to the data
// start) of record lr of each group of rpi = 64 / nq records (nq = quads per
// slot; rpi = 1 and a quad loop when nq > 64), CDR_RUN groups per round so
// several 16-B loads per lane are in flight.  A 976-byte array is one load +
// one store per lane and record.  The header word of STRING / SEQ slots is
// stored by the lane with lq == 0.
__device__ __forceinline__ void wide_slot(const CdrProg& P, const CdrSlot& S, const CdrArgs& a, uint32_t hdr,
                                          uint32_t nv, uint32_t lane, const uint32_t* meta, const uint64_t* vbase,
                                          const uint32_t* posT, const uint32_t* lenT, uint8_t* rowc) {
  const uint32_t dwd = S.dwords - hdr;  // data words of the slot
  const uint32_t nq = (dwd + 3) >> 2;
  const uint32_t rpi = nq >= 64 ? 1u : 64u / nq;
  const uint32_t lr = nq >= 64 ? 0u : lane / nq;
  const uint32_t lq = nq >= 64 ? lane : lane - lr * nq;
  if (lr >= rpi) return;  // idle lanes (64 not a multiple of nq)
  for (uint32_t q0 = 0; q0 < nq; q0 += 64) {
    const uint32_t q = q0 + lq;
    const uint32_t bq = 16u * q;
    for (uint32_t r = 0; r < nv; r += rpi * CDR_RUN) {
      uint4 x[CDR_RUN];
      uint32_t nbv[CDR_RUN];
      bool own[CDR_RUN];  // this slot writes record rr (segments vs their member slots)
#pragma unroll
      for (uint32_t u = 0; u < CDR_RUN; ++u) {
        const uint32_t rr = r + u * rpi + lr;
        const uint32_t rec = min(rr, nv - 1);
        const uint32_t m = meta[rec];
        const bool okrec = (m & 0xffu) == RTPS_CDR_OK, le = ((m >> 8) & 1u) != 0;
        const bool ok = rr < nv && okrec && S.kind != CDR_SLOT_ZERO;
        const uint32_t ln = hdr ? lenT[S.op * 64u + rec] : 0u;
        const uint32_t nb = S.kind == CDR_SLOT_SEG ? 4u * S.dwords
                          : S.kind == RTPS_CDR_STRING ? ln : (S.kind == RTPS_CDR_SEQ ? ln * S.size : S.count * S.size);
        nbv[u] = ok ? nb : 0u;
        own[u] = S.kind == CDR_SLOT_SEG ? (okrec && le) : (S.flags & CDR_IN_SEG) ? !(okrec && le) : true;
        const uint32_t dpos = S.kind == CDR_SLOT_SEG ? S.count : posT[S.op * 64u + rec];
        const uint64_t abs = vbase[rec] + dpos + bq;
        const bool fast = own[u] && q < nq && bq < nbv[u] && abs + 16 <= a.arena_len;
        x[u] = ld16u(fast ? a.arena + abs : (const uint8_t*)a.records);
      }
#pragma unroll
      for (uint32_t u = 0; u < CDR_RUN; ++u) {
        const uint32_t rr = r + u * rpi + lr;
        if (rr >= nv) break;
        if (!own[u]) continue;
        const uint32_t m = meta[rr];
        const bool le = ((m >> 8) & 1u) != 0;
        const uint32_t nb = nbv[u];
        uint8_t* rowp = rowc + (uint64_t)rr * P.row_bytes + S.out_off;
        if (hdr && q == 0) *(uint32_t*)rowp = nb ? lenT[S.op * 64u + rr] : 0u;  // nb == 0 <=> length 0 or failed row
        if (q >= nq) continue;
        uint32_t w[4] = {x[u].x, x[u].y, x[u].z, x[u].w};
        if (bq < nb) {
          const uint64_t abs = vbase[rr] + (S.kind == CDR_SLOT_SEG ? S.count : posT[S.op * 64u + rr]) + bq;
          if (abs + 16 > a.arena_len) {  // quad runs past the arena end (rare)
#pragma unroll
            for (uint32_t t = 0; t < 4; ++t) {
              w[t] = 0;
              for (uint32_t c = 0; c < 4; ++c)
                if (abs + 4 * t + c < a.arena_len) w[t] |= (uint32_t)a.arena[abs + 4 * t + c] << (8 * c);
            }
          }
        }
        if (!le && S.size == 8) {
          uint32_t t0 = w[0], t2 = w[2];
          w[0] = w[1]; w[1] = t0; w[2] = w[3]; w[3] = t2;
        }
        uint4 o;
        o.x = fix_word(w[0], bq, nb, S.size, le);
        o.y = fix_word(w[1], bq + 4, nb, S.size, le);
        o.z = fix_word(w[2], bq + 8, nb, S.size, le);
        o.w = fix_word(w[3], bq + 12, nb, S.size, le);
        uint8_t* d = rowp + 4u * hdr + bq;
        if (4 * q + 4 <= dwd) {
          st16u(d, o);
        } else {
          const uint32_t nw = dwd - 4 * q;
          *(uint32_t*)d = o.x;
          if (nw > 1) *(uint32_t*)(d + 4) = o.y;
          if (nw > 2) *(uint32_t*)(d + 8) = o.z;
        }
      }
    }
  }
}

// Segment of an all-little-endian chunk: a plain block copy of dwords*4 bytes
// per record from value + wire_off, 16 B per lane, rpi records per pass.
// WIDE (a separate kernel instantiation, for programs with a segment of more than
// 32 quads: one record per pass, T's 976-B arrays): four records' quads are loaded
// before any is stored, so a lane's loads are in flight together (a store between
// them would order them).  T 446 -> 433-441 us; in the instantiation every program
// uses it cost C2 (four records per pass) 145 -> 162-198 us, hence the template.
template <bool WIDE>
__device__ __forceinline__ void seg_copy(const CdrProg& P, const CdrSlot& S, const CdrArgs& a, uint32_t nv,
                                         uint32_t lane, const uint64_t* vbase, uint8_t* rowc) {
  const uint32_t nb = 4u * S.dwords;
  const uint32_t nq = (S.dwords + 3) >> 2;
  const uint32_t rpi = nq >= 64 ? 1u : 64u / nq;
  const uint32_t lr = nq >= 64 ? 0u : lane / nq;
  const uint32_t lq = nq >= 64 ? lane : lane - lr * nq;
  if (lr >= rpi) return;
  for (uint32_t q0 = 0; q0 < nq; q0 += 64) {
    const uint32_t q = q0 + lq;
    if (q >= nq) break;
    const uint32_t bq = 16u * q;
    const bool full = bq + 16 <= nb;
    uint32_t rr = lr;
    if (WIDE && rpi == 1u && full && a.arena_len >= 16) {
      for (; rr + 3u < nv; rr += 4u) {
        uint4 v[4];
        bool fast = true;
#pragma unroll
        for (uint32_t u = 0; u < 4u; ++u) {
          const uint64_t abs = vbase[rr + u] + S.count + bq;
          fast = fast && abs + 16 <= a.arena_len;
          v[u] = ld16u(a.arena + (abs + 16 <= a.arena_len ? abs : 0));
        }
        if (!fast) break;  // the arena tail: the per-record loop below
#pragma unroll
        for (uint32_t u = 0; u < 4u; ++u) st16u(rowc + (uint64_t)(rr + u) * P.row_bytes + S.out_off + bq, v[u]);
      }
    }
    for (; rr < nv; rr += rpi) {
      const uint64_t abs = vbase[rr] + S.count + bq;
      uint8_t* d = rowc + (uint64_t)rr * P.row_bytes + S.out_off + bq;
      if (full && abs + 16 <= a.arena_len) {
        st16u(d, ld16u(a.arena + abs));
      } else {  // last partial quad (whole words) or the arena tail
        for (uint32_t b = bq; b < nb && b < bq + 16; b += 4) {
          uint32_t w = 0;
          const uint64_t o = abs + (b - bq);
          if (o + 4 <= a.arena_len) w = *(const u32u*)(a.arena + o);
          else for (uint32_t c = 0; c < 4; ++c) if (o + c < a.arena_len) w |= (uint32_t)a.arena[o + c] << (8 * c);
          *(uint32_t*)(d + (b - bq)) = w;
        }
      }
    }
  }
}

#ifndef CDR_OST_STAGE
#define CDR_OST_STAGE 0  // output-stationary: the first 32 B of every value staged in LDS by phase A
#endif
constexpr uint32_t CDR_STAGE_BYTES = 32;  // per row; + 16 B of pad per wave (the funnel's second word)
#ifndef CDR_OST_MASKED
#define CDR_OST_MASKED 1  // words without data skip their load (exec-masked): C3 list 190 -> 186 us
#endif
#ifndef CDR_OQ
#define CDR_OQ 1  // output quads per lane per round of the output-stationary path: one at 8 waves / SIMD
                  // (63 VGPRs) 183.5 us on C3, two at 6 waves 186, three at 5 waves 208, four at 4 285
#endif
#ifndef CDR_OST_WAVES_PER_EU
#define CDR_OST_WAVES_PER_EU 8
#endif

// Output-stationary phase B (programs with a string or a sequence, rows up to CDR_OSTAT_ROW
// bytes): the chunk's rows are contiguous (nv * row_bytes bytes), so lane = 16-B output quad
// and every row store is a whole coalesced quad; each word finds its slot in the block's word
// table wt[row_bytes / 4] = {kind | size << 8 | op << 16, k | static bytes << 16} (k = word of
// the slot; segments are overlays and are not in it).  The narrow slot-by-slot walk stores one
// word per row per instruction (64 rows, 64 lines) and waits for each slot's loads in turn:
// C3's 3 one-word slots cost 86 of its 284 us, 56 of them the scattered stores (diagnosis builds).
// Word ctl: bits 0-2 bytes kept (0: the word is zero), 3-4 bytes clamped at the arena end,
// 5-6 swap (1: 16-bit halves, 2: 32-bit), bit 7 immediate (val is the word).
__device__ __forceinline__ void ostat_word(const CdrArgs& a, const uint2* wt, uint32_t r, uint32_t w, bool in,
                                           const uint32_t* meta, const uint64_t* vbase, const uint32_t* posT,
                                           const uint32_t* lenT, const uint32_t* stg, uint32_t& val, uint32_t& ctl) {
  const uint2 d = wt[in ? w : 0u];
  const uint32_t kind = d.x & 0xffu, size = (d.x >> 8) & 0xffu, op = d.x >> 16;
  const uint32_t k = d.y & 0xffffu;
  const uint32_t m = meta[r];
  const bool le = ((m >> 8) & 1u) != 0, ok = in && (m & 0xffu) == RTPS_CDR_OK && kind != CDR_SLOT_ZERO;
  const bool hdr = kind == RTPS_CDR_STRING || kind == RTPS_CDR_SEQ;
  const uint32_t ln = hdr ? lenT[op * 64u + r] : 0u;
  const uint32_t nb = kind == RTPS_CDR_STRING ? ln : (kind == RTPS_CDR_SEQ ? ln * size : d.y >> 16);
  const uint32_t bb = 4u * (k - (hdr ? 1u : 0u));
  const bool data = ok && !(hdr && k == 0u) && bb < nb;
  const uint32_t off = posT[op * 64u + r] + ((!le && size == 8u) ? (bb ^ 4u) : bb);  // in the value
  uint64_t abs = vbase[r] + off;
  abs = data ? abs : 0ull;
  // a word inside the row's staged window (meta bits 16-23: its length) is read from LDS
  const bool staged = CDR_OST_STAGE && data && off + 4u <= ((m >> 16) & 0xffu);
  const uint32_t over = (abs + 4 > a.arena_len) ? (uint32_t)(abs + 4 - a.arena_len) : 0u;
  const uint32_t rem = nb - bb;
  const uint32_t keep = data ? (rem >= 4u ? 4u : rem) : 0u;
  const uint32_t sw = le ? 0u : (size == 2u ? 1u : (size >= 4u ? 2u : 0u));
  const bool imm = ok && hdr && k == 0u;
  ctl = keep | (over << 3) | (sw << 5) | (imm ? 0x80u : 0u);
#if CDR_OST_MASKED
  if (CDR_OST_STAGE && staged) {
    const uint32_t i = r * (CDR_STAGE_BYTES / 4u) + (off >> 2);
    val = __builtin_amdgcn_alignbyte(stg[i + 1], stg[i], off & 3u);
  } else {
    val = imm ? ln : (data ? *(const u32u*)(a.arena + (abs - over)) : 0u);
  }
#else
  // words without data read a record word instead (in bounds, cached)
  const uint8_t* pa = data ? a.arena + (abs - over) : (const uint8_t*)a.records;
  val = imm ? ln : *(const u32u*)pa;
#endif
}
__device__ __forceinline__ uint32_t ostat_fix(uint32_t x, uint32_t ctl) {
  if (ctl & 0x80u) return x;
  const uint32_t keep = ctl & 7u;
  if (keep == 0u) return 0u;
  x >>= 8u * ((ctl >> 3) & 3u);
  if (keep < 4u) x &= (1u << (8u * keep)) - 1u;
  const uint32_t sw = (ctl >> 5) & 3u;
  if (sw == 1u) x = ((x & 0xff00ff00u) >> 8) | ((x & 0x00ff00ffu) << 8);
  else if (sw == 2u) x = __builtin_bswap32(x);
  return x;
}
__device__ __forceinline__ void ostat_rows(const CdrArgs& a, const uint2* wt, uint32_t rdw, uint32_t nv,
                                           uint32_t lane, const uint32_t* meta, const uint64_t* vbase,
                                           const uint32_t* posT, const uint32_t* lenT, const uint32_t* stg,
                                           uint8_t* rowc) {
  const uint32_t nwords = nv * rdw, nquads = (nwords + 3u) >> 2;
  const float inv = 1.0f / (float)rdw;
  for (uint32_t q0 = 0; q0 < nquads; q0 += 64u * CDR_OQ) {
    uint32_t val[4 * CDR_OQ], ctl[CDR_OQ];  // ctl: a byte per word
#pragma unroll
    for (uint32_t u = 0; u < CDR_OQ; ++u) {
      const uint32_t wd = 4u * (q0 + u * 64u + lane);
      uint32_t r = (uint32_t)((float)wd * inv);
      r = (r * rdw > wd) ? r - 1u : r;
      r = ((r + 1u) * rdw <= wd) ? r + 1u : r;
      uint32_t w = wd - r * rdw;
      ctl[u] = 0u;
#pragma unroll
      for (uint32_t t = 0; t < 4u; ++t) {
        const bool in = wd + t < nwords;
        uint32_t c;
        ostat_word(a, wt, in ? r : 0u, w, in, meta, vbase, posT, lenT, stg, val[4 * u + t], c);
        ctl[u] |= c << (8u * t);
        if (++w == rdw) { w = 0u; ++r; }
      }
    }
#pragma unroll
    for (uint32_t u = 0; u < CDR_OQ; ++u) {
      const uint32_t q = q0 + u * 64u + lane;
      if (q >= nquads) break;
      uint4 o;
      o.x = ostat_fix(val[4 * u], ctl[u] & 0xffu);
      o.y = ostat_fix(val[4 * u + 1], (ctl[u] >> 8) & 0xffu);
      o.z = ostat_fix(val[4 * u + 2], (ctl[u] >> 16) & 0xffu);
      o.w = ostat_fix(val[4 * u + 3], ctl[u] >> 24);
      uint8_t* d = rowc + 16u * q;
      if (4u * q + 4u <= nwords) {
        st16u(d, o);
      } else {
        const uint32_t nw = nwords - 4u * q;
        *(uint32_t*)d = o.x;
        if (nw > 1) *(uint32_t*)(d + 4) = o.y;
        if (nw > 2) *(uint32_t*)(d + 8) = o.z;
      }
    }
  }
}

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

extern __shared__ uint8_t cdr_lds[];

// One wave per chunk of 64 rows (a row = a record, or in list mode a list entry
// naming a record).  Phase A: lane = row (validation, LDS table).  Phase B: the wave writes the chunk's rows slot by slot, one 4-byte
// word per lane and item (item = record x word of the slot), so consecutive
// lanes store consecutive words and every row byte is written exactly once.
template <bool WIDE, bool OSTAT>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(OSTAT ? CDR_OST_WAVES_PER_EU : CDR_WAVES_PER_EU)))
void cdr_decode_kernel(CdrProg P, CdrArgs a) {
  const uint32_t lane = threadIdx.x & 63u, wpb = blockDim.x >> 6;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // (uniform: LDS bases in SGPRs)
  uint8_t* T = cdr_lds + wave * P.lds_per_wave;
  uint2* wt = (uint2*)(cdr_lds + wpb * P.lds_per_wave);  // OSTAT: the block's word table
  const uint32_t rdw = P.row_bytes >> 2;
  if (OSTAT) {
    for (uint32_t si = 0; si < P.n_slots; ++si) {
      const CdrSlot S = P.slots[si];
      if (S.kind == CDR_SLOT_SEG) continue;  // an overlay: its member slots cover its words
      const uint32_t info = S.kind | ((uint32_t)S.size << 8) | ((uint32_t)S.op << 16);
      const uint32_t nbs = S.count * S.size;
      for (uint32_t t = threadIdx.x; t < S.dwords; t += blockDim.x)
        wt[(S.out_off >> 2) + t] = make_uint2(info, t | (nbs << 16));
    }
    __syncthreads();
  }
  uint32_t* meta = (uint32_t*)T;             // [64] status | le << 8
  uint64_t* vbase = (uint64_t*)(T + 256);    // [64] arena offset of the value
  uint32_t* posT = (uint32_t*)(T + 768);     // [n_ops][64]
  uint32_t* lenT = posT + P.n_ops * 64u;     // [n_ops][64]
  uint32_t* stg = lenT + P.n_ops * 64u;      // OSTAT: [64][CDR_STAGE_BYTES / 4] + pad, the staged values
  const uint64_t n = a.list ? min(*a.n_list, a.max_list) : min(*a.n_records, a.max_records);
  const uint64_t nrec = min(*a.n_records, a.max_records);
  const uint64_t chunks = (n + 63) / 64;
  for (uint64_t c = (uint64_t)blockIdx.x * wpb + wave; c < chunks; c += (uint64_t)gridDim.x * wpb) {
    const uint64_t r0 = c * 64;
    const uint32_t nv = (uint32_t)min<uint64_t>(64, n - r0);
    // ---- phase A ----
    uint32_t st = 0xff, le = 1, wl = 0;
    uint64_t vb = 0;
    if (lane < nv) {
      // the row's record: the row itself, or its list entry (a delivery, a sample index)
      const uint64_t ri = a.list ? *reinterpret_cast<const uint32_t*>(a.list + (r0 + lane) * a.list_stride) : r0 + lane;
      // bytes 0..31 (dgram_idx @0, kind @6, payload_kind @31) and 40..47 (pl_off, pl_len, rep_id); a list
      // entry past the records loads nothing (nrec may be 0)
      uint4 h0 = {0u, 0u, 0u, 0u}, h1 = h0;
      uint2 u0 = {0u, 0u};
      if (ri < nrec) {
        const rtps_record* rec = a.records + ri;
        h0 = *(const uint4*)rec;
        h1 = *(const uint4*)((const uint8_t*)rec + 16);
        u0 = *(const uint2*)((const uint8_t*)rec + 40);
      }
      const uint32_t kind = (h0.y >> 16) & 0xff, pk = h1.w >> 24;
      const uint32_t pl_off = u0.x & 0xffff, pl_len = u0.x >> 16;
      const uint32_t id0 = u0.y & 0xff, id1 = (u0.y >> 8) & 0xff;
      if (ri >= nrec || kind != RTPS_DATA || pk != RTPS_PK_DATA || pl_len < 4) {
        st = RTPS_CDR_NOT_DATA;
      } else if (id0 != 0 || (id1 != 0 && id1 != 1 && id1 != 3)) {
        st = RTPS_CDR_BAD_ENCODING;
      } else {
        vb = a.dgram_off[h0.x] + pl_off + 4;
        const uint32_t len = pl_len - 4;
        le = id1 != 0;
        if (OSTAT && CDR_OST_STAGE) {  // the value's first 32 B, in flight beside the validation's loads
          const bool sw = vb + CDR_STAGE_BYTES <= a.arena_len;
          const uint4 s0 = ld16u(a.arena + (sw ? vb : 0ull)), s1 = ld16u(a.arena + (sw ? vb + 16u : 0ull));
          *(uint4*)(stg + lane * (CDR_STAGE_BYTES / 4u)) = s0;
          *(uint4*)(stg + lane * (CDR_STAGE_BYTES / 4u) + 4u) = s1;
          wl = sw ? min(len, CDR_STAGE_BYTES) : 0u;
        }
        st = (vb + len > a.arena_len) ? (uint32_t)RTPS_CDR_NOT_DATA  // cannot happen for parse outputs
             : CDR_PROBE == 4 ? (a.arena[vb] == 0xee ? 0u : 1u)
                                      : cdr_validate(P, a.arena + vb, len, a.arena_len - vb, le, posT, lenT, lane);
      }
      a.row_status[r0 + lane] = (uint8_t)st;
    }
    meta[lane] = st | (le << 8) | (wl << 16);
    vbase[lane] = vb;
    // every record of the chunk decoded little-endian: segments are plain copies
    // and their member slots have nothing to write
    const bool all_okle = __all(lane >= nv || (st == RTPS_CDR_OK && le));
    const bool all_fail = __all(lane >= nv || st != RTPS_CDR_OK);
    wave_sync();
    // ---- phase B ----
    if (CDR_PROBE == 1 || CDR_PROBE == 4) { wave_sync(); continue; }
    uint8_t* rowc = a.rows + r0 * P.row_bytes;
    if (all_fail) {  // every row of the chunk is zero: one contiguous fill
      const uint32_t bytes = nv * P.row_bytes;
      for (uint32_t b = 16u * lane; b < bytes; b += 1024u) {
        if (b + 16 <= bytes) st16u(rowc + b, make_uint4(0, 0, 0, 0));
        else for (uint32_t t = b; t < bytes; t += 4) *(uint32_t*)(rowc + t) = 0u;
      }
      wave_sync();
      continue;
    }
    if (OSTAT) {
      ostat_rows(a, wt, rdw, nv, lane, meta, vbase, posT, lenT, stg, rowc);
      wave_sync();
      continue;
    }
    for (uint32_t si = 0; si < P.n_slots; ++si) {
      const CdrSlot S = P.slots[si];
      const uint32_t hdr = (S.kind == RTPS_CDR_STRING || S.kind == RTPS_CDR_SEQ) ? 1u : 0u;
      if (all_okle && (S.flags & CDR_IN_SEG)) continue;
      if (all_okle && S.kind == CDR_SLOT_SEG) {
        seg_copy<WIDE>(P, S, a, nv, lane, vbase, rowc);
        continue;
      }
      if (S.dwords >= CDR_WIDE_DWORDS) {
        if (CDR_PROBE == 2) continue;
        wide_slot(P, S, a, hdr, nv, lane, meta, vbase, posT, lenT, rowc);
        continue;
      }
      if (CDR_PROBE == 3) continue;
      const uint32_t total = nv * S.dwords;
      const bool swap8 = S.size == 8;
      const float inv_dwords = 1.0f / (float)S.dwords;
      // CDR_UNROLL independent words per lane per round, branch-free: every
      // load of the round is in flight before the first store waits
      for (uint32_t it0 = 0; it0 < total; it0 += 64u * CDR_UNROLL) {
        uint32_t val[CDR_UNROLL], dst[CDR_UNROLL], keep[CDR_UNROLL], shift[CDR_UNROLL], flags[CDR_UNROLL];
#pragma unroll
        for (uint32_t u = 0; u < CDR_UNROLL; ++u) {
          const uint32_t item = it0 + u * 64u + lane;
          const bool in = item < total;
          uint32_t rec = (uint32_t)((float)item * inv_dwords);
          rec = (rec * S.dwords > item) ? rec - 1 : rec;
          rec = ((rec + 1) * S.dwords <= item) ? rec + 1 : rec;
          rec = in ? rec : 0u;
          const uint32_t k = item - rec * S.dwords;
          const uint32_t m = meta[rec];
          const bool le = ((m >> 8) & 1u) != 0;
          const bool okrec = (m & 0xffu) == RTPS_CDR_OK;
          const bool mine = S.kind == CDR_SLOT_SEG ? (okrec && le) : (S.flags & CDR_IN_SEG) ? !(okrec && le) : true;
          dst[u] = (in && mine) ? rec * P.row_bytes + S.out_off + 4u * k : ~0u;
          const bool ok = in && mine && okrec && S.kind != CDR_SLOT_ZERO;
          const uint32_t ln = hdr ? lenT[S.op * 64u + rec] : 0u;
          const uint32_t nb = S.kind == RTPS_CDR_STRING ? ln : (S.kind == RTPS_CDR_SEQ ? ln * S.size : S.count * S.size);
          const uint32_t nbs = S.kind == CDR_SLOT_SEG ? 4u * S.dwords : nb;
          const uint32_t j = k - hdr;  // data word index (wraps for the header word)
          const uint32_t bb = 4u * j;
          const bool data = ok && k >= hdr && bb < nbs;
          // absolute arena offset of the word; 8-byte big-endian elements take the other half
          const uint32_t dpos = S.kind == CDR_SLOT_SEG ? S.count : posT[S.op * 64u + rec];
          uint64_t abs = vbase[rec] + dpos + ((!le && swap8) ? (bb ^ 4u) : bb);
          abs = data ? abs : 0ull;
          // clamp a word that would run past the arena end; its valid bytes shift down
          const uint64_t over = (abs + 4 > a.arena_len) ? abs + 4 - a.arena_len : 0ull;
          shift[u] = (uint32_t)over * 8u;
          const uint32_t rem = nbs - bb;
          keep[u] = !data ? 0u : (rem >= 4 ? 0xffffffffu : ((1u << (8u * rem)) - 1u));
          flags[u] = (ok && k < hdr ? 1u : 0u) | (le ? 2u : 0u);
          // lanes without data read a record word instead (always in bounds, cached)
          const uint8_t* pa = data ? a.arena + (abs - over) : (const uint8_t*)a.records;
          val[u] = ok && k < hdr ? ln : (CDR_PROBE == 6 ? (uint32_t)(uintptr_t)pa : *(const u32u*)pa);
        }
#pragma unroll
        for (uint32_t u = 0; u < CDR_UNROLL; ++u) {
          uint32_t x = val[u];
          if (!(flags[u] & 1u)) {
            x = (x >> shift[u]) & keep[u];
            if (!(flags[u] & 2u)) {
              if (S.size == 2) x = ((x & 0xff00ff00u) >> 8) | ((x & 0x00ff00ffu) << 8);
              else if (S.size >= 4) x = __builtin_bswap32(x);
            }
          }
          if (CDR_PROBE == 5) { if (dst[u] != ~0u) *(uint32_t*)(rowc + 4u * lane + 256u * ((u + si) % 9u)) = x; }
          else if (dst[u] != ~0u) *(uint32_t*)(rowc + dst[u]) = x;
        }
      }
    }
    wave_sync();  // the LDS table is reused by the wave's next chunk
  }
}

// ---- composite programs ----------------------------------------------------
// Lane-serial decode of one row with the restated cdr-encoding rules of
// cdr_validate, plus elements: SEQ_BEGIN reads a u32 count (aligned to 4),
// ARRAY_BEGIN has none; each element is the ops up to the matching END, with
// no alignment of its own (serde's Vec<T> / [T; N] through deserialize_seq /
// deserialize_tuple).  Elements past the slot (n > count) are read and
// validated but not stored; the sequence is then TOO_LONG (at once when its
// element reads no bytes, as it cannot fail).  The lane zeroed its row first
// (its own stores: program order), and zeroes it again when the decode fails.
__device__ __forceinline__ void copy_bytes(uint8_t* d, const uint8_t* s, uint32_t m) {
  uint32_t i = 0;
  for (; i + 4 <= m; i += 4) *(uint32_t*)(d + i) = *(const u32u*)(s + i);  // d is 4-aligned
  for (; i < m; ++i) d[i] = s[i];
}
// Open elements live in LDS, one 16-B frame per (depth, lane):
// {n, i, elem0, base | begin << 24 | write << 31} (base, elem0 < 2^20: row offsets).
__device__ uint8_t nest_decode(const rtps_cdr_op* ops, const uint8_t* match, const uint8_t* zero_el, uint32_t n_ops,
                               const uint8_t* v, uint32_t len, bool le, uint8_t* row, uint4* fr) {
  uint32_t depth = 0, base = 0, pos = 0;
  bool write = true;
  for (uint32_t k = 0; k < n_ops; ++k) {
    const rtps_cdr_op op = ops[k];
    const uint32_t size = op.size;
    uint8_t* d = row + base + op.out_off;
    switch (op.kind) {
      case RTPS_CDR_PRIM:
      case RTPS_CDR_ARRAY: {
        const uint32_t cnt = op.kind == RTPS_CDR_PRIM ? 1u : op.count;
        if (cnt == 0) break;
        const uint32_t pad = pad_to(pos, size);
        if ((uint64_t)pos + pad + (uint64_t)cnt * size > len) return RTPS_CDR_EOF;
        pos += pad;
        if (write)
          for (uint32_t e = 0; e < cnt; ++e) store_prim(d + e * size, load_prim(v + pos + e * size, size, le), size);
        pos += cnt * size;
        break;
      }
      case RTPS_CDR_BOOL:
        if (pos + 1 > len) return RTPS_CDR_EOF;
        if (v[pos] > 1) return RTPS_CDR_BAD_BOOL;
        if (write) d[0] = v[pos];
        pos += 1;
        break;
      case RTPS_CDR_STRING: {
        pos += pad_to(pos, 4);
        if ((uint64_t)pos + 4 > len) return RTPS_CDR_EOF;
        const uint32_t l = (uint32_t)load_prim(v + pos, 4, le);
        pos += 4;
        if ((uint64_t)pos + l > len) return RTPS_CDR_EOF;
        const uint32_t m = l ? l - 1 : 0;
        if (!utf8_ok(v + pos, m)) return RTPS_CDR_BAD_UTF8;
        if (m > op.count) return RTPS_CDR_TOO_LONG;
        if (write) {
          *(uint32_t*)d = m;
          copy_bytes(d + 4, v + pos, m);
        }
        pos += l;
        break;
      }
      case RTPS_CDR_SEQ: {
        pos += pad_to(pos, 4);
        if ((uint64_t)pos + 4 > len) return RTPS_CDR_EOF;
        const uint32_t n = (uint32_t)load_prim(v + pos, 4, le);
        pos += 4;
        if (n) {
          const uint32_t pe = pad_to(pos, size);
          if ((uint64_t)pos + pe + (uint64_t)n * size > len) return RTPS_CDR_EOF;
          if (n > op.count) return RTPS_CDR_TOO_LONG;
          pos += pe;
          if (write)
            for (uint32_t e = 0; e < n; ++e) store_prim(d + 4 + e * size, load_prim(v + pos + e * size, size, le), size);
          pos += n * size;
        }
        if (write) *(uint32_t*)d = n;
        break;
      }
      case RTPS_CDR_SEQ_BEGIN:
      case RTPS_CDR_ARRAY_BEGIN: {
        const bool seq = op.kind == RTPS_CDR_SEQ_BEGIN;
        uint32_t n = op.count;
        if (seq) {
          pos += pad_to(pos, 4);
          if ((uint64_t)pos + 4 > len) return RTPS_CDR_EOF;
          n = (uint32_t)load_prim(v + pos, 4, le);
          pos += 4;
          if (write) *(uint32_t*)d = n;
        }
        if (n > op.count && zero_el[k]) return RTPS_CDR_TOO_LONG;
        // elements that read no wire bytes also write nothing (zero-count arrays only): skipped,
        // so a crafted count cannot make the walk loop without consuming bytes
        if (n == 0 || zero_el[k]) { k = match[k]; break; }
        // base < 2^20 always (a row offset; 0 while nothing is stored), so it packs beside k
        const uint32_t elem0 = write ? base + op.out_off + (seq ? 4u : 0u) : 0u;
        fr[depth * 64u] = make_uint4(n, 0u, elem0, base | (k << 24) | (write ? 0x80000000u : 0u));
        write = write && op.count > 0;
        base = write ? elem0 : 0u;
        depth++;
        break;
      }
      case RTPS_CDR_END: {
        uint4 f = fr[(depth - 1) * 64u];
        const uint32_t begin = (f.w >> 24) & 63u;
        const bool fw = (f.w >> 31) != 0;
        const rtps_cdr_op b = ops[begin];
        if (++f.y < f.x) {
          fr[(depth - 1) * 64u].y = f.y;
          write = fw && f.y < b.count;
          base = write ? f.z + f.y * b.stride : 0u;  // (elements past the slot store nothing)
          k = begin;  // ++k: the element's first op
        } else {
          depth--;
          base = f.w & 0xfffffu;
          write = fw;
          if (f.x > b.count) return RTPS_CDR_TOO_LONG;
        }
        break;
      }
      default:
        return RTPS_CDR_TOO_LONG;
    }
  }
  return RTPS_CDR_OK;
}

__device__ __forceinline__ void zero_row(uint8_t* r, uint32_t bytes) {
  uint32_t b = 0;
  for (; b + 16 <= bytes; b += 16) st16u(r + b, make_uint4(0, 0, 0, 0));
  for (; b < bytes; b += 4) *(uint32_t*)(r + b) = 0u;
}

// One wave per chunk of 64 rows: lane = row.  The chunk's values (up to NEST_VCAP
// bytes each) are staged in LDS by the whole wave (16-B loads, all in flight
// together), so the lane-serial walk reads LDS, not HBM; longer values are read in
// place.
#ifndef CDR_NEST_VCAP
#define CDR_NEST_VCAP 128  // LDS 49 KB per block: 3 blocks (12 waves) per CU
#endif
constexpr uint32_t NEST_WAVES = 4, NEST_VCAP = CDR_NEST_VCAP, NEST_VQ = NEST_VCAP / 16;
__global__ __launch_bounds__(64 * NEST_WAVES) void cdr_nested_kernel(CdrNest N, CdrArgs a) {
  __shared__ rtps_cdr_op s_ops[RTPS_CDR_MAX_OPS];
  __shared__ uint8_t s_match[RTPS_CDR_MAX_OPS], s_zero[RTPS_CDR_MAX_OPS];
  __shared__ uint4 s_val[NEST_WAVES][64][NEST_VQ];
  __shared__ uint4 s_fr[NEST_WAVES][RTPS_CDR_MAX_DEPTH * 64];
  __shared__ uint64_t s_vb[NEST_WAVES][64];
  __shared__ uint32_t s_len[NEST_WAVES][64];
  if (threadIdx.x < N.n_ops) {
    s_ops[threadIdx.x] = N.ops[threadIdx.x];
    s_match[threadIdx.x] = N.match[threadIdx.x];
    s_zero[threadIdx.x] = N.zero_el[threadIdx.x];
  }
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63u, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t n = a.list ? min(*a.n_list, a.max_list) : min(*a.n_records, a.max_records);
  const uint64_t nrec = min(*a.n_records, a.max_records);
  const uint64_t chunks = (n + 63) / 64;
  for (uint64_t c = (uint64_t)blockIdx.x * NEST_WAVES + wave; c < chunks; c += (uint64_t)gridDim.x * NEST_WAVES) {
    const uint64_t r = c * 64 + lane;
    uint32_t st = RTPS_CDR_NOT_DATA, len = 0;
    uint64_t vb = 0;
    bool le = true;
    if (r < n) {
      const uint64_t ri = a.list ? *reinterpret_cast<const uint32_t*>(a.list + r * a.list_stride) : r;
      if (ri < nrec) {
        const uint8_t* rec = (const uint8_t*)(a.records + ri);
        const uint4 h0 = *(const uint4*)rec, h1 = *(const uint4*)(rec + 16);
        const uint2 u0 = *(const uint2*)(rec + 40);
        const uint32_t kind = (h0.y >> 16) & 0xff, pk = h1.w >> 24;
        const uint32_t pl_off = u0.x & 0xffff, pl_len = u0.x >> 16;
        const uint32_t id0 = u0.y & 0xff, id1 = (u0.y >> 8) & 0xff;
        if (kind != RTPS_DATA || pk != RTPS_PK_DATA || pl_len < 4) {
          st = RTPS_CDR_NOT_DATA;
        } else if (id0 != 0 || (id1 != 0 && id1 != 1 && id1 != 3)) {
          st = RTPS_CDR_BAD_ENCODING;
        } else {
          vb = a.dgram_off[h0.x] + pl_off + 4;
          len = pl_len - 4;
          le = id1 != 0;
          st = vb + len > a.arena_len ? (uint32_t)RTPS_CDR_NOT_DATA : 0xffu;  // 0xff: decode
        }
      }
    }
    s_vb[wave][lane] = vb;
    s_len[wave][lane] = (st == 0xffu && len <= NEST_VCAP) ? len : 0u;
    wave_sync();
#pragma unroll 8
    for (uint32_t k = 0; k < NEST_VQ; ++k) {  // unit u: row u / NEST_VQ, quad u % NEST_VQ
      const uint32_t u = k * 64u + lane, rw = u / NEST_VQ, q = u % NEST_VQ;
      const uint32_t L = s_len[wave][rw];
      if (16u * q < L) {
        const uint64_t abs = s_vb[wave][rw] + 16u * q;
        uint4 x;
        if (abs + 16 <= a.arena_len) {
          x = ld16u(a.arena + abs);
        } else {  // the arena's last bytes
          uint32_t w[4] = {0u, 0u, 0u, 0u};
          for (uint32_t b = 0; b < 16 && abs + b < a.arena_len; ++b) w[b >> 2] |= (uint32_t)a.arena[abs + b] << (8 * (b & 3));
          x = make_uint4(w[0], w[1], w[2], w[3]);
        }
        s_val[wave][rw][q] = x;
      }
    }
    {  // the chunk's rows zeroed by the whole wave (16 B per lane, consecutive), complete before any
       // lane stores into them (vmcnt(0): the stores are acknowledged)
      const uint64_t r0 = c * 64, nv = n - r0 < 64 ? n - r0 : 64;
      uint8_t* rowc = a.rows + r0 * N.row_bytes;
      const uint64_t bytes = nv * N.row_bytes;
      for (uint64_t b = 16u * lane; b < bytes; b += 1024u) {
        if (b + 16 <= bytes) st16u(rowc + b, make_uint4(0, 0, 0, 0));
        else for (uint64_t t2 = b; t2 < bytes; t2 += 4) *(uint32_t*)(rowc + t2) = 0u;
      }
      __builtin_amdgcn_s_waitcnt(0);  // (vector counters only: no scalar stores are issued)
    }
    wave_sync();
    if (r < n) {
      uint8_t* row = a.rows + r * N.row_bytes;
      if (st == 0xffu) {
        const uint8_t* v = len <= NEST_VCAP ? (const uint8_t*)&s_val[wave][lane][0] : a.arena + vb;
        st = nest_decode(s_ops, s_match, s_zero, N.n_ops, v, len, le, row, &s_fr[wave][lane]);
        if (st != RTPS_CDR_OK) zero_row(row, N.row_bytes);
      }
      a.row_status[r] = (uint8_t)st;
    }
    wave_sync();  // s_val / s_len are reused by the wave's next chunk
  }
}

}  // namespace

bool rtps_cdr_is_composite(const rtps_cdr_op* prog, uint32_t n_ops) {
  for (uint32_t k = 0; k < n_ops; ++k)
    if (prog[k].kind == RTPS_CDR_SEQ_BEGIN || prog[k].kind == RTPS_CDR_ARRAY_BEGIN || prog[k].kind == RTPS_CDR_END)
      return true;
  return false;
}

bool rtps_cdr_build_nested(const rtps_cdr_op* prog, uint32_t n_ops, uint32_t row_bytes, CdrNest& N) {
  if (n_ops > RTPS_CDR_MAX_OPS) return false;
  // the composite walk packs a slot's row offset into 20 bits beside its op index
  // (the LDS frame word restored with `f.w & 0xfffff`): wider rows cannot be framed
  if (row_bytes > (1u << 20)) return false;
  memset(&N, 0, sizeof(N));
  // open containers: the row, then one per open BEGIN (its element)
  struct Box { uint32_t begin, limit; uint64_t min_wire; };
  Box box[RTPS_CDR_MAX_DEPTH + 1];
  uint32_t iv_lo[RTPS_CDR_MAX_OPS], iv_hi[RTPS_CDR_MAX_OPS];
  uint32_t n_iv = 0, depth = 0;
  box[0] = Box{0u, row_bytes, 0u};
  auto close_box = [&](uint32_t from) -> bool {  // sibling slots of the box: no overlap
    for (uint32_t i = from; i < n_iv; ++i)
      for (uint32_t j = i + 1; j < n_iv; ++j)
        if (iv_lo[i] < iv_hi[j] && iv_lo[j] < iv_hi[i]) return false;
    return true;
  };
  uint32_t box_first[RTPS_CDR_MAX_DEPTH + 1] = {0};
  for (uint32_t k = 0; k < n_ops; ++k) {
    const rtps_cdr_op& op = prog[k];
    const uint64_t sz = op.size, cnt = op.count;
    const bool pow2 = sz == 1 || sz == 2 || sz == 4 || sz == 8;
    uint64_t slot = 0, wire = 0;
    switch (op.kind) {
      case RTPS_CDR_PRIM: if (!pow2) return false; slot = (sz + 3) / 4 * 4; wire = sz; break;
      case RTPS_CDR_BOOL: slot = 4; wire = 1; break;
      case RTPS_CDR_STRING: slot = 4 + (cnt + 3) / 4 * 4; wire = 4; break;
      case RTPS_CDR_SEQ: if (!pow2) return false; slot = 4 + (sz * cnt + 3) / 4 * 4; wire = 4; break;
      case RTPS_CDR_ARRAY: if (!pow2) return false; slot = (sz * cnt + 3) / 4 * 4; wire = sz * cnt; break;
      case RTPS_CDR_SEQ_BEGIN:
      case RTPS_CDR_ARRAY_BEGIN:
        if (op.stride < 4 || (op.stride & 3u) || depth >= RTPS_CDR_MAX_DEPTH) return false;
        slot = (op.kind == RTPS_CDR_SEQ_BEGIN ? 4u : 0u) + cnt * op.stride;
        break;
      case RTPS_CDR_END: {
        if (depth == 0) return false;
        Box& b = box[depth];
        if (!close_box(box_first[depth])) return false;
        n_iv = box_first[depth];
        const rtps_cdr_op& bo = prog[b.begin];
        N.match[b.begin] = (uint8_t)k;
        N.match[k] = (uint8_t)b.begin;
        N.zero_el[b.begin] = b.min_wire == 0;
        depth--;
        box[depth].min_wire += bo.kind == RTPS_CDR_SEQ_BEGIN ? 4u : b.min_wire * bo.count;
        N.ops[k] = op;
        continue;
      }
      default: return false;
    }
    if ((op.out_off & 3u) || (uint64_t)op.out_off + slot > box[depth].limit) return false;
    iv_lo[n_iv] = op.out_off;
    iv_hi[n_iv] = (uint32_t)(op.out_off + slot);
    n_iv++;
    box[depth].min_wire += wire;
    N.ops[k] = op;
    if (op.kind == RTPS_CDR_SEQ_BEGIN || op.kind == RTPS_CDR_ARRAY_BEGIN) {
      depth++;
      box[depth] = Box{k, op.stride, 0u};
      box_first[depth] = n_iv;
    }
  }
  if (depth != 0 || !close_box(0)) return false;
  N.n_ops = n_ops;
  N.row_bytes = row_bytes;
  return true;
}

int rtps_cdr_launch_nested(hipStream_t s, const CdrNest& N, const CdrArgs& a, uint32_t max_blocks) {
  const uint64_t rows = a.list ? a.max_list : a.max_records;
  uint64_t blocks = (rows + 64 * NEST_WAVES - 1) / (64 * NEST_WAVES);
  if (blocks > max_blocks) blocks = max_blocks;
  if (blocks == 0) return 0;
  hipLaunchKernelGGL(cdr_nested_kernel, dim3((uint32_t)blocks), dim3(64 * NEST_WAVES), 0, s, N, a);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

static uint32_t slot_dwords(const rtps_cdr_op& op) {
  const uint64_t sz = op.size;
  switch (op.kind) {
    case RTPS_CDR_PRIM: return (uint32_t)((sz + 3) / 4);
    case RTPS_CDR_BOOL: return 1;
    case RTPS_CDR_STRING: return (uint32_t)(1 + ((uint64_t)op.count + 3) / 4);
    case RTPS_CDR_SEQ: return (uint32_t)(1 + (sz * op.count + 3) / 4);
    default: return (uint32_t)((sz * op.count + 3) / 4);  // ARRAY
  }
}

static bool rtps_cdr_ostat(const CdrProg& P);

bool rtps_cdr_build_slots(CdrProg& P) {
  // op slots sorted by out_off (insertion sort: n_ops <= 64)
  uint32_t order[RTPS_CDR_MAX_OPS];
  for (uint32_t k = 0; k < P.n_ops; ++k) order[k] = k;
  for (uint32_t i = 1; i < P.n_ops; ++i)
    for (uint32_t j = i; j > 0 && P.ops[order[j - 1]].out_off > P.ops[order[j]].out_off; --j) {
      uint32_t t = order[j]; order[j] = order[j - 1]; order[j - 1] = t;
    }
  uint32_t ns = 0;
  uint64_t at = 0;
  bool full = false;
  auto push = [&](uint8_t kind, uint8_t size, uint32_t op, uint64_t off, uint64_t dw, uint32_t count) -> CdrSlot* {
    if (ns >= CDR_MAX_SLOTS) { full = true; return nullptr; }
    CdrSlot& S = P.slots[ns++];
    S = CdrSlot{};
    S.kind = kind; S.size = size; S.op = (uint16_t)op; S.out_off = (uint32_t)off; S.dwords = (uint32_t)dw;
    S.count = count;
    return &S;
  };
  uint32_t slot_of[RTPS_CDR_MAX_OPS];
  for (uint32_t i = 0; i < P.n_ops; ++i) {
    const rtps_cdr_op& op = P.ops[order[i]];
    slot_of[order[i]] = 0xffffffffu;
    if (op.out_off & 3u) return false;
    if (op.out_off < at) return false;  // overlap
    const uint64_t dw = slot_dwords(op);
    if (op.out_off + 4 * dw > P.row_bytes) return false;
    if (op.out_off > at) push(CDR_SLOT_ZERO, 0, 0, at, (op.out_off - at) / 4, 0);
    if (dw) {
      slot_of[order[i]] = ns;
      push(op.kind, op.size, order[i], op.out_off, dw, op.kind == RTPS_CDR_PRIM ? 1u : op.count);
    }
    at = op.out_off + 4 * dw;
  }
  if (at < P.row_bytes) push(CDR_SLOT_ZERO, 0, 0, at, (P.row_bytes - at) / 4, 0);
  // segments over the static prefix of the program (wire offsets known here)
  uint64_t w = 0;
  uint32_t k = 0, run0 = 0, run_n = 0;
  uint64_t run_wire = 0, run_out = 0, run_bytes = 0;
  auto close_run = [&]() {
    if (run_n >= 2) {
      CdrSlot* S = push(CDR_SLOT_SEG, 4, run0, run_out, run_bytes / 4, (uint32_t)run_wire);
      if (S)
        for (uint32_t t = run0; t < run0 + run_n; ++t) P.slots[slot_of[t]].flags |= CDR_IN_SEG;
    }
    run_n = 0;
  };
  for (; k < P.n_ops; ++k) {
    const rtps_cdr_op& op = P.ops[k];
    if (op.kind == RTPS_CDR_STRING || op.kind == RTPS_CDR_SEQ) break;  // wire offsets turn dynamic
    const uint64_t cnt = op.kind == RTPS_CDR_ARRAY ? op.count : 1u;
    const uint64_t sz = op.kind == RTPS_CDR_BOOL ? 1u : op.size;
    if (cnt == 0) {  // no bytes, no slot: ends a run (runs are consecutive op indices)
      close_run();
      continue;
    }
    w = (w + sz - 1) / sz * sz;
    const uint64_t bytes = sz * cnt;
    const bool cand = (op.kind == RTPS_CDR_PRIM || op.kind == RTPS_CDR_ARRAY) && sz >= 4 && w < (1ull << 32);
    if (cand && run_n && run_out + run_bytes == op.out_off && run_wire + run_bytes == w) {
      run_n++;
      run_bytes += bytes;
    } else {
      close_run();
      if (cand) { run0 = k; run_n = 1; run_wire = w; run_out = op.out_off; run_bytes = bytes; }
    }
    w += bytes;
  }
  close_run();
  if (full) return false;
  P.n_slots = ns;
  // output-stationary programs stage 32 B of every value per wave (+ the funnel's pad)
  P.lds_per_wave = 768u + 512u * P.n_ops + (CDR_OST_STAGE && rtps_cdr_ostat(P) ? 64u * CDR_STAGE_BYTES + 16u : 0u);
  return true;
}

// The output-stationary phase B: flat programs whose field offsets turn dynamic (a string or a
// sequence: no segment covers the fields behind it) with rows up to CDR_OSTAT_ROW bytes (the word
// table is 2 B per row byte of LDS).  RTPS_CDR_OSTAT=0 / 1 overrides (diagnosis).
#ifndef CDR_OSTAT_ROW
#define CDR_OSTAT_ROW 1024u
#endif
static bool rtps_cdr_ostat(const CdrProg& P) {
  static const int force = [] { const char* e = getenv("RTPS_CDR_OSTAT"); return e ? (e[0] == '1' ? 1 : 0) : -1; }();
  if (force >= 0) return force == 1 && P.row_bytes <= 8192u;
  if (P.row_bytes > CDR_OSTAT_ROW) return false;
  for (uint32_t k = 0; k < P.n_ops; ++k)
    if (P.ops[k].kind == RTPS_CDR_STRING || P.ops[k].kind == RTPS_CDR_SEQ) return true;
  return false;
}

// Grid cap: the kernel's own residency (its VGPRs and LDS) on every CU, cached per thread for the
// last (kernel, block, LDS) asked.  The context's resident_blocks is the parse kernel's; under it
// the 8-wave output-stationary kernel ran with a part of the chip idle (C3 list 183.6 -> 179.4 us,
// per-record 416 -> 387 us).  CDR_OCC_CAP=0: the old cap (diagnosis builds).
#ifndef CDR_OCC_CAP
#define CDR_OCC_CAP 1
#endif
static uint64_t cdr_grid_cap(const void* fn, uint32_t threads, size_t lds, uint32_t max_blocks) {
  if (!CDR_OCC_CAP) return (uint64_t)max_blocks * CDR_GRID_MULT;
  thread_local const void* c_fn = nullptr;
  thread_local uint32_t c_threads = 0;
  thread_local size_t c_lds = 0;
  thread_local int c_dev = -1;
  thread_local uint64_t c_cap = 0;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return max_blocks;
  if (fn != c_fn || threads != c_threads || lds != c_lds || dev != c_dev) {
    int cus = 0, per = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0 ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, fn, (int)threads, lds) != hipSuccess || per <= 0)
      return max_blocks;
    c_fn = fn; c_threads = threads; c_lds = lds; c_dev = dev;
    c_cap = (uint64_t)cus * (uint64_t)per * CDR_GRID_MULT;
  }
  return c_cap;
}

// Host launcher, called by rtps_rx_cdr_decode / _list (rtps_rx.hip) after validation.
int rtps_cdr_launch(hipStream_t s, const CdrProg& P, const CdrArgs& a, uint32_t max_blocks) {
#ifndef CDR_OST_WPB
#define CDR_OST_WPB 1  // one wave per block for the output-stationary kernel: C3 list 180.5 -> 177.7 us (2: 179.3)
#endif
  uint32_t wpb = 65536u / P.lds_per_wave;
  const uint32_t wmax = rtps_cdr_ostat(P) ? CDR_OST_WPB : 4u;
  wpb = wpb < 1 ? 1 : (wpb > wmax ? wmax : wpb);
  const uint64_t chunks = ((a.list ? a.max_list : a.max_records) + 63) / 64;
  uint64_t blocks = (chunks + wpb - 1) / wpb;
  bool wide = false;  // a segment of more than 32 quads: one record per pass (seg_copy<true>)
  for (uint32_t i = 0; i < P.n_slots; ++i)
    wide = wide || (P.slots[i].kind == CDR_SLOT_SEG && (P.slots[i].dwords + 3u) / 4u > 32u);
  const bool ost = rtps_cdr_ostat(P);
  const void* fn = ost ? (const void*)cdr_decode_kernel<false, true>
                 : wide ? (const void*)cdr_decode_kernel<true, false> : (const void*)cdr_decode_kernel<false, false>;
  const size_t lds = wpb * P.lds_per_wave + (ost ? 2u * P.row_bytes : 0u);
  // (the staged values live in each wave's table: lds_per_wave counts them for output-stationary programs)
  // the slot-walk kernels keep the context's cap: C2 at its own residency took 148 -> 172 us (T unchanged)
  const uint64_t cap = ost ? cdr_grid_cap(fn, 64 * wpb, lds, max_blocks) : (uint64_t)max_blocks * CDR_GRID_MULT;
  if (blocks > cap) blocks = cap;
  if (blocks == 0) return 0;
  if (ost) {
    hipLaunchKernelGGL((cdr_decode_kernel<false, true>), dim3((uint32_t)blocks), dim3(64 * wpb), lds, s, P, a);
  } else if (wide) {
    hipLaunchKernelGGL((cdr_decode_kernel<true, false>), dim3((uint32_t)blocks), dim3(64 * wpb), lds, s, P, a);
  } else {
    hipLaunchKernelGGL((cdr_decode_kernel<false, false>), dim3((uint32_t)blocks), dim3(64 * wpb), lds, s, P, a);
  }
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
