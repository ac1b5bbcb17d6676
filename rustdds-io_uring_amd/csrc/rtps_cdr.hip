// rtps_cdr.hip — batch CDR primitive decode of DATA payloads.
//
// Replaces, for fixed-layout sample types, the per-sample decode chain
//   SimpleDataReader::deserialize_with      io_uring/dds/with_key/simpledatareader.rs:137-160
//   -> CDRDeserializerAdapter (REPR_IDS)     serialization/cdr_adapters.rs:96-100
//   -> deserialize_from_cdr_with_decoder_and_rep_id   cdr_adapters.rs:246-275
//   -> cdr_encoding::CdrDeserializer         (external crate cdr-encoding 0.10)
// The sample type is a flat program of ops (rtps_cdr_op), wave-uniform (a
// kernel argument).  A wave takes 64 records: each lane validates one record
// and leaves its per-op data offsets in LDS; then the whole wave writes the 64
// rows slot by slot, one 4-byte word per lane, so row stores are coalesced and
// every row byte is written once (failed rows as zeros).
//
// Roofline: HBM-bound.  Algorithmic bytes per record = 40 B of the record +
// the value bytes a decoded row consumes + row_bytes + 1 status byte written.
#include <hip/hip_runtime.h>
#include <stdint.h>

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

// std::str::from_utf8 acceptance over m bytes.
__device__ bool utf8_ok(const uint8_t* s, uint32_t m) {
  uint32_t i = 0;
  while (i < m) {
    // ASCII fast path: 4 bytes at a time
    if (i + 4 <= m) {
      uint32_t w = *(const u32u*)(s + i);
      if ((w & 0x80808080u) == 0) { i += 4; continue; }
    }
    uint32_t c = s[i];
    if (c < 0x80) { i++; continue; }
    uint32_t need, lo = 0x80, hi = 0xBF;
    if (c >= 0xC2 && c <= 0xDF) need = 1;
    else if (c >= 0xE0 && c <= 0xEF) { need = 2; lo = (c == 0xE0) ? 0xA0 : 0x80; hi = (c == 0xED) ? 0x9F : 0xBF; }
    else if (c >= 0xF0 && c <= 0xF4) { need = 3; lo = (c == 0xF0) ? 0x90 : 0x80; hi = (c == 0xF4) ? 0x8F : 0xBF; }
    else return false;
    if (i + need >= m) return false;
    uint32_t b1 = s[i + 1];
    if (b1 < lo || b1 > hi) return false;
    for (uint32_t k = 2; k <= need; ++k) {
      uint32_t b = s[i + k];
      if (b < 0x80 || b > 0xBF) return false;
    }
    i += need + 1;
  }
  return true;
}

// Phase A (one lane per record): walk the program, return the status and
// record each op's data start (pos) and run-time length (string chars /
// sequence elements) in the wave's LDS table.  Reads only lengths, bools and
// string bytes.
__device__ uint8_t cdr_validate(const CdrProg& P, const uint8_t* v, uint32_t len, bool le, uint32_t* posT,
                                uint32_t* lenT, uint32_t lane) {
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
        const uint32_t l = (uint32_t)load_prim(v + pos, 4, le);
        pos += 4;
        if ((uint64_t)pos + l > len) return RTPS_CDR_EOF;
        const uint32_t m = l ? l - 1 : 0;
        if (!utf8_ok(v + pos, m)) return RTPS_CDR_BAD_UTF8;
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

// Word j of a run of nb bytes of `size`-byte elements at src, in host order;
// bytes at or past nb are zero and never read.
__device__ __forceinline__ uint32_t data_word(const uint8_t* src, uint32_t j, uint32_t nb, uint32_t size, bool le) {
  const uint32_t b = 4u * j;
  if (b >= nb) return 0u;
  uint32_t x;
  if (b + 4 <= nb) {
    x = *(const u32u*)(src + ((!le && size == 8) ? (b ^ 4u) : b));
  } else {  // 1..3 trailing bytes (size 1 or 2 only)
    x = 0;
    for (uint32_t t = 0; t < nb - b; ++t) x |= (uint32_t)src[b + t] << (8 * t);
  }
  if (!le) {
    if (size == 2) x = ((x & 0xff00ff00u) >> 8) | ((x & 0x00ff00ffu) << 8);
    else if (size >= 4) x = __builtin_bswap32(x);
  }
  return x;
}

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

extern __shared__ uint8_t cdr_lds[];

// One wave per chunk of 64 records.  Phase A: lane = record (validation, LDS
// table).  Phase B: the wave writes the chunk's rows slot by slot, one 4-byte
// word per lane and item (item = record x word of the slot), so consecutive
// lanes store consecutive words and every row byte is written exactly once.
__global__ __launch_bounds__(256) void cdr_decode_kernel(CdrProg P, CdrArgs a) {
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6, wpb = blockDim.x >> 6;
  uint8_t* T = cdr_lds + wave * P.lds_per_wave;
  uint32_t* meta = (uint32_t*)T;             // [64] status | le << 8
  uint64_t* vbase = (uint64_t*)(T + 256);    // [64] arena offset of the value
  uint32_t* posT = (uint32_t*)(T + 768);     // [n_ops][64]
  uint32_t* lenT = posT + P.n_ops * 64u;     // [n_ops][64]
  const uint64_t n = min(*a.n_records, a.max_records);
  const uint64_t chunks = (n + 63) / 64;
  for (uint64_t c = (uint64_t)blockIdx.x * wpb + wave; c < chunks; c += (uint64_t)gridDim.x * wpb) {
    const uint64_t r0 = c * 64;
    const uint32_t nv = (uint32_t)min<uint64_t>(64, n - r0);
    // ---- phase A ----
    uint32_t st = 0xff, le = 1;
    uint64_t vb = 0;
    if (lane < nv) {
      const rtps_record* rec = a.records + r0 + lane;
      // bytes 0..31 (dgram_idx @0, kind @6, payload_kind @31) and 40..47 (pl_off, pl_len, rep_id)
      const uint4 h0 = *(const uint4*)rec;
      const uint4 h1 = *(const uint4*)((const uint8_t*)rec + 16);
      const uint2 u0 = *(const uint2*)((const uint8_t*)rec + 40);
      const uint32_t kind = (h0.y >> 16) & 0xff, pk = h1.w >> 24;
      const uint32_t pl_off = u0.x & 0xffff, pl_len = u0.x >> 16;
      const uint32_t id0 = u0.y & 0xff, id1 = (u0.y >> 8) & 0xff;
      if (kind != RTPS_DATA || pk != RTPS_PK_DATA || pl_len < 4) {
        st = RTPS_CDR_NOT_DATA;
      } else if (id0 != 0 || (id1 != 0 && id1 != 1 && id1 != 3)) {
        st = RTPS_CDR_BAD_ENCODING;
      } else {
        vb = a.dgram_off[h0.x] + pl_off + 4;
        const uint32_t len = pl_len - 4;
        le = id1 != 0;
        st = (vb + len > a.arena_len) ? (uint32_t)RTPS_CDR_NOT_DATA  // cannot happen for parse outputs
                                      : cdr_validate(P, a.arena + vb, len, le, posT, lenT, lane);
      }
      a.row_status[r0 + lane] = (uint8_t)st;
    }
    meta[lane] = st | (le << 8);
    vbase[lane] = vb;
    wave_sync();
    // ---- phase B ----
    uint8_t* rowc = a.rows + r0 * P.row_bytes;
    for (uint32_t si = 0; si < P.n_slots; ++si) {
      const CdrSlot S = P.slots[si];
      const uint32_t total = nv * S.dwords;
      for (uint32_t item = lane; item < total; item += 64) {
        uint32_t rec = (uint32_t)((float)item * S.inv_dwords);
        if (rec * S.dwords > item) rec--;
        else if ((rec + 1) * S.dwords <= item) rec++;
        const uint32_t k = item - rec * S.dwords;
        const uint32_t m = meta[rec];
        uint32_t val = 0;
        if ((m & 0xffu) == RTPS_CDR_OK && S.kind != CDR_SLOT_ZERO) {
          const bool lle = (m >> 8) != 0;
          const uint8_t* src = a.arena + vbase[rec] + posT[S.op * 64u + rec];
          switch (S.kind) {
            case RTPS_CDR_PRIM:
            case RTPS_CDR_ARRAY: val = data_word(src, k, S.count * S.size, S.size, lle); break;
            case RTPS_CDR_BOOL: val = src[0]; break;
            case RTPS_CDR_STRING: {
              const uint32_t ln = lenT[S.op * 64u + rec];
              val = k == 0 ? ln : data_word(src, k - 1, ln, 1, lle);
              break;
            }
            default: {  // SEQ
              const uint32_t ln = lenT[S.op * 64u + rec];
              val = k == 0 ? ln : data_word(src, k - 1, ln * S.size, S.size, lle);
              break;
            }
          }
        }
        *(uint32_t*)(rowc + (uint64_t)rec * P.row_bytes + S.out_off + 4u * k) = val;
      }
    }
    wave_sync();  // the LDS table is reused by the wave's next chunk
  }
}

}  // namespace

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
  auto push = [&](uint8_t kind, uint8_t size, uint32_t op, uint64_t off, uint64_t dw, uint32_t count) {
    CdrSlot& S = P.slots[ns++];
    S.kind = kind; S.size = size; S.op = (uint16_t)op; S.out_off = (uint32_t)off; S.dwords = (uint32_t)dw;
    S.count = count; S.inv_dwords = 1.0f / (float)dw;
  };
  for (uint32_t i = 0; i < P.n_ops; ++i) {
    const rtps_cdr_op& op = P.ops[order[i]];
    if (op.out_off & 3u) return false;
    if (op.out_off < at) return false;  // overlap
    const uint64_t dw = slot_dwords(op);
    if (op.out_off + 4 * dw > P.row_bytes) return false;
    if (op.out_off > at) push(CDR_SLOT_ZERO, 0, 0, at, (op.out_off - at) / 4, 0);
    if (dw) push(op.kind, op.size, order[i], op.out_off, dw, op.kind == RTPS_CDR_PRIM ? 1u : op.count);
    at = op.out_off + 4 * dw;
  }
  if (at < P.row_bytes) push(CDR_SLOT_ZERO, 0, 0, at, (P.row_bytes - at) / 4, 0);
  P.n_slots = ns;
  P.lds_per_wave = 768u + 512u * P.n_ops;
  return true;
}

// Host launcher, called by rtps_rx_cdr_decode (rtps_rx.hip) after validation.
int rtps_cdr_launch(hipStream_t s, const CdrProg& P, const CdrArgs& a, uint32_t max_blocks) {
  uint32_t wpb = 65536u / P.lds_per_wave;
  wpb = wpb < 1 ? 1 : (wpb > 4 ? 4 : wpb);
  const uint64_t chunks = (a.max_records + 63) / 64;
  uint64_t blocks = (chunks + wpb - 1) / wpb;
  if (blocks > max_blocks) blocks = max_blocks;
  if (blocks == 0) return 0;
  hipLaunchKernelGGL(cdr_decode_kernel, dim3((uint32_t)blocks), dim3(64 * wpb), wpb * P.lds_per_wave, s, P, a);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
