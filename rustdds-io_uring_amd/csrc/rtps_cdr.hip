// rtps_cdr.hip — batch CDR primitive decode of DATA payloads.
//
// Replaces, for fixed-layout sample types, the per-sample decode chain
//   SimpleDataReader::deserialize_with      io_uring/dds/with_key/simpledatareader.rs:137-160
//   -> CDRDeserializerAdapter (REPR_IDS)     serialization/cdr_adapters.rs:96-100
//   -> deserialize_from_cdr_with_decoder_and_rep_id   cdr_adapters.rs:246-275
//   -> cdr_encoding::CdrDeserializer         (external crate cdr-encoding 0.10)
// The sample type is a flat program of ops (rtps_cdr_op); every record of the
// parse output is one lane.  The program is wave-uniform (kernel argument),
// the byte offsets are per lane.  Two passes per lane: validate (reads only
// lengths, bools and string bytes) then write, so an error never leaves a
// half-written row and no byte of a row is written twice except the zero fill.
//
// Roofline: HBM-bound.  Algorithmic bytes per record = the decoded payload
// bytes read + row_bytes written.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/rtps_rx.h"
#include "rtps_cdr.h"

namespace {

typedef uint16_t u16u __attribute__((aligned(1)));
typedef uint32_t u32u __attribute__((aligned(1)));
typedef uint64_t u64u __attribute__((aligned(1)));

constexpr int CDR_TILE = 256;

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

// Pass 1: walk the program, return status.  Reads lengths, bools, strings.
__device__ uint8_t cdr_validate(const CdrProg& P, const uint8_t* v, uint32_t len, bool le) {
  uint32_t pos = 0;
  for (uint32_t k = 0; k < P.n_ops; ++k) {
    const rtps_cdr_op op = P.ops[k];
    const uint32_t size = op.size;
    switch (op.kind) {
      case RTPS_CDR_PRIM:
      case RTPS_CDR_ARRAY: {
        const uint32_t cnt = op.kind == RTPS_CDR_PRIM ? 1u : op.count;
        if (cnt == 0) break;
        const uint32_t pad = pad_to(pos, size);
        if ((uint64_t)pos + pad + (uint64_t)cnt * size > len) return RTPS_CDR_EOF;
        pos += pad + cnt * size;
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
          pos += pe + n * size;
        }
        break;
      }
      default:
        return RTPS_CDR_TOO_LONG;
    }
  }
  return RTPS_CDR_OK;
}

// Pass 2: the payload is known to hold the whole type; write the fields.
// The row was zero-filled before, so slot tails stay zero.
__device__ void cdr_write(const CdrProg& P, const uint8_t* v, bool le, uint8_t* row) {
  uint32_t pos = 0;
  for (uint32_t k = 0; k < P.n_ops; ++k) {
    const rtps_cdr_op op = P.ops[k];
    const uint32_t size = op.size;
    uint8_t* d = row + op.out_off;
    switch (op.kind) {
      case RTPS_CDR_PRIM:
      case RTPS_CDR_ARRAY: {
        const uint32_t cnt = op.kind == RTPS_CDR_PRIM ? 1u : op.count;
        if (cnt == 0) break;
        pos += pad_to(pos, size);
        if (le) {  // bulk copy, 4 bytes at a time
          const uint32_t nb = cnt * size;
          uint32_t b = 0;
          for (; b + 4 <= nb; b += 4) *(u32u*)(d + b) = *(const u32u*)(v + pos + b);
          for (; b < nb; ++b) d[b] = v[pos + b];
        } else {
          for (uint32_t e = 0; e < cnt; ++e) store_prim(d + e * size, load_prim(v + pos + e * size, size, false), size);
        }
        pos += cnt * size;
        break;
      }
      case RTPS_CDR_BOOL:
        d[0] = v[pos];
        pos += 1;
        break;
      case RTPS_CDR_STRING: {
        pos += pad_to(pos, 4);
        const uint32_t l = (uint32_t)load_prim(v + pos, 4, le);
        pos += 4;
        const uint32_t m = l ? l - 1 : 0;
        *(u32u*)d = m;
        uint32_t b = 0;
        for (; b + 4 <= m; b += 4) *(u32u*)(d + 4 + b) = *(const u32u*)(v + pos + b);
        for (; b < m; ++b) d[4 + b] = v[pos + b];
        pos += l;
        break;
      }
      case RTPS_CDR_SEQ: {
        pos += pad_to(pos, 4);
        const uint32_t n = (uint32_t)load_prim(v + pos, 4, le);
        pos += 4;
        *(u32u*)d = n;
        if (n) {
          pos += pad_to(pos, size);
          for (uint32_t e = 0; e < n; ++e)
            store_prim(d + 4 + e * size, load_prim(v + pos + e * size, size, le), size);
          pos += n * size;
        }
        break;
      }
      default:
        break;
    }
  }
}

__global__ __launch_bounds__(CDR_TILE) void cdr_decode_kernel(CdrProg P, CdrArgs a) {
  const uint64_t n = min(*a.n_records, a.max_records);
  const uint64_t stride = (uint64_t)gridDim.x * CDR_TILE;
  for (uint64_t r = (uint64_t)blockIdx.x * CDR_TILE + threadIdx.x; r < n; r += stride) {
    const rtps_record* rec = a.records + r;
    // bytes 0..31 (dgram_idx @0, kind @6, payload_kind @31) and 40..47 (pl_off, pl_len, rep_id)
    const uint4 h0 = *(const uint4*)rec;
    const uint4 h1 = *(const uint4*)((const uint8_t*)rec + 16);
    const uint2 u0 = *(const uint2*)((const uint8_t*)rec + 40);
    const uint32_t dgram = h0.x;
    const uint32_t kind = (h0.y >> 16) & 0xff;
    const uint32_t pk = h1.w >> 24;
    const uint32_t pl_off = u0.x & 0xffff, pl_len = u0.x >> 16;
    const uint32_t id0 = u0.y & 0xff, id1 = (u0.y >> 8) & 0xff;

    uint8_t* row = a.rows + r * (uint64_t)P.row_bytes;
    for (uint32_t b = 0; b < P.row_bytes; b += 4) *(uint32_t*)(row + b) = 0u;

    uint8_t st;
    if (kind != RTPS_DATA || pk != RTPS_PK_DATA || pl_len < 4) {
      st = RTPS_CDR_NOT_DATA;
    } else if (id0 != 0 || (id1 != 0 && id1 != 1 && id1 != 3)) {
      st = RTPS_CDR_BAD_ENCODING;
    } else {
      const uint64_t base = a.dgram_off[dgram] + pl_off + 4;
      const uint32_t len = pl_len - 4;
      if (base + len > a.arena_len) {
        st = RTPS_CDR_NOT_DATA;  // cannot happen for parse outputs; never read out of bounds
      } else {
        const uint8_t* v = a.arena + base;
        const bool le = id1 != 0;
        st = cdr_validate(P, v, len, le);
        if (st == RTPS_CDR_OK) cdr_write(P, v, le, row);
      }
    }
    a.row_status[r] = st;
  }
}

}  // namespace

// Host launcher, called by rtps_rx_cdr_decode (rtps_rx.hip) after validation.
int rtps_cdr_launch(hipStream_t s, const CdrProg& P, const CdrArgs& a, uint32_t max_blocks) {
  uint64_t blocks = (a.max_records + CDR_TILE - 1) / CDR_TILE;
  if (blocks > max_blocks) blocks = max_blocks;
  if (blocks == 0) return 0;
  hipLaunchKernelGGL(cdr_decode_kernel, dim3((uint32_t)blocks), dim3(CDR_TILE), 0, s, P, a);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
