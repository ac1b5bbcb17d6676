// Diagnostic ceiling kernels for the parse's memory-traffic shape (not product code).
// mode 0: read 12 B (off,len) + 64-B head per datagram, write 64-B record + 1 B + 4 B (per-lane stores)
// mode 1: reads only (off,len + head), 1 B status write
// mode 2: writes only (records + status + rec_begin)
// mode 3: as 0 but the record is transposed through LDS and stored as contiguous 16-B pieces
#include <hip/hip_runtime.h>
#include <stdint.h>
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
template <int MODE>
__global__ __launch_bounds__(256) void ceil_kernel(const uint8_t* arena, const uint64_t* off, const uint32_t* len,
                                                   uint32_t n, u32x4* rec, uint8_t* status, uint32_t* rb) {
  __shared__ u32x4 lds[256 * 4];
  uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  u32x4 a = {0, 0, 0, 0}, b = a, c = a, d = a;
  uint32_t L = 0;
  if (MODE != 2) {
    uint64_t o = off[i];
    L = len[i];
    const u32x4* h = reinterpret_cast<const u32x4*>(arena + o);
    a = h[0]; b = h[1]; c = h[2]; d = h[3];
  } else {
    a[0] = i; b[1] = i; c[2] = i; d[3] = i;
  }
  a[1] ^= L;
  status[i] = (uint8_t)(a[0] ^ b[0] ^ c[0] ^ d[0]);
  if (MODE == 1) return;
  rb[i] = i;
  if (MODE == 3) {
    uint32_t t = threadIdx.x;
    lds[t * 4 + 0] = a; lds[t * 4 + 1] = b; lds[t * 4 + 2] = c; lds[t * 4 + 3] = d;
    __syncthreads();
    u32x4* base = rec + (uint64_t)blockIdx.x * 256 * 4;
    for (int k = 0; k < 4; ++k) base[k * 256 + t] = lds[k * 256 + t];
  } else {
    u32x4* r = rec + (uint64_t)i * 4;
    r[0] = a; r[1] = b; r[2] = c; r[3] = d;
  }
}
extern "C" int diag_ceiling(int mode, const uint8_t* arena, const uint64_t* off, const uint32_t* len, uint32_t n,
                            void* rec, uint8_t* status, uint32_t* rb, void* stream) {
  dim3 g((n + 255) / 256), b(256);
  hipStream_t s = (hipStream_t)stream;
  switch (mode) {
    case 0: hipLaunchKernelGGL(ceil_kernel<0>, g, b, 0, s, arena, off, len, n, (u32x4*)rec, status, rb); break;
    case 1: hipLaunchKernelGGL(ceil_kernel<1>, g, b, 0, s, arena, off, len, n, (u32x4*)rec, status, rb); break;
    case 2: hipLaunchKernelGGL(ceil_kernel<2>, g, b, 0, s, arena, off, len, n, (u32x4*)rec, status, rb); break;
    case 3: hipLaunchKernelGGL(ceil_kernel<3>, g, b, 0, s, arena, off, len, n, (u32x4*)rec, status, rb); break;
    default: return -1;
  }
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

// ---- copy ceilings for the CDR decode (T: 976 value bytes per datagram -> 976-B rows) ----
// mode 0: one wave per record, 16 B per lane (the decode's wide-slot shape)
// mode 1: flat grid, one 16-B quad per thread (pure streaming gather)
typedef uint4 u128u __attribute__((aligned(1)));
typedef uint4 u128u_v;
__global__ __launch_bounds__(256) void copy_wave_kernel(const uint8_t* arena, const uint64_t* off, uint32_t n,
                                                        uint8_t* rows, uint32_t row_bytes, uint32_t skip) {
  const uint32_t lane = threadIdx.x & 63, nq = row_bytes / 16;
  for (uint64_t r = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6); r < n; r += (uint64_t)gridDim.x * 4) {
    const uint8_t* src = arena + off[r] + skip;
    for (uint32_t q = lane; q < nq; q += 64)
      *(u128u*)(rows + r * row_bytes + 16 * q) = *(const u128u*)(src + 16 * q);
  }
}
__global__ __launch_bounds__(256) void copy_flat_kernel(const uint8_t* arena, const uint64_t* off, uint32_t n,
                                                        uint8_t* rows, uint32_t row_bytes, uint32_t skip) {
  const uint32_t nq = row_bytes / 16;
  const uint64_t total = (uint64_t)n * nq;
  for (uint64_t t = (uint64_t)blockIdx.x * 256 + threadIdx.x; t < total; t += (uint64_t)gridDim.x * 256) {
    const uint64_t r = t / nq, q = t - r * nq;
    *(u128u*)(rows + r * row_bytes + 16 * q) = *(const u128u*)(arena + off[r] + skip + 16 * q);
  }
}
// ---- copy ceilings for the DataFrag reassembly's shape (C4: 1344 B at datagram offset 56 -> heap) ----
// one wave per record, W-byte elements (W = 4 / 8 / 16), U elements in flight per lane, optional
// non-temporal stores; src alignment is whatever skip gives (56: 8-B aligned in the 16-B-aligned arena)
template <int W, int U, bool NT>
__global__ __launch_bounds__(256) void copy_w_kernel(const uint8_t* arena, const uint64_t* off, uint32_t n,
                                                     uint8_t* rows, uint32_t row_bytes, uint32_t skip) {
  typedef uint32_t e_t __attribute__((ext_vector_type(W / 4)));
  const uint32_t lane = threadIdx.x & 63, ne = row_bytes / W;
  for (uint64_t r = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6); r < n; r += (uint64_t)gridDim.x * 4) {
    const uint8_t* src = arena + off[r] + skip;
    uint8_t* dst = rows + r * row_bytes;
    for (uint32_t q0 = lane; q0 < ne; q0 += 64 * U) {
      e_t v[U];
#pragma unroll
      for (int k = 0; k < U; ++k) {
        const uint32_t q = q0 + 64 * k;
        if (q < ne) __builtin_memcpy(&v[k], src + (uint64_t)W * q, W);
      }
#pragma unroll
      for (int k = 0; k < U; ++k) {
        const uint32_t q = q0 + 64 * k;
        if (q < ne) {
          if (NT) __builtin_nontemporal_store(v[k], reinterpret_cast<e_t*>(dst + (uint64_t)W * q));
          else *reinterpret_cast<e_t*>(dst + (uint64_t)W * q) = v[k];
        }
      }
    }
  }
}
// R consecutive rows per wave as one flat list of 16-B chunks (lane l takes chunks l, l + 64, ...):
// every lane's loads of the R rows are in flight together (R x 1344 B per wave), and no lane idles
// on a row's 20-chunk tail
template <int R, bool NT>
__global__ __launch_bounds__(256) void copy_group_kernel(const uint8_t* arena, const uint64_t* off, uint32_t n,
                                                         uint8_t* rows, uint32_t row_bytes, uint32_t skip) {
  constexpr int MAXC = (R * 84 + 63) / 64;  // chunks per lane for rows of <= 1344 B
  const uint32_t lane = threadIdx.x & 63, ne = row_bytes / 16, tot = R * ne;
  const uint64_t nw = (uint64_t)gridDim.x * 4;
  for (uint64_t g = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6); g * R < n; g += nw) {
    u128u_v v[MAXC];
#pragma unroll
    for (int k = 0; k < MAXC; ++k) {
      const uint32_t c = lane + 64u * k, j = c / ne, q = c - j * ne;
      const uint64_t r = g * R + j;
      if (c < tot && r < n) v[k] = *(const u128u*)(arena + off[r] + skip + 16 * q);
    }
#pragma unroll
    for (int k = 0; k < MAXC; ++k) {
      const uint32_t c = lane + 64u * k, j = c / ne, q = c - j * ne;
      const uint64_t r = g * R + j;
      if (c < tot && r < n) {
        uint4* d = reinterpret_cast<uint4*>(rows + r * row_bytes + 16 * q);
        if (NT) {
          u32x4 w = {v[k].x, v[k].y, v[k].z, v[k].w};
          __builtin_nontemporal_store(w, reinterpret_cast<u32x4*>(d));
        } else {
          *d = v[k];
        }
      }
    }
  }
}
extern "C" int diag_copy_group(int r, int nt, const uint8_t* arena, const uint64_t* off, uint32_t n, uint8_t* rows,
                               uint32_t row_bytes, uint32_t skip, uint32_t blocks, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (row_bytes > 1344) return -1;
#define V(R, NT)                                                                                              \
  if (r == R && nt == NT) {                                                                                   \
    hipLaunchKernelGGL((copy_group_kernel<R, NT>), dim3(blocks), dim3(256), 0, s, arena, off, n, rows, row_bytes, skip); \
    return hipGetLastError() == hipSuccess ? 0 : -2;                                                          \
  }
  V(1, 1) V(2, 1) V(3, 1) V(4, 1) V(6, 1) V(3, 0)
#undef V
  return -1;
}
extern "C" int diag_copy_w(int w, int u, int nt, const uint8_t* arena, const uint64_t* off, uint32_t n, uint8_t* rows,
                           uint32_t row_bytes, uint32_t skip, uint32_t blocks, void* stream) {
  hipStream_t s = (hipStream_t)stream;
#define V(W, U, NT)                                                                                        \
  if (w == W && u == U && nt == NT) {                                                                      \
    hipLaunchKernelGGL((copy_w_kernel<W, U, NT>), dim3(blocks), dim3(256), 0, s, arena, off, n, rows, row_bytes, skip); \
    return hipGetLastError() == hipSuccess ? 0 : -2;                                                       \
  }
  V(16, 1, 0) V(16, 2, 0) V(16, 1, 1) V(16, 2, 1) V(8, 1, 1) V(8, 2, 1) V(8, 3, 1) V(4, 3, 1) V(4, 6, 1)
#undef V
  return -1;
}

extern "C" int diag_copy(int mode, const uint8_t* arena, const uint64_t* off, uint32_t n, uint8_t* rows,
                         uint32_t row_bytes, uint32_t skip, uint32_t blocks, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (mode == 0) hipLaunchKernelGGL(copy_wave_kernel, dim3(blocks), dim3(256), 0, s, arena, off, n, rows, row_bytes, skip);
  else if (mode == 1) hipLaunchKernelGGL(copy_flat_kernel, dim3(blocks), dim3(256), 0, s, arena, off, n, rows, row_bytes, skip);
  else return -1;
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

// ---- variants of mode 0 (read head + write record) probing the attainable rate ----
// HB: head bytes read (32/48/64); NTL/NTS: non-temporal loads / stores; PER: datagrams per lane
template <int HB, bool NTL, bool NTS, int PER>
__global__ __launch_bounds__(256) void ceil_var_kernel(const uint8_t* arena, const uint64_t* off, const uint32_t* len,
                                                       uint32_t n, u32x4* rec, uint8_t* status, uint32_t* rb) {
  const uint32_t base = blockIdx.x * 256 * PER + threadIdx.x;
  u32x4 a[PER], b[PER], c[PER], d[PER];
  uint32_t L[PER];
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const uint32_t i = base + k * 256;
    a[k] = b[k] = c[k] = d[k] = u32x4{0, 0, 0, 0};
    L[k] = 0;
    if (i < n) {
      const u32x4* h = reinterpret_cast<const u32x4*>(arena + off[i]);
      L[k] = len[i];
      if (NTL) {
        a[k] = __builtin_nontemporal_load(h);
        b[k] = __builtin_nontemporal_load(h + 1);
        if (HB >= 48) c[k] = __builtin_nontemporal_load(h + 2);
        if (HB >= 64) d[k] = __builtin_nontemporal_load(h + 3);
      } else {
        a[k] = h[0];
        b[k] = h[1];
        if (HB >= 48) c[k] = h[2];
        if (HB >= 64) d[k] = h[3];
      }
    }
  }
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const uint32_t i = base + k * 256;
    if (i >= n) continue;
    a[k][1] ^= L[k];
    status[i] = (uint8_t)(a[k][0] ^ b[k][0] ^ c[k][0] ^ d[k][0]);
    rb[i] = i;
    u32x4* r = rec + (uint64_t)i * 4;
    if (NTS) {
      __builtin_nontemporal_store(a[k], r);
      __builtin_nontemporal_store(b[k], r + 1);
      __builtin_nontemporal_store(c[k], r + 2);
      __builtin_nontemporal_store(d[k], r + 3);
    } else {
      r[0] = a[k]; r[1] = b[k]; r[2] = c[k]; r[3] = d[k];
    }
  }
}
extern "C" int diag_ceiling_var(int hb, int ntl, int nts, int per, const uint8_t* arena, const uint64_t* off,
                                const uint32_t* len, uint32_t n, void* rec, uint8_t* status, uint32_t* rb,
                                void* stream) {
  hipStream_t s = (hipStream_t)stream;
  dim3 b(256);
#define V(HB, L, S, P)                                                                                   \
  if (hb == HB && ntl == L && nts == S && per == P) {                                                    \
    hipLaunchKernelGGL((ceil_var_kernel<HB, L, S, P>), dim3((n + 256 * P - 1) / (256 * P)), b, 0, s, arena, off, \
                       len, n, (u32x4*)rec, status, rb);                                                 \
    return hipGetLastError() == hipSuccess ? 0 : -2;                                                     \
  }
  V(64, 0, 0, 1) V(48, 0, 0, 1) V(32, 0, 0, 1) V(64, 1, 0, 1) V(64, 0, 1, 1) V(64, 1, 1, 1) V(48, 1, 1, 1)
  V(64, 0, 0, 2) V(64, 0, 0, 4) V(48, 0, 1, 2) V(64, 1, 1, 2)
#undef V
  return -1;
}

// ---- the mixed-traffic (C3) floor: the parse's dependent header hops + its record stores ----
// Lane per datagram.  One hop per submessage: a 16-B load at the submessage start (the first
// from the 64-B head, as the parse), its length from the header (octetsToNextHeader in the
// submessage's byte order; 0 = to the end), then the next.  Every submessage the parse
// materialises gets a 64-B record built from the loaded window (no field decode, no validation,
// no classification) at the parse's own position (rec_begin, from the real parse; datagrams the
// parse dropped store nothing).  WALKS = 2: a first walk without stores before the storing one,
// as a count-then-write parse does.
__device__ __forceinline__ uint32_t hop_e16(uint32_t raw, bool le) {
  const uint32_t v = raw >> 16;
  return le ? v : (((v & 0xffu) << 8) | (v >> 8));
}
template <int WALKS>
__global__ __launch_bounds__(256) void ceil_hops_kernel(const uint8_t* arena, uint64_t arena_len, const uint64_t* off,
                                                        const uint32_t* len, uint32_t n, const uint8_t* status,
                                                        const uint32_t* rb, u32x4* rec) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const uint8_t* d = arena + off[i];
  const uint32_t L = len[i];
  const u32x4* h = reinterpret_cast<const u32x4*>(d);
  u32x4 h0 = {0u, 0u, 0u, 0u}, h1 = h0, h2 = h0, h3 = h0;
  if (off[i] + 64u <= arena_len) { h0 = h[0]; h1 = h[1]; h2 = h[2]; h3 = h[3]; }
  const bool ok = status[i] == 0;
  uint64_t r = rb[i];
  uint32_t guard = 0;
#pragma unroll 1
  for (int walk = 0; walk < WALKS; ++walk) {
    const bool store = walk == WALKS - 1 && ok;
    uint32_t o = 20;
    while (o + 4u <= L && guard < 20000u) {
      ++guard;
      u32x4 w;
      if (o == 20u) {
        w = u32x4{h1[1], h1[2], h1[3], h2[0]};
      } else if (o + 16u <= ((L + 15u) & ~15u)) {  // inside the datagram's 16-B slot of the arena
        __builtin_memcpy(&w, d + o, 16);
      } else {
        w = u32x4{0u, 0u, 0u, 0u};
        for (uint32_t k = 0; k < 4; ++k) w[0] |= (uint32_t)d[o + k] << (8u * k);
      }
      const uint32_t kind = w[0] & 0xffu;
      const bool le = (w[0] >> 8) & 1u;
      uint32_t blen = hop_e16(w[0], le);
      if (blen == 0u && kind != 0x01u && kind != 0x09u) blen = L - o - 4u;
      const bool emits = kind == 0x06u || kind == 0x07u || kind == 0x08u || kind == 0x09u || kind == 0x0cu ||
                         kind == 0x0eu || kind == 0x0fu || kind == 0x12u || kind == 0x13u || kind == 0x15u ||
                         kind == 0x16u;
      if (store && emits) {
        u32x4* q = rec + r * 4;
        q[0] = u32x4{i, o | (kind << 16), h0[2], h0[3]};
        q[1] = u32x4{h1[0], w[1], w[2], blen};
        q[2] = u32x4{w[3], w[1] ^ w[2], h3[0], h3[1]};
        q[3] = u32x4{w[0], h2[1], h2[2], h2[3]};
        ++r;
      }
      o += 4u + blen;
    }
  }
}
extern "C" int diag_ceiling_hops(int walks, const uint8_t* arena, uint64_t arena_len, const uint64_t* off,
                                 const uint32_t* len, uint32_t n, const uint8_t* status, const uint32_t* rb, void* rec,
                                 void* stream) {
  hipStream_t s = (hipStream_t)stream;
  dim3 g((n + 255) / 256), b(256);
  if (walks == 1)
    hipLaunchKernelGGL(ceil_hops_kernel<1>, g, b, 0, s, arena, arena_len, off, len, n, status, rb, (u32x4*)rec);
  else if (walks == 2)
    hipLaunchKernelGGL(ceil_hops_kernel<2>, g, b, 0, s, arena, arena_len, off, len, n, status, rb, (u32x4*)rec);
  else return -1;
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

// ---- the history-cache ingest's floor ----
// The bytes the ingest must move, at its real scatter pattern, and nothing else: every 64-B
// record read (one 16-B load per lane of a quad: the record's four quads by four lanes, so a
// wave reads 16 records back to back), 1 accept byte written per record; per EVENT (a writer
// record that passes and reaches a proxy: DATA / HEARTBEAT / GAP with MATCHED) the proxy's 8-B
// state read and 4 B of its change-set bitmap written at the SN's word (a plain store: the
// traffic, not the atomics; the window's layout: 2^17 bits per proxy); per DELIVERY (a DATA
// sample with a proxy) 8 B written at the record's index (the deliveries' compaction is a
// scan in the ingest; a counter here would serialise on one address).  The proxy is the
// record's target set (one proxy per writer set when one reader subscribes to every writer,
// as in bench.py).
constexpr uint32_t ING_WW = (1u << 17) / 32u;  // change-set words per proxy
__global__ __launch_bounds__(256) void ceil_ingest_kernel(const u32x4* rec, const uint32_t* target, uint64_t n_rec,
                                                          const uint64_t* state, uint32_t* bits, uint8_t* accept,
                                                          uint64_t* dels, unsigned long long* n_del,
                                                          uint32_t n_sets) {
  const uint64_t t = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  const uint64_t i = t >> 2;  // the record of this lane's quad
  const uint32_t q = threadIdx.x & 3u, lane = threadIdx.x & 63u;
  u32x4 v = {0u, 0u, 0u, 0u};
  if (i < n_rec) v = rec[i * 4 + q];
  // quad 0 has dgram_idx, sub_off | kind << 16; quad 1 word 3 = aux16 | route << 16 | pk << 24; quad 2 = sn
  const uint32_t w1 = __shfl(v[1], (lane & ~3u) + 0u, 64), w7 = __shfl(v[3], (lane & ~3u) + 1u, 64);
  const uint32_t sn = __shfl(v[0], (lane & ~3u) + 2u, 64);
  const uint32_t kind = (w1 >> 16) & 0xffu, route = (w7 >> 16) & 0xffu;
  bool event = false, del = false;
  if (q == 0 && i < n_rec) {
    accept[i] = 0;
    const bool matched = (route & 0x01u) && (route & 0x20u);  // PASS and MATCHED
    event = matched && (kind == 0x15u || kind == 0x07u || kind == 0x08u);
    del = event && kind == 0x15u;
  }
  if (event) {
    const uint32_t e = target[i] < n_sets ? target[i] : 0u;
    const uint64_t st = state[e];
    bits[(uint64_t)e * ING_WW + ((sn + (uint32_t)st) & ((1u << 17) - 1u)) / 32u] = 1u << (sn & 31u);
  }
  if (del) dels[i] = i | ((uint64_t)1 << 32);
  (void)n_del;
}
extern "C" int diag_ceiling_ingest(const void* rec, const uint32_t* target, uint64_t n_rec, const uint64_t* state,
                                   uint32_t* bits, uint8_t* accept, uint64_t* dels, uint64_t* n_del, uint32_t n_sets,
                                   void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (hipMemsetAsync(n_del, 0, 8, s) != hipSuccess) return -2;
  const uint64_t threads = 4 * n_rec;
  hipLaunchKernelGGL(ceil_ingest_kernel, dim3((uint32_t)((threads + 255) / 256)), dim3(256), 0, s,
                     (const u32x4*)rec, target, n_rec, state, bits, accept, dels, (unsigned long long*)n_del, n_sets);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
