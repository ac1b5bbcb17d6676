// rtps_bsort.h — the reassembly's key sort: a stable sort of (32-bit hash key,
// record index) pairs, index = position, keys of 0xffffffff (records that are not
// assembled) last.  Replaces rocprim's device sort for batches of up to MAX_N
// records: at 1M pairs rocprim runs a ten-pass merge sort (~150 us, twenty
// launches) and Onesweep needs four 8-bit digits (~30 us each); the keys are
// uniform hashes, so one bucket pass on the top byte plus an LDS sort of each
// bucket's low 24 bits does the same work in four launches.
//
//  1 hist     per 4096-key tile, the count of each bucket (the top BB key bits;
//             the 0xffffffff keys get the last bucket), stored bucket-major
//  2 colscan  one workgroup per bucket: exclusive scan over the tiles, and the
//             bucket's total
//  3 scatter  per tile, each key's stable rank inside its bucket (wave ballots on
//             the bucket bits, then the waves in order), written as key:index at
//             bucket base (a scan of the totals, redone per workgroup from L2) +
//             tile offset + rank
//  4 sub      one workgroup per bucket: rocprim's block radix sort of up to SCAP
//             pairs on the key's low 32 - BB bits (stable: the bucket holds them
//             in index order).  A larger bucket that is already in key order (one
//             large sample's fragments) is copied; any other larger bucket takes
//             an LSD pass per key byte through global memory, SCAP pairs at a time.
//             The last bucket (keys 0xffffffff, in index order) is copied by every
//             workgroup's share.
// The result is the one a stable radix sort on all 32 key bits gives.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <rocprim/block/block_radix_sort.hpp>

namespace rtps_bsort {

#ifndef RTPS_BSORT_BITS
#define RTPS_BSORT_BITS 8
#endif
#ifndef RTPS_BSORT_ST
#define RTPS_BSORT_ST 1024
#endif
constexpr uint32_t KSENT = 0xffffffffu;
constexpr uint32_t BT = 256, BI = 16, TILE = BT * BI;  // tile: 4096 keys per workgroup
constexpr uint32_t BB = RTPS_BSORT_BITS;               // bucket bits (top of the key)
constexpr uint32_t NR = 1u << BB, NB = NR + 1;         // key buckets, then the 0xffffffff one
constexpr uint32_t LOW = 32 - BB;                      // key bits sorted inside a bucket
constexpr uint32_t ST = RTPS_BSORT_ST, SI = 8, SCAP = ST * SI;  // bucket sort: pairs per LDS pass
constexpr uint64_t MAX_N = 3ull << 19;                 // 1.5M keys: uniform buckets stay under SCAP
static_assert(MAX_N / TILE <= 2 * BT, "colscan: two tiles per thread");
static_assert(MAX_N / NR * 5 / 4 <= SCAP, "uniform buckets fit one LDS pass");

__device__ __forceinline__ uint32_t bucket_of(uint32_t k) { return k == KSENT ? NR : k >> LOW; }

__global__ __launch_bounds__(BT) void k_hist(const uint32_t* keys, uint32_t n, uint32_t T, uint32_t* H) {
  __shared__ uint32_t h[NB];
  for (uint32_t b = threadIdx.x; b < NB; b += BT) h[b] = 0u;
  __syncthreads();
  const uint32_t t = blockIdx.x, lane = threadIdx.x & 63u;
  for (uint32_t r = 0; r < BI; ++r) {
    const uint32_t i = t * TILE + r * BT + threadIdx.x;
    const bool v = i < n;
    const uint32_t b = v ? bucket_of(keys[i]) : 0u;
    const uint32_t b0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)b);
    const uint64_t all = __ballot(v), same = __ballot(v && b == b0);
    if (same == all) {  // one bucket for the whole wave (the 0xffffffff tail, one sample's run)
      if (lane == 0) atomicAdd(&h[b0], (uint32_t)__popcll(all));
    } else if (v) {
      atomicAdd(&h[b], 1u);
    }
  }
  __syncthreads();
  for (uint32_t b = threadIdx.x; b < NB; b += BT) H[(uint64_t)b * T + t] = h[b];
}

// per bucket b: H[b][t] -> exclusive prefix over tiles t, tot[b] = the bucket's count.
// Workgroups past the NB buckets run the caller's side job (side(i), i < side.wgs,
// BT threads): work that needs the keys' producer finished and must be done
// before the sorted output is used, without a launch of its own.
struct NoSide {
  uint32_t wgs = 0;
  __device__ void operator()(uint32_t) const {}
};
template <class Side>
__global__ __launch_bounds__(BT) void k_colscan(uint32_t* H, uint32_t T, uint32_t* tot, Side side) {
  if (blockIdx.x >= NB) { side(blockIdx.x - NB); return; }
  __shared__ uint32_t s[BT];
  uint32_t* h = H + (uint64_t)blockIdx.x * T;
  const uint32_t t0 = 2 * threadIdx.x;
  const uint32_t a = t0 < T ? h[t0] : 0u, b = t0 + 1 < T ? h[t0 + 1] : 0u;
  s[threadIdx.x] = a + b;
  __syncthreads();
  for (uint32_t d = 1; d < BT; d <<= 1) {
    const uint32_t v = threadIdx.x >= d ? s[threadIdx.x - d] : 0u;
    __syncthreads();
    s[threadIdx.x] += v;
    __syncthreads();
  }
  const uint32_t ex = s[threadIdx.x] - a - b;
  if (t0 < T) h[t0] = ex;
  if (t0 + 1 < T) h[t0 + 1] = ex + a;
  if (threadIdx.x == BT - 1) tot[blockIdx.x] = s[BT - 1];
}

// exclusive scan of the NB bucket totals into LDS (every workgroup redoes it: NB loads from L2)
__device__ __forceinline__ void bucket_bases(const uint32_t* tot, uint32_t* base, uint32_t* tmp, uint32_t nthr) {
  for (uint32_t b = threadIdx.x; b < NB; b += nthr) tmp[b] = tot[b];
  __syncthreads();
  if (threadIdx.x < 64) {  // one wave: 64-lane chunks with a running carry
    uint32_t carry = 0;
    for (uint32_t c = 0; c < NB; c += 64) {
      const uint32_t b = c + threadIdx.x;
      uint32_t v = b < NB ? tmp[b] : 0u, x = v;
      for (uint32_t d = 1; d < 64; d <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)x, d, 64);
        if (threadIdx.x >= d) x += y;
      }
      if (b < NB) base[b] = carry + x - v;
      carry += (uint32_t)__shfl((int)x, 63, 64);
    }
  }
  __syncthreads();
}

__global__ __launch_bounds__(BT) void k_scatter(const uint32_t* keys, uint32_t n, uint32_t T, const uint32_t* H,
                                                const uint32_t* tot, uint64_t* out) {
  __shared__ uint32_t run[NB];
  __shared__ uint32_t wc[BT / 64][NB];
  const uint32_t t = blockIdx.x, lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
  bucket_bases(tot, run, wc[0], BT);
  for (uint32_t b = threadIdx.x; b < NB; b += BT) {
    run[b] += H[(uint64_t)b * T + t];
    for (uint32_t k = 0; k < BT / 64; ++k) wc[k][b] = 0u;
  }
  __syncthreads();
  const uint64_t lt = (1ull << lane) - 1ull;
  for (uint32_t r = 0; r < BI; ++r) {
    const uint32_t i = t * TILE + r * BT + threadIdx.x;
    const bool v = i < n;
    const uint32_t key = v ? keys[i] : KSENT;
    const uint32_t b = bucket_of(key);
    uint64_t peers = __ballot(v);
#pragma unroll
    for (uint32_t k = 0; k <= BB; ++k) {  // lanes of the same bucket
      const uint64_t m = __ballot((b >> k) & 1u);
      peers &= ((b >> k) & 1u) ? m : ~m;
    }
    const uint32_t rank = (uint32_t)__popcll(peers & lt);
    if (v && rank == 0) wc[w][b] = (uint32_t)__popcll(peers);
    __syncthreads();
    if (v) {
      uint32_t base = run[b];
      for (uint32_t k = 0; k < w; ++k) base += wc[k][b];
      out[base + rank] = ((uint64_t)key << 32) | i;
    }
    __syncthreads();
    for (uint32_t b2 = threadIdx.x; b2 < NB; b2 += BT) {
      uint32_t s = 0;
      for (uint32_t k = 0; k < BT / 64; ++k) { s += wc[k][b2]; wc[k][b2] = 0u; }
      run[b2] += s;
    }
    __syncthreads();
  }
}

typedef rocprim::block_radix_sort<uint32_t, ST, SI, uint32_t> sort_t;

// one LSD pass of an oversized bucket [s, e) on key byte d, 8192 pairs at a time
// in index order: each chunk is sorted on the byte in LDS (stable) and its runs
// appended to the byte's running output position
__device__ void lsd_pass(const uint64_t* src, uint64_t* dst, uint32_t* dk, uint32_t* dv, uint32_t s, uint32_t e,
                         uint32_t d, sort_t::storage_type& st, uint32_t* run, uint32_t* cc, uint32_t* cs) {
  const uint32_t sh = 8u * d;
  for (uint32_t k = threadIdx.x; k < 256u; k += ST) run[k] = 0u;
  __syncthreads();
  for (uint32_t p = s + threadIdx.x; p < e; p += ST) atomicAdd(&run[(uint32_t)(src[p] >> (32 + sh)) & 255u], 1u);
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t a = s;
    for (uint32_t k = 0; k < 256u; ++k) { const uint32_t c = run[k]; run[k] = a; a += c; }
  }
  __syncthreads();
  for (uint32_t c0 = s; c0 < e; c0 += SCAP) {
    const uint32_t cnt = min(SCAP, e - c0);
    for (uint32_t k = threadIdx.x; k < 256u; k += ST) cc[k] = 0u;
    __syncthreads();
    uint32_t kk[SI], vv[SI];
#pragma unroll
    for (uint32_t j = 0; j < SI; ++j) {
      const uint32_t pos = threadIdx.x * SI + j;
      kk[j] = KSENT;  // padding: byte 255, after every real pair (stable)
      vv[j] = 0u;
      if (pos < cnt) {
        const uint64_t x = src[c0 + pos];
        kk[j] = (uint32_t)(x >> 32);
        vv[j] = (uint32_t)x;
        atomicAdd(&cc[(kk[j] >> sh) & 255u], 1u);
      }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      uint32_t a = 0;
      for (uint32_t k = 0; k < 256u; ++k) { cs[k] = a; a += cc[k]; }
    }
    sort_t().sort(kk, vv, st, sh, sh + 8u);
    __syncthreads();
#pragma unroll
    for (uint32_t j = 0; j < SI; ++j) {
      const uint32_t pos = threadIdx.x * SI + j;
      if (pos < cnt) {
        const uint32_t b = (kk[j] >> sh) & 255u;
        const uint32_t o = run[b] + (pos - cs[b]);
        if (dst) dst[o] = ((uint64_t)kk[j] << 32) | vv[j];
        else { dk[o] = kk[j]; dv[o] = vv[j]; }
      }
    }
    __syncthreads();
    for (uint32_t k = threadIdx.x; k < 256u; k += ST) run[k] += cc[k];
    __syncthreads();
  }
}

__global__ __launch_bounds__(ST) void k_sub(uint64_t* bk, uint64_t* tmp, uint32_t n, const uint32_t* tot,
                                            uint32_t* skeys, uint32_t* svals) {
  __shared__ sort_t::storage_type st;
  __shared__ uint32_t base[NB], btmp[NB];
  __shared__ uint32_t run[256], cc[256], cs[256];
  __shared__ int unordered;
  bucket_bases(tot, base, btmp, ST);
  const uint32_t tail = base[NR];
  for (uint32_t p = tail + blockIdx.x * ST + threadIdx.x; p < n; p += gridDim.x * ST) {
    skeys[p] = KSENT;
    svals[p] = (uint32_t)bk[p];
  }
  const uint32_t b = blockIdx.x, s = base[b], e = base[b + 1], m = e - s;
  if (m == 0) return;
  if (m <= SCAP) {
    uint32_t kk[SI], vv[SI];
#pragma unroll
    for (uint32_t j = 0; j < SI; ++j) {
      const uint32_t pos = threadIdx.x * SI + j;
      kk[j] = KSENT;
      vv[j] = 0u;
      if (pos < m) {
        const uint64_t x = bk[s + pos];
        kk[j] = (uint32_t)(x >> 32);
        vv[j] = (uint32_t)x;
      }
    }
    sort_t().sort(kk, vv, st, 0, LOW);  // the bucket's keys share their top BB bits
#pragma unroll
    for (uint32_t j = 0; j < SI; ++j) {
      const uint32_t pos = threadIdx.x * SI + j;
      if (pos < m) { skeys[s + pos] = kk[j]; svals[s + pos] = vv[j]; }
    }
    return;
  }
  if (threadIdx.x == 0) unordered = 0;
  __syncthreads();
  for (uint32_t p = s + 1 + threadIdx.x; p < e; p += ST)
    if ((uint32_t)(bk[p - 1] >> 32) > (uint32_t)(bk[p] >> 32)) unordered = 1;
  __syncthreads();
  if (!unordered) {
    for (uint32_t p = s + threadIdx.x; p < e; p += ST) {
      const uint64_t x = bk[p];
      skeys[p] = (uint32_t)(x >> 32);
      svals[p] = (uint32_t)x;
    }
    return;
  }
  static_assert(LOW > 16 && LOW <= 24, "three LSD byte passes");
  lsd_pass(bk, tmp, nullptr, nullptr, s, e, 0, st, run, cc, cs);
  lsd_pass(tmp, bk, nullptr, nullptr, s, e, 1, st, run, cc, cs);
  lsd_pass(bk, nullptr, skeys, svals, s, e, 2, st, run, cc, cs);
}

// scratch: H = NB x ceil(n / 4096) + NB u32, bk and tmp = n u64 each; n <= MAX_N
inline size_t hist_words(uint64_t n) { return (size_t)NB * (size_t)((n + TILE - 1) / TILE) + NB; }

template <class Side = NoSide>
inline hipError_t sort_pairs(const uint32_t* keys, uint32_t n, uint32_t* H, uint64_t* bk, uint64_t* tmp,
                             uint32_t* skeys, uint32_t* svals, hipStream_t st, const Side& side = Side()) {
  if (n == 0 || n > MAX_N) return hipErrorInvalidValue;
  const uint32_t T = (n + TILE - 1) / TILE;
  uint32_t* tot = H + (size_t)NB * T;
  hipLaunchKernelGGL(k_hist, dim3(T), dim3(BT), 0, st, keys, n, T, H);
  hipLaunchKernelGGL(k_colscan<Side>, dim3(NB + side.wgs), dim3(BT), 0, st, H, T, tot, side);
  hipLaunchKernelGGL(k_scatter, dim3(T), dim3(BT), 0, st, keys, n, T, H, tot, bk);
  hipLaunchKernelGGL(k_sub, dim3(NR), dim3(ST), 0, st, bk, tmp, n, tot, skeys, svals);
  return hipGetLastError();
}

}  // namespace rtps_bsort
