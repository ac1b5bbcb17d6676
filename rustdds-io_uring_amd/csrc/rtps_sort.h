// rtps_sort.h — the device radix sort the reassembly and the ingest use.
// rocprim's default configuration sorts up to 1M items by merge sort (about ten
// passes, each a separate launch: ~115 us for 0.57M pairs on the ingest's
// HEARTBEAT sort) whatever the key width; a merge-sort limit of 0 selects Onesweep
// (a histogram pass + one pass per 8-bit digit, ~30 us per digit at 1M pairs
// including its state resets).  So: Onesweep for keys of at most 16 bits (one or
// two digits: proxy indices), the default otherwise (32-bit hashes: four digits
// cost more than the merge sort, measured 180 us against 150 us at 1M pairs).
#pragma once
#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>

using rtps_sort_config = rocprim::radix_sort_config<rocprim::default_config, rocprim::default_config,
                                                    rocprim::default_config, 0>;

// stable ascending sort of (key, value) pairs on key bits [0, bits).  Temporary
// storage: query with the largest `bits` the caller will use (both configurations).
template <class K, class V>
inline hipError_t rtps_sort_pairs(void* tmp, size_t& bytes, K* keys_in, K* keys_out, V* vals_in, V* vals_out,
                                  uint32_t n, int bits, hipStream_t st) {
  if (bits <= 16) {
    if (!tmp) {  // size for both, so that one query covers every later call
      size_t a = 0, b = 0;
      hipError_t e = rocprim::radix_sort_pairs<rtps_sort_config>(nullptr, a, keys_in, keys_out, vals_in, vals_out, n,
                                                                 0, bits, st);
      if (e == hipSuccess)
        e = rocprim::radix_sort_pairs(nullptr, b, keys_in, keys_out, vals_in, vals_out, n, 0, bits, st);
      bytes = a > b ? a : b;
      return e;
    }
    return rocprim::radix_sort_pairs<rtps_sort_config>(tmp, bytes, keys_in, keys_out, vals_in, vals_out, n, 0, bits,
                                                       st);
  }
  if (!tmp) {
    size_t a = 0, b = 0;
    hipError_t e = rocprim::radix_sort_pairs<rtps_sort_config>(nullptr, a, keys_in, keys_out, vals_in, vals_out, n, 0,
                                                               bits, st);
    if (e == hipSuccess) e = rocprim::radix_sort_pairs(nullptr, b, keys_in, keys_out, vals_in, vals_out, n, 0, bits, st);
    bytes = a > b ? a : b;
    return e;
  }
  return rocprim::radix_sort_pairs(tmp, bytes, keys_in, keys_out, vals_in, vals_out, n, 0, bits, st);
}
