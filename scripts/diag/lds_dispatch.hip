// Dispatch cost of workgroups with a large LDS allocation (diagnostic, not product code):
// 256 workgroups x 512 threads, dynamic LDS of 0 / 64 / 151 KB, a body that only touches its
// LDS, timed with HIP events over back-to-back launches.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ __launch_bounds__(512) void k_lds(uint32_t* out, uint32_t words) {
  extern __shared__ uint32_t s[];
  for (uint32_t i = threadIdx.x; i < words; i += blockDim.x) s[i] = i;
  __syncthreads();
  if (threadIdx.x == 0) out[blockIdx.x] = words ? s[words - 1] : 0u;
}
int main() {
  uint32_t* out;
  if (hipMalloc(&out, 4096 * 4) != hipSuccess) return 1;
  const uint32_t sizes[3] = {0u, 64u * 1024u, 151u * 1024u};
  hipEvent_t a, b;
  (void)hipEventCreate(&a); (void)hipEventCreate(&b);
  for (uint32_t grid : {256u, 512u}) {
    for (uint32_t sz : sizes) {
      if (hipFuncSetAttribute((const void*)k_lds, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sz) != hipSuccess) return 2;
      for (int touch = 0; touch < 2; ++touch) {
        const uint32_t words = touch ? sz / 4 : 0u;
        for (int w = 0; w < 5; ++w) hipLaunchKernelGGL(k_lds, dim3(grid), dim3(512), sz, 0, out, words);
        (void)hipEventRecord(a, 0);
        for (int k = 0; k < 100; ++k) hipLaunchKernelGGL(k_lds, dim3(grid), dim3(512), sz, 0, out, words);
        (void)hipEventRecord(b, 0);
        (void)hipEventSynchronize(b);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, a, b);
        printf("grid %u lds %6u B touch %d: %.2f us per launch\n", grid, sz, touch, ms * 10.0f);
      }
    }
  }
  return hipDeviceSynchronize() == hipSuccess ? 0 : 3;
}
