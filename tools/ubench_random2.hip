// ubench_random2.hip -- random independent 16-byte loads vs table footprint (development tool):
// the split-block layer-1 access pattern.  Each lane issues ITERS rounds of K independent loads.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
typedef uint32_t v4u32 __attribute__((ext_vector_type(4)));
template <int K, bool NT>
__global__ __launch_bounds__(256) void k_rand16(const v4u32 *t, uint64_t blocks, uint32_t iters, uint32_t *out) {
  uint64_t g = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  uint64_t h = g * 0x9E3779B97F4A7C15ULL + 1;
  uint32_t acc = 0;
  for (uint32_t it = 0; it < iters; it++) {
    v4u32 v[K];
#pragma unroll
    for (int k = 0; k < K; k++) {
      h = h * 6364136223846793005ULL + 1442695040888963407ULL;
      const v4u32 *p = t + (h >> 24) % blocks;
      v[k] = NT ? __builtin_nontemporal_load(p) : *p;
    }
#pragma unroll
    for (int k = 0; k < K; k++) acc += v[k].x ^ v[k].w;
  }
  out[g] = acc;
}
int main() {
  const uint64_t maxbytes = 24ULL << 30;
  v4u32 *t;
  if (hipMalloc(&t, maxbytes) != hipSuccess) { printf("alloc failed\n"); return 1; }
  (void)hipMemset(t, 1, maxbytes);
  uint32_t *out;
  const int lanes = 4096 * 256;
  (void)hipMalloc(&out, lanes * 4);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  for (uint64_t mb : {64ULL, 256ULL, 2048ULL, 6144ULL, 24576ULL}) {
    uint64_t blocks = (mb << 20) / 16;
    for (int variant = 0; variant < 4; variant++) {
      uint32_t iters = 64;
      auto go = [&]() {
        switch (variant) {
          case 0: hipLaunchKernelGGL((k_rand16<1, false>), dim3(lanes / 256), dim3(256), 0, 0, t, blocks, iters, out); break;
          case 1: hipLaunchKernelGGL((k_rand16<4, false>), dim3(lanes / 256), dim3(256), 0, 0, t, blocks, iters, out); break;
          case 2: hipLaunchKernelGGL((k_rand16<1, true>), dim3(lanes / 256), dim3(256), 0, 0, t, blocks, iters, out); break;
          case 3: hipLaunchKernelGGL((k_rand16<4, true>), dim3(lanes / 256), dim3(256), 0, 0, t, blocks, iters, out); break;
        }
      };
      go();
      (void)hipEventRecord(a);
      go();
      (void)hipEventRecord(b);
      (void)hipEventSynchronize(b);
      float ms;
      (void)hipEventElapsedTime(&ms, a, b);
      int K = (variant & 1) ? 4 : 1;
      double loads = (double)lanes * iters * K;
      printf("footprint %6llu MB  K=%d %s: %7.2f G loads/s\n", (unsigned long long)mb, K, variant >= 2 ? "nt " : "   ",
             loads / ms / 1e6);
    }
  }
  return 0;
}
