// ubench_random.hip -- random 1-byte read throughput into a large table (the layer-1 bloom access
// pattern): each lane does CHAIN dependent reads at hash-derived addresses, PAIRS independent chains.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
__global__ void k_rand(const uint8_t *t, uint64_t bytes, uint32_t iters, uint32_t *out, int pairs) {
  uint64_t g = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  uint64_t h1 = g * 0x9E3779B97F4A7C15ULL + 1, h2 = g * 0xC2B2AE3D27D4EB4FULL + 7;
  uint32_t acc = 0;
  for (uint32_t it = 0; it < iters; it++) {
    h1 = h1 * 6364136223846793005ULL + 1442695040888963407ULL;
    uint32_t v = t[(h1 >> 20) % bytes];
    acc += v;
    if (pairs == 2) {
      h2 = h2 * 6364136223846793005ULL + 1442695040888963407ULL + v;  // keep it dependent-ish
      acc += t[(h2 >> 20) % bytes];
    }
    h1 += v;
  }
  out[g] = acc;
}
int main() {
  uint64_t bytes = 1930000000ULL;
  uint8_t *t;
  hipMalloc(&t, bytes);
  hipMemset(t, 1, bytes);
  uint32_t *out;
  int lanes = 16384 * 256;  // >= the largest grid below
  hipMalloc(&out, lanes * 4);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int pairs = 1; pairs <= 2; pairs++)
    for (int blk : {256, 1024, 4096, 16384}) {
      int n = blk * 256;
      uint32_t iters = 256;
      hipLaunchKernelGGL(k_rand, dim3(blk), dim3(256), 0, 0, t, bytes, iters, out, pairs);
      hipEventRecord(a);
      hipLaunchKernelGGL(k_rand, dim3(blk), dim3(256), 0, 0, t, bytes, iters, out, pairs);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      double reads = (double)n * iters * pairs;
      printf("pairs=%d lanes=%8d: %.2f G random reads/s (%.2f TB/s at 64 B)\n", pairs, n, reads / ms / 1e6,
             reads * 64 / ms / 1e9);
    }
  return 0;
}
