// ubench_field4.hip -- cycles per field op for hipcc fe_mul vs the generated asm forms, and the asm
// product / reduction alone (development tool).  Needs the experiment header:
//   KH_GEN_EXPERIMENTS=1 python3 tools/gen_field_asm.py tools/kh_field_asm_x.h
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <vector>
#include "../keyhunt_amd/csrc/kh_math.h"
#include "kh_field_asm_x.h"  // includes the experiment functions too
using namespace kh;
__device__ __noinline__ void fe_mul_slow(fe &r, const fe &a, const fe &b) { fe_mul(r, a, b); }
template <int V>
__global__ __launch_bounds__(256, 4) void k_bench(const uint32_t *in, uint32_t *out, int iters) {
  uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  fe a, b, c, d;
  for (int i = 0; i < 8; i++) { a.d[i] = in[g * 32 + i]; b.d[i] = in[g * 32 + 8 + i]; c.d[i] = in[g * 32 + 16 + i]; d.d[i] = in[g * 32 + 24 + i]; }
  uint32_t acc = 0;
  for (int it = 0; it < iters; it++) {
    fe r, s;
    if (V == 0) { fe_mul(r, a, b); fe_mul(s, c, d); }
    if (V == 1) { acc += fe_mul_asm(r, a, b); acc += fe_mul_asm(s, c, d); }
    if (V == 2) { acc += fe_mulP_asm(r, a, b); acc += fe_mulP_asm(s, c, d); }
    if (V == 3) { acc += fe_red_asm(r, a, b); acc += fe_red_asm(s, c, d); }
    if (V == 4) { acc += fe_sqr_asm(r, a); acc += fe_sqr_asm(s, c); }
    if (V == 5) { acc += fe_mul2_asm(r, a, b, s, c, d); }
    if (V == 6) {  // with the portable fallback on a set flag, as the walk would use it
      fe t, u;
      if (fe_mul_asm(t, a, b) == 0xFFFFFFFFu) fe_mul(t, a, b);
      if (fe_mul_asm(u, c, d) == 0xFFFFFFFFu) fe_mul(u, c, d);
      r = t;
      s = u;
    }
    if (V == 7) {  // fallback through a non-inlined call
      fe t, u;
      if (fe_mul_asm(t, a, b) == 0xFFFFFFFFu) fe_mul_slow(t, a, b);
      if (fe_mul_asm(u, c, d) == 0xFFFFFFFFu) fe_mul_slow(u, c, d);
      r = t;
      s = u;
    }
    b = a; d = c; a = r; c = s;
  }
  for (int i = 0; i < 8; i++) { out[g * 16 + i] = a.d[i] + acc; out[g * 16 + 8 + i] = c.d[i]; }
}
int main() {
  const int lanes = 256 * 1024, iters = 1000;
  std::vector<uint32_t> h((size_t)lanes * 32);
  uint64_t s = 88172645463325252ULL;
  for (auto &x : h) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; x = (uint32_t)s & 0x7FFFFFFF; }
  uint32_t *din, *dout;
  (void)hipMalloc(&din, h.size() * 4);
  (void)hipMalloc(&dout, (size_t)lanes * 64);
  (void)hipMemcpy(din, h.data(), h.size() * 4, hipMemcpyHostToDevice);
  hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  const char *names[] = {"hipcc fe_mul", "asm mul", "asm product only", "asm reduce only", "asm sqr", "asm mul2", "asm mul + fallback", "asm mul + call"};
  for (int v = 0; v < 8; v++) {
    for (int rep = 0; rep < 2; rep++) {
      (void)hipEventRecord(e0);
      switch (v) {
#define L(n) case n: hipLaunchKernelGGL(k_bench<n>, dim3(lanes / 256), dim3(256), 0, 0, din, dout, iters); break;
        L(0) L(1) L(2) L(3) L(4) L(5) L(6) L(7)
      }
      (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
      float ms; (void)hipEventElapsedTime(&ms, e0, e1);
      if (rep) printf("%-20s %8.3f ms  %7.1f cycles per wave-op per SIMD\n", names[v], ms, ms * 1e-3 * 2.4e9 / (4.0 * 2 * iters));
    }
  }
  return 0;
}
