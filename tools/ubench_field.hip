// ubench_field.hip -- microbenchmark of 256-bit field multiplication formulations on gfx950.
// Development tool: each lane runs a chain of ITERS multiplications; prints ns per mul per lane
// and chip throughput, and checks every variant against variant 0.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <vector>
#include "../keyhunt_amd/csrc/kh_math.h"

using namespace kh;

// ---- variant 1: product scanning, 64-bit accumulator + carry counter ---------------------
__device__ __forceinline__ void mul_ps(fe &r, const fe &a, const fe &b) {
  uint32_t t[16];
  uint64_t acc = 0;
  uint32_t cnt = 0;
#pragma unroll
  for (int k = 0; k < 15; k++) {
#pragma unroll
    for (int i = 0; i < 8; i++) {
      int j = k - i;
      if (j < 0 || j > 7) continue;
      uint64_t p = (uint64_t)a.d[i] * b.d[j];
      uint64_t s = acc + p;
      cnt += (s < p);
      acc = s;
    }
    t[k] = (uint32_t)acc;
    acc = (acc >> 32) | ((uint64_t)cnt << 32);
    cnt = 0;
  }
  t[15] = (uint32_t)acc;
  fe_reduce512(r, t);
}

// ---- variant 2: inline-asm v_mad_u64_u32 with carry-out into a lane mask ------------------
__device__ __forceinline__ uint64_t mad_co(uint32_t a, uint32_t b, uint64_t c, uint32_t &cnt) {
  uint64_t d;
  uint64_t m;
  asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=v"(d), "=s"(m) : "v"(a), "v"(b), "v"(c));
  uint32_t o;
  asm volatile("v_addc_co_u32 %0, vcc, 0, %1, %2" : "=v"(o) : "v"(cnt), "s"(m) : "vcc");
  cnt = o;
  return d;
}
__device__ __forceinline__ void mul_asm(fe &r, const fe &a, const fe &b) {
  uint32_t t[16];
  uint64_t acc = 0;
  uint32_t cnt = 0;
#pragma unroll
  for (int k = 0; k < 15; k++) {
#pragma unroll
    for (int i = 0; i < 8; i++) {
      int j = k - i;
      if (j < 0 || j > 7) continue;
      acc = mad_co(a.d[i], b.d[j], acc, cnt);
    }
    t[k] = (uint32_t)acc;
    acc = (acc >> 32) | ((uint64_t)cnt << 32);
    cnt = 0;
  }
  t[15] = (uint32_t)acc;
  fe_reduce512(r, t);
}

// ---- variant 3: 32-bit mul_lo/mul_hi + add-with-carry chains (Comba, 3-word accumulator) ----
__device__ __forceinline__ void mul_comba32(fe &r, const fe &a, const fe &b) {
  uint32_t t[16];
  uint32_t c0 = 0, c1 = 0, c2 = 0;
#pragma unroll
  for (int k = 0; k < 15; k++) {
#pragma unroll
    for (int i = 0; i < 8; i++) {
      int j = k - i;
      if (j < 0 || j > 7) continue;
      uint32_t lo = a.d[i] * b.d[j];
      uint32_t hi = __umulhi(a.d[i], b.d[j]);
      uint32_t cy;
      c0 = addc(c0, lo, 0, cy);
      c1 = addc(c1, hi, cy, cy);
      c2 += cy;
    }
    t[k] = c0;
    c0 = c1;
    c1 = c2;
    c2 = 0;
  }
  t[15] = c0;
  fe_reduce512(r, t);
}

template <int V>
__global__ void k_bench(const uint32_t *in, uint32_t *out, int iters) {
  uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  fe a, b;
  for (int i = 0; i < 8; i++) {
    a.d[i] = in[g * 16 + i];
    b.d[i] = in[g * 16 + 8 + i];
  }
  fe_canon(a);
  fe_canon(b);
  for (int it = 0; it < iters; it++) {
    fe r;
    if (V == 0) fe_mul(r, a, b);
    if (V == 1) mul_ps(r, a, b);
    if (V == 2) mul_asm(r, a, b);
    if (V == 3) mul_comba32(r, a, b);
    if (V == 4) fe_sqr(r, a);
    b = a;
    a = r;
  }
  for (int i = 0; i < 8; i++) out[g * 8 + i] = a.d[i];
}

int main() {
  const int lanes = 256 * 1024, iters = 2000;
  std::vector<uint32_t> h(lanes * 16);
  uint64_t s = 88172645463325252ULL;
  for (auto &x : h) {
    s ^= s << 13; s ^= s >> 7; s ^= s << 17;
    x = (uint32_t)s;
  }
  uint32_t *din, *dout;
  hipMalloc(&din, h.size() * 4);
  hipMalloc(&dout, lanes * 32);
  hipMemcpy(din, h.data(), h.size() * 4, hipMemcpyHostToDevice);
  std::vector<uint32_t> ref(lanes * 8), got(lanes * 8);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const char *names[] = {"fe_mul (u64 carry)", "product-scan u64+cnt", "asm mad_u64 carry-out", "comba mul_lo/hi", "fe_sqr"};
  for (int v = 0; v < 5; v++) {
    auto launch = [&]() {
      switch (v) {
        case 0: hipLaunchKernelGGL(k_bench<0>, dim3(lanes / 256), dim3(256), 0, 0, din, dout, iters); break;
        case 1: hipLaunchKernelGGL(k_bench<1>, dim3(lanes / 256), dim3(256), 0, 0, din, dout, iters); break;
        case 2: hipLaunchKernelGGL(k_bench<2>, dim3(lanes / 256), dim3(256), 0, 0, din, dout, iters); break;
        case 3: hipLaunchKernelGGL(k_bench<3>, dim3(lanes / 256), dim3(256), 0, 0, din, dout, iters); break;
        case 4: hipLaunchKernelGGL(k_bench<4>, dim3(lanes / 256), dim3(256), 0, 0, din, dout, iters); break;
      }
    };
    launch();
    hipDeviceSynchronize();
    hipEventRecord(e0);
    launch();
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    hipMemcpy(got.data(), dout, lanes * 32, hipMemcpyDeviceToHost);
    if (v == 0) ref = got;
    bool ok = (v == 4) || got == ref;
    double muls = (double)lanes * iters;
    printf("%-26s %8.3f ms  %8.2f Gmul/s  %s\n", names[v], ms, muls / ms / 1e6, ok ? "match" : "MISMATCH");
  }
  return 0;
}
