// ubench_field2.hip -- field multiplication formulations for the walk (development tool).
//   v0  fe_mul (kh_math.h: 8x32 limbs, asm v_mad_u64_u32 + carry count), 2 chains per lane
//   v1  same two chains, calls interleaved statement by statement (fe_mul2)
//   v2  9x29-bit limbs, column sums without carries (pure C), 2 chains per lane
//   v3  fe_sqr (kh_math.h), 2 chains
//   v4  9x29 squaring, 2 chains
// Launch bounds (256, 4) as in the BSGS walk.  Every variant's result is checked against v0/v3.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <vector>
#include "../keyhunt_amd/csrc/kh_math.h"

using namespace kh;

// ------------------------------------------------------------------ 9 x 29-bit limbs
struct f29 {
  uint32_t v[9];
};
constexpr uint32_t M29 = (1u << 29) - 1;

__device__ __forceinline__ void f29_from_fe(f29 &r, const fe &a) {
  // 256 bits -> 9 x 29
#pragma unroll
  for (int k = 0; k < 9; k++) {
    int bit = 29 * k, w = bit >> 5, s = bit & 31;
    uint64_t x = a.d[w];
    if (w + 1 < 8) x |= (uint64_t)a.d[w + 1] << 32;
    r.v[k] = (uint32_t)(x >> s) & M29;
  }
}
__device__ __forceinline__ void f29_to_fe(fe &r, const f29 &a) {
  // full carry normalisation, then 2^256 fold, then canonical
  uint32_t l[9];
  uint64_t c = 0;
#pragma unroll
  for (int k = 0; k < 9; k++) {
    uint64_t t = (uint64_t)a.v[k] + c;
    l[k] = (k < 8) ? (uint32_t)t & M29 : (uint32_t)t;
    c = (k < 8) ? t >> 29 : 0;
  }
  // l[8] may exceed 24 bits: hi = l[8] >> 24 ; value = lo + hi*2^256 = lo + hi*(2^32+977)
  uint32_t hi = l[8] >> 24;
  l[8] &= (1u << 24) - 1;
  uint64_t acc[4] = {0, 0, 0, 0};
  (void)acc;
  uint32_t d[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
  for (int k = 0; k < 9; k++) {
    int bit = 29 * k, w = bit >> 5, s = bit & 31;
    uint64_t x = (uint64_t)l[k] << s;
    d[w] |= (uint32_t)x;
    if (w + 1 < 8) d[w + 1] |= (uint32_t)(x >> 32);
  }
  fe t;
#pragma unroll
  for (int i = 0; i < 8; i++) t.d[i] = d[i];
  fe h;
  fe_set_u32(h, 0);
  uint64_t v = (uint64_t)hi * 977u;
  h.d[0] = (uint32_t)v;
  h.d[1] = (uint32_t)(v >> 32) + hi;
  fe_canon(t);
  fe_add(r, t, h);
}

// columns c_k = sum a_i b_j (81 products, no carries), then carry pass, fold 2^261 = 2^37 + 31264,
// carry pass, fold the bits >= 2^256 by 2^32 + 977.  Inputs: limbs <= 2^30.  Output: limbs < 2^29
// except limb 2 (< 2^29 + 2^21) and limb 8 (< 2^24): value < 2^256 + 2^79, weakly reduced.
__device__ __forceinline__ void f29_reduce(f29 &r, const uint64_t c[17]) {
  uint32_t l[18];
  uint64_t carry = 0;
#pragma unroll
  for (int k = 0; k < 17; k++) {
    uint64_t t = c[k] + carry;
    l[k] = (uint32_t)t & M29;
    carry = t >> 29;
  }
  l[17] = (uint32_t)carry;
  uint64_t d[10];
  d[0] = (uint64_t)l[9] * 31264u + l[0];
#pragma unroll
  for (int k = 1; k < 9; k++) d[k] = (uint64_t)l[9 + k] * 31264u + ((uint64_t)l[8 + k] << 8) + l[k];
  d[9] = (uint64_t)l[17] << 8;
  uint32_t e[9];
  carry = 0;
#pragma unroll
  for (int k = 0; k < 9; k++) {
    uint64_t t = d[k] + carry;
    e[k] = (uint32_t)t & M29;
    carry = t >> 29;
  }
  uint64_t top = d[9] + carry;                     // weight 2^261
  uint64_t t256 = (top << 5) | (e[8] >> 24);       // bits >= 256
  e[8] &= (1u << 24) - 1;
  uint64_t x0 = t256 * 977u + e[0];
  r.v[0] = (uint32_t)x0 & M29;
  uint64_t x1 = (t256 << 3) + e[1] + (x0 >> 29);
  r.v[1] = (uint32_t)x1 & M29;
  r.v[2] = e[2] + (uint32_t)(x1 >> 29);
#pragma unroll
  for (int k = 3; k < 9; k++) r.v[k] = e[k];
}
__device__ __forceinline__ void f29_mul(f29 &r, const f29 &a, const f29 &b) {
  uint64_t c[17];
#pragma unroll
  for (int k = 0; k < 17; k++) {
    uint64_t s = 0;
#pragma unroll
    for (int i = 0; i < 9; i++) {
      int j = k - i;
      if (j < 0 || j > 8) continue;
      s += (uint64_t)a.v[i] * b.v[j];
    }
    c[k] = s;
  }
  f29_reduce(r, c);
}
__device__ __forceinline__ void f29_sqr(f29 &r, const f29 &a) {
  uint32_t a2[9];
#pragma unroll
  for (int i = 0; i < 9; i++) a2[i] = a.v[i] << 1;
  uint64_t c[17];
#pragma unroll
  for (int k = 0; k < 17; k++) {
    uint64_t s = 0;
#pragma unroll
    for (int i = 0; i < 9; i++) {
      int j = k - i;
      if (j <= i || j > 8) continue;
      s += (uint64_t)a2[i] * a.v[j];
    }
    if ((k & 1) == 0 && k / 2 < 9) s += (uint64_t)a.v[k / 2] * a.v[k / 2];
    c[k] = s;
  }
  f29_reduce(r, c);
}

// ------------------------------------------------------------------ interleaved pair, 8 x 32
__device__ __forceinline__ void fe_mul2(fe &r1, const fe &a1, const fe &b1, fe &r2, const fe &a2, const fe &b2) {
#if defined(__HIP_DEVICE_COMPILE__)
  uint32_t t1[16], t2[16];
  uint64_t acc1 = 0, acc2 = 0;
  uint32_t cnt1 = 0, cnt2 = 0;
#pragma unroll
  for (int k = 0; k < 15; k++) {
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const int j = k - i;
      if (j < 0 || j > 7) continue;
      acc1 = mad_acc(a1.d[i], b1.d[j], acc1, cnt1);
      acc2 = mad_acc(a2.d[i], b2.d[j], acc2, cnt2);
    }
    t1[k] = (uint32_t)acc1;
    acc1 = (acc1 >> 32) | ((uint64_t)cnt1 << 32);
    cnt1 = 0;
    t2[k] = (uint32_t)acc2;
    acc2 = (acc2 >> 32) | ((uint64_t)cnt2 << 32);
    cnt2 = 0;
  }
  t1[15] = (uint32_t)acc1;
  t2[15] = (uint32_t)acc2;
  fe_reduce512(r1, t1);
  fe_reduce512(r2, t2);
#endif
}

// ------------------------------------------------------------------ software-pipelined carries
// The carry SGPR of product n is consumed after the mad of product n+1 has issued, so the
// "VALU writes SGPR -> VALU reads it as carry" wait state is filled by useful work.
__device__ __forceinline__ uint64_t mad_co2(uint32_t a, uint32_t b, uint64_t acc, uint64_t &m) {
  uint64_t d;
  asm("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=v"(d), "=s"(m) : "v"(a), "v"(b), "v"(acc));
  return d;
}
__device__ __forceinline__ uint32_t addc_m(uint32_t cnt, uint64_t m) {
  uint32_t o;
  asm("v_addc_co_u32 %0, vcc, 0, %1, %2" : "=v"(o) : "v"(cnt), "s"(m) : "vcc");
  return o;
}
__device__ __forceinline__ void fe_mul_sp(fe &r, const fe &a, const fe &b) {
#if defined(__HIP_DEVICE_COMPILE__)
  uint32_t t[16];
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 15; k++) {
    uint32_t cnt = 0;
    uint64_t mp = 0;
    bool have = false;
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const int j = k - i;
      if (j < 0 || j > 7) continue;
      uint64_t m;
      acc = mad_co2(a.d[i], b.d[j], acc, m);
      if (have) cnt = addc_m(cnt, mp);
      mp = m;
      have = true;
    }
    cnt = addc_m(cnt, mp);
    t[k] = (uint32_t)acc;
    acc = (acc >> 32) | ((uint64_t)cnt << 32);
  }
  t[15] = (uint32_t)acc;
  fe_reduce512(r, t);
#endif
}

// two products interleaved AND software-pipelined carries: between a carry's write, its read, and
// the next write of the same SGPR pair there is always an instruction of the other product
__device__ __forceinline__ void fe_mul2_sp(fe &r1, const fe &a1, const fe &b1, fe &r2, const fe &a2, const fe &b2) {
#if defined(__HIP_DEVICE_COMPILE__)
  uint32_t t1[16], t2[16];
  uint64_t acc1 = 0, acc2 = 0;
#pragma unroll
  for (int k = 0; k < 15; k++) {
    uint32_t cnt1 = 0, cnt2 = 0;
    uint64_t mp1 = 0, mp2 = 0;
    bool have = false;
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const int j = k - i;
      if (j < 0 || j > 7) continue;
      uint64_t m1, m2;
      acc1 = mad_co2(a1.d[i], b1.d[j], acc1, m1);
      acc2 = mad_co2(a2.d[i], b2.d[j], acc2, m2);
      if (have) {
        cnt1 = addc_m(cnt1, mp1);
        cnt2 = addc_m(cnt2, mp2);
      }
      mp1 = m1;
      mp2 = m2;
      have = true;
    }
    cnt1 = addc_m(cnt1, mp1);
    cnt2 = addc_m(cnt2, mp2);
    t1[k] = (uint32_t)acc1;
    acc1 = (acc1 >> 32) | ((uint64_t)cnt1 << 32);
    t2[k] = (uint32_t)acc2;
    acc2 = (acc2 >> 32) | ((uint64_t)cnt2 << 32);
  }
  t1[15] = (uint32_t)acc1;
  t2[15] = (uint32_t)acc2;
  fe_reduce512(r1, t1);
  fe_reduce512(r2, t2);
#endif
}

template <int V>
__global__ __launch_bounds__(256, 4) void k_bench(const uint32_t *in, uint32_t *out, int iters) {
  uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  fe a, b, c, d;
  for (int i = 0; i < 8; i++) {
    a.d[i] = in[g * 32 + i];
    b.d[i] = in[g * 32 + 8 + i];
    c.d[i] = in[g * 32 + 16 + i];
    d.d[i] = in[g * 32 + 24 + i];
  }
  fe_canon(a);
  fe_canon(b);
  fe_canon(c);
  fe_canon(d);
  if (V == 2 || V == 4) {
    f29 A, B, C, D;
    f29_from_fe(A, a);
    f29_from_fe(B, b);
    f29_from_fe(C, c);
    f29_from_fe(D, d);
    for (int it = 0; it < iters; it++) {
      f29 R, S;
      if (V == 2) {
        f29_mul(R, A, B);
        f29_mul(S, C, D);
        B = A;
        A = R;
        D = C;
        C = S;
      } else {
        f29_sqr(R, A);
        f29_sqr(S, C);
        A = R;
        C = S;
      }
    }
    f29_to_fe(a, A);
    f29_to_fe(c, C);
  } else {
    for (int it = 0; it < iters; it++) {
      fe r, s;
      if (V == 0) {
        fe_mul(r, a, b);
        fe_mul(s, c, d);
      } else if (V == 1) {
        fe_mul2(r, a, b, s, c, d);
      } else if (V == 6) {
        fe_mul2_sp(r, a, b, s, c, d);
      } else if (V == 5) {
        fe_mul_sp(r, a, b);
        fe_mul_sp(s, c, d);
      } else {
        fe_sqr(r, a);
        fe_sqr(s, c);
      }
      if (V != 3 && V != 4) {
        b = a;
        d = c;
      }
      a = r;
      c = s;
    }
  }
  for (int i = 0; i < 8; i++) {
    out[g * 16 + i] = a.d[i];
    out[g * 16 + 8 + i] = c.d[i];
  }
}

int main() {
  const int lanes = 256 * 1024, iters = 1000;
  std::vector<uint32_t> h((size_t)lanes * 32);
  uint64_t s = 88172645463325252ULL;
  for (auto &x : h) {
    s ^= s << 13;
    s ^= s >> 7;
    s ^= s << 17;
    x = (uint32_t)s;
  }
  uint32_t *din, *dout;
  (void)hipMalloc(&din, h.size() * 4);
  (void)hipMalloc(&dout, (size_t)lanes * 64);
  (void)hipMemcpy(din, h.data(), h.size() * 4, hipMemcpyHostToDevice);
  std::vector<uint32_t> ref_mul, ref_sqr, got((size_t)lanes * 16);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const char *names[] = {"fe_mul x2", "fe_mul2 interleaved", "f29_mul x2", "fe_sqr x2", "f29_sqr x2",
                         "fe_mul_sp x2", "fe_mul2_sp"};
  for (int v = 0; v < 7; v++) {
    auto launch = [&]() {
      dim3 g(lanes / 256), b(256);
      switch (v) {
        case 0: hipLaunchKernelGGL(k_bench<0>, g, b, 0, 0, din, dout, iters); break;
        case 1: hipLaunchKernelGGL(k_bench<1>, g, b, 0, 0, din, dout, iters); break;
        case 2: hipLaunchKernelGGL(k_bench<2>, g, b, 0, 0, din, dout, iters); break;
        case 3: hipLaunchKernelGGL(k_bench<3>, g, b, 0, 0, din, dout, iters); break;
        case 4: hipLaunchKernelGGL(k_bench<4>, g, b, 0, 0, din, dout, iters); break;
        case 5: hipLaunchKernelGGL(k_bench<5>, g, b, 0, 0, din, dout, iters); break;
        case 6: hipLaunchKernelGGL(k_bench<6>, g, b, 0, 0, din, dout, iters); break;
      }
    };
    launch();
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(e0);
    launch();
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    (void)hipMemcpy(got.data(), dout, (size_t)lanes * 64, hipMemcpyDeviceToHost);
    const char *ok = "";
    if (v == 0) ref_mul = got;
    if (v == 3) ref_sqr = got;
    if (v == 1 || v == 2 || v == 5 || v == 6) ok = got == ref_mul ? "match" : "MISMATCH";
    if (v == 4) ok = got == ref_sqr ? "match" : "MISMATCH";
    double ops = 2.0 * lanes * iters;
    printf("%-22s %8.3f ms  %8.2f Gop/s  %s\n", names[v], ms, ops / ms / 1e6, ok);
  }
  return 0;
}
