// ubench_field_cf.hip -- the shipped 8x32-bit field multiplication (kh_math.h fe_mul / fe_sqr: product
// scanning with carry counts, multiply-add fold) against a carry-free 10x26-bit form (VERDICT round 4
// item 2: carry ops are 60 % of the BSGS walk's cycles).  Development tool, built as a shared library
// and driven by tools/field_cf_energy.py, which times each variant with HIP events and reads the
// board's energy accumulator around it (multiplications per second AND per joule).
//
// The 10x26 form: a = sum n_i 2^(26 i), limbs below 2^26 (magnitude 1).  A product's 19 columns are
// sums of at most 10 products of 52 bits, so they accumulate in 64 bits with no carry to count (plain
// C: LLVM emits v_mad_u64_u32 chains).  The high columns 10..18 are normalized to 26-bit limbs h_j and
// folded with 2^260 == R = 0x1000003D10 = R1 2^26 + R0 (R1 = 0x400, R0 = 0x3D10): h_j R0 at column j,
// h_j R1 at column j + 1, while the low columns are normalized; the part left above 2^260 folds once
// more into limbs 0..2.  Every chain's result is converted back to canonical bytes and compared with
// the shipped form's.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <vector>
#include "../keyhunt_amd/csrc/kh_math.h"

using namespace kh;

struct f26 {
  uint32_t n[10];
};

__device__ __forceinline__ void to26(f26 &o, const fe &a) {
#pragma unroll
  for (int i = 0; i < 10; i++) {
    const int bit = 26 * i, w = bit >> 5, s = bit & 31;
    uint64_t v = a.d[w];
    if (w + 1 < 8) v |= (uint64_t)a.d[w + 1] << 32;
    o.n[i] = (uint32_t)(v >> s) & 0x3FFFFFFu;
  }
}

// carry-normalize to limbs < 2^26 (top limb < 2^22 after the fold), then to canonical 8x32 (< p)
__device__ __forceinline__ void from26(fe &o, const f26 &a) {
  uint32_t n[10];
  uint64_t c = 0;
  for (int pass = 0; pass < 3; pass++) {
    c = 0;
#pragma unroll
    for (int i = 0; i < 10; i++) {
      c += pass ? n[i] : a.n[i];
      n[i] = (uint32_t)c & 0x3FFFFFFu;
      c >>= 26;
    }
    // bits at 2^260 and above (c) plus bits 256..259 of limb 9: t * 2^256 == t * 0x1000003D1
    const uint64_t t = (c << 4) | (n[9] >> 22);
    n[9] &= 0x3FFFFFu;
    uint64_t v = (uint64_t)n[0] + t * 0x3D1u;
    n[0] = (uint32_t)v & 0x3FFFFFFu;
    v = (v >> 26) + n[1] + (t << 6);  // 2^32 = 2^6 at limb 1
    n[1] = (uint32_t)v & 0x3FFFFFFu;
    n[2] += (uint32_t)(v >> 26);
  }
  // pack 256 bits
  uint32_t w[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
  for (int i = 0; i < 10; i++) {
    const int bit = 26 * i, k = bit >> 5, s = bit & 31;
    const uint64_t v = (uint64_t)n[i] << s;
    w[k] |= (uint32_t)v;
    if (k + 1 < 8) w[k + 1] |= (uint32_t)(v >> 32);
  }
#pragma unroll
  for (int i = 0; i < 8; i++) o.d[i] = w[i];
  fe_canon(o);
}

__device__ __forceinline__ void fold26(f26 &r, uint64_t acc, const uint32_t h9) {
  const uint32_t M = 0x3FFFFFFu, R0 = 0x3D10u, R1 = 0x400u;
  // what is left at 2^260: the low columns' last carry plus h9 * R1
  const uint64_t T = acc + (uint64_t)h9 * R1;  // < 2^43
  const uint32_t tl = (uint32_t)T & M, th = (uint32_t)(T >> 26);
  uint64_t v = (uint64_t)tl * R0 + r.n[0];
  r.n[0] = (uint32_t)v & M;
  v = (v >> 26) + (uint64_t)tl * R1 + (uint64_t)th * R0 + r.n[1];
  r.n[1] = (uint32_t)v & M;
  v = (v >> 26) + (uint64_t)th * R1 + r.n[2];
  r.n[2] = (uint32_t)v & M;
  r.n[3] += (uint32_t)(v >> 26);
}

__device__ __forceinline__ void mul26(f26 &r, const f26 &a, const f26 &b) {
  const uint32_t M = 0x3FFFFFFu, R0 = 0x3D10u, R1 = 0x400u;
  uint32_t h[10];
  uint64_t acc = 0;
#pragma unroll
  for (int k = 10; k < 19; k++) {
#pragma unroll
    for (int i = k - 9; i <= 9; i++) acc += (uint64_t)a.n[i] * b.n[k - i];
    h[k - 10] = (uint32_t)acc & M;
    acc >>= 26;
  }
  h[9] = (uint32_t)acc;  // < 2^32
  acc = 0;
#pragma unroll
  for (int k = 0; k < 10; k++) {
#pragma unroll
    for (int i = 0; i <= k; i++) acc += (uint64_t)a.n[i] * b.n[k - i];
    acc += (uint64_t)h[k] * R0;
    if (k) acc += (uint64_t)h[k - 1] * R1;
    r.n[k] = (uint32_t)acc & M;
    acc >>= 26;
  }
  fold26(r, acc, h[9]);
}

__device__ __forceinline__ void sqr26(f26 &r, const f26 &a) {
  const uint32_t M = 0x3FFFFFFu, R0 = 0x3D10u, R1 = 0x400u;
  uint32_t d[10];
#pragma unroll
  for (int i = 0; i < 10; i++) d[i] = a.n[i] << 1;
  uint32_t h[10];
  uint64_t acc = 0;
  // column k = sum_{i<j, i+j=k} 2 a_i a_j (+ a_{k/2}^2)
#pragma unroll
  for (int k = 10; k < 19; k++) {
#pragma unroll
    for (int i = k - 9; 2 * i < k; i++) acc += (uint64_t)d[i] * a.n[k - i];
    if ((k & 1) == 0) acc += (uint64_t)a.n[k / 2] * a.n[k / 2];
    h[k - 10] = (uint32_t)acc & M;
    acc >>= 26;
  }
  h[9] = (uint32_t)acc;
  acc = 0;
#pragma unroll
  for (int k = 0; k < 10; k++) {
#pragma unroll
    for (int i = 0; 2 * i < k; i++) acc += (uint64_t)d[i] * a.n[k - i];
    if ((k & 1) == 0) acc += (uint64_t)a.n[k / 2] * a.n[k / 2];
    acc += (uint64_t)h[k] * R0;
    if (k) acc += (uint64_t)h[k - 1] * R1;
    r.n[k] = (uint32_t)acc & M;
    acc >>= 26;
  }
  fold26(r, acc, h[9]);
}

// one carry sweep with the fold above 2^256: any magnitude (limbs below 2^31) back to limbs < 2^26
// (limb 9 < 2^22, limbs 1..3 a few bits over) -- what a lazy sum needs before it may enter mul26, whose
// columns stay below 2^58 only for limbs under 2^27
__device__ __forceinline__ void norm26(f26 &r) {
  uint64_t c = 0;
#pragma unroll
  for (int i = 0; i < 10; i++) {
    c += r.n[i];
    r.n[i] = (uint32_t)c & 0x3FFFFFFu;
    c >>= 26;
  }
  const uint64_t t = (c << 4) | (r.n[9] >> 22);
  r.n[9] &= 0x3FFFFFu;
  uint64_t v = (uint64_t)r.n[0] + t * 0x3D1u;
  r.n[0] = (uint32_t)v & 0x3FFFFFFu;
  v = (v >> 26) + r.n[1] + (t << 6);
  r.n[1] = (uint32_t)v & 0x3FFFFFFu;
  r.n[2] += (uint32_t)(v >> 26);
}

// lazy add and subtract (a + 4p - b, for b of magnitude <= 4): no carry chains
__device__ __forceinline__ void add26(f26 &r, const f26 &a, const f26 &b) {
#pragma unroll
  for (int i = 0; i < 10; i++) r.n[i] = a.n[i] + b.n[i];
}
__device__ __forceinline__ void sub26(f26 &r, const f26 &a, const f26 &b) {
  // 4p in 26-bit limbs: p = 2^256 - 0x1000003D1
  const uint32_t P2[10] = {4u * 0x3FFFC2Fu, 4u * 0x3FFFFBFu, 4u * 0x3FFFFFFu, 4u * 0x3FFFFFFu, 4u * 0x3FFFFFFu,
                           4u * 0x3FFFFFFu, 4u * 0x3FFFFFFu, 4u * 0x3FFFFFFu, 4u * 0x3FFFFFFu, 4u * 0x3FFFFFu};
#pragma unroll
  for (int i = 0; i < 10; i++) r.n[i] = a.n[i] + P2[i] - b.n[i];
}

// ---- 9x29: a = sum n_i 2^(29 i), limbs below 2^29 (the top one below 2^24).  2^261 == R = 0x2000007A20
// = R1 2^29 + R0 (R1 = 0x100, R0 = 0x7A20).  Columns of at most 9 products of 58 bits stay below 2^62 for
// limbs under 1.5 x 2^29, so the inputs must be (almost) normalized.
struct f29 {
  uint32_t n[9];
};
__device__ __forceinline__ void to29(f29 &o, const fe &a) {
#pragma unroll
  for (int i = 0; i < 9; i++) {
    const int bit = 29 * i, w = bit >> 5, s = bit & 31;
    uint64_t v = a.d[w];
    if (w + 1 < 8) v |= (uint64_t)a.d[w + 1] << 32;
    o.n[i] = (uint32_t)(v >> s) & 0x1FFFFFFFu;
  }
}
__device__ __forceinline__ void from29(fe &o, const f29 &a) {
  uint32_t n[9];
  for (int pass = 0; pass < 3; pass++) {
    uint64_t c = 0;
#pragma unroll
    for (int i = 0; i < 9; i++) {
      c += pass ? n[i] : a.n[i];
      n[i] = (uint32_t)c & 0x1FFFFFFFu;
      c >>= 29;
    }
    // bits at 2^261 and above (c) plus bits 256..260 of limb 8 (limb 8 holds bits 232..260)
    const uint64_t t = (c << 5) | (n[8] >> 24);
    n[8] &= 0xFFFFFFu;
    uint64_t v = (uint64_t)n[0] + t * 0x3D1u;
    n[0] = (uint32_t)v & 0x1FFFFFFFu;
    v = (v >> 29) + n[1] + (t << 3);  // 2^32 = 2^3 at limb 1
    n[1] = (uint32_t)v & 0x1FFFFFFFu;
    n[2] += (uint32_t)(v >> 29);
  }
  uint32_t w[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
  for (int i = 0; i < 9; i++) {
    const int bit = 29 * i, k = bit >> 5, s = bit & 31;
    const uint64_t v = (uint64_t)n[i] << s;
    w[k] |= (uint32_t)v;
    if (k + 1 < 8) w[k + 1] |= (uint32_t)(v >> 32);
  }
#pragma unroll
  for (int i = 0; i < 8; i++) o.d[i] = w[i];
  fe_canon(o);
}
__device__ __forceinline__ void fold29(f29 &r, uint64_t acc, const uint32_t h8) {
  const uint32_t M = 0x1FFFFFFFu, R0 = 0x7A20u, R1 = 0x100u;
  const uint64_t T = acc + (uint64_t)h8 * R1;  // at 2^261
  const uint32_t tl = (uint32_t)T & M, th = (uint32_t)(T >> 29);
  uint64_t v = (uint64_t)tl * R0 + r.n[0];
  r.n[0] = (uint32_t)v & M;
  v = (v >> 29) + (uint64_t)tl * R1 + (uint64_t)th * R0 + r.n[1];
  r.n[1] = (uint32_t)v & M;
  v = (v >> 29) + (uint64_t)th * R1 + r.n[2];
  r.n[2] = (uint32_t)v & M;
  r.n[3] += (uint32_t)(v >> 29);
}
__device__ __forceinline__ void mul29(f29 &r, const f29 &a, const f29 &b) {
  const uint32_t M = 0x1FFFFFFFu, R0 = 0x7A20u, R1 = 0x100u;
  uint32_t h[9];
  uint64_t acc = 0;
#pragma unroll
  for (int k = 9; k < 17; k++) {
#pragma unroll
    for (int i = k - 8; i <= 8; i++) acc += (uint64_t)a.n[i] * b.n[k - i];
    h[k - 9] = (uint32_t)acc & M;
    acc >>= 29;
  }
  h[8] = (uint32_t)acc;  // < 2^33: kept below 2^32 by the input bound
  acc = 0;
#pragma unroll
  for (int k = 0; k < 9; k++) {
#pragma unroll
    for (int i = 0; i <= k; i++) acc += (uint64_t)a.n[i] * b.n[k - i];
    acc += (uint64_t)h[k] * R0;
    if (k) acc += (uint64_t)h[k - 1] * R1;
    r.n[k] = (uint32_t)acc & M;
    acc >>= 29;
  }
  fold29(r, acc, h[8]);
}
__device__ __forceinline__ void sqr29(f29 &r, const f29 &a) {
  const uint32_t M = 0x1FFFFFFFu, R0 = 0x7A20u, R1 = 0x100u;
  uint32_t d[9];
#pragma unroll
  for (int i = 0; i < 9; i++) d[i] = a.n[i] << 1;
  uint32_t h[9];
  uint64_t acc = 0;
#pragma unroll
  for (int k = 9; k < 17; k++) {
#pragma unroll
    for (int i = k - 8; 2 * i < k; i++) acc += (uint64_t)d[i] * a.n[k - i];
    if ((k & 1) == 0) acc += (uint64_t)a.n[k / 2] * a.n[k / 2];
    h[k - 9] = (uint32_t)acc & M;
    acc >>= 29;
  }
  h[8] = (uint32_t)acc;
  acc = 0;
#pragma unroll
  for (int k = 0; k < 9; k++) {
#pragma unroll
    for (int i = 0; 2 * i < k; i++) acc += (uint64_t)d[i] * a.n[k - i];
    if ((k & 1) == 0) acc += (uint64_t)a.n[k / 2] * a.n[k / 2];
    acc += (uint64_t)h[k] * R0;
    if (k) acc += (uint64_t)h[k - 1] * R1;
    r.n[k] = (uint32_t)acc & M;
    acc >>= 29;
  }
  fold29(r, acc, h[8]);
}

// V: 0 fe_mul, 1 fe_sqr, 2 mul26, 3 sqr26, 4 two fe_add + two fe_sub, 5 two add26 + two sub26 + one norm26
// (the sweep the lazy sums need before a multiplication), 6 from26 + to26 (canonical bytes, as every probe needs)
template <int V>
__global__ void __launch_bounds__(256, 4) k_chain(const uint32_t *in, uint32_t *out, int iters) {
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  fe a, b;
  for (int i = 0; i < 8; i++) {
    a.d[i] = in[g * 16 + i];
    b.d[i] = in[g * 16 + 8 + i];
  }
  fe_canon(a);
  fe_canon(b);
  if constexpr (V <= 1 || V == 4) {
    for (int it = 0; it < iters; it++) {
      fe r;
      if constexpr (V == 0) fe_mul(r, a, b);
      if constexpr (V == 1) fe_sqr(r, a);
      if constexpr (V == 4) {
        fe s;
        fe_add(s, a, b);
        fe_sub(r, s, b);  // == a: the chain keeps a data dependence
        fe_sub(r, r, s);
        fe_add(r, r, a);
      }
      b = a;
      a = r;
    }
    for (int i = 0; i < 8; i++) out[g * 8 + i] = a.d[i];
  } else {
    f26 x, y;
    to26(x, a);
    to26(y, b);
    for (int it = 0; it < iters; it++) {
      f26 r;
      if constexpr (V == 2) mul26(r, x, y);
      if constexpr (V == 3) sqr26(r, x);
      if constexpr (V == 5) {
        f26 s;
        add26(s, x, y);
        sub26(r, s, y);
        sub26(r, r, s);
        add26(r, r, x);
        norm26(r);  // magnitude ~9 back to 1 before the next step (a mul would need it)
      }
      if constexpr (V == 6) {
        fe t;
        from26(t, x);
        to26(r, t);
        r.n[0] ^= y.n[0] & 1u;  // keep a dependence on y
      }
      y = x;
      x = r;
    }
    fe o;
    from26(o, x);
    for (int i = 0; i < 8; i++) out[g * 8 + i] = o.d[i];
  }
}
// V 7: mul29, 8: sqr29
template <int V>
__global__ void __launch_bounds__(256, 4) k_chain29(const uint32_t *in, uint32_t *out, int iters) {
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  fe a, b;
  for (int i = 0; i < 8; i++) {
    a.d[i] = in[g * 16 + i];
    b.d[i] = in[g * 16 + 8 + i];
  }
  fe_canon(a);
  fe_canon(b);
  f29 x, y;
  to29(x, a);
  to29(y, b);
  for (int it = 0; it < iters; it++) {
    f29 r;
    if constexpr (V == 7) mul29(r, x, y);
    if constexpr (V == 8) sqr29(r, x);
    y = x;
    x = r;
  }
  fe o;
  from29(o, x);
  for (int i = 0; i < 8; i++) out[g * 8 + i] = o.d[i];
}

namespace {
uint32_t *d_in = nullptr, *d_out = nullptr;
uint32_t g_lanes = 0;
}

extern "C" int ub_setup(uint32_t lanes) {
  g_lanes = lanes;
  std::vector<uint32_t> h((size_t)lanes * 16);
  uint64_t s = 88172645463325252ULL;
  for (auto &x : h) {
    s ^= s << 13;
    s ^= s >> 7;
    s ^= s << 17;
    x = (uint32_t)s;
  }
  if (hipMalloc(&d_in, h.size() * 4) != hipSuccess || hipMalloc(&d_out, (size_t)lanes * 32) != hipSuccess) return -1;
  return hipMemcpy(d_in, h.data(), h.size() * 4, hipMemcpyHostToDevice) == hipSuccess ? 0 : -1;
}

// reps launches of `iters` chained operations per lane; returns the events' milliseconds
extern "C" double ub_run(int v, int iters, int reps) {
  dim3 grid(g_lanes / 256), block(256);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0, 0);
  for (int r = 0; r < reps; r++) {
    switch (v) {
      case 0: hipLaunchKernelGGL(k_chain<0>, grid, block, 0, 0, d_in, d_out, iters); break;
      case 1: hipLaunchKernelGGL(k_chain<1>, grid, block, 0, 0, d_in, d_out, iters); break;
      case 2: hipLaunchKernelGGL(k_chain<2>, grid, block, 0, 0, d_in, d_out, iters); break;
      case 3: hipLaunchKernelGGL(k_chain<3>, grid, block, 0, 0, d_in, d_out, iters); break;
      case 4: hipLaunchKernelGGL(k_chain<4>, grid, block, 0, 0, d_in, d_out, iters); break;
      case 5: hipLaunchKernelGGL(k_chain<5>, grid, block, 0, 0, d_in, d_out, iters); break;
      case 6: hipLaunchKernelGGL(k_chain<6>, grid, block, 0, 0, d_in, d_out, iters); break;
      case 7: hipLaunchKernelGGL(k_chain29<7>, grid, block, 0, 0, d_in, d_out, iters); break;
      case 8: hipLaunchKernelGGL(k_chain29<8>, grid, block, 0, 0, d_in, d_out, iters); break;
      default: return -1;
    }
  }
  hipEventRecord(e1, 0);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  hipEventDestroy(e0);
  hipEventDestroy(e1);
  return hipGetLastError() == hipSuccess ? ms : -1;
}

extern "C" int ub_result(uint32_t *out) {
  return hipMemcpy(out, d_out, (size_t)g_lanes * 32, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
