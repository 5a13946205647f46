// ubench_field3.hip -- field mul/sqr: hipcc-scheduled (kh_math.h) vs the generated single-statement
// asm forms (kh_field_asm.h, generated: python3 tools/gen_field_asm.py), single and paired (development tool).
//   timing: 2 independent chains per lane, ITERS steps, launch bounds (256, 4) as in the BSGS walk;
//   correctness: every variant's final values equal the kh_math.h device result, and a one-step
//   check of 2^18 lanes x edge-case inputs against the host (portable) code.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <vector>
#include "../keyhunt_amd/csrc/kh_math.h"
#include "kh_field_asm.h"

using namespace kh;

__device__ __forceinline__ void mul_a(fe &r, const fe &a, const fe &b) {
  fe t;
  if (fe_mul_asm(t, a, b) == 0xFFFFFFFFu) fe_mul(t, a, b);
  r = t;
}
__device__ __forceinline__ void sqr_a(fe &r, const fe &a) {
  fe t;
  if (fe_sqr_asm(t, a) == 0xFFFFFFFFu) fe_sqr(t, a);
  r = t;
}
__device__ __forceinline__ void mul2_a(fe &r, const fe &a, const fe &b, fe &s, const fe &c, const fe &d) {
  fe t, u;
  if (fe_mul2_asm(t, a, b, u, c, d) == 0xFFFFFFFFu) {
    fe_mul(t, a, b);
    fe_mul(u, c, d);
  }
  r = t;
  s = u;
}
__device__ __forceinline__ void sqr2_a(fe &r, const fe &a, fe &s, const fe &c) {
  fe t, u;
  if (fe_sqr2_asm(t, a, u, c) == 0xFFFFFFFFu) {
    fe_sqr(t, a);
    fe_sqr(u, c);
  }
  r = t;
  s = u;
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
  for (int it = 0; it < iters; it++) {
    fe r, s;
    if (V == 0) {
      fe_mul(r, a, b);
      fe_mul(s, c, d);
    } else if (V == 1) {
      mul_a(r, a, b);
      mul_a(s, c, d);
    } else if (V == 2) {
      mul2_a(r, a, b, s, c, d);
    } else if (V == 3) {
      fe_sqr(r, a);
      fe_sqr(s, c);
    } else if (V == 4) {
      sqr_a(r, a);
      sqr_a(s, c);
    } else {
      sqr2_a(r, a, s, c);
    }
    if (V < 3) {
      b = a;
      d = c;
    }
    a = r;
    c = s;
  }
  for (int i = 0; i < 8; i++) {
    out[g * 16 + i] = a.d[i];
    out[g * 16 + 8 + i] = c.d[i];
  }
}

// one step of each op on given inputs (no canonicalisation of inputs: < 2^256 is allowed)
__global__ void k_once(const uint32_t *in, uint32_t n, uint32_t *out) {
  uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= n) return;
  fe a, b, c, d;
  for (int i = 0; i < 8; i++) {
    a.d[i] = in[g * 32 + i];
    b.d[i] = in[g * 32 + 8 + i];
    c.d[i] = in[g * 32 + 16 + i];
    d.d[i] = in[g * 32 + 24 + i];
  }
  fe r[8];
  mul_a(r[0], a, b);
  sqr_a(r[1], a);
  mul2_a(r[2], a, b, r[3], c, d);
  sqr2_a(r[4], a, r[5], c);
  uint32_t f1 = fe_mul_asm(r[6], a, b);
  uint32_t f2 = fe_sqr_asm(r[7], c);
  for (int k = 0; k < 8; k++)
    for (int i = 0; i < 8; i++) out[((size_t)g * 8 + k) * 8 + i] = r[k].d[i];
  out[(size_t)n * 64 + 2 * g] = f1;
  out[(size_t)n * 64 + 2 * g + 1] = f2;
}

static uint64_t rs = 88172645463325252ULL;
static uint32_t rnd() {
  rs ^= rs << 13;
  rs ^= rs >> 7;
  rs ^= rs << 17;
  return (uint32_t)rs;
}

int main(int argc, char **argv) {
  const int lanes = 256 * 1024, iters = argc > 1 ? atoi(argv[1]) : 1000;
  std::vector<uint32_t> h((size_t)lanes * 32);
  for (size_t i = 0; i < h.size(); i++) {
    uint32_t x = rnd();
    // edge cases: limbs of all ones / zeros / p's limbs in some lanes
    uint32_t sel = (uint32_t)(i / 32) % 16;
    if (sel == 1) x = 0xFFFFFFFFu;
    if (sel == 2 && (i % 8) >= 2) x = 0xFFFFFFFFu;
    if (sel == 3) x = (i % 8) == 0 ? 0xFFFFFC2Eu : (i % 8) == 1 ? 0xFFFFFFFEu : 0xFFFFFFFFu;
    if (sel == 4 && (i % 8) < 4) x = 0;
    if (sel == 5 && (i % 8) >= 4) x = 0xFFFFFFFFu;
    h[i] = x;
  }
  uint32_t *din, *dout;
  (void)hipMalloc(&din, h.size() * 4);
  (void)hipMalloc(&dout, (size_t)lanes * 64 * 4 + (size_t)lanes * 8);
  (void)hipMemcpy(din, h.data(), h.size() * 4, hipMemcpyHostToDevice);

  // correctness, one step, against the host code
  hipLaunchKernelGGL(k_once, dim3(lanes / 256), dim3(256), 0, 0, din, (uint32_t)lanes, dout);
  std::vector<uint32_t> got((size_t)lanes * 64 + (size_t)lanes * 2);
  (void)hipMemcpy(got.data(), dout, got.size() * 4, hipMemcpyDeviceToHost);
  size_t bad = 0, slow1 = 0, slow2 = 0;
  for (int g = 0; g < lanes; g++) {
    fe a, b, c, d;
    for (int i = 0; i < 8; i++) {
      a.d[i] = h[g * 32 + i];
      b.d[i] = h[g * 32 + 8 + i];
      c.d[i] = h[g * 32 + 16 + i];
      d.d[i] = h[g * 32 + 24 + i];
    }
    fe e[6];
    fe_mul(e[0], a, b);
    fe_sqr(e[1], a);
    e[2] = e[0];
    fe_mul(e[3], c, d);
    e[4] = e[1];
    fe_sqr(e[5], c);
    for (int k = 0; k < 6; k++)
      for (int i = 0; i < 8; i++)
        if (got[((size_t)g * 8 + k) * 8 + i] != e[k].d[i]) {
          if (bad < 5) printf("MISMATCH lane %d op %d limb %d: %08x vs %08x\n", g, k, i, got[((size_t)g * 8 + k) * 8 + i], e[k].d[i]);
          bad++;
        }
    slow1 += got[(size_t)lanes * 64 + 2 * g] == 0xFFFFFFFFu;
    slow2 += got[(size_t)lanes * 64 + 2 * g + 1] == 0xFFFFFFFFu;
  }
  printf("one-step check over %d lanes: %zu mismatches; slow-path flags mul %zu sqr %zu\n", lanes, bad, slow1, slow2);

  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const char *names[] = {"fe_mul x2 (hipcc)", "fe_mul_asm x2", "fe_mul2_asm", "fe_sqr x2 (hipcc)", "fe_sqr_asm x2",
                         "fe_sqr2_asm"};
  std::vector<uint32_t> ref_mul, ref_sqr, res((size_t)lanes * 16);
  for (int v = 0; v < 6; v++) {
    auto launch = [&]() {
      dim3 g(lanes / 256), b(256);
      switch (v) {
        case 0: hipLaunchKernelGGL(k_bench<0>, g, b, 0, 0, din, dout, iters); break;
        case 1: hipLaunchKernelGGL(k_bench<1>, g, b, 0, 0, din, dout, iters); break;
        case 2: hipLaunchKernelGGL(k_bench<2>, g, b, 0, 0, din, dout, iters); break;
        case 3: hipLaunchKernelGGL(k_bench<3>, g, b, 0, 0, din, dout, iters); break;
        case 4: hipLaunchKernelGGL(k_bench<4>, g, b, 0, 0, din, dout, iters); break;
        case 5: hipLaunchKernelGGL(k_bench<5>, g, b, 0, 0, din, dout, iters); break;
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
    (void)hipMemcpy(res.data(), dout, (size_t)lanes * 64, hipMemcpyDeviceToHost);
    const char *ok = "";
    if (v == 0) ref_mul = res;
    if (v == 3) ref_sqr = res;
    if (v == 1 || v == 2) ok = res == ref_mul ? "match" : "MISMATCH";
    if (v == 4 || v == 5) ok = res == ref_sqr ? "match" : "MISMATCH";
    double ops = 2.0 * lanes * iters;
    printf("%-22s %8.3f ms  %8.2f Gop/s  %s\n", names[v], ms, ops / ms / 1e6, ok);
  }
  return 0;
}
