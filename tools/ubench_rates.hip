// ubench_rates.hip -- issue rate of single VALU instructions on gfx950 (development tool).
// Each lane runs 8 independent chains of ITERS instructions; prints cycles per wave-instruction per
// SIMD (chip-wide, at 2.4 GHz nominal) for: v_mad_u64_u32, v_mul_lo_u32, v_mul_hi_u32, v_fma_f64,
// v_add_co/addc pairs, v_mad_u32_u24, v_fma_f32.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define ITERS 4096

template <int V>
__global__ __launch_bounds__(256) void k_rate(uint64_t *out, uint32_t seed) {
  uint32_t t = blockIdx.x * 256 + threadIdx.x;
  uint64_t a[8];
  double f[8];
  uint32_t u[8];
  for (int i = 0; i < 8; i++) {
    a[i] = (uint64_t)(t * 2654435761u + i * 97u + seed) | 1;
    f[i] = (double)(t + i) * 1.0000001;
    u[i] = t * 7 + i;
  }
  uint32_t m = seed | 3;
  double fm = 1.0000000001;
  for (int it = 0; it < ITERS; it++) {
#pragma unroll
    for (int i = 0; i < 8; i++) {
      if (V == 0) asm volatile("v_mad_u64_u32 %0, s[100:101], %1, %2, %0" : "+v"(a[i]) : "v"(u[i]), "v"(m) : "s100", "s101");
      if (V == 1) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(u[i]) : "v"(m));
      if (V == 2) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(u[i]) : "v"(m));
      if (V == 3) asm volatile("v_fma_f64 %0, %0, %1, %1" : "+v"(f[i]) : "v"(fm));
      if (V == 4) asm volatile("v_add_co_u32 %0, vcc, %0, %1\n v_addc_co_u32 %0, vcc, %0, %1, vcc" : "+v"(u[i]) : "v"(m) : "vcc");
      if (V == 5) asm volatile("v_mad_u32_u24 %0, %0, %1, %0" : "+v"(u[i]) : "v"(m));
      if (V == 6) asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(u[i]) : "v"(m));
      if (V == 7) asm volatile("v_mul_f64 %0, %0, %1" : "+v"(f[i]) : "v"(fm));
      if (V == 8) asm volatile("v_add_u32 %0, %0, %1" : "+v"(u[i]) : "v"(m));
    }
  }
  uint64_t s = 0;
  for (int i = 0; i < 8; i++) s += a[i] + u[i] + (uint64_t)f[i];
  out[t] = s;
}

int main() {
  const int blocks = 256 * 16;   // 16 waves... 4 blocks of 4 waves per CU-SIMD set
  uint64_t *out;
  hipMalloc(&out, (size_t)blocks * 256 * 8);
  const char *names[] = {"v_mad_u64_u32", "v_mul_lo_u32", "v_mul_hi_u32", "v_fma_f64", "v_add_co+v_addc (2 instr)",
                         "v_mad_u32_u24", "v_fma_f32", "v_mul_f64", "v_add_u32"};
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int v = 0; v < 9; v++) {
    for (int rep = 0; rep < 2; rep++) {
      hipEventRecord(e0);
      switch (v) {
        case 0: hipLaunchKernelGGL(k_rate<0>, dim3(blocks), dim3(256), 0, 0, out, 1u); break;
        case 1: hipLaunchKernelGGL(k_rate<1>, dim3(blocks), dim3(256), 0, 0, out, 1u); break;
        case 2: hipLaunchKernelGGL(k_rate<2>, dim3(blocks), dim3(256), 0, 0, out, 1u); break;
        case 3: hipLaunchKernelGGL(k_rate<3>, dim3(blocks), dim3(256), 0, 0, out, 1u); break;
        case 4: hipLaunchKernelGGL(k_rate<4>, dim3(blocks), dim3(256), 0, 0, out, 1u); break;
        case 5: hipLaunchKernelGGL(k_rate<5>, dim3(blocks), dim3(256), 0, 0, out, 1u); break;
        case 6: hipLaunchKernelGGL(k_rate<6>, dim3(blocks), dim3(256), 0, 0, out, 1u); break;
        case 7: hipLaunchKernelGGL(k_rate<7>, dim3(blocks), dim3(256), 0, 0, out, 1u); break;
        case 8: hipLaunchKernelGGL(k_rate<8>, dim3(blocks), dim3(256), 0, 0, out, 1u); break;
      }
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      if (rep) {
        double wave_instr = (double)blocks * 4 * ITERS * 8 * (v == 4 ? 2 : 1);
        double per_simd = wave_instr / 1024.0;
        printf("%-28s %8.3f ms  %6.2f cycles per wave-instruction per SIMD (2.4 GHz)\n", names[v], ms,
               ms * 1e-3 * 2.4e9 / per_simd);
      }
    }
  }
  return 0;
}
