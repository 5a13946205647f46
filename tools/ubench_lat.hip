// ubench_lat.hip -- gfx950 VALU issue cost and dependent latency of the instructions the field
// arithmetic is built from (development tool).  Each pattern is one asm statement of 32
// instructions per loop trip; printed: cycles per wave-instruction per SIMD at 1 and 4 waves/SIMD
// (2.4 GHz nominal).  At 1 wave/SIMD a dependent pattern shows its latency; at 4 its throughput.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define ITERS 2048
#define R4(x) x x x x
#define R8(x) R4(x) R4(x)

template <int P>
__global__ __launch_bounds__(256) void k_pat(uint64_t *out, uint32_t seed) {
  uint32_t t = blockIdx.x * 256 + threadIdx.x;
  uint64_t x0 = t * 3 + seed, x1 = t * 5, x2 = t * 7, x3 = t * 11, x4 = t * 13, x5 = t * 17, x6 = t * 19, x7 = t * 23;
  uint32_t a = t * 2654435761u + seed, b = a ^ 0x5bd1e995u, u0 = t, u1 = t + 1, u2 = t + 2, u3 = t + 3;
  uint64_t s0 = seed, s1, s2, s3;
  for (int it = 0; it < ITERS; it++) {
    if (P == 0)  // 8 independent accumulate chains, carries into one SGPR pair
      asm volatile(R4("v_mad_u64_u32 %0, %8, %9, %10, %0\n v_mad_u64_u32 %1, %8, %9, %10, %1\n"
                      "v_mad_u64_u32 %2, %8, %9, %10, %2\n v_mad_u64_u32 %3, %8, %9, %10, %3\n"
                      "v_mad_u64_u32 %4, %8, %9, %10, %4\n v_mad_u64_u32 %5, %8, %9, %10, %5\n"
                      "v_mad_u64_u32 %6, %8, %9, %10, %6\n v_mad_u64_u32 %7, %8, %9, %10, %7\n")
                   : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(x4), "+v"(x5), "+v"(x6), "+v"(x7), "=s"(s0)
                   : "v"(a), "v"(b));
    if (P == 1)  // one dependent accumulate chain
      asm volatile(R8(R4("v_mad_u64_u32 %0, %1, %2, %3, %0\n")) : "+v"(x0), "=s"(s0) : "v"(a), "v"(b));
    if (P == 3)  // 4 interleaved chains
      asm volatile(R8("v_mad_u64_u32 %0, %4, %5, %6, %0\n v_mad_u64_u32 %1, %4, %5, %6, %1\n"
                      "v_mad_u64_u32 %2, %4, %5, %6, %2\n v_mad_u64_u32 %3, %4, %5, %6, %3\n")
                   : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "=s"(s0)
                   : "v"(a), "v"(b));
    if (P == 4)  // 8 independent, non-accumulating (src2 = 0)
      asm volatile(R4("v_mad_u64_u32 %0, %8, %9, %10, 0\n v_mad_u64_u32 %1, %8, %9, %10, 0\n"
                      "v_mad_u64_u32 %2, %8, %9, %10, 0\n v_mad_u64_u32 %3, %8, %9, %10, 0\n"
                      "v_mad_u64_u32 %4, %8, %9, %10, 0\n v_mad_u64_u32 %5, %8, %9, %10, 0\n"
                      "v_mad_u64_u32 %6, %8, %9, %10, 0\n v_mad_u64_u32 %7, %8, %9, %10, 0\n")
                   : "=v"(x0), "=v"(x1), "=v"(x2), "=v"(x3), "=v"(x4), "=v"(x5), "=v"(x6), "=v"(x7), "=s"(s0)
                   : "v"(a), "v"(b));
    if (P == 5)  // dependent v_add_u32 chain
      asm volatile(R8(R4("v_add_u32 %0, %0, %1\n")) : "+v"(u0) : "v"(a));
    if (P == 6)  // 4 independent v_add_u32 chains
      asm volatile(R8("v_add_u32 %0, %0, %4\n v_add_u32 %1, %1, %4\n v_add_u32 %2, %2, %4\n v_add_u32 %3, %3, %4\n")
                   : "+v"(u0), "+v"(u1), "+v"(u2), "+v"(u3) : "v"(a));
    if (P == 7)  // 64-bit shifts, 4 independent
      asm volatile(R8("v_lshrrev_b64 %0, 1, %0\n v_lshrrev_b64 %1, 1, %1\n v_lshrrev_b64 %2, 1, %2\n v_lshrrev_b64 %3, 1, %3\n")
                   : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3));
    if (P == 8)  // add-with-carry pairs, 4 independent chains, carries in 4 SGPR pairs, reads 3 later
      asm volatile(R4("v_add_co_u32 %0, %4, %0, %8\n v_add_co_u32 %1, %5, %1, %8\n"
                      "v_add_co_u32 %2, %6, %2, %8\n v_addc_co_u32 %0, %4, %0, %8, %4\n"
                      "v_add_co_u32 %3, %7, %3, %8\n v_addc_co_u32 %1, %5, %1, %8, %5\n"
                      "v_addc_co_u32 %2, %6, %2, %8, %6\n v_addc_co_u32 %3, %7, %3, %8, %7\n")
                   : "+v"(u0), "+v"(u1), "+v"(u2), "+v"(u3), "=s"(s0), "=s"(s1), "=s"(s2), "=s"(s3)
                   : "v"(a));
    if (P == 9)  // v_mad_u64_u32 with mul-by-1 (64-bit accumulate of a 32-bit word), 4 independent chains
      asm volatile(R8("v_mad_u64_u32 %0, %4, %5, 1, %0\n v_mad_u64_u32 %1, %4, %5, 1, %1\n"
                      "v_mad_u64_u32 %2, %4, %5, 1, %2\n v_mad_u64_u32 %3, %4, %5, 1, %3\n")
                   : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "=s"(s0)
                   : "v"(a));
    if (P == 10)  // v_mov_b32 independent
      asm volatile(R8("v_mov_b32 %0, %4\n v_mov_b32 %1, %4\n v_mov_b32 %2, %4\n v_mov_b32 %3, %4\n")
                   : "=v"(u0), "=v"(u1), "=v"(u2), "=v"(u3) : "v"(a));
    if (P == 11)  // v_mul_lo_u32 + v_mul_hi_u32, 4 independent
      asm volatile(R4("v_mul_lo_u32 %0, %0, %4\n v_mul_hi_u32 %1, %1, %4\n v_mul_lo_u32 %2, %2, %4\n v_mul_hi_u32 %3, %3, %4\n"
                      "v_mul_lo_u32 %0, %0, %4\n v_mul_hi_u32 %1, %1, %4\n v_mul_lo_u32 %2, %2, %4\n v_mul_hi_u32 %3, %3, %4\n")
                   : "+v"(u0), "+v"(u1), "+v"(u2), "+v"(u3) : "v"(a));
    if (P == 12)  // product-scanning column as generated: mad chain + carry count 2 instructions behind
      asm volatile(R4("v_mad_u64_u32 %0, %2, %6, %7, %0\n v_mad_u64_u32 %0, %3, %6, %7, %0\n"
                      "v_mad_u64_u32 %0, %4, %6, %7, %0\n v_addc_co_u32_e64 %1, %2, 0, %1, %2\n"
                      "v_mad_u64_u32 %0, %2, %6, %7, %0\n v_addc_co_u32_e64 %1, %3, 0, %1, %3\n"
                      "v_mad_u64_u32 %0, %3, %6, %7, %0\n v_addc_co_u32_e64 %1, %4, 0, %1, %4\n")
                   : "+v"(x0), "+v"(u0), "=s"(s0), "=s"(s1), "=s"(s2), "=s"(s3)
                   : "v"(a), "v"(b));
    if (P == 13)  // the same pairs as hipcc schedules them around single-instruction asm (s_nop 0 each side)
      asm volatile(R8("v_mad_u64_u32 %0, %2, %4, %5, %0\n s_nop 0\n v_addc_co_u32_e64 %1, %2, 0, %1, %2\n s_nop 0\n")
                   : "+v"(x0), "+v"(u0), "=s"(s0), "=s"(s1)
                   : "v"(a), "v"(b));
    if (P == 14)  // two independent columns interleaved
      asm volatile(R4("v_mad_u64_u32 %0, %4, %8, %9, %0\n v_mad_u64_u32 %1, %5, %8, %9, %1\n"
                      "v_mad_u64_u32 %0, %6, %8, %9, %0\n v_addc_co_u32_e64 %2, %4, 0, %2, %4\n"
                      "v_mad_u64_u32 %1, %7, %8, %9, %1\n v_addc_co_u32_e64 %3, %5, 0, %3, %5\n"
                      "v_addc_co_u32_e64 %2, %6, 0, %2, %6\n v_addc_co_u32_e64 %3, %7, 0, %3, %7\n")
                   : "+v"(x0), "+v"(x1), "+v"(u0), "+v"(u1), "=s"(s0), "=s"(s1), "=s"(s2), "=s"(s3)
                   : "v"(a), "v"(b));
    if (P == 15)  // v_cndmask from an SGPR mask
      asm volatile(R8("v_cndmask_b32_e64 %0, 0, 1, %4\n v_cndmask_b32_e64 %1, 0, 1, %4\n v_cndmask_b32_e64 %2, 0, 1, %4\n v_cndmask_b32_e64 %3, 0, 1, %4\n")
                   : "=v"(u0), "=v"(u1), "=v"(u2), "=v"(u3) : "s"(s0));
    if (P == 16)  // mad chain, fixed registers: X banks 0,1, a bank 2, b bank 3 (no bank conflict)
      asm volatile(R8(R4("v_mad_u64_u32 v[40:41], s[90:91], v42, v43, v[40:41]\n")) ::: "v40", "v41", "v42", "v43", "s90", "s91");
    if (P == 17)  // same, a and b both in bank 0 (= X.lo's bank)
      asm volatile(R8(R4("v_mad_u64_u32 v[40:41], s[90:91], v44, v48, v[40:41]\n")) ::: "v40", "v41", "v44", "v48", "s90", "s91");
    if (P == 18)  // a in bank 0, b in bank 1 (X.lo, X.hi banks)
      asm volatile(R8(R4("v_mad_u64_u32 v[40:41], s[90:91], v44, v45, v[40:41]\n")) ::: "v40", "v41", "v44", "v45", "s90", "s91");
    if (P == 19)  // a, b in bank 2 both
      asm volatile(R8(R4("v_mad_u64_u32 v[40:41], s[90:91], v42, v46, v[40:41]\n")) ::: "v40", "v41", "v42", "v46", "s90", "s91");
    if (P == 20)
      asm volatile(R8("v_add_u32_e64 %0, %0, %4\n v_add_u32_e64 %1, %1, %4\n v_add_u32_e64 %2, %2, %4\n v_add_u32_e64 %3, %3, %4\n") : "+v"(u0), "+v"(u1), "+v"(u2), "+v"(u3), "+v"(a), "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3) : : "vcc");
    if (P == 21)
      asm volatile(R8("v_add3_u32 %0, %0, %4, %1\n v_add3_u32 %1, %1, %4, %2\n v_add3_u32 %2, %2, %4, %3\n v_add3_u32 %3, %3, %4, %0\n") : "+v"(u0), "+v"(u1), "+v"(u2), "+v"(u3), "+v"(a), "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3) : : "vcc");
    if (P == 22)
      asm volatile(R8("v_bitop3_b32 %0, %0, %4, %1 bitop3:0x96\n v_bitop3_b32 %1, %1, %4, %2 bitop3:0x96\n v_bitop3_b32 %2, %2, %4, %3 bitop3:0x96\n v_bitop3_b32 %3, %3, %4, %0 bitop3:0x96\n") : "+v"(u0), "+v"(u1), "+v"(u2), "+v"(u3), "+v"(a), "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3) : : "vcc");
    if (P == 23)
      asm volatile(R8("v_alignbit_b32 %0, %0, %0, 7\n v_alignbit_b32 %1, %1, %1, 7\n v_alignbit_b32 %2, %2, %2, 7\n v_alignbit_b32 %3, %3, %3, 7\n") : "+v"(u0), "+v"(u1), "+v"(u2), "+v"(u3), "+v"(a), "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3) : : "vcc");
    if (P == 24)
      asm volatile(R8("v_xor_b32 %0, %4, %0\n v_xor_b32 %1, %4, %1\n v_xor_b32 %2, %4, %2\n v_xor_b32 %3, %4, %3\n") : "+v"(u0), "+v"(u1), "+v"(u2), "+v"(u3), "+v"(a), "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3) : : "vcc");
    if (P == 25)
      asm volatile(R8("v_lshlrev_b32 %0, 3, %0\n v_lshlrev_b32 %1, 3, %1\n v_lshlrev_b32 %2, 3, %2\n v_lshlrev_b32 %3, 3, %3\n") : "+v"(u0), "+v"(u1), "+v"(u2), "+v"(u3), "+v"(a), "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3) : : "vcc");
    if (P == 26)
      asm volatile(R8("v_add_co_u32 %0, vcc, %4, %0\n v_add_co_u32 %1, vcc, %4, %1\n v_add_co_u32 %2, vcc, %4, %2\n v_add_co_u32 %3, vcc, %4, %3\n") : "+v"(u0), "+v"(u1), "+v"(u2), "+v"(u3), "+v"(a), "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3) : : "vcc");
    if (P == 27)
      asm volatile(R8("v_xad_u32 %0, %0, %4, %1\n v_xad_u32 %1, %1, %4, %2\n v_xad_u32 %2, %2, %4, %3\n v_xad_u32 %3, %3, %4, %0\n") : "+v"(u0), "+v"(u1), "+v"(u2), "+v"(u3), "+v"(a), "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3) : : "vcc");
    if (P == 28)
      asm volatile(R8("v_add_lshl_u32 %0, %0, %4, 3\n v_add_lshl_u32 %1, %1, %4, 3\n v_add_lshl_u32 %2, %2, %4, 3\n v_add_lshl_u32 %3, %3, %4, 3\n") : "+v"(u0), "+v"(u1), "+v"(u2), "+v"(u3), "+v"(a), "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3) : : "vcc");
    if (P == 29)
      asm volatile(R8("v_perm_b32 %0, %0, %4, %1\n v_perm_b32 %1, %1, %4, %2\n v_perm_b32 %2, %2, %4, %3\n v_perm_b32 %3, %3, %4, %0\n") : "+v"(u0), "+v"(u1), "+v"(u2), "+v"(u3), "+v"(a), "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3) : : "vcc");
    if (P == 30)
      asm volatile(R8("v_pk_add_u16 %0, %0, %4\n v_pk_add_u16 %1, %1, %4\n v_pk_add_u16 %2, %2, %4\n v_pk_add_u16 %3, %3, %4\n") : "+v"(u0), "+v"(u1), "+v"(u2), "+v"(u3), "+v"(a), "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3) : : "vcc");
    if (P == 31)
      asm volatile(R8("v_mad_u32_u24 %0, %0, %4, %1\n v_mad_u32_u24 %1, %1, %4, %2\n v_mad_u32_u24 %2, %2, %4, %3\n v_mad_u32_u24 %3, %3, %4, %0\n") : "+v"(u0), "+v"(u1), "+v"(u2), "+v"(u3), "+v"(a), "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3) : : "vcc");
    if (P == 32)
      asm volatile(R8("v_lshl_add_u64 %5, %5, 0, %6\n v_lshl_add_u64 %6, %6, 0, %5\n v_lshl_add_u64 %7, %7, 0, %8\n v_lshl_add_u64 %8, %8, 0, %7\n") : "+v"(u0), "+v"(u1), "+v"(u2), "+v"(u3), "+v"(a), "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3) : : "vcc");
    if (P == 33)
      asm volatile(R8("v_mov_b64 %5, %6\n v_mov_b64 %6, %7\n v_mov_b64 %7, %8\n v_mov_b64 %8, %5\n") : "+v"(u0), "+v"(u1), "+v"(u2), "+v"(u3), "+v"(a), "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3) : : "vcc");
    if (P == 34)
      asm volatile(R8("v_cndmask_b32 %0, %4, %0, vcc\n v_cndmask_b32 %1, %4, %1, vcc\n v_cndmask_b32 %2, %4, %2, vcc\n v_cndmask_b32 %3, %4, %3, vcc\n") : "+v"(u0), "+v"(u1), "+v"(u2), "+v"(u3), "+v"(a), "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3) : : "vcc");
    if (P == 35)
      asm volatile(R8("v_mul_u32_u24 %0, %4, %0\n v_mul_u32_u24 %1, %4, %1\n v_mul_u32_u24 %2, %4, %2\n v_mul_u32_u24 %3, %4, %3\n") : "+v"(u0), "+v"(u1), "+v"(u2), "+v"(u3), "+v"(a), "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3) : : "vcc");
  }
  out[t] = x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7 + u0 + u1 + u2 + u3;
}

int main() {
  uint64_t *out;
  (void)hipMalloc(&out, (size_t)16384 * 256 * 8);
  const char *names[] = {"mad acc x8 indep", "mad acc 1 chain", "(unused)", "mad acc 4 chains",
                         "mad src2=0 x8 indep", "add_u32 1 chain", "add_u32 4 chains", "lshrrev_b64 4 chains",
                         "add_co/addc 4 chains", "mad-by-1 4 chains", "mov_b32", "mul_lo/hi 4 chains",
                         "column: mad+addc, no nop", "mad,nop,addc,nop (hipcc)", "2 columns interleaved", "cndmask sgpr",
                         "mad X01 a2 b3", "mad X01 a0 b0", "mad X01 a0 b1", "mad X01 a2 b2", "add_u32_e64 (VOP3 enc)", "add3_u32", "bitop3_b32", "alignbit_b32", "xor_b32_e32", "lshlrev_b32_e32", "add_co_u32_e32 (vcc)", "xad_u32", "add_lshl_u32", "perm_b32", "pk_add_u16", "mad_u32_u24", "lshl_add_u64", "mov_b64", "cndmask_b32_e32 (vcc)", "mul_u32_u24 e32"};
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int p = 0; p < 36; p++) {
    if (p == 2) continue;
    double cyc[3];
    for (int w = 0; w < 3; w++) {
      const int blocks = w == 0 ? 256 : w == 1 ? 1024 : 2048;  // 256 threads = 4 waves/block: 1, 4, 8 waves per SIMD
      for (int rep = 0; rep < 2; rep++) {
        (void)hipEventRecord(e0);
        switch (p) {
#define L(n) case n: hipLaunchKernelGGL(k_pat<n>, dim3(blocks), dim3(256), 0, 0, out, 1u); break;
          L(0) L(1) L(3) L(4) L(5) L(6) L(7) L(8) L(9) L(10) L(11) L(12) L(13) L(14) L(15) L(16) L(17) L(18) L(19) L(20) L(21) L(22) L(23) L(24) L(25) L(26) L(27) L(28) L(29) L(30) L(31) L(32) L(33) L(34) L(35)
        }
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        double per_simd = (double)blocks * 4 / 1024.0 * ITERS * 32;  // wave-instructions per SIMD (P13: 16 + 16 nops)
        cyc[w] = ms * 1e-3 * 2.4e9 / per_simd;
      }
    }
    printf("%-26s waves/SIMD 1: %5.2f  4: %5.2f  8: %5.2f  cycles/wave-instr\n", names[p], cyc[0], cyc[1], cyc[2]);
  }
  return 0;
}
