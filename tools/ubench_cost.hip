// ubench_cost.hip -- gfx950 VALU issue cost per instruction class in SHADER CYCLES (development
// tool for the class-weighted roofline, bench.py "frac_mix").  tools/ubench_lat.hip priced the
// classes from wall time at a nominal 2.4 GHz, which folds the chip's clock into every figure; here
// every wave stamps s_memtime (shader clock) around its loop, and the host also derives the clock
// from s_memtime / s_memrealtime (100 MHz), so the table is clock-free.
//
// Each pattern is one asm statement of 32 wave-instructions (s_nop included where the pattern has
// them) per loop trip.  Printed per pattern and waves/SIMD (1, 2, 4, 8), two figures:
//   span  SIMD cycles per wave-instruction from the whole launch: (last wave's end - first wave's
//         start, s_memrealtime) x the in-kernel clock / (wave-instructions / 1024 SIMDs) -- the
//         SIMD's throughput whether or not the waves all overlap;
//   wave  the median wave's own (delta s_memtime) / (trips x 32): its issue interval per
//         instruction while sharing the SIMD (4.2 alone for most classes),
// and the in-kernel clock (delta s_memtime / delta s_memrealtime x 100 MHz).
//
// build: hipcc --offload-arch=gfx950 -O3 tools/ubench_cost.hip -o tools/ubench_cost
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

#define TRIPS 1024
#define R2(x) x x
#define R4(x) R2(x) R2(x)
#define R8(x) R4(x) R4(x)

struct stamp {
  uint64_t t0, t1, r0, r1;
};

template <int P>
__global__ __launch_bounds__(256) void k_pat(stamp *out, uint32_t seed) {
  const uint32_t t = blockIdx.x * 256 + threadIdx.x;
  uint64_t x0 = t * 3 + seed, x1 = t * 5, x2 = t * 7, x3 = t * 11;
  uint32_t a = t * 2654435761u + seed, b = a ^ 0x5bd1e995u, u0 = t, u1 = t + 1, u2 = t + 2, u3 = t + 3;
  uint64_t s0 = seed, s1 = seed + 1, s2 = seed + 2, s3 = seed + 3;
  uint32_t v0 = t * 13, v1 = t * 17, v2 = t * 19, v3 = t * 23;  // 32-bit operands of the run patterns
  __syncthreads();
  const uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < TRIPS; it++) {
    // --- 64-bit multiply-add and the product-scanning carry count
    if (P == 0)  // 4 independent accumulate chains, carry-outs into one SGPR pair
      asm volatile(R8("v_mad_u64_u32 %0, %4, %5, %6, %0\n v_mad_u64_u32 %1, %4, %5, %6, %1\n"
                      "v_mad_u64_u32 %2, %4, %5, %6, %2\n v_mad_u64_u32 %3, %4, %5, %6, %3\n")
                   : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "=s"(s0)
                   : "v"(a), "v"(b));
    if (P == 1)  // column as hipcc emits it around single-instruction asm: mad, s_nop 0, addc, s_nop 0
      asm volatile(R8("v_mad_u64_u32 %0, %2, %4, %5, %0\n s_nop 0\n v_addc_co_u32 %1, %3, 0, %1, %2\n s_nop 0\n")
                   : "+v"(x0), "+v"(u0), "=s"(s0), "=s"(s1)
                   : "v"(a), "v"(b));
    if (P == 2)  // the same 16 mad + 16 addc with the hazards covered by scheduling (no s_nop):
                 // each count reads a mask written two instructions earlier
      asm volatile(R4("v_mad_u64_u32 %0, %2, %6, %7, %0\n v_mad_u64_u32 %0, %3, %6, %7, %0\n"
                      "v_addc_co_u32 %1, %5, 0, %1, %2\n v_mad_u64_u32 %0, %4, %6, %7, %0\n"
                      "v_addc_co_u32 %1, %5, 0, %1, %3\n v_mad_u64_u32 %0, %2, %6, %7, %0\n"
                      "v_addc_co_u32 %1, %5, 0, %1, %4\n v_addc_co_u32 %1, %5, 0, %1, %2\n")
                   : "+v"(x0), "+v"(u0), "=s"(s0), "=s"(s1), "=s"(s2), "=s"(s3)
                   : "v"(a), "v"(b));
    if (P == 3)  // VCC carry chain as emitted: v_addc_co_u32_e32, s_nop 1, ... (16 + 16 nops)
      asm volatile(R8("v_add_co_u32_e32 %0, vcc, %4, %0\n s_nop 1\n v_addc_co_u32_e32 %1, vcc, %4, %1, vcc\n s_nop 1\n")
                   : "+v"(u0), "+v"(u1), "+v"(u2), "+v"(u3) : "v"(a) : "vcc");
    if (P == 4)  // add/addc pairs of 4 independent chains through 4 SGPR pairs, no s_nop needed
      asm volatile(R4("v_add_co_u32 %0, %4, %0, %8\n v_add_co_u32 %1, %5, %1, %8\n"
                      "v_add_co_u32 %2, %6, %2, %8\n v_addc_co_u32 %0, %4, %0, %8, %4\n"
                      "v_add_co_u32 %3, %7, %3, %8\n v_addc_co_u32 %1, %5, %1, %8, %5\n"
                      "v_addc_co_u32 %2, %6, %2, %8, %6\n v_addc_co_u32 %3, %7, %3, %8, %7\n")
                   : "+v"(u0), "+v"(u1), "+v"(u2), "+v"(u3), "=s"(s0), "=s"(s1), "=s"(s2), "=s"(s3)
                   : "v"(a));
    // --- full-rate candidates
    if (P == 5)
      asm volatile(R8("v_mov_b32 %0, %4\n v_mov_b32 %1, %4\n v_mov_b32 %2, %4\n v_mov_b32 %3, %4\n")
                   : "=v"(u0), "=v"(u1), "=v"(u2), "=v"(u3) : "v"(a));
    if (P == 6)
      asm volatile(R8("v_add_u32 %0, %0, %4\n v_add_u32 %1, %1, %4\n v_add_u32 %2, %2, %4\n v_add_u32 %3, %3, %4\n")
                   : "+v"(u0), "+v"(u1), "+v"(u2), "+v"(u3) : "v"(a));
    if (P == 7)
      asm volatile(R8("v_and_b32 %0, %4, %0\n v_and_b32 %1, %4, %1\n v_and_b32 %2, %4, %2\n v_and_b32 %3, %4, %3\n")
                   : "+v"(u0), "+v"(u1), "+v"(u2), "+v"(u3) : "v"(a));
    if (P == 8)
      asm volatile(R8("v_bitop3_b32 %0, %0, %4, %1 bitop3:0x96\n v_bitop3_b32 %1, %1, %4, %2 bitop3:0x96\n"
                      "v_bitop3_b32 %2, %2, %4, %3 bitop3:0x96\n v_bitop3_b32 %3, %3, %4, %0 bitop3:0x96\n")
                   : "+v"(u0), "+v"(u1), "+v"(u2), "+v"(u3) : "v"(a));
    if (P == 9)
      asm volatile(R8("v_alignbit_b32 %0, %0, %0, 7\n v_alignbit_b32 %1, %1, %1, 7\n v_alignbit_b32 %2, %2, %2, 7\n"
                      "v_alignbit_b32 %3, %3, %3, 7\n")
                   : "+v"(u0), "+v"(u1), "+v"(u2), "+v"(u3));
    if (P == 10)
      asm volatile(R8("v_add3_u32 %0, %0, %4, %1\n v_add3_u32 %1, %1, %4, %2\n v_add3_u32 %2, %2, %4, %3\n"
                      "v_add3_u32 %3, %3, %4, %0\n")
                   : "+v"(u0), "+v"(u1), "+v"(u2), "+v"(u3) : "v"(a));
    if (P == 11)
      asm volatile(R8("v_lshrrev_b32 %0, 3, %0\n v_lshrrev_b32 %1, 3, %1\n v_lshrrev_b32 %2, 3, %2\n v_lshrrev_b32 %3, 3, %3\n")
                   : "+v"(u0), "+v"(u1), "+v"(u2), "+v"(u3));
    if (P == 12)
      asm volatile(R8("v_pk_lshlrev_b16 %0, %4, %0\n v_pk_lshlrev_b16 %1, %4, %1\n v_pk_lshlrev_b16 %2, %4, %2\n"
                      "v_pk_lshlrev_b16 %3, %4, %3\n")
                   : "+v"(u0), "+v"(u1), "+v"(u2), "+v"(u3) : "v"(a));
    if (P == 13)
      asm volatile(R8("v_perm_b32 %0, %0, %4, %1\n v_perm_b32 %1, %1, %4, %2\n v_perm_b32 %2, %2, %4, %3\n"
                      "v_perm_b32 %3, %3, %4, %0\n")
                   : "+v"(u0), "+v"(u1), "+v"(u2), "+v"(u3) : "v"(a));
    // --- compares, selects, carries to VCC
    if (P == 14)
      asm volatile(R8("v_cmp_eq_u32_e32 vcc, %0, %4\n v_cmp_eq_u32_e32 vcc, %1, %4\n v_cmp_eq_u32_e32 vcc, %2, %4\n"
                      "v_cmp_eq_u32_e32 vcc, %3, %4\n")
                   : "+v"(u0), "+v"(u1), "+v"(u2), "+v"(u3) : "v"(a) : "vcc");
    if (P == 15)
      asm volatile(R8("v_cndmask_b32_e64 %0, 0, 1, %4\n v_cndmask_b32_e64 %1, 0, 1, %4\n v_cndmask_b32_e64 %2, 0, 1, %4\n"
                      "v_cndmask_b32_e64 %3, 0, 1, %4\n")
                   : "=v"(u0), "=v"(u1), "=v"(u2), "=v"(u3) : "s"(s0));
    if (P == 16)  // independent adds writing VCC
      asm volatile(R8("v_add_co_u32_e32 %0, vcc, %4, %0\n v_add_co_u32_e32 %1, vcc, %4, %1\n"
                      "v_add_co_u32_e32 %2, vcc, %4, %2\n v_add_co_u32_e32 %3, vcc, %4, %3\n")
                   : "+v"(u0), "+v"(u1), "+v"(u2), "+v"(u3) : "v"(a) : "vcc");
    // --- 64-bit ALU
    if (P == 17)
      asm volatile(R8("v_lshrrev_b64 %0, 1, %0\n v_lshrrev_b64 %1, 1, %1\n v_lshrrev_b64 %2, 1, %2\n v_lshrrev_b64 %3, 1, %3\n")
                   : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3));
    if (P == 18)
      asm volatile(R8("v_lshl_add_u64 %0, %0, 0, %1\n v_lshl_add_u64 %1, %1, 0, %2\n v_lshl_add_u64 %2, %2, 0, %3\n"
                      "v_lshl_add_u64 %3, %3, 0, %0\n")
                   : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3));
    if (P == 19)
      asm volatile(R8("v_mov_b64 %0, %1\n v_mov_b64 %1, %2\n v_mov_b64 %2, %3\n v_mov_b64 %3, %0\n")
                   : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3));
    if (P == 20)
      asm volatile(R8("v_mul_lo_u32 %0, %0, %4\n v_mul_hi_u32 %1, %1, %4\n v_mul_lo_u32 %2, %2, %4\n v_mul_hi_u32 %3, %3, %4\n")
                   : "+v"(u0), "+v"(u1), "+v"(u2), "+v"(u3) : "v"(a));
    // --- s_nop and mixes
    if (P == 21)  // s_nop 0 only
      asm volatile(R8(R4("s_nop 0\n")));
    if (P == 22)  // 16 v_add_u32 + 16 s_nop 0
      asm volatile(R8("v_add_u32 %0, %0, %4\n s_nop 0\n v_add_u32 %1, %1, %4\n s_nop 0\n")
                   : "+v"(u0), "+v"(u1), "+v"(u2), "+v"(u3) : "v"(a));
    if (P == 23)  // 16 independent mads + 16 s_nop 0 (nops that cover no hazard)
      asm volatile(R8("v_mad_u64_u32 %0, %4, %5, %6, %0\n s_nop 0\n v_mad_u64_u32 %1, %4, %5, %6, %1\n s_nop 0\n")
                   : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "=s"(s0)
                   : "v"(a), "v"(b));
    if (P == 25)  // 16 mads (4 chains) + 16 independent SALU ops on 64-bit masks, interleaved
      asm volatile(R4("v_mad_u64_u32 %0, %4, %5, %6, %0\n s_xor_b64 %7, %7, %8\n v_mad_u64_u32 %1, %4, %5, %6, %1\n"
                      "s_and_b64 %8, %8, %7\n v_mad_u64_u32 %2, %4, %5, %6, %2\n s_or_b64 %7, %7, %8\n"
                      "v_mad_u64_u32 %3, %4, %5, %6, %3\n s_xor_b64 %8, %8, %7\n")
                   : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "=s"(s0), "+v"(a), "+v"(b), "+s"(s1), "+s"(s2)
                   :
                   : "scc");  // SALU ops write SCC: the loop's own compare-and-branch must not see it
    if (P == 26)  // SALU only: 32 s_xor_b64 / s_and_b64 on 4 independent mask pairs
      asm volatile(R8("s_xor_b64 %0, %0, %1\n s_and_b64 %1, %1, %2\n s_or_b64 %2, %2, %3\n s_xor_b64 %3, %3, %0\n")
                   : "+s"(s0), "+s"(s1), "+s"(s2), "+s"(s3)
                   :
                   : "scc");
    if (P == 27)  // a 7-product column counted by 7 v_addc (masks 3 apart) -- 14 VALU; x2 + 4 filler adds
      asm volatile(R2("v_mad_u64_u32 %0, %2, %9, %10, %0\n v_mad_u64_u32 %0, %3, %9, %10, %0\n v_mad_u64_u32 %0, %4, %9, %10, %0\n"
                      "v_addc_co_u32 %1, %2, 0, %1, %2\n v_mad_u64_u32 %0, %2, %9, %10, %0\n v_addc_co_u32 %1, %3, 0, %1, %3\n"
                      "v_mad_u64_u32 %0, %3, %9, %10, %0\n v_addc_co_u32 %1, %4, 0, %1, %4\n v_mad_u64_u32 %0, %4, %9, %10, %0\n"
                      "v_addc_co_u32 %1, %2, 0, %1, %2\n v_mad_u64_u32 %0, %2, %9, %10, %0\n v_addc_co_u32 %1, %3, 0, %1, %3\n"
                      "v_addc_co_u32 %1, %4, 0, %1, %4\n v_addc_co_u32 %1, %2, 0, %1, %2\n"
                      "v_add_u32 %5, %5, %9\n v_add_u32 %6, %6, %9\n")
                   : "+v"(x0), "+v"(u0), "=&s"(s0), "=&s"(s1), "=&s"(s2), "+v"(u1), "+v"(u2), "+v"(u3), "+v"(x1)
                   : "v"(a), "v"(b));
    if (P == 28)  // the same column counted on the SALU: 7 masks -> bit-sliced full adders (20 SALU) ->
                  // 3 VALU to materialize cnt = b0 + 2 b1 + 4 b2 -- 10 VALU + 20 SALU; x2 + 12 filler
      asm volatile(R2("v_mad_u64_u32 %0, s[40:41], %9, %10, %0\n v_mad_u64_u32 %0, s[42:43], %9, %10, %0\n"
                      "v_mad_u64_u32 %0, s[44:45], %9, %10, %0\n v_mad_u64_u32 %0, s[46:47], %9, %10, %0\n"
                      "s_xor_b64 s[60:61], s[40:41], s[42:43]\n v_mad_u64_u32 %0, s[48:49], %9, %10, %0\n"
                      "s_xor_b64 s[62:63], s[60:61], s[44:45]\n s_and_b64 s[64:65], s[40:41], s[42:43]\n"
                      "v_mad_u64_u32 %0, s[50:51], %9, %10, %0\n s_and_b64 s[60:61], s[60:61], s[44:45]\n"
                      "s_or_b64 s[64:65], s[64:65], s[60:61]\n v_mad_u64_u32 %0, s[52:53], %9, %10, %0\n"
                      "s_xor_b64 s[66:67], s[46:47], s[48:49]\n s_xor_b64 s[68:69], s[66:67], s[50:51]\n"
                      "s_and_b64 s[70:71], s[46:47], s[48:49]\n s_and_b64 s[66:67], s[66:67], s[50:51]\n"
                      "s_or_b64 s[70:71], s[70:71], s[66:67]\n"
                      "s_xor_b64 s[72:73], s[62:63], s[68:69]\n s_xor_b64 s[74:75], s[72:73], s[52:53]\n"
                      "s_and_b64 s[76:77], s[62:63], s[68:69]\n s_and_b64 s[72:73], s[72:73], s[52:53]\n"
                      "s_or_b64 s[76:77], s[76:77], s[72:73]\n"
                      "s_xor_b64 s[78:79], s[64:65], s[70:71]\n s_xor_b64 s[80:81], s[78:79], s[76:77]\n"
                      "s_and_b64 s[82:83], s[64:65], s[70:71]\n s_and_b64 s[78:79], s[78:79], s[76:77]\n"
                      "s_or_b64 s[82:83], s[82:83], s[78:79]\n"
                      "v_cndmask_b32_e64 %5, 0, 2, s[80:81]\n v_cndmask_b32_e64 %6, 0, 4, s[82:83]\n"
                      "v_addc_co_u32 %1, s[84:85], %5, %6, s[74:75]\n"
                      "v_add_u32 %7, %7, %9\n v_add_u32 %7, %7, %9\n v_add_u32 %7, %7, %9\n")
                   : "+v"(x0), "+v"(u0), "=&s"(s0), "=&s"(s1), "=&s"(s2), "=&v"(u1), "=&v"(u2), "+v"(u3), "+v"(x1)
                   : "v"(a), "v"(b)
                   : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53",
                     "s60", "s61", "s62", "s63", "s64", "s65", "s66", "s67", "s68", "s69", "s70", "s71", "s72", "s73",
                     "s74", "s75", "s76", "s77", "s78", "s79", "s80", "s81", "s82", "s83", "s84", "s85", "scc");
    // --- round 4: rotate encodings for the hash walks (SHA-256 / RIPEMD-160) and mixed-rate streams
    if (P == 29)  // byte-multiple rotates: v_alignbyte_b32
      asm volatile(R8("v_alignbyte_b32 %0, %0, %0, 1\n v_alignbyte_b32 %1, %1, %1, 1\n v_alignbyte_b32 %2, %2, %2, 1\n"
                      "v_alignbyte_b32 %3, %3, %3, 1\n")
                   : "+v"(u0), "+v"(u1), "+v"(u2), "+v"(u3));
    if (P == 30)  // shift-or fused: (x << n) | y
      asm volatile(R8("v_lshl_or_b32 %0, %0, 7, %1\n v_lshl_or_b32 %1, %1, 7, %2\n v_lshl_or_b32 %2, %2, 7, %3\n"
                      "v_lshl_or_b32 %3, %3, 7, %0\n")
                   : "+v"(u0), "+v"(u1), "+v"(u2), "+v"(u3));
    if (P == 31)  // a rotate as a shift pair: t = x >> 25; r = (x << 7) | t  (16 rotates per trip)
      asm volatile(R4("v_lshrrev_b32 %4, 25, %0\n v_lshrrev_b32 %5, 25, %1\n v_lshl_or_b32 %0, %0, 7, %4\n"
                      "v_lshl_or_b32 %1, %1, 7, %5\n v_lshrrev_b32 %4, 25, %2\n v_lshrrev_b32 %5, 25, %3\n"
                      "v_lshl_or_b32 %2, %2, 7, %4\n v_lshl_or_b32 %3, %3, 7, %5\n")
                   : "+v"(u0), "+v"(u1), "+v"(u2), "+v"(u3), "=&v"(a), "=&v"(b));
    if (P == 32)
      asm volatile(R8("v_or3_b32 %0, %0, %4, %1\n v_or3_b32 %1, %1, %4, %2\n v_or3_b32 %2, %2, %4, %3\n"
                      "v_or3_b32 %3, %3, %4, %0\n")
                   : "+v"(u0), "+v"(u1), "+v"(u2), "+v"(u3) : "v"(a));
    if (P == 33)
      asm volatile(R8("v_xad_u32 %0, %0, %4, %1\n v_xad_u32 %1, %1, %4, %2\n v_xad_u32 %2, %2, %4, %3\n"
                      "v_xad_u32 %3, %3, %4, %0\n")
                   : "+v"(u0), "+v"(u1), "+v"(u2), "+v"(u3) : "v"(a));
    if (P == 34)  // 16 alignbit + 16 v_add_u32, interleaved: does a full-rate op fill a half-rate op's slot?
      asm volatile(R8("v_alignbit_b32 %0, %0, %0, 7\n v_add_u32 %1, %1, %4\n v_alignbit_b32 %2, %2, %2, 7\n"
                      "v_add_u32 %3, %3, %4\n")
                   : "+v"(u0), "+v"(u1), "+v"(u2), "+v"(u3) : "v"(a));
    if (P == 35)  // 16 alignbit + 16 bitop3, interleaved
      asm volatile(R8("v_alignbit_b32 %0, %0, %0, 7\n v_bitop3_b32 %1, %1, %4, %3 bitop3:0x96\n"
                      "v_alignbit_b32 %2, %2, %2, 7\n v_bitop3_b32 %3, %3, %4, %1 bitop3:0x96\n")
                   : "+v"(u0), "+v"(u1), "+v"(u2), "+v"(u3) : "v"(a));
    if (P == 36)
      asm volatile(R8("v_lshl_add_u32 %0, %0, 3, %1\n v_lshl_add_u32 %1, %1, 3, %2\n v_lshl_add_u32 %2, %2, 3, %3\n"
                      "v_lshl_add_u32 %3, %3, 3, %0\n")
                   : "+v"(u0), "+v"(u1), "+v"(u2), "+v"(u3));
    if (P == 37)  // 16 add3 + 16 bitop3, interleaved
      asm volatile(R8("v_add3_u32 %0, %0, %4, %1\n v_bitop3_b32 %1, %1, %4, %3 bitop3:0x96\n"
                      "v_add3_u32 %2, %2, %4, %3\n v_bitop3_b32 %3, %3, %4, %0 bitop3:0x96\n")
                   : "+v"(u0), "+v"(u1), "+v"(u2), "+v"(u3) : "v"(a));
    if (P == 38)  // 16 mads + 16 bitop3, interleaved (the field math beside logic)
      asm volatile(R8("v_mad_u64_u32 %0, %4, %5, %6, %0\n v_bitop3_b32 %7, %7, %5, %8 bitop3:0x96\n"
                      "v_mad_u64_u32 %1, %4, %5, %6, %1\n v_bitop3_b32 %8, %8, %6, %7 bitop3:0x96\n")
                   : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "=s"(s0), "+v"(a), "+v"(b), "+v"(u0), "+v"(u1));
    if (P == 39)  // 16 add_u32 + 16 v_add_u32 writing... two full-rate streams (control for 34/35)
      asm volatile(R8("v_add_u32 %0, %0, %4\n v_xor_b32 %1, %1, %4\n v_add_u32 %2, %2, %4\n v_xor_b32 %3, %3, %4\n")
                   : "+v"(u0), "+v"(u1), "+v"(u2), "+v"(u3) : "v"(a));
    if (P == 40)  // rotate by 16 with SDWA word selects: t = x << 16 (dst WORD_1), r = (x >> 16) | t
      asm volatile(R4("v_mov_b32_sdwa %4, %0 dst_sel:WORD_1 dst_unused:UNUSED_PAD src0_sel:WORD_0\n"
                      "v_mov_b32_sdwa %5, %1 dst_sel:WORD_1 dst_unused:UNUSED_PAD src0_sel:WORD_0\n"
                      "v_or_b32_sdwa %0, %0, %4 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:DWORD\n"
                      "v_or_b32_sdwa %1, %1, %5 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:DWORD\n"
                      "v_mov_b32_sdwa %4, %2 dst_sel:WORD_1 dst_unused:UNUSED_PAD src0_sel:WORD_0\n"
                      "v_mov_b32_sdwa %5, %3 dst_sel:WORD_1 dst_unused:UNUSED_PAD src0_sel:WORD_0\n"
                      "v_or_b32_sdwa %2, %2, %4 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:DWORD\n"
                      "v_or_b32_sdwa %3, %3, %5 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:DWORD\n")
                   : "+v"(u0), "+v"(u1), "+v"(u2), "+v"(u3), "=&v"(a), "=&v"(b));
    if (P == 41)  // runs of 4: 4 alignbit then 4 v_add_u32 (does grouping let full-rate ops pair up?)
      asm volatile(R4("v_alignbit_b32 %0, %0, %0, 7\n v_alignbit_b32 %1, %1, %1, 7\n v_alignbit_b32 %2, %2, %2, 7\n"
                      "v_alignbit_b32 %3, %3, %3, 7\n v_add_u32 %4, %4, %8\n v_add_u32 %5, %5, %8\n"
                      "v_add_u32 %6, %6, %8\n v_add_u32 %7, %7, %8\n")
                   : "+v"(u0), "+v"(u1), "+v"(u2), "+v"(u3), "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3) : "v"(a));
    if (P == 42)  // runs of 16: 16 alignbit then 16 bitop3
      asm volatile(R4("v_alignbit_b32 %0, %0, %0, 7\n v_alignbit_b32 %1, %1, %1, 7\n v_alignbit_b32 %2, %2, %2, 7\n"
                      "v_alignbit_b32 %3, %3, %3, 7\n")
                   R4("v_bitop3_b32 %4, %4, %8, %5 bitop3:0x96\n v_bitop3_b32 %5, %5, %8, %6 bitop3:0x96\n"
                      "v_bitop3_b32 %6, %6, %8, %7 bitop3:0x96\n v_bitop3_b32 %7, %7, %8, %4 bitop3:0x96\n")
                   : "+v"(u0), "+v"(u1), "+v"(u2), "+v"(u3), "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3) : "v"(a));
    if (P == 43)  // pairs: 2 alignbit then 2 v_add_u32
      asm volatile(R8("v_alignbit_b32 %0, %0, %0, 7\n v_alignbit_b32 %1, %1, %1, 7\n v_add_u32 %2, %2, %4\n"
                      "v_add_u32 %3, %3, %4\n")
                   : "+v"(u0), "+v"(u1), "+v"(u2), "+v"(u3) : "v"(a));
    if (P == 24)  // 16 mads + 16 v_mov (the product-scanning column shift), interleaved
      asm volatile(R8("v_mad_u64_u32 %0, %4, %5, %6, %0\n v_mov_b32 %7, %5\n v_mad_u64_u32 %1, %4, %5, %6, %1\n"
                      "v_mov_b32 %8, %6\n")
                   : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "=s"(s0), "+v"(a), "+v"(b), "=v"(u0), "=v"(u1));
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  if ((threadIdx.x & 63) == 0) {
    stamp s;
    s.t0 = t0;
    s.t1 = t1 + (x0 ^ x1 ^ x2 ^ x3 ^ u0 ^ u1 ^ u2 ^ u3 ^ s0 ^ s1 ^ s2 ^ s3 ^ a ^ b ^ v0 ^ v1 ^ v2 ^ v3) * 0;  // keep results live
    s.r0 = r0;
    s.r1 = r1;
    out[t >> 6] = s;
  }
}

typedef void (*kfn)(stamp *, uint32_t);
#define K(n) k_pat<n>
static const kfn kernels[] = {K(0),  K(1),  K(2),  K(3),  K(4),  K(5),  K(6),  K(7),  K(8),  K(9),  K(10), K(11), K(12),
                              K(13), K(14), K(15), K(16), K(17), K(18), K(19), K(20), K(21), K(22), K(23), K(24),
                              K(25), K(26), K(27), K(28), K(29), K(30), K(31), K(32), K(33), K(34), K(35), K(36),
                              K(37), K(38), K(39), K(40), K(41), K(42), K(43)};
static const char *names[] = {
    "mad_u64_u32 acc, 4 chains",      "mad,nop,addc,nop (as hipcc)",  "mad+addc, hazards scheduled", "addc_e32 vcc chain + s_nop 1",
    "add_co/addc, 4 sgpr chains",     "v_mov_b32",                    "v_add_u32",                   "v_and_b32",
    "v_bitop3_b32",                   "v_alignbit_b32",               "v_add3_u32",                  "v_lshrrev_b32",
    "v_pk_lshlrev_b16",               "v_perm_b32",                   "v_cmp_eq_u32 (vcc)",          "v_cndmask_b32_e64 (sgpr)",
    "v_add_co_u32_e32 (vcc) indep",   "v_lshrrev_b64",                "v_lshl_add_u64",              "v_mov_b64",
    "v_mul_lo/hi_u32",                "s_nop 0 only",                 "v_add_u32 + s_nop 0",         "mad + s_nop 0 (no hazard)",
    "mad + v_mov interleaved",        "mad + SALU interleaved",       "SALU only (s_xor/and/or_b64)", "7-col: 7 addc (+2 add)",
    "7-col: SALU count (+3 add)",     "v_alignbyte_b32",              "v_lshl_or_b32",               "rotate = lshrrev + lshl_or",
    "v_or3_b32",                      "v_xad_u32 (xor-add)",                   "alignbit + v_add_u32 mix",    "alignbit + bitop3 mix",
    "v_lshl_add_u32",                 "add3 + bitop3 mix",            "mad + bitop3 mix",            "v_add_u32 + v_xor_b32 mix",
    "rot16 = 2 sdwa ops",             "runs: 4 alignbit, 4 add",      "runs: 16 alignbit, 16 bitop3", "runs: 2 alignbit, 2 add"};

int main(int argc, char **argv) {
  // optional: the pattern numbers to run (default all)
  setvbuf(stdout, nullptr, _IOLBF, 0);
  const int NP = sizeof(kernels) / sizeof(kernels[0]);
  std::vector<int> only;
  for (int i = 1; i < argc; i++) only.push_back(atoi(argv[i]));
  const int waves_per_simd[] = {1, 2, 4, 8};
  stamp *d;
  const int max_blocks = 256 * 8;
  (void)hipMalloc(&d, sizeof(stamp) * max_blocks * 4);
  std::vector<stamp> h(max_blocks * 4);
  printf("%-32s %s\n", "pattern (32 instr per trip)",
         "at W waves/SIMD: span = SIMD cycles per wave-instruction (whole launch), wave = one wave's cycles per instruction [in-kernel GHz]");
  for (int p = 0; p < NP; p++) {
    if (!only.empty() && std::find(only.begin(), only.end(), p) == only.end()) continue;
    printf("%-32s", names[p]);
    for (int w : waves_per_simd) {
      const int blocks = 256 * w;  // 256 CUs x w blocks of 4 waves: w waves per SIMD
      double cyc = 0, ghz = 0, span = 0;
      for (int rep = 0; rep < 2; rep++) {  // the first launch warms the clock
        hipLaunchKernelGGL(kernels[p], dim3(blocks), dim3(256), 0, 0, d, 1u);
        (void)hipDeviceSynchronize();
        (void)hipMemcpy(h.data(), d, sizeof(stamp) * blocks * 4, hipMemcpyDeviceToHost);
        std::vector<double> c, g;
        uint64_t rmin = ~0ull, rmax = 0;
        for (int i = 0; i < blocks * 4; i++) {
          const double dt = (double)(h[i].t1 - h[i].t0), dr = (double)(h[i].r1 - h[i].r0);
          c.push_back(dt / (TRIPS * 32.0));
          if (dr > 0) g.push_back(dt / dr * 0.1);  // s_memrealtime ticks at 100 MHz
          rmin = std::min(rmin, h[i].r0);
          rmax = std::max(rmax, h[i].r1);
        }
        std::sort(c.begin(), c.end());
        std::sort(g.begin(), g.end());
        cyc = c[c.size() / 2];
        ghz = g.empty() ? 0 : g[g.size() / 2];
        // whole-launch SIMD cycles / wave-instructions per SIMD (blocks x 4 waves over 1024 SIMDs)
        span = (double)(rmax - rmin) * 10.0 * ghz / ((double)blocks * 4 * TRIPS * 32 / 1024.0);
      }
      printf("  W%d span %5.2f wave %5.2f [%.2f]", w, span, cyc, ghz);
    }
    printf("\n");
  }
  return 0;
}
