// kh_math.h -- secp256k1 field/group arithmetic, SHA-256, RIPEMD-160, XXH64 and libbloom probes,
// written once for CDNA4 device code and for the engine's host side (hipcc compiles both).
//
// Field elements are 8 x 32-bit little-endian limbs: the 32x32->64 multiply-add that gfx950
// executes natively (v_mad_u64_u32) is the unit of work, and carry chains use v_add_co/v_addc.
// In memory (HBM tables, host API) values are the reference's 4 x 64-bit little-endian limbs
// (secp256k1/Int.h:178-181) -- the same bytes.  All results are canonical (< p); the reference's
// ModMulK1 omits the final subtraction (secp256k1/IntMod.cpp:912), which can only differ with
// probability ~2^-224 and never on an emitted X coordinate.
//
// Reference behaviour restated here (paths relative to the reference checkout):
//   fe_mul / fe_sqr ........ secp256k1/IntMod.cpp:855-915, 977-1093 (fold by 0x1000003D1)
//   fe_add / fe_sub / neg .. secp256k1/IntMod.cpp:41-108
//   fe_inv ................. secp256k1/IntMod.cpp:382-511 (DRS62 there; Fermat chain here: same value)
//   sha256 / ripemd160 ..... hash/sha256_sse.cpp:95-554, hash/ripemd160_sse.cpp:323-361
//   hash160 packing ........ secp256k1/SECP256K1.cpp:974-1024 (04||X||Y), 1187-1250 (02/03||X)
//   xxh64 .................. xxhash/xxhash.h:2290-2529 (v0.8.0)
//   keccak-256 / eth ....... sha3/sha3.c (KECCAK_256_Final), keyhunt.cpp:5647-5669
//   bloom probe/add ........ bloom/bloom.cpp:122-146, 189-212
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define KH_HD __host__ __device__ __forceinline__
#else
#define KH_HD static inline
#endif

namespace kh {

struct fe {
  uint32_t d[8];
};

// ------------------------------------------------------------------------------------------
// carry helpers
// ------------------------------------------------------------------------------------------
// add/sub with carry: clang's __builtin_addc/__builtin_subc select v_add_co_u32/v_addc_co_u32
// (v_sub_co/v_subb_co) carry chains on gfx950; the portable form is for g++ host builds.
KH_HD uint32_t addc(uint32_t a, uint32_t b, uint32_t cin, uint32_t &cout) {
#if defined(__clang__)
  unsigned int co;
  uint32_t r = __builtin_addc(a, b, cin, &co);
  cout = co;
  return r;
#else
  uint64_t s = (uint64_t)a + b + cin;
  cout = (uint32_t)(s >> 32);
  return (uint32_t)s;
#endif
}
KH_HD uint32_t subb(uint32_t a, uint32_t b, uint32_t bin, uint32_t &bout) {
#if defined(__clang__)
  unsigned int bo;
  uint32_t r = __builtin_subc(a, b, bin, &bo);
  bout = bo;
  return r;
#else
  uint64_t s = (uint64_t)a - b - bin;
  bout = (uint32_t)(s >> 63);
  return (uint32_t)s;
#endif
}

// p = 2^256 - 0x1000003D1
#define KH_P0 0xFFFFFC2Fu
#define KH_P1 0xFFFFFFFEu

KH_HD void fe_set_u32(fe &r, uint32_t v) {
  r.d[0] = v;
#pragma unroll
  for (int i = 1; i < 8; i++) r.d[i] = 0;
}
KH_HD bool fe_is_zero(const fe &a) {
  uint32_t o = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) o |= a.d[i];
  return o == 0;
}
KH_HD bool fe_eq(const fe &a, const fe &b) {
  uint32_t o = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) o |= a.d[i] ^ b.d[i];
  return o == 0;
}
// r >= p ?
KH_HD bool fe_geq_p(const fe &r) {
  uint32_t hi = r.d[7] & r.d[6] & r.d[5] & r.d[4] & r.d[3] & r.d[2];
  if (hi != 0xFFFFFFFFu) return false;
  if (r.d[1] != KH_P1) return r.d[1] > KH_P1;
  return r.d[0] >= KH_P0;
}
// r -= p  (== r += 0x1000003D1 mod 2^256)
KH_HD void fe_sub_p(fe &r) {
  uint32_t c;
  r.d[0] = addc(r.d[0], 0x3D1u, 0, c);
  r.d[1] = addc(r.d[1], 1u, c, c);
#pragma unroll
  for (int i = 2; i < 8; i++) r.d[i] = addc(r.d[i], 0, c, c);
}
KH_HD void fe_canon(fe &r) {
  if (fe_geq_p(r)) fe_sub_p(r);
}

// KH_ISA_MARKS (analysis builds only, tools/valu_mix.py): every rarely executed fix-up block carries
// an empty asm statement whose comment marks it in the ISA listing
#if defined(__HIP_DEVICE_COMPILE__) && defined(KH_ISA_MARKS)
#define KH_RARE_MARK() asm volatile(";@kh_rare")
#else
#define KH_RARE_MARK() ((void)0)
#endif

#if defined(__HIP_DEVICE_COMPILE__)
// true iff `v` holds on any lane of the wave: a wave-uniform branch around a rarely needed fix-up
// (a carry rippling past limb 1, a value in [p, 2^256)).  When no lane needs it the wave jumps
// over it with one scalar branch; when taken, lanes that do not need it run it as a no-op.
__device__ __forceinline__ bool kh_any(bool v) { return __builtin_amdgcn_ballot_w64(v) != 0; }
__device__ __forceinline__ uint32_t kh_lane() {
  return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
}
#endif

// KH_ADDSUB_MAD: the +-0x1000003D1 fix-up of fe_add / fe_sub on limbs 0..1 as ONE 64-bit
// multiply-add.  0x1000003D1 = 3 * 1431656091, so with a selector s in {0, 3} (add) or {0, -3}
// (sub, signed v_mad_i64_i32), {r0, r1} + s * 1431656091 is the fix-up mod 2^64; the multiply-add's
// carry-out (add) or a grown limb 1 (sub: subtracting 0x1000003D1 < 2^33 wraps iff the new limb 1
// exceeds the old) flags the rare ripple past limb 1 as a lane mask the SALU tests.  Replaces two
// selects, an add pair and a bool-to-mask round trip per call.
#ifndef KH_ADDSUB_MAD
#define KH_ADDSUB_MAD 1
#endif
#define KH_P_DIV3 1431656091u

#if defined(__HIP_DEVICE_COMPILE__)
// a*b + c with b wave-uniform (an SGPR); m = the lane mask of the sum's 65th bit
__device__ __forceinline__ uint64_t mad_co(uint32_t a, uint32_t b, uint64_t c, uint64_t &m) {
  uint64_t d;
  asm("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=v"(d), "=s"(m) : "v"(a), "s"(b), "v"(c));
  return d;
}
// signed a*b + c mod 2^64 with b wave-uniform
__device__ __forceinline__ uint64_t mad_i_s(uint32_t a, uint32_t b, uint64_t c) {
  uint64_t d, m;
  asm("v_mad_i64_i32 %0, %1, %2, %3, %4" : "=v"(d), "=s"(m) : "v"(a), "s"(b), "v"(c));
  return d;
}
__device__ __forceinline__ uint64_t pack64(uint32_t lo, uint32_t hi) { return ((uint64_t)hi << 32) | lo; }
#endif

#if defined(__HIP_DEVICE_COMPILE__)
// The pieces of the KH_ADDSUB_MAD forms.  Tail of an addition: limbs 0..1 of r += c * 0x1000003D1;
// m = lanes whose fix-up carries past limb 1; returns the lanes that need fe_add_fix (m, or a top
// limb of all ones: r may be in [p, 2^256)).
__device__ __forceinline__ uint64_t fe_add_tail(fe &r, uint32_t c, uint64_t &m) {
  const uint64_t lo = mad_co(c ? 3u : 0u, KH_P_DIV3, pack64(r.d[0], r.d[1]), m);
  r.d[0] = (uint32_t)lo;
  r.d[1] = (uint32_t)(lo >> 32);
  return m | __builtin_amdgcn_ballot_w64(r.d[7] == 0xFFFFFFFFu);
}
__device__ __forceinline__ void fe_add_fix(fe &r, uint64_t m) {
  uint32_t c1 = (uint32_t)(m >> kh_lane()) & 1u;
#pragma unroll
  for (int i = 2; i < 8; i++) r.d[i] = addc(r.d[i], 0, c1, c1);
  fe_canon(r);
}
// Tail of a subtraction: limbs 0..1 of r -= br * 0x1000003D1; returns the lanes whose borrow
// ripples past limb 1 (limb 1 grew)
__device__ __forceinline__ uint64_t fe_sub_tail(fe &r, uint32_t br) {
  const uint32_t r1 = r.d[1];
  const uint64_t lo = mad_i_s(br ? 0xFFFFFFFDu : 0u, KH_P_DIV3, pack64(r.d[0], r.d[1]));  // -3 * ...
  r.d[0] = (uint32_t)lo;
  r.d[1] = (uint32_t)(lo >> 32);
  uint64_t m;
  asm("v_cmp_gt_u32 %0, %1, %2" : "=s"(m) : "v"(r.d[1]), "v"(r1));
  return m;
}
__device__ __forceinline__ void fe_sub_fix(fe &r, uint64_t m) {
  uint32_t b2 = (uint32_t)(m >> kh_lane()) & 1u;
#pragma unroll
  for (int i = 2; i < 8; i++) r.d[i] = subb(r.d[i], 0, b2, b2);
}
#endif

KH_HD void fe_add(fe &r, const fe &a, const fe &b) {
#if defined(__HIP_DEVICE_COMPILE__)
  if constexpr (KH_ADDSUB_MAD) {
    uint32_t c = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) r.d[i] = addc(a.d[i], b.d[i], c, c);
    uint64_t m;
    if (fe_add_tail(r, c, m) != 0) {
      KH_RARE_MARK();
      fe_add_fix(r, m);
    }
    return;
  }
  // a, b < p.  r = a + b; on a carry out of 2^256 (a + b - 2^256 < p) add 2^256 - p = 0x1000003D1:
  // the carry past limb 1 is rare.  Without a carry r < 2^256 is >= p only if its top limb is
  // all ones (rare).
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) r.d[i] = addc(a.d[i], b.d[i], c, c);
  uint32_t c1;
  r.d[0] = addc(r.d[0], c ? 0x3D1u : 0u, 0, c1);
  r.d[1] = addc(r.d[1], c, c1, c1);
  if (kh_any(c1 != 0 || r.d[7] == 0xFFFFFFFFu)) {
    KH_RARE_MARK();
#pragma unroll
    for (int i = 2; i < 8; i++) r.d[i] = addc(r.d[i], 0, c1, c1);
    fe_canon(r);
  }
#else
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) r.d[i] = addc(a.d[i], b.d[i], c, c);
  // if carry or r >= p: r -= p  (t = r + 0x1000003D1 carries out iff r >= p)
  fe t;
  uint32_t c2;
  t.d[0] = addc(r.d[0], 0x3D1u, 0, c2);
  t.d[1] = addc(r.d[1], 1u, c2, c2);
#pragma unroll
  for (int i = 2; i < 8; i++) t.d[i] = addc(r.d[i], 0, c2, c2);
  bool sel = (c | c2) != 0;
#pragma unroll
  for (int i = 0; i < 8; i++) r.d[i] = sel ? t.d[i] : r.d[i];
#endif
}
KH_HD void fe_sub(fe &r, const fe &a, const fe &b) {
  uint32_t br = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) r.d[i] = subb(a.d[i], b.d[i], br, br);
#if defined(__HIP_DEVICE_COMPILE__)
  if constexpr (KH_ADDSUB_MAD) {
    const uint64_t m = fe_sub_tail(r, br);
    if (m != 0) {
      KH_RARE_MARK();
      fe_sub_fix(r, m);
    }
    return;
  }
  // borrow: r += p == r -= 0x1000003D1 (mod 2^256); the borrow past limb 1 is rare
  {
    uint32_t b2;
    r.d[0] = subb(r.d[0], br ? 0x3D1u : 0u, 0, b2);
    r.d[1] = subb(r.d[1], br, b2, b2);
    if (kh_any(b2 != 0)) {
      KH_RARE_MARK();
#pragma unroll
      for (int i = 2; i < 8; i++) r.d[i] = subb(r.d[i], 0, b2, b2);
    }
    return;
  }
#endif
  // borrow: r += p  == r -= 0x1000003D1 (mod 2^256)
  uint32_t k0 = br ? 0x3D1u : 0u, k1 = br ? 1u : 0u, b2;
  r.d[0] = subb(r.d[0], k0, 0, b2);
  r.d[1] = subb(r.d[1], k1, b2, b2);
#pragma unroll
  for (int i = 2; i < 8; i++) r.d[i] = subb(r.d[i], 0, b2, b2);
}
KH_HD void fe_neg(fe &r, const fe &a) {
  fe z;
  fe_set_u32(z, 0);
  fe_sub(r, z, a);
}

// r = a (+|-) b and q = x (+|-) y (SUB1 / SUB2 pick subtraction), two independent operations with
// their carry chains interleaved limb by limb (KH_CHAIN2): each chain's next link reads a carry
// the other chain's link separates from its write, filling the pad a lone chain needs per link.
// Same results as the two single calls; r may alias a or b, q may alias x or y (never across).
#ifndef KH_CHAIN2
#define KH_CHAIN2 1
#endif
template <bool SUB1, bool SUB2>
KH_HD void fe_addsub2(fe &r, const fe &a, const fe &b, fe &q, const fe &x, const fe &y) {
#if defined(__HIP_DEVICE_COMPILE__)
  if constexpr (KH_ADDSUB_MAD && KH_CHAIN2) {
    uint32_t c = 0, d = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
      r.d[i] = SUB1 ? subb(a.d[i], b.d[i], c, c) : addc(a.d[i], b.d[i], c, c);
      q.d[i] = SUB2 ? subb(x.d[i], y.d[i], d, d) : addc(x.d[i], y.d[i], d, d);
    }
    uint64_t m1 = 0, m2 = 0, f1, f2;
    if constexpr (SUB1) f1 = fe_sub_tail(r, c); else f1 = fe_add_tail(r, c, m1);
    if constexpr (SUB2) f2 = fe_sub_tail(q, d); else f2 = fe_add_tail(q, d, m2);
    if ((f1 | f2) != 0) {
      KH_RARE_MARK();
      if (f1 != 0) {
        if constexpr (SUB1) fe_sub_fix(r, f1); else fe_add_fix(r, m1);
      }
      if (f2 != 0) {
        if constexpr (SUB2) fe_sub_fix(q, f2); else fe_add_fix(q, m2);
      }
    }
    return;
  }
#endif
  if constexpr (SUB1) fe_sub(r, a, b); else fe_add(r, a, b);
  if constexpr (SUB2) fe_sub(q, x, y); else fe_add(q, x, y);
}

// 512-bit t (16 limbs) -> canonical r.  t = lo + hi*2^256 == lo + hi*(2^32 + 977) (mod p).
KH_HD void fe_reduce512_gen(fe &r, const uint32_t t[16]) {
  uint32_t u[10];
  uint64_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    uint64_t v = (uint64_t)t[8 + i] * 977u + t[i] + c;
    u[i] = (uint32_t)v;
    c = v >> 32;
  }
  u[8] = (uint32_t)c;
  uint32_t cy = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) u[i + 1] = addc(u[i + 1], t[8 + i], cy, cy);
  u[9] = cy;
  // second fold: h = u[8] + u[9]*2^32 (< 2^34); r = u[0..7] + h*977 + h*2^32
  uint64_t v = (uint64_t)u[8] * 977u + u[0];
  r.d[0] = (uint32_t)v;
  c = v >> 32;
  v = (uint64_t)u[9] * 977u + u[1] + c + u[8];
  r.d[1] = (uint32_t)v;
  c = v >> 32;
  v = (uint64_t)u[2] + u[9] + c;
  r.d[2] = (uint32_t)v;
  uint32_t cc = (uint32_t)(v >> 32);
#if defined(__HIP_DEVICE_COMPILE__)
  // the carry past limb 2 and a result in [p, 2^256) are both rare
#pragma unroll
  for (int i = 3; i < 8; i++) r.d[i] = u[i];
  if (kh_any(cc != 0 || r.d[7] == 0xFFFFFFFFu)) {
    KH_RARE_MARK();
#pragma unroll
    for (int i = 3; i < 8; i++) r.d[i] = addc(r.d[i], 0, cc, cc);
    if (cc) fe_sub_p(r);
    if (r.d[7] == 0xFFFFFFFFu) fe_canon(r);
  }
#else
#pragma unroll
  for (int i = 3; i < 8; i++) r.d[i] = addc(u[i], 0, cc, cc);
  if (cc) fe_sub_p(r);  // wrapped past 2^256: add 0x1000003D1 (cannot wrap again)
  if (r.d[7] == 0xFFFFFFFFu) fe_canon(r);
#endif
}

#if defined(__HIP_DEVICE_COMPILE__)
// acc += a*b with the 64-bit carry-out of v_mad_u64_u32 counted into cnt (product scanning).
// The carry lands in an SGPR lane mask and is folded by v_addc_co_u32.
__device__ __forceinline__ uint64_t mad_acc(uint32_t a, uint32_t b, uint64_t acc, uint32_t &cnt) {
  uint64_t d, m, junk;
  asm("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=v"(d), "=s"(m) : "v"(a), "v"(b), "v"(acc));
  uint32_t o;
#ifdef KH_TIMING_EXTRA_NOPS
  // timing-only build (same results): one more s_nop per carry count prices the hazard pads
  asm("v_addc_co_u32 %0, %1, 0, %2, %3\n s_nop 1" : "=v"(o), "=s"(junk) : "v"(cnt), "s"(m));
#else
  asm("v_addc_co_u32 %0, %1, 0, %2, %3" : "=v"(o), "=s"(junk) : "v"(cnt), "s"(m));
#endif
  cnt = o;
  return d;
}
#endif

#if defined(__HIP_DEVICE_COMPILE__)
// acc + a*b where the sum provably fits 64 bits (no carry to count)
__device__ __forceinline__ uint64_t mad_nc(uint32_t a, uint32_t b, uint64_t acc) {
  uint64_t d, m;
  asm("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=v"(d), "=s"(m) : "v"(a), "v"(b), "v"(acc));
  return d;
}
#endif
#ifndef KH_SAFE_ADDC
#define KH_SAFE_ADDC 1
#endif
#ifndef KH_RED2
#define KH_RED2 1
#endif
// KH_COLS: fe_mul / fe_sqr columns as one scheduled asm statement each (kh_cols.h, tools/gen_cols.py)
#ifndef KH_COLS
#define KH_COLS 1
#endif
// KH_MULRED: fe_mul's reduction slices and chain links issued inside its last column statements
// (kh_cols.h mul_red_cols), so the chain's carries wait behind column work instead of s_nop pads
#ifndef KH_MULRED
#define KH_MULRED 1
#endif
#include "kh_cols.h"

// The fold with 64-bit multiply-adds only (device): with h = t[8..15], l = t[0..7],
//   t == sum_{j even} V_j 2^(32j) + sum_{i odd} W_i 2^(32i)  (mod p),
//   V_j = h_j*977 + l_j + l_{j+1} 2^32,   W_i = h_i*977 + h_{i-1} + h_i 2^32,
// since h_j (2^32 + 977) 2^(32j) is h_j*977 at limb j (in V_j) plus h_j at limb j+1 (in W_{j+1}
// for even j, in W_j's own 2^32 term for odd j).  The V_j are disjoint 64-bit slices (A) and so are
// the W_i one limb up (B): R = A + B 2^32 is one 8-limb carry chain, and its limb 8 folds again.
// Each V_j / W_i exceeds 64 bits with probability ~2^-22; the mad's carry-out lane mask keeps the
// lost bit.  A wave with such a lane, or whose second fold overflows, ripples past limb 2 or lands
// in [p, 2^256), puts the lost bits back into R and redoes the second fold the long way -- from R
// and the masks only, so t is dead after the mads.  Replaces the 64-bit adds and zero-extension
// moves of the long form (fe_reduce512_gen) by multiply-adds.
#if defined(__HIP_DEVICE_COMPILE__)
// The second fold and the rare block, from the chain's limbs R[0..8] (R = A + B 2^32) and the slice
// masks; r9() gives a lane's carry out of limb 8 (0/1), read in the rare block only.
template <typename R9F>
__device__ __forceinline__ void fe_reduce_tail(fe &r, uint32_t R[9], uint64_t m0, uint64_t m1, uint64_t m2,
                                               uint64_t m3, uint64_t m4, uint64_t m5, uint64_t m6, uint64_t m7,
                                               R9F r9) {
  const uint32_t K = 977u;
  uint64_t m8;
  // second fold: R8 (2^32 + 977) at limb 0
  const uint64_t X = mad_co(R[8], K, pack64(R[0], R[1]), m8);
  r.d[0] = (uint32_t)X;
#pragma unroll
  for (int i = 3; i < 8; i++) r.d[i] = R[i];
  // limbs 1..2 (+ R8 at limb 1) with the carry past limb 2 and the [p, 2^256) candidates as SGPR
  // lane masks (a bool carry read back through a ballot would round-trip through a VGPR); a
  // carry out of limb 8 (R9) leaves R8 = 0, so the mask of R8 == 0 stands for it
  uint64_t c2m, f7, c1m;
  asm("v_add_co_u32 %0, %3, %5, %6\n\tv_cmp_eq_u32 %4, -1, %8\n\ts_nop 0\n\tv_addc_co_u32 %1, %2, %7, 0, %3"
      : "=&v"(r.d[1]), "=v"(r.d[2]), "=s"(c2m), "=&s"(c1m), "=&s"(f7)
      : "v"((uint32_t)(X >> 32)), "v"(R[8]), "v"(R[2]), "v"(R[7]));
  if ((m0 | m1 | m2 | m3 | m4 | m5 | m6 | m7 | m8 | c2m | f7 | __builtin_amdgcn_ballot_w64(R[8] == 0)) != 0) {
    // rare: put back the 2^64 each overflowing V_j / W_i lost (limb j+2 / i+2; lane bits of
    // the masks), then the second fold the long way from R: h = R8 + R9 2^32 < 2^34
    KH_RARE_MARK();
    const uint32_t lane = kh_lane();
    const uint64_t ms[8] = {m0, m1, m2, m3, m4, m5, m6, m7};
    uint32_t cc = 0, Rq[9];
#pragma unroll
    for (int q = 0; q < 9; q++) Rq[q] = R[q];
#pragma unroll
    for (int q = 2; q < 9; q++) Rq[q] = addc(Rq[q], (uint32_t)(ms[q - 2] >> lane) & 1u, cc, cc);
    const uint32_t R9 = r9() + cc + ((uint32_t)(m7 >> lane) & 1u);
    const uint64_t h = (uint64_t)Rq[8] + ((uint64_t)R9 << 32);
    uint64_t v = h * 977u + Rq[0];
    r.d[0] = (uint32_t)v;
    v = (v >> 32) + Rq[1] + (h & 0xFFFFFFFFu);
    r.d[1] = (uint32_t)v;
    v = (v >> 32) + Rq[2] + (h >> 32);
    r.d[2] = (uint32_t)v;
    cc = (uint32_t)(v >> 32);
#pragma unroll
    for (int i = 3; i < 8; i++) r.d[i] = addc(Rq[i], 0, cc, cc);
    if (cc) fe_sub_p(r);  // wrapped past 2^256 once: + 0x1000003D1 cannot wrap again
    fe_canon(r);
  }
}
#endif

KH_HD void fe_reduce512(fe &r, const uint32_t t[16]) {
#if defined(__HIP_DEVICE_COMPILE__)
  if constexpr (KH_RED2) {
    const uint32_t K = 977u;
    uint64_t m0, m1, m2, m3, m4, m5, m6, m7;
    const uint64_t V0 = mad_co(t[8], K, pack64(t[0], t[1]), m0);
    const uint64_t W1 = mad_co(t[9], K, pack64(t[8], t[9]), m1);
    const uint64_t V2 = mad_co(t[10], K, pack64(t[2], t[3]), m2);
    const uint64_t W3 = mad_co(t[11], K, pack64(t[10], t[11]), m3);
    const uint64_t V4 = mad_co(t[12], K, pack64(t[4], t[5]), m4);
    const uint64_t W5 = mad_co(t[13], K, pack64(t[12], t[13]), m5);
    const uint64_t V6 = mad_co(t[14], K, pack64(t[6], t[7]), m6);
    const uint64_t W7 = mad_co(t[15], K, pack64(t[14], t[15]), m7);
    uint32_t R[9], c, R9;
    R[0] = (uint32_t)V0;
    R[1] = addc((uint32_t)(V0 >> 32), (uint32_t)W1, 0, c);
    R[2] = addc((uint32_t)V2, (uint32_t)(W1 >> 32), c, c);
    R[3] = addc((uint32_t)(V2 >> 32), (uint32_t)W3, c, c);
    R[4] = addc((uint32_t)V4, (uint32_t)(W3 >> 32), c, c);
    R[5] = addc((uint32_t)(V4 >> 32), (uint32_t)W5, c, c);
    R[6] = addc((uint32_t)V6, (uint32_t)(W5 >> 32), c, c);
    R[7] = addc((uint32_t)(V6 >> 32), (uint32_t)W7, c, c);
    R[8] = addc((uint32_t)(W7 >> 32), 0, c, R9);
    fe_reduce_tail(r, R, m0, m1, m2, m3, m4, m5, m6, m7, [&]() { return R9; });
    return;
  }
#endif
  fe_reduce512_gen(r, t);
}

KH_HD void fe_mul(fe &r, const fe &a, const fe &b) {
  uint32_t t[16];
#if defined(__HIP_DEVICE_COMPILE__)
  if constexpr (KH_COLS && KH_RED2 && KH_MULRED) {
    // the columns with the reduction's slices and first chain links interleaved (kh_cols.h)
    uint32_t R[9];
    uint64_t mk[8], r9;
    mul_red_cols(a.d, b.d, R, mk, r9);
    (void)t;
    fe_reduce_tail(r, R, mk[0], mk[1], mk[2], mk[3], mk[4], mk[5], mk[6], mk[7],
                   [&]() { return (uint32_t)(r9 >> kh_lane()) & 1u; });
    return;
  }
  if constexpr (KH_COLS) {
    mul_cols(a.d, b.d, t);  // the same columns, one scheduled asm statement each (kh_cols.h)
    fe_reduce512(r, t);
    return;
  }
  // product scanning: column k = sum_{i+j=k} a_i*b_j in a 64-bit accumulator + carry count
  uint64_t acc = 0;
  uint32_t cnt = 0;
#pragma unroll
  for (int k = 0; k < 15; k++) {
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const int j = k - i;
      if (j < 0 || j > 7) continue;
      // column 0 and the first product of column 1 cannot carry: (2^32-1)^2 + 2^32 - 1 < 2^64
      if (KH_SAFE_ADDC && (k == 0 || (k == 1 && i == 0)))
        acc = mad_nc(a.d[i], b.d[j], acc);
      else
        acc = mad_acc(a.d[i], b.d[j], acc, cnt);
    }
    t[k] = (uint32_t)acc;
    acc = (acc >> 32) | ((uint64_t)cnt << 32);
    cnt = 0;
  }
  t[15] = (uint32_t)acc;
#else
  {
    uint64_t c = 0;
    for (int j = 0; j < 8; j++) {
      uint64_t v = (uint64_t)a.d[0] * b.d[j] + c;
      t[j] = (uint32_t)v;
      c = v >> 32;
    }
    t[8] = (uint32_t)c;
  }
  for (int i = 1; i < 8; i++) {
    uint64_t c = 0;
    for (int j = 0; j < 8; j++) {
      uint64_t v = (uint64_t)a.d[i] * b.d[j] + t[i + j] + c;
      t[i + j] = (uint32_t)v;
      c = v >> 32;
    }
    t[i + 8] = (uint32_t)c;
  }
#endif
  fe_reduce512(r, t);
}

KH_HD void fe_sqr(fe &r, const fe &a) {
  uint32_t t[16];
#if defined(__HIP_DEVICE_COMPILE__)
  // cross products a_i*a_j (i<j) by product scanning, doubled, plus the squares a_i^2
  if constexpr (KH_COLS) {
    sqr_cross_cols(a.d, t);  // one scheduled asm statement per column (kh_cols.h)
  } else {
  uint64_t acc = 0;
  uint32_t cnt = 0;
  t[0] = 0;
#pragma unroll
  for (int k = 1; k < 14; k++) {
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const int j = k - i;
      if (j <= i || j > 7) continue;
      // columns 1 and 2 hold one cross product each and column 3 starts on an accumulator of at
      // most 2^32 - 1: their first products cannot carry
      if (KH_SAFE_ADDC && k <= 3 && i == 0)
        acc = mad_nc(a.d[i], a.d[j], acc);
      else
        acc = mad_acc(a.d[i], a.d[j], acc, cnt);
    }
    t[k] = (uint32_t)acc;
    acc = (acc >> 32) | ((uint64_t)cnt << 32);
    cnt = 0;
  }
  t[14] = (uint32_t)acc;
  t[15] = (uint32_t)(acc >> 32);
  }
  // double
#pragma unroll
  for (int i = 15; i > 0; i--) t[i] = __builtin_amdgcn_alignbit(t[i], t[i - 1], 31);
  t[0] = 0;
  // add squares: pair (t[2i], t[2i+1]) += a_i^2, carries rippled into the next pair
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    uint64_t sq = (uint64_t)a.d[i] * a.d[i];
    uint32_t c1;
    t[2 * i] = addc(t[2 * i], (uint32_t)sq, c, c1);
    t[2 * i + 1] = addc(t[2 * i + 1], (uint32_t)(sq >> 32), c1, c);
  }
#else
  for (int i = 0; i < 16; i++) t[i] = 0;
  for (int i = 0; i < 7; i++) {
    uint64_t c = 0;
    for (int j = i + 1; j < 8; j++) {
      uint64_t v = (uint64_t)a.d[i] * a.d[j] + t[i + j] + c;
      t[i + j] = (uint32_t)v;
      c = v >> 32;
    }
    t[i + 8] = (uint32_t)c;
  }
  t[15] = (t[15] << 1) | (t[14] >> 31);
  for (int i = 14; i > 0; i--) t[i] = (t[i] << 1) | (t[i - 1] >> 31);
  t[0] = t[0] << 1;
  uint64_t c = 0;
  for (int i = 0; i < 8; i++) {
    uint64_t v = (uint64_t)a.d[i] * a.d[i] + t[2 * i] + c;
    t[2 * i] = (uint32_t)v;
    v = (v >> 32) + t[2 * i + 1];
    t[2 * i + 1] = (uint32_t)v;
    c = v >> 32;
  }
#endif
  fe_reduce512(r, t);
}

KH_HD void fe_sqr_n(fe &r, const fe &a, int n) {
  fe_sqr(r, a);
#pragma unroll 1
  for (int i = 1; i < n; i++) fe_sqr(r, r);
}

// a^(p-2): 255 squarings + 15 multiplications (addition chain for p-2 = 2^256 - 2^32 - 979).
// The squaring runs stay rolled loops: the inversion runs once per 2H points.
KH_HD void fe_inv(fe &r, const fe &a) {
  fe x2, x3, x6, x9, x11, x22, x44, x88, x176, x220, x223, t;
  fe_sqr(x2, a);
  fe_mul(x2, x2, a);
  fe_sqr(x3, x2);
  fe_mul(x3, x3, a);
  fe_sqr_n(x6, x3, 3);
  fe_mul(x6, x6, x3);
  fe_sqr_n(x9, x6, 3);
  fe_mul(x9, x9, x3);
  fe_sqr_n(x11, x9, 2);
  fe_mul(x11, x11, x2);
  fe_sqr_n(x22, x11, 11);
  fe_mul(x22, x22, x11);
  fe_sqr_n(x44, x22, 22);
  fe_mul(x44, x44, x22);
  fe_sqr_n(x88, x44, 44);
  fe_mul(x88, x88, x44);
  fe_sqr_n(x176, x88, 88);
  fe_mul(x176, x176, x88);
  fe_sqr_n(x220, x176, 44);
  fe_mul(x220, x220, x44);
  fe_sqr_n(x223, x220, 3);
  fe_mul(x223, x223, x3);
  fe_sqr_n(t, x223, 23);
  fe_mul(t, t, x22);
  fe_sqr_n(t, t, 5);
  fe_mul(t, t, a);
  fe_sqr_n(t, t, 3);
  fe_mul(t, t, x2);
  fe_sqr_n(t, t, 2);
  fe_mul(r, t, a);
}

// a^((p+1)/4): square root when one exists (p == 3 mod 4).  Returns false if a is a non-residue.
KH_HD bool fe_sqrt(fe &r, const fe &a) {
  // (p+1)/4 = 2^254 - 2^30 - 244: chain from libsecp256k1's layout
  fe x2, x3, x6, x9, x11, x22, x44, x88, x176, x220, x223, t;
  fe_sqr(x2, a);
  fe_mul(x2, x2, a);
  fe_sqr(x3, x2);
  fe_mul(x3, x3, a);
  fe_sqr_n(x6, x3, 3);
  fe_mul(x6, x6, x3);
  fe_sqr_n(x9, x6, 3);
  fe_mul(x9, x9, x3);
  fe_sqr_n(x11, x9, 2);
  fe_mul(x11, x11, x2);
  fe_sqr_n(x22, x11, 11);
  fe_mul(x22, x22, x11);
  fe_sqr_n(x44, x22, 22);
  fe_mul(x44, x44, x22);
  fe_sqr_n(x88, x44, 44);
  fe_mul(x88, x88, x44);
  fe_sqr_n(x176, x88, 88);
  fe_mul(x176, x176, x88);
  fe_sqr_n(x220, x176, 44);
  fe_mul(x220, x220, x44);
  fe_sqr_n(x223, x220, 3);
  fe_mul(x223, x223, x3);
  fe_sqr_n(t, x223, 23);
  fe_mul(t, t, x22);
  fe_sqr_n(t, t, 6);
  fe_mul(t, t, x2);
  fe_sqr(t, t);
  fe_sqr(r, t);
  fe chk;
  fe_sqr(chk, r);
  return fe_eq(chk, a);
}

// 4 x u64 little-endian limbs <-> fe
KH_HD void fe_from_u64(fe &r, const uint64_t v[4]) {
#pragma unroll
  for (int i = 0; i < 4; i++) {
    r.d[2 * i] = (uint32_t)v[i];
    r.d[2 * i + 1] = (uint32_t)(v[i] >> 32);
  }
}
KH_HD void fe_to_u64(uint64_t v[4], const fe &a) {
#pragma unroll
  for (int i = 0; i < 4; i++) v[i] = (uint64_t)a.d[2 * i] | ((uint64_t)a.d[2 * i + 1] << 32);
}
// 32-byte big-endian (Int::Get32Bytes, secp256k1/Int.cpp:308-316)
KH_HD void fe_from_be(fe &r, const uint8_t b[32]) {
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint8_t *p = b + 28 - 4 * i;
    r.d[i] = ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
  }
}
KH_HD void fe_to_be(uint8_t b[32], const fe &a) {
#pragma unroll
  for (int i = 0; i < 8; i++) {
    uint8_t *p = b + 28 - 4 * i;
    p[0] = (uint8_t)(a.d[i] >> 24);
    p[1] = (uint8_t)(a.d[i] >> 16);
    p[2] = (uint8_t)(a.d[i] >> 8);
    p[3] = (uint8_t)a.d[i];
  }
}

// ------------------------------------------------------------------------------------------
// Group: affine points; the walk itself lives in the kernels.
// ------------------------------------------------------------------------------------------
struct ge {
  fe x, y;
};
struct gej {
  fe x, y, z;
  bool inf;
};

// Jacobian += affine (madd-2007-bl without the doubling/inverse cases: callers never hit them,
// see kh_kernels.hip scalar-mult comment).
KH_HD void gej_add_ge(gej &r, const ge &q) {
  if (r.inf) {
    r.x = q.x;
    r.y = q.y;
    fe_set_u32(r.z, 1);
    r.inf = false;
    return;
  }
  fe z1z1, u2, s2, h, hh, i, j, rr, v, t;
  fe_sqr(z1z1, r.z);
  fe_mul(u2, q.x, z1z1);
  fe_mul(s2, q.y, r.z);
  fe_mul(s2, s2, z1z1);
  fe_sub(h, u2, r.x);
  fe_sqr(hh, h);
  fe_add(i, hh, hh);
  fe_add(i, i, i);
  fe_mul(j, h, i);
  fe_sub(rr, s2, r.y);
  fe_add(rr, rr, rr);
  fe_mul(v, r.x, i);
  fe x3, y3, z3;
  fe_sqr(x3, rr);
  fe_sub(x3, x3, j);
  fe_sub(x3, x3, v);
  fe_sub(x3, x3, v);
  fe_sub(t, v, x3);
  fe_mul(y3, rr, t);
  fe_mul(t, r.y, j);
  fe_add(t, t, t);
  fe_sub(y3, y3, t);
  fe_add(z3, r.z, h);
  fe_sqr(z3, z3);
  fe_sub(z3, z3, z1z1);
  fe_sub(z3, z3, hh);
  r.x = x3;
  r.y = y3;
  r.z = z3;
}
KH_HD void gej_to_ge(ge &r, const gej &p) {
  fe zi, zi2, zi3;
  fe_inv(zi, p.z);
  fe_sqr(zi2, zi);
  fe_mul(zi3, zi2, zi);
  fe_mul(r.x, p.x, zi2);
  fe_mul(r.y, p.y, zi3);
}
// affine r = p + q with its own inversion (AddDirect, SECP256K1.cpp:455-478); p != +-q.
KH_HD void ge_add(ge &r, const ge &p, const ge &q) {
  fe dx, dy, s, s2, t;
  fe_sub(dx, q.x, p.x);
  fe_sub(dy, q.y, p.y);
  fe_inv(dx, dx);
  fe_mul(s, dy, dx);
  fe_sqr(s2, s);
  fe rx, ry;
  fe_sub(rx, s2, p.x);
  fe_sub(rx, rx, q.x);
  fe_sub(t, p.x, rx);
  fe_mul(ry, s, t);
  fe_sub(ry, ry, p.y);
  r.x = rx;
  r.y = ry;
}
// affine doubling (DoubleDirect, SECP256K1.cpp:589-614)
KH_HD void ge_double(ge &r, const ge &p) {
  fe x2, n3, d2, s, s2, t, rx, ry;
  fe_sqr(x2, p.x);
  fe_add(n3, x2, x2);
  fe_add(n3, n3, x2);
  fe_add(d2, p.y, p.y);
  fe_inv(d2, d2);
  fe_mul(s, n3, d2);
  fe_sqr(s2, s);
  fe_sub(rx, s2, p.x);
  fe_sub(rx, rx, p.x);
  fe_sub(t, p.x, rx);
  fe_mul(ry, s, t);
  fe_sub(ry, ry, p.y);
  r.x = rx;
  r.y = ry;
}

// ------------------------------------------------------------------------------------------
// SHA-256 / RIPEMD-160 (single 64-byte blocks, fully unrolled)
// ------------------------------------------------------------------------------------------
KH_HD uint32_t rotr32(uint32_t x, int n) {
#if defined(__HIP_DEVICE_COMPILE__)
  // llvm.fshr: one v_alignbit_b32, and constant-folded when x is a constant (the target-specific
  // alignbit builtin was not, which kept the hash IVs' rotations and every bitop3 on them live)
  return __builtin_rotateright32(x, (uint32_t)n);
#else
  return (x >> n) | (x << (32 - n));
#endif
}
KH_HD uint32_t rotl32(uint32_t x, int n) { return rotr32(x, (32 - n) & 31); }
KH_HD uint32_t bswap32(uint32_t x) {
  return (x >> 24) | ((x >> 8) & 0xFF00u) | ((x << 8) & 0xFF0000u) | (x << 24);
}
// Any 3-input boolean function in one gfx950 v_bitop3_b32: IMM is the truth table evaluated on
// a = 0xF0, b = 0xCC, c = 0xAA (so xor3 = 0x96, ch = 0xCA, maj = 0xE8).
// The truth table as plain logic: what the host runs, and what the device runs when an operand is a
// compile-time constant (below).
template <uint32_t IMM>
KH_HD uint32_t bitop3_logic(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t r = 0;
#pragma unroll
  for (int i = 0; i < 8; i++)
    if ((IMM >> i) & 1) {
      uint32_t m = ((i & 4) ? a : ~a) & ((i & 2) ? b : ~b) & ((i & 1) ? c : ~c);
      r |= m;
    }
  return r;
}
#ifndef KH_BITOP3_FOLD
#define KH_BITOP3_FOLD 1
#endif
template <uint32_t IMM>
KH_HD uint32_t bitop3(uint32_t a, uint32_t b, uint32_t c) {
#if defined(__HIP_DEVICE_COMPILE__)
  // An operand that is a constant after unrolling (the hash IVs and padding words: SHA-256's first
  // rounds, sigma of the zero schedule words, RIPEMD-160's first steps) goes through plain logic,
  // which LLVM folds; asm would pin each constant in a VGPR and keep the instruction.
  // __builtin_constant_p is resolved after inlining and unrolling (llvm.is.constant).
  if (KH_BITOP3_FOLD && __builtin_constant_p(a) && __builtin_constant_p(b) && __builtin_constant_p(c))
    return bitop3_logic<IMM>(a, b, c);
  uint32_t r;
  // one constant operand may come from an SGPR (the VOP3 constant-bus allows one scalar read): the
  // hash IVs of the first rounds then cost no VGPR across the walk's loop
  if (KH_BITOP3_FOLD && __builtin_constant_p(c))
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:%4" : "=v"(r) : "v"(a), "v"(b), "s"(c), "i"(IMM));
  else if (KH_BITOP3_FOLD && __builtin_constant_p(b))
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:%4" : "=v"(r) : "v"(a), "s"(b), "v"(c), "i"(IMM));
  else if (KH_BITOP3_FOLD && __builtin_constant_p(a))
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:%4" : "=v"(r) : "s"(a), "v"(b), "v"(c), "i"(IMM));
  else
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:%4" : "=v"(r) : "v"(a), "v"(b), "v"(c), "i"(IMM));
  return r;
#else
  return bitop3_logic<IMM>(a, b, c);
#endif
}
KH_HD uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) { return bitop3<0x96>(a, b, c); }

#define KH_SHA_K                                                                                          \
  {0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u, 0xab1c5ed5u, \
   0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u, 0xc19bf174u, \
   0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu, 0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau, \
   0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u, \
   0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu, 0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u, \
   0xa2bfe8a1u, 0xa81a664bu, 0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u, \
   0x19a4c116u, 0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u, \
   0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u, 0xc67178f2u}

KH_HD void sha256_init(uint32_t st[8]) {
  st[0] = 0x6a09e667u; st[1] = 0xbb67ae85u; st[2] = 0x3c6ef372u; st[3] = 0xa54ff53au;
  st[4] = 0x510e527fu; st[5] = 0x9b05688cu; st[6] = 0x1f83d9abu; st[7] = 0x5be0cd19u;
}
// st = compress(st, w) ; w is consumed (rolling schedule)
KH_HD void sha256_transform(uint32_t st[8], uint32_t w[16]) {
  const uint32_t K[64] = KH_SHA_K;
  uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
#pragma unroll
  for (int i = 0; i < 64; i++) {
    uint32_t wi;
    if (i < 16) {
      wi = w[i];
    } else {
      uint32_t w15 = w[(i - 15) & 15], w2 = w[(i - 2) & 15];
      uint32_t s0 = xor3(rotr32(w15, 7), rotr32(w15, 18), w15 >> 3);
      uint32_t s1 = xor3(rotr32(w2, 17), rotr32(w2, 19), w2 >> 10);
      wi = w[i & 15] + s0 + w[(i - 7) & 15] + s1;
      w[i & 15] = wi;
    }
    uint32_t t1 = h + xor3(rotr32(e, 6), rotr32(e, 11), rotr32(e, 25)) + bitop3<0xCA>(e, f, g) + K[i] + wi;
    uint32_t t2 = xor3(rotr32(a, 2), rotr32(a, 13), rotr32(a, 22)) + bitop3<0xE8>(a, b, c);
    h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
  }
  st[0] += a; st[1] += b; st[2] += c; st[3] += d; st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}


// Two independent SHA-256 compressions advanced round by round together (two dependency chains in
// flight per lane: hash160(02||X) and hash160(03||X) differ only in the first message byte).
KH_HD void sha256_transform2(uint32_t sa[8], uint32_t wa[16], uint32_t sb[8], uint32_t wb[16]) {
  const uint32_t K[64] = KH_SHA_K;
  uint32_t a = sa[0], b = sa[1], c = sa[2], d = sa[3], e = sa[4], f = sa[5], g = sa[6], h = sa[7];
  uint32_t a2 = sb[0], b2 = sb[1], c2 = sb[2], d2 = sb[3], e2 = sb[4], f2 = sb[5], g2 = sb[6], h2 = sb[7];
#pragma unroll
  for (int i = 0; i < 64; i++) {
    uint32_t wi, wj;
    if (i < 16) {
      wi = wa[i];
      wj = wb[i];
    } else {
      uint32_t w15 = wa[(i - 15) & 15], w2v = wa[(i - 2) & 15];
      wi = wa[i & 15] + xor3(rotr32(w15, 7), rotr32(w15, 18), w15 >> 3) + wa[(i - 7) & 15] +
           xor3(rotr32(w2v, 17), rotr32(w2v, 19), w2v >> 10);
      wa[i & 15] = wi;
      uint32_t v15 = wb[(i - 15) & 15], v2 = wb[(i - 2) & 15];
      wj = wb[i & 15] + xor3(rotr32(v15, 7), rotr32(v15, 18), v15 >> 3) + wb[(i - 7) & 15] +
           xor3(rotr32(v2, 17), rotr32(v2, 19), v2 >> 10);
      wb[i & 15] = wj;
    }
    uint32_t t1 = h + xor3(rotr32(e, 6), rotr32(e, 11), rotr32(e, 25)) + bitop3<0xCA>(e, f, g) + K[i] + wi;
    uint32_t t2 = xor3(rotr32(a, 2), rotr32(a, 13), rotr32(a, 22)) + bitop3<0xE8>(a, b, c);
    uint32_t u1 = h2 + xor3(rotr32(e2, 6), rotr32(e2, 11), rotr32(e2, 25)) + bitop3<0xCA>(e2, f2, g2) + K[i] + wj;
    uint32_t u2 = xor3(rotr32(a2, 2), rotr32(a2, 13), rotr32(a2, 22)) + bitop3<0xE8>(a2, b2, c2);
    h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    h2 = g2; g2 = f2; f2 = e2; e2 = d2 + u1; d2 = c2; c2 = b2; b2 = a2; a2 = u1 + u2;
  }
  sa[0] += a; sa[1] += b; sa[2] += c; sa[3] += d; sa[4] += e; sa[5] += f; sa[6] += g; sa[7] += h;
  sb[0] += a2; sb[1] += b2; sb[2] += c2; sb[3] += d2; sb[4] += e2; sb[5] += f2; sb[6] += g2; sb[7] += h2;
}

// RIPEMD-160 of a 32-byte message given as 8 little-endian words; out: 5 state words (LE bytes)
KH_HD uint32_t rmd_f(int j, uint32_t x, uint32_t y, uint32_t z) {
  // x^y^z, (x&y)|(~x&z), (x|~y)^z, (x&z)|(y&~z), x^(y|~z) as single v_bitop3_b32 truth tables
  return j < 16 ? bitop3<0x96>(x, y, z)
       : j < 32 ? bitop3<0xCA>(x, y, z)
       : j < 48 ? bitop3<0x59>(x, y, z)
       : j < 64 ? bitop3<0xE4>(x, y, z)
                : bitop3<0x2D>(x, y, z);
}
KH_HD void ripemd160_32(const uint32_t m[8], uint32_t out[5]) {
  const uint8_t RL[80] = {0, 1, 2,  3,  4,  5,  6,  7,  8,  9,  10, 11, 12, 13, 14, 15, 7,  4,  13, 1,
                          10, 6, 15, 3,  12, 0,  9,  5,  2,  14, 11, 8,  3,  10, 14, 4,  9,  15, 8,  1,
                          2,  7, 0,  6,  13, 11, 5,  12, 1,  9,  11, 10, 0,  8,  12, 4,  13, 3,  7,  15,
                          14, 5, 6,  2,  4,  0,  5,  9,  7,  12, 2,  10, 14, 1,  3,  8,  11, 6,  15, 13};
  const uint8_t RR[80] = {5,  14, 7,  0,  9, 2,  11, 4,  13, 6,  15, 8,  1,  10, 3,  12, 6,  11, 3,  7,
                          0,  13, 5,  10, 14, 15, 8, 12, 4,  9,  1,  2,  15, 5,  1,  3,  7,  14, 6,  9,
                          11, 8,  12, 2,  10, 0,  4, 13, 8,  6,  4,  1,  3,  11, 15, 0,  5,  12, 2,  13,
                          9,  7,  10, 14, 12, 15, 10, 4, 1,  5,  8,  7,  6,  2,  13, 14, 0,  3,  9,  11};
  const uint8_t SL[80] = {11, 14, 15, 12, 5,  8,  7,  9,  11, 13, 14, 15, 6,  7,  9,  8,  7,  6,  8,  13,
                          11, 9,  7,  15, 7,  12, 15, 9,  11, 7,  13, 12, 11, 13, 6,  7,  14, 9,  13, 15,
                          14, 8,  13, 6,  5,  12, 7,  5,  11, 12, 14, 15, 14, 15, 9,  8,  9,  14, 5,  6,
                          8,  6,  5,  12, 9,  15, 5,  11, 6,  8,  13, 12, 5,  12, 13, 14, 11, 8,  5,  6};
  const uint8_t SR[80] = {8,  9,  9,  11, 13, 15, 15, 5,  7,  7,  8,  11, 14, 14, 12, 6,  9,  13, 15, 7,
                          12, 8,  9,  11, 7,  7,  12, 7,  6,  15, 13, 11, 9,  7,  15, 11, 8,  6,  6,  14,
                          12, 13, 5,  14, 13, 13, 7,  5,  15, 5,  8,  11, 14, 14, 6,  14, 6,  9,  12, 9,
                          12, 5,  15, 8,  8,  5,  12, 9,  12, 5,  14, 6,  8,  13, 6,  5,  15, 13, 11, 11};
  const uint32_t KL[5] = {0x00000000u, 0x5A827999u, 0x6ED9EBA1u, 0x8F1BBCDCu, 0xA953FD4Eu};
  const uint32_t KR[5] = {0x50A28BE6u, 0x5C4DD124u, 0x6D703EF3u, 0x7A6D76E9u, 0x00000000u};
  uint32_t x[16];
#pragma unroll
  for (int i = 0; i < 8; i++) x[i] = m[i];
  x[8] = 0x80u;
#pragma unroll
  for (int i = 9; i < 16; i++) x[i] = 0;
  x[14] = 256u;
  const uint32_t h0 = 0x67452301u, h1 = 0xEFCDAB89u, h2 = 0x98BADCFEu, h3 = 0x10325476u, h4 = 0xC3D2E1F0u;
  uint32_t al = h0, bl = h1, cl = h2, dl = h3, el = h4;
  uint32_t ar = h0, br = h1, cr = h2, dr = h3, er = h4;
#pragma unroll
  for (int j = 0; j < 80; j++) {
    uint32_t t = rotl32(al + rmd_f(j, bl, cl, dl) + x[RL[j]] + KL[j / 16], SL[j]) + el;
    al = el; el = dl; dl = rotl32(cl, 10); cl = bl; bl = t;
    t = rotl32(ar + rmd_f(79 - j, br, cr, dr) + x[RR[j]] + KR[j / 16], SR[j]) + er;
    ar = er; er = dr; dr = rotl32(cr, 10); cr = br; br = t;
  }
  out[0] = h1 + cl + dr;
  out[1] = h2 + dl + er;
  out[2] = h3 + el + ar;
  out[3] = h4 + al + br;
  out[4] = h0 + bl + cr;
}

// hash160(prefix || X) for prefix 0x02/0x03, X canonical.  out: 5 LE words = the 20 digest bytes.
// Message packing as KEYBUFFPREFIX (secp256k1/SECP256K1.cpp:1187-1203).
KH_HD void hash160_comp(const fe &x, uint32_t prefix, uint32_t out[5]) {
  uint32_t w[16];
  w[0] = (prefix << 24) | (x.d[7] >> 8);
#pragma unroll
  for (int i = 1; i < 8; i++) w[i] = (x.d[8 - i] << 24) | (x.d[7 - i] >> 8);
  w[8] = (x.d[0] << 24) | 0x00800000u;
#pragma unroll
  for (int i = 9; i < 15; i++) w[i] = 0;
  w[15] = 0x108u;
  uint32_t st[8];
  sha256_init(st);
  sha256_transform(st, w);
  uint32_t m[8];
#pragma unroll
  for (int i = 0; i < 8; i++) m[i] = bswap32(st[i]);
  ripemd160_32(m, out);
}

// hash160(02||X) and hash160(03||X) with the two SHA-256 compressions interleaved.
KH_HD void hash160_comp2(const fe &x, uint32_t out02[5], uint32_t out03[5]) {
  uint32_t wa[16], wb[16];
  wa[0] = (2u << 24) | (x.d[7] >> 8);
#pragma unroll
  for (int i = 1; i < 8; i++) wa[i] = (x.d[8 - i] << 24) | (x.d[7 - i] >> 8);
  wa[8] = (x.d[0] << 24) | 0x00800000u;
#pragma unroll
  for (int i = 9; i < 15; i++) wa[i] = 0;
  wa[15] = 0x108u;
#pragma unroll
  for (int i = 0; i < 16; i++) wb[i] = wa[i];
  wb[0] = (3u << 24) | (x.d[7] >> 8);
  uint32_t sa[8], sb[8];
  sha256_init(sa);
  sha256_init(sb);
  sha256_transform2(sa, wa, sb, wb);
  // the two RIPEMD-160s run one after the other: interleaving them (4 lines in flight) spills
  // and halves the rmd160 rate (measured: 7.7 vs 14.4 Gkeys/s)
  uint32_t m[8];
#pragma unroll
  for (int i = 0; i < 8; i++) m[i] = bswap32(sa[i]);
  ripemd160_32(m, out02);
#pragma unroll
  for (int i = 0; i < 8; i++) m[i] = bswap32(sb[i]);
  ripemd160_32(m, out03);
}

// hash160(04 || X || Y) (KEYBUFFUNCOMP, secp256k1/SECP256K1.cpp:992-1024): two SHA-256 blocks.
KH_HD void hash160_uncomp(const fe &x, const fe &y, uint32_t out[5]) {
  uint32_t w[16];
  w[0] = 0x04000000u | (x.d[7] >> 8);
#pragma unroll
  for (int i = 1; i < 8; i++) w[i] = (x.d[8 - i] << 24) | (x.d[7 - i] >> 8);
  w[8] = (x.d[0] << 24) | (y.d[7] >> 8);
#pragma unroll
  for (int i = 1; i < 8; i++) w[8 + i] = (y.d[8 - i] << 24) | (y.d[7 - i] >> 8);
  uint32_t st[8];
  sha256_init(st);
  sha256_transform(st, w);
  w[0] = (y.d[0] << 24) | 0x00800000u;
#pragma unroll
  for (int i = 1; i < 15; i++) w[i] = 0;
  w[15] = 0x208u;
  sha256_transform(st, w);
  uint32_t m[8];
#pragma unroll
  for (int i = 0; i < 8; i++) m[i] = bswap32(st[i]);
  ripemd160_32(m, out);
}

// ------------------------------------------------------------------------------------------
// XXH64 for the two input shapes on the hot path (xxhash/xxhash.h:2468-2529).
// ------------------------------------------------------------------------------------------
#define KH_XP1 0x9E3779B185EBCA87ULL
#define KH_XP2 0xC2B2AE3D27D4EB4FULL
#define KH_XP3 0x165667B19E3779F9ULL
#define KH_XP4 0x85EBCA77C2B2AE63ULL
#define KH_XP5 0x27D4EB2F165667C5ULL
#define KH_BLOOM_SEED 0x59f2815b16f81798ULL

KH_HD uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
KH_HD uint64_t xxh_round(uint64_t acc, uint64_t in) {
  acc += in * KH_XP2;
  acc = rotl64(acc, 31);
  return acc * KH_XP1;
}
KH_HD uint64_t xxh_merge(uint64_t acc, uint64_t v) {
  v = xxh_round(0, v);
  acc ^= v;
  return acc * KH_XP1 + KH_XP4;
}
KH_HD uint64_t xxh_avalanche(uint64_t h) {
  h ^= h >> 33;
  h *= KH_XP2;
  h ^= h >> 29;
  h *= KH_XP3;
  h ^= h >> 32;
  return h;
}
// 32-byte input as 4 little-endian u64 lanes
KH_HD uint64_t xxh64_32(const uint64_t in[4], uint64_t seed) {
  uint64_t v1 = seed + KH_XP1 + KH_XP2, v2 = seed + KH_XP2, v3 = seed, v4 = seed - KH_XP1;
  v1 = xxh_round(v1, in[0]);
  v2 = xxh_round(v2, in[1]);
  v3 = xxh_round(v3, in[2]);
  v4 = xxh_round(v4, in[3]);
  uint64_t h = rotl64(v1, 1) + rotl64(v2, 7) + rotl64(v3, 12) + rotl64(v4, 18);
  h = xxh_merge(h, v1);
  h = xxh_merge(h, v2);
  h = xxh_merge(h, v3);
  h = xxh_merge(h, v4);
  h += 32;
  return xxh_avalanche(h);
}
// 20-byte input as 5 little-endian u32 words
KH_HD uint64_t xxh64_20(const uint32_t w[5], uint64_t seed) {
  uint64_t h = seed + KH_XP5 + 20;
  uint64_t k0 = (uint64_t)w[0] | ((uint64_t)w[1] << 32);
  uint64_t k1 = (uint64_t)w[2] | ((uint64_t)w[3] << 32);
  h ^= xxh_round(0, k0);
  h = rotl64(h, 27) * KH_XP1 + KH_XP4;
  h ^= xxh_round(0, k1);
  h = rotl64(h, 27) * KH_XP1 + KH_XP4;
  h ^= (uint64_t)w[4] * KH_XP1;
  h = rotl64(h, 23) * KH_XP2 + KH_XP3;
  return xxh_avalanche(h);
}

// word i of w[5] without dynamic register indexing
KH_HD uint32_t w5_at(const uint32_t w[5], uint32_t i) {
  uint32_t v = w[0];
  v = i == 1 ? w[1] : v;
  v = i == 2 ? w[2] : v;
  v = i == 3 ? w[3] : v;
  v = i == 4 ? w[4] : v;
  return v;
}
// XXH64 of the first len <= 20 bytes of 5 LE u32 words (XXH64 short-input path,
// xxhash/xxhash.h:2468-2529): the vanity bloom hashes a hash160 prefix (keyhunt.cpp:6680)
KH_HD uint64_t xxh64_prefix(const uint32_t w[5], uint32_t len, uint64_t seed) {
  uint64_t h = seed + KH_XP5 + len;
  uint32_t p = 0;
  for (; p + 8 <= len; p += 8) {
    const uint64_t k = (uint64_t)w5_at(w, p / 4) | ((uint64_t)w5_at(w, p / 4 + 1) << 32);
    h ^= xxh_round(0, k);
    h = rotl64(h, 27) * KH_XP1 + KH_XP4;
  }
  if (p + 4 <= len) {
    h ^= (uint64_t)w5_at(w, p / 4) * KH_XP1;
    h = rotl64(h, 23) * KH_XP2 + KH_XP3;
    p += 4;
  }
  for (; p < len; p++) {
    const uint64_t b = (w5_at(w, p / 4) >> (8 * (p % 4))) & 0xFFu;
    h ^= b * KH_XP5;
    h = rotl64(h, 11) * KH_XP1;
  }
  return xxh_avalanche(h);
}

// ------------------------------------------------------------------------------------------
// Keccak-256 with the original 0x01 padding (sha3/sha3.c:229, KECCAK_256_Final) of the 64-byte
// X||Y: the Ethereum address is digest bytes 12..31 (generate_binaddress_eth, keyhunt.cpp:5663-5669).
// ------------------------------------------------------------------------------------------
KH_HD void keccak_f1600(uint64_t a[25]) {
  const uint64_t RC[24] = {0x0000000000000001ULL, 0x0000000000008082ULL, 0x800000000000808aULL, 0x8000000080008000ULL,
                           0x000000000000808bULL, 0x0000000080000001ULL, 0x8000000080008081ULL, 0x8000000000008009ULL,
                           0x000000000000008aULL, 0x0000000000000088ULL, 0x0000000080008009ULL, 0x000000008000000aULL,
                           0x000000008000808bULL, 0x800000000000008bULL, 0x8000000000008089ULL, 0x8000000000008003ULL,
                           0x8000000000008002ULL, 0x8000000000000080ULL, 0x000000000000800aULL, 0x800000008000000aULL,
                           0x8000000080008081ULL, 0x8000000000008080ULL, 0x0000000080000001ULL, 0x8000000080008008ULL};
  // rho rotation and pi destination of lane 1, 10, 7, ... (the standard walk of the 24 lanes)
  const int ROT[24] = {1, 3, 6, 10, 15, 21, 28, 36, 45, 55, 2, 14, 27, 41, 56, 8, 25, 43, 62, 18, 39, 61, 20, 44};
  const int PI[24] = {10, 7, 11, 17, 18, 3, 5, 16, 8, 21, 24, 4, 15, 23, 19, 13, 12, 2, 20, 14, 22, 9, 6, 1};
#pragma unroll 1
  for (int r = 0; r < 24; r++) {
    uint64_t c[5];
#pragma unroll
    for (int x = 0; x < 5; x++) c[x] = a[x] ^ a[x + 5] ^ a[x + 10] ^ a[x + 15] ^ a[x + 20];
#pragma unroll
    for (int x = 0; x < 5; x++) {
      const uint64_t d = c[(x + 4) % 5] ^ ((c[(x + 1) % 5] << 1) | (c[(x + 1) % 5] >> 63));
#pragma unroll
      for (int y = 0; y < 25; y += 5) a[y + x] ^= d;
    }
    uint64_t t = a[1];
#pragma unroll
    for (int i = 0; i < 24; i++) {
      const uint64_t u = a[PI[i]];
      a[PI[i]] = (t << ROT[i]) | (t >> (64 - ROT[i]));
      t = u;
    }
#pragma unroll
    for (int y = 0; y < 25; y += 5) {
      const uint64_t b0 = a[y], b1 = a[y + 1], b2 = a[y + 2], b3 = a[y + 3], b4 = a[y + 4];
      a[y] = b0 ^ (~b1 & b2);
      a[y + 1] = b1 ^ (~b2 & b3);
      a[y + 2] = b2 ^ (~b3 & b4);
      a[y + 3] = b3 ^ (~b4 & b0);
      a[y + 4] = b4 ^ (~b0 & b1);
    }
    a[0] ^= RC[r];
  }
}
// Ethereum address of (x, y) as 5 LE u32 words = its 20 bytes in order
KH_HD void eth_address(const fe &x, const fe &y, uint32_t out[5]) {
  uint64_t a[25];
#pragma unroll
  for (int i = 0; i < 25; i++) a[i] = 0;
#pragma unroll
  for (int k = 0; k < 4; k++) {  // the 32 big-endian bytes of X, then of Y, as LE u64 lanes
    a[k] = (uint64_t)bswap32(x.d[7 - 2 * k]) | ((uint64_t)bswap32(x.d[6 - 2 * k]) << 32);
    a[4 + k] = (uint64_t)bswap32(y.d[7 - 2 * k]) | ((uint64_t)bswap32(y.d[6 - 2 * k]) << 32);
  }
  a[8] = 0x01ULL;                  // padding: 0x01 after the 64 message bytes ...
  a[16] = 0x8000000000000000ULL;   // ... and 0x80 in the last byte of the 136-byte rate
  keccak_f1600(a);
  out[0] = (uint32_t)(a[1] >> 32);
  out[1] = (uint32_t)a[2];
  out[2] = (uint32_t)(a[2] >> 32);
  out[3] = (uint32_t)a[3];
  out[4] = (uint32_t)(a[3] >> 32);
}

// ------------------------------------------------------------------------------------------
// libbloom2 geometry.  bit index x_i = (a + b*i) mod bits (u64 wrap-around, bloom.cpp:201),
// computed as h_i = h_{i-1} + b and an exact Barrett reduction by the per-filter reciprocal
// recip = floor((2^64-1) / bits) (bits < 2^32 on every filter keyhunt builds).
// ------------------------------------------------------------------------------------------
struct bloom_desc {
  uint64_t bits;     // number of bits
  uint64_t bytes;    // bytes per filter (shard)
  uint64_t stride;   // bytes between consecutive shards in the device buffer (>= bytes)
  uint64_t recip;    // floor((2^64-1)/bits)
  uint32_t hashes;   // number of hash functions
  uint32_t pad;
};

KH_HD uint64_t mulhi64(uint64_t a, uint64_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __umul64hi(a, b);
#else
  return (uint64_t)(((unsigned __int128)a * b) >> 64);
#endif
}
KH_HD uint64_t mod_bits(uint64_t h, uint64_t bits, uint64_t recip) {
  uint64_t q = mulhi64(h, recip);
  uint64_t r = h - q * bits;
  if (r >= bits) r -= bits;
  if (r >= bits) r -= bits;
  return r;
}

}  // namespace kh
