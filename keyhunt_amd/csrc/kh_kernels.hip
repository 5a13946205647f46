// kh_kernels.hip -- CDNA4 (gfx950) kernels for keyhunt's hot path.
//
// One walk kernel serves every mode.  A LANE owns a contiguous run of points on an arithmetic
// progression P(t) = P0 + t*D (address family: D = stride*G, t = key offset; BSGS giant steps:
// D = -2M*G, t = giant index; BSGS baby build: D = G, t = baby index).  Per GROUP the lane sits on
// a centre C and emits the 2H points C + o*D, o in [-H, H-1]: C itself, C +- T[i] (T[i] = (i+1)*D,
// i < H-1) and C - T[H-1]; then C += T[H] (= 2H*D).  The H+1 differences T[i].x - C.x are inverted
// together with one Fermat inversion (Montgomery trick, secp256k1/IntGroup.cpp:36-58) whose prefix
// products live in a per-lane HBM scratch pad ([i][lane][32 B], coalesced 2 KB per wave-access).
// This is the reference's group geometry (keyhunt.cpp:3349-3461, 4644-4716, 5318-5393) with the
// group's delta table T read through the scalar cache: i is wave-uniform, so every lane of a wave
// reads the same T[i] (s_load into SGPRs, no VGPRs and no LDS bank traffic for the table).
//
// Why per-lane batching rather than a cross-lane product tree: on a SIMD machine an inversion
// executed by a wave costs the same whether it serves 1 lane's batch or 64 lanes' batches, so a
// lane's share of inversion work is I / (elements per lane per inversion) either way; a wave-wide
// prefix/suffix tree only adds 12+ multiplications per lane.  The lever is elements per lane per
// inversion (H = 512 here: 0.26 field-mul-equivalents per point), which needs the HBM pad.
//
// Probe modes (template MODE):
//   KM_H160C / KM_H160U / KM_H160B  hash160 of 02/03||X, 04||X||Y or both -> 20-byte target bloom
//                                    (thread_process, keyhunt.cpp:3475-3830)
//   KM_XPOINT                        X[0..20) -> target bloom (keyhunt.cpp:3801-3824)
//   KM_ETH                           Keccak-256(X||Y)[12..32) -> target bloom (-c eth, 3524-3760)
//   KM_BSGS                          32-byte X -> bloom_bP[X[0]] (keyhunt.cpp:4819-4822)
//   KM_BUILD                         baby X -> bloom layers 1/2/3 + bP rows (keyhunt.cpp:5394-5443)
//   KM_BSGSB / KM_BUILDB             same with the BLOCKED layer-1 layout (kh_kernels.h): an item's
//                                    16 bits lie in one 16-byte block, so a probe is one 16-B load
//                                    and a 4-word mask test; layers 2/3 keep the reference layout
//   KM_DUMP                          write X (and Y) -- parity tests only
#include <hip/hip_runtime.h>
#include "kh_math.h"
#include "kh_kernels.h"

using namespace kh;

namespace {

__device__ __forceinline__ void load_fe(fe &r, const uint32_t *__restrict__ p) {
#pragma unroll
  for (int i = 0; i < 8; i++) r.d[i] = p[i];
}
// Read-only tables indexed wave-uniformly (the walk's delta table) are accessed through the
// constant address space so that uniform reads become s_load_dwordx8 into SGPRs.
typedef const __attribute__((address_space(4))) uint32_t *kconst_ptr;
__device__ __forceinline__ void load_fe_k(fe &r, kconst_ptr p) {
#pragma unroll
  for (int i = 0; i < 8; i++) r.d[i] = p[i];
}
// SoA centre arrays: word w of lane g at base[w * L + g]
__device__ __forceinline__ void load_soa(fe &r, const uint32_t *__restrict__ base, uint32_t L, uint32_t g) {
#pragma unroll
  for (int i = 0; i < 8; i++) r.d[i] = base[(size_t)i * L + g];
}
__device__ __forceinline__ void store_soa(uint32_t *__restrict__ base, uint32_t L, uint32_t g, const fe &r) {
#pragma unroll
  for (int i = 0; i < 8; i++) base[(size_t)i * L + g] = r.d[i];
}
// Pad entry `slot` = row * L + g (lane g) as two 16-B halves.  KH_PAD_PLANES: the halves of a row
// live in two planes of L entries each, so one 16-B access of a wave covers 1 KB contiguously
// (16 lines) instead of 2 KB with 16-B holes (32 lines, each touched again by the other half)
__device__ __forceinline__ size_t pad_idx(size_t slot, uint32_t g, size_t L, int h) {
  if constexpr (KH_PAD_PLANES) return 2 * slot - g + (h ? L : 0);
  (void)g;
  (void)L;
  return 2 * slot + h;
}
typedef uint32_t pad4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void scr_store(uint4 *__restrict__ scr, size_t slot, const fe &a, uint32_t g, size_t L) {
  if constexpr (KH_PAD_NT & 1) {
    pad4 *p = reinterpret_cast<pad4 *>(scr);
    __builtin_nontemporal_store(pad4{a.d[0], a.d[1], a.d[2], a.d[3]}, p + pad_idx(slot, g, L, 0));
    __builtin_nontemporal_store(pad4{a.d[4], a.d[5], a.d[6], a.d[7]}, p + pad_idx(slot, g, L, 1));
    return;
  }
  scr[pad_idx(slot, g, L, 0)] = make_uint4(a.d[0], a.d[1], a.d[2], a.d[3]);
  scr[pad_idx(slot, g, L, 1)] = make_uint4(a.d[4], a.d[5], a.d[6], a.d[7]);
}
// a pad entry as its two loaded 16-B halves (kept as loaded across a loop edge, see k_walk)
__device__ __forceinline__ void scr_load_raw(pad4 &u, pad4 &v, const uint4 *__restrict__ scr, size_t slot, uint32_t g,
                                             size_t L) {
  const pad4 *p = reinterpret_cast<const pad4 *>(scr);
  if constexpr (KH_PAD_NT & 2) {
    u = __builtin_nontemporal_load(p + pad_idx(slot, g, L, 0));
    v = __builtin_nontemporal_load(p + pad_idx(slot, g, L, 1));
  } else {
    u = p[pad_idx(slot, g, L, 0)];
    v = p[pad_idx(slot, g, L, 1)];
  }
}
__device__ __forceinline__ void pad_unpack(fe &a, const pad4 &u, const pad4 &v) {
  a.d[0] = u.x; a.d[1] = u.y; a.d[2] = u.z; a.d[3] = u.w;
  a.d[4] = v.x; a.d[5] = v.y; a.d[6] = v.z; a.d[7] = v.w;
}
__device__ __forceinline__ void scr_load(fe &a, const uint4 *__restrict__ scr, size_t slot, uint32_t g, size_t L) {
  pad4 u, v;
  scr_load_raw(u, v, scr, slot, g, L);
  pad_unpack(a, u, v);
}

// bloom_check (bloom/bloom.cpp:189-212) on one filter at `bf`
__device__ __forceinline__ bool bloom_probe(const uint8_t *__restrict__ bf, const bloom_desc &bd, uint64_t a,
                                            uint64_t b) {
  uint64_t h = a;
  for (uint32_t i = 0; i < bd.hashes; i++) {
    uint64_t x = mod_bits(h, bd.bits, bd.recip);
    if (!((bf[x >> 3] >> (x & 7)) & 1)) return false;
    h += b;
  }
  return true;
}
// Same result, but the second hash b = XXH64(buf, a) is only computed once bit 0 (which depends on
// a alone) is set: a negative probe usually stops there.
template <typename HashB>
__device__ __forceinline__ bool bloom_probe_lazy(const uint8_t *__restrict__ bf, const bloom_desc &bd, uint64_t a,
                                                 HashB hash_b) {
  uint64_t x = mod_bits(a, bd.bits, bd.recip);
  if (!((bf[x >> 3] >> (x & 7)) & 1)) return false;
  uint64_t b = hash_b(a);
  uint64_t h = a + b;
  for (uint32_t i = 1; i < bd.hashes; i++) {
    x = mod_bits(h, bd.bits, bd.recip);
    if (!((bf[x >> 3] >> (x & 7)) & 1)) return false;
    h += b;
  }
  return true;
}
// bloom_add (bloom/bloom.cpp:122-146, add=1): set every bit with a 32-bit atomic OR
__device__ __forceinline__ void bloom_insert(uint8_t *__restrict__ bf_base, uint64_t shard_off,
                                             const bloom_desc &bd, uint64_t a, uint64_t b) {
  uint64_t h = a;
  uint32_t *w = reinterpret_cast<uint32_t *>(bf_base);
  for (uint32_t i = 0; i < bd.hashes; i++) {
    uint64_t x = mod_bits(h, bd.bits, bd.recip);
    uint64_t byte = shard_off + (x >> 3);
    atomicOr(&w[byte >> 2], 1u << ((uint32_t)((byte & 3) * 8) + (uint32_t)(x & 7)));
    h += b;
  }
}


// Blocked layer-1 (split-block) geometry, kh_kernels.h: desc.bits = blocks per shard.  The item
// is an x-coordinate, already uniform, so the block and the bit positions are taken from its words
// directly (no XXH64): block = (X[8..12) * blocks) >> 32 (limb 5); positions from X[12..20) (limbs
// 4, 3) by kh_blk_masks (kh_kernels.h).
__device__ __forceinline__ uint32_t blk_index(uint32_t w5, const bloom_desc &bd) {
  return (uint32_t)(((uint64_t)w5 * bd.bits) >> 32);
}
// masks of the four block words from s0 = limb 4, s1 = limb 3, s2 = limb 2 (kh_kernels.h
// kh_blk_masks: packed 16-bit shifts, or `1u << (s >> k)` per 5-bit field with KH_PK_MASKS=0)
__device__ __forceinline__ void blk_masks(uint32_t s0, uint32_t s1, uint32_t s2, uint32_t m[4]) {
  kh_blk_masks(s0, s1, s2, m);
}
__device__ __forceinline__ bool blk_match(const uint4 &v, uint32_t s0, uint32_t s1, uint32_t s2) {
  uint32_t m[4];
#ifdef KH_TIMING_CHEAP_MASKS
  // timing-only build: the probe without mask arithmetic (hits are wrong); prices the masks
  m[0] = s0 | 0x80000001u; m[1] = s1 | 0x80000001u; m[2] = s2 | 0x80000001u; m[3] = (s0 ^ s1) | 0x80000001u;
#else
  blk_masks(s0, s1, s2, m);
#endif
  // a miss is a mask bit its block word lacks: OR the four words' misses and compare once
  return ((m[0] & ~v.x) | (m[1] & ~v.y) | (m[2] & ~v.z) | (m[3] & ~v.w)) == 0;
}
__device__ __forceinline__ void blk_insert(uint8_t *__restrict__ bf_shard, const bloom_desc &bd, const fe &x) {
  uint32_t m[4];
  blk_masks(x.d[4], x.d[3], x.d[2], m);
  uint32_t *w = reinterpret_cast<uint32_t *>(bf_shard + (size_t)blk_index(x.d[5], bd) * 16);
#pragma unroll
  for (int k = 0; k < 4; k++) atomicOr(&w[k], m[k]);
}

__device__ __forceinline__ void record_hit(const walk_args &A, uint64_t idx, uint32_t kind) {
  KH_RARE_MARK();
  uint32_t slot = atomicAdd(A.hit_count, 1u);
  if (slot < A.hit_cap) {
    A.hits[slot].idx = idx;
    A.hits[slot].kind = kind;
    A.hits[slot].aux = 0;
  }
}

// X as the 4 little-endian u64 words of its 32 big-endian bytes (Int::Get32Bytes order)
__device__ __forceinline__ void x_bytes_u64(const fe &x, uint64_t in[4]) {
#pragma unroll
  for (int k = 0; k < 4; k++)
    in[k] = (uint64_t)bswap32(x.d[7 - 2 * k]) | ((uint64_t)bswap32(x.d[6 - 2 * k]) << 32);
}

// Exact 20-byte targets (hash160, X[0..20), eth address) are uniform, so they go to a split-block
// filter keyed on their own words, like the blocked BSGS layer 1: with w = the little-endian u32s
// of the 20 bytes, the 16-byte block is (w0 * blocks) >> 32 and the bit positions come from w1, w2
// (kh_blk_masks).  One 16-B load, no XXH64.  Every filter hit is still confirmed by the
// host's exact table search (searchbinary), so the reported hits are the reference's.
__device__ __forceinline__ bool tblk_probe(const walk_args &A, const uint32_t w[5]) {
  const uint32_t blk = (uint32_t)(((uint64_t)w[0] * A.tblocks) >> 32);
  return blk_match(A.tblk[blk], w[1], w[2], w[3]);
}

// one 20-byte hash into the target bloom: the whole hash (address/rmd160), or its first
// A.probe_len bytes (vanity prefixes, vanityrmdmatch keyhunt.cpp:6677-6703)
__device__ __forceinline__ bool probe_h160(const walk_args &A, const uint32_t h[5]) {
  if (A.tblk) return tblk_probe(A, h);
  if (A.probe_len == 20) {
    const uint64_t a = xxh64_20(h, KH_BLOOM_SEED);
    return bloom_probe_lazy(A.bloom, A.bd, a, [&](uint64_t s) { return xxh64_20(h, s); });
  }
  const uint64_t a = xxh64_prefix(h, A.probe_len, KH_BLOOM_SEED);
  return bloom_probe_lazy(A.bloom, A.bd, a, [&](uint64_t s) { return xxh64_prefix(h, A.probe_len, s); });
}

// hash160(02||X) and hash160(03||X) of one x-coordinate into the target bloom; kinds 0/1 | tag
__device__ __forceinline__ void probe_comp(const walk_args &A, const fe &x, uint64_t idx, uint32_t tag) {
#if KH_HASH_PAIR
  uint32_t hh[2][5];
  hash160_comp2(x, hh[0], hh[1]);
#pragma unroll 1
  for (uint32_t k = 0; k < 2; k++) {
    uint32_t h[5];
#pragma unroll
    for (int q = 0; q < 5; q++) h[q] = k ? hh[1][q] : hh[0][q];
    if (probe_h160(A, h)) record_hit(A, idx, k | tag);
  }
#else
#pragma unroll 1
  for (uint32_t pfx = 2; pfx <= 3; pfx++) {
    uint32_t h[5];
    hash160_comp(x, pfx, h);
    if (probe_h160(A, h)) record_hit(A, idx, (pfx - 2) | tag);
  }
#endif
}
// hash160(04||X||Y); kind 2 | tag
__device__ __forceinline__ void probe_uncomp(const walk_args &A, const fe &x, const fe &y, uint64_t idx, uint32_t tag) {
  uint32_t h[5];
  hash160_uncomp(x, y, h);
  if (probe_h160(A, h)) record_hit(A, idx, 2 | tag);
}
// X[0..20); kind 3 | tag
__device__ __forceinline__ void probe_xpoint(const walk_args &A, const fe &x, uint64_t idx, uint32_t tag) {
  uint32_t w[5];
#pragma unroll
  for (int j = 0; j < 5; j++) w[j] = bswap32(x.d[7 - j]);
  if (A.tblk) {
    if (tblk_probe(A, w)) record_hit(A, idx, 3 | tag);
    return;
  }
  uint64_t a = xxh64_20(w, KH_BLOOM_SEED);
  if (bloom_probe_lazy(A.bloom, A.bd, a, [&](uint64_t s) { return xxh64_20(w, s); })) record_hit(A, idx, 3 | tag);
}
// beta and beta^2 (cube roots of unity mod p): lambda*(x, y) = (beta*x, y) (-e, keyhunt.cpp:926-930)
__device__ __forceinline__ void endo_beta(fe &b, int e) {
  const uint32_t B1[8] = {0x719501eeu, 0xc1396c28u, 0x12f58995u, 0x9cf04975u,
                          0xac3434e9u, 0x6e64479eu, 0x657c0710u, 0x7ae96a2bu};
  const uint32_t B2[8] = {0x8e6afa40u, 0x3ec693d6u, 0xed0a766au, 0x630fb68au,
                          0x53cbcb16u, 0x919bb861u, 0x9a83f8efu, 0x851695d4u};
#pragma unroll
  for (int i = 0; i < 8; i++) b.d[i] = e == 1 ? B1[i] : B2[i];
}

// Ethereum address (Keccak-256 of X||Y, bytes 12..31); kind 5 | tag (keyhunt.cpp:3524-3548, 3703-3760)
__device__ __forceinline__ void probe_eth(const walk_args &A, const fe &x, const fe &y, uint64_t idx,
                                          uint32_t tag = 0) {
  uint32_t w[5];
  eth_address(x, y, w);
  if (A.tblk) {
    if (tblk_probe(A, w)) record_hit(A, idx, 5 | tag);
    return;
  }
  uint64_t a = xxh64_20(w, KH_BLOOM_SEED);
  if (bloom_probe_lazy(A.bloom, A.bd, a, [&](uint64_t s) { return xxh64_20(w, s); })) record_hit(A, idx, 5 | tag);
}

template <int MODE>
__device__ __forceinline__ void probe_point(const walk_args &A, const fe &x, const fe &y, uint64_t idx) {
  if (idx >= A.n_points) return;
  if constexpr (MODE == KM_H160CB) {
    // hash160(02||X), hash160(03||X) against the blocked target filter only: the filter reads digest
    // words 0..2, so the RIPEMD-160 steps that feed only words 3..4 are dead code here
    uint32_t hh[2][5];
    hash160_comp2(x, hh[0], hh[1]);
#pragma unroll 1
    for (uint32_t k = 0; k < 2; k++) {
      uint32_t h[5];
#pragma unroll
      for (int q = 0; q < 5; q++) h[q] = k ? hh[1][q] : hh[0][q];
      if (tblk_probe(A, h)) record_hit(A, idx, k);
    }
    return;
  }
  if constexpr (MODE == KM_ETH) {
    probe_eth(A, x, y, idx);
    return;
  }
  if constexpr (MODE == (KM_ETH | KM_ENDO)) {
    // -e -c eth (keyhunt.cpp:3524-3536): the reference's six images per point are eth(P), eth(-P),
    // eth(beta P), eth(-beta P), eth(beta P) again (it passes endomorphism_beta where beta2 is
    // meant, 3533) and eth(-beta^2 P).  The repeated image is probed once; the host reports its
    // second hit (kind ETH | ENDO2 without NEG) with the key the reference derives for it.
    fe ny;
    fe_neg(ny, y);
    probe_eth(A, x, y, idx, 0);
    probe_eth(A, x, ny, idx, KH_DKIND_NEG);
    fe b, xe;
    endo_beta(b, 1);
    fe_mul(xe, x, b);
    probe_eth(A, xe, y, idx, 1u << KH_DKIND_ENDO_SHIFT);
    probe_eth(A, xe, ny, idx, (1u << KH_DKIND_ENDO_SHIFT) | KH_DKIND_NEG);
    endo_beta(b, 2);
    fe_mul(xe, x, b);
    probe_eth(A, xe, ny, idx, (2u << KH_DKIND_ENDO_SHIFT) | KH_DKIND_NEG);
    return;
  }
  constexpr int BASE = MODE & 15;
  constexpr bool ENDO = (MODE & KM_ENDO) != 0;
  if constexpr (BASE == KM_H160C || BASE == KM_H160B || BASE == KM_H160U || BASE == KM_XPOINT) {
    // images e = 0 (X), then with -e: 1 (beta*X) and 2 (beta^2*X); per point the reference
    // checks every compressed variant before the uncompressed ones (keyhunt.cpp:3476-3700)
    if constexpr (BASE == KM_H160C || BASE == KM_H160B) {
      probe_comp(A, x, idx, 0);
      if constexpr (ENDO) {
#pragma unroll 1
        for (int e = 1; e <= 2; e++) {
          fe b, xe;
          endo_beta(b, e);
          fe_mul(xe, x, b);
          probe_comp(A, xe, idx, (uint32_t)e << KH_DKIND_ENDO_SHIFT);
        }
      }
    }
    if constexpr (BASE == KM_H160U || BASE == KM_H160B) {
      probe_uncomp(A, x, y, idx, 0);
      if constexpr (ENDO) {  // (X, -Y) and both images with +-Y
        fe ny;
        fe_neg(ny, y);
        probe_uncomp(A, x, ny, idx, KH_DKIND_NEG);
#pragma unroll 1
        for (int e = 1; e <= 2; e++) {
          fe b, xe;
          endo_beta(b, e);
          fe_mul(xe, x, b);
          probe_uncomp(A, xe, y, idx, (uint32_t)e << KH_DKIND_ENDO_SHIFT);
          probe_uncomp(A, xe, ny, idx, ((uint32_t)e << KH_DKIND_ENDO_SHIFT) | KH_DKIND_NEG);
        }
      }
    }
    if constexpr (BASE == KM_XPOINT) {
      probe_xpoint(A, x, idx, 0);
      if constexpr (ENDO) {
#pragma unroll 1
        for (int e = 1; e <= 2; e++) {
          fe b, xe;
          endo_beta(b, e);
          fe_mul(xe, x, b);
          probe_xpoint(A, xe, idx, (uint32_t)e << KH_DKIND_ENDO_SHIFT);
        }
      }
    }
    return;
  }
  if constexpr (MODE == KM_BSGS) {
    uint64_t in[4];
    x_bytes_u64(x, in);
    uint64_t a = xxh64_32(in, KH_BLOOM_SEED);
    const uint8_t *bf = A.bloom + (size_t)(x.d[7] >> 24) * A.bd.stride;
    if (bloom_probe_lazy(bf, A.bd, a, [&](uint64_t s) { return xxh64_32(in, s); })) record_hit(A, idx, 4);
  }
  if constexpr (MODE == KM_BUILD || MODE == KM_BUILDB) {
    // baby index idx -> point (idx+1)G; layers by index (keyhunt.cpp:5394-5443)
    uint32_t shard = x.d[7] >> 24;
    if constexpr (MODE == KM_BUILDB) {
      blk_insert(A.bl1 + (size_t)shard * A.bd.stride, A.bd, x);
      if (idx >= A.m2) return;  // layers 2/3 hold only the first M2 / M3 babies
    }
    uint64_t in[4];
    x_bytes_u64(x, in);
    uint64_t a = xxh64_32(in, KH_BLOOM_SEED);
    uint64_t b = xxh64_32(in, a);
    if constexpr (MODE == KM_BUILD) bloom_insert(A.bl1, (uint64_t)shard * A.bd.stride, A.bd, a, b);
    if (idx < A.m2) bloom_insert(A.bl2, (uint64_t)shard * A.bd2.stride, A.bd2, a, b);
    if (idx < A.m3) {
      bloom_insert(A.bl3, (uint64_t)shard * A.bd3.stride, A.bd3, a, b);
      // bsgs_xvalue {X[16..22), index}: sort key = those 6 bytes big-endian
      A.rows_key[idx] = ((uint64_t)x.d[3] << 16) | (x.d[2] >> 16);
      A.rows_val[idx] = idx;
    }
  }
  if constexpr (MODE == KM_DUMP) {
    uint32_t *o = A.dump_x + (size_t)idx * 8;
#pragma unroll
    for (int i = 0; i < 8; i++) o[i] = x.d[i];
    if (A.dump_y) {
      uint32_t *q = A.dump_y + (size_t)idx * 8;
#pragma unroll
      for (int i = 0; i < 8; i++) q[i] = y.d[i];
    }
  }
}

// Blocked layer-1 probes: each point costs one 16-byte load (its split block) and the word-mask
// test.  The walk issues a pair's loads one step later and tests them after that step's field
// math (see k_walk).
typedef uint32_t v4u32 __attribute__((ext_vector_type(4)));
// 16-byte load with the nontemporal hint: each block is read once, at a random address
__device__ __forceinline__ uint4 ld_nt16(const uint4 *p) {
  v4u32 v = __builtin_nontemporal_load(reinterpret_cast<const v4u32 *>(p));
  return make_uint4(v.x, v.y, v.z, v.w);
}
// {block index within the shard, limbs 4, 3, and the shard byte in the top 8 bits of the last word}
// of one point (KH_PK_MASKS=0: limb 2, whose bits 0..19 are all its masks read).  The record
// addresses any layer whose shards are < 4 GB (the whole layer < 1 TB; a global 16-B block index in
// 32 bits would stop at 64 GB).
__device__ __forceinline__ uint4 blk_record(const walk_args &A, const fe &x) {
  // the packed-shift masks read limbs 4 and 3 only: the shard byte rides as limb 7 itself
  if constexpr (KH_PK_MASKS) return make_uint4(blk_index(x.d[5], A.bd), x.d[4], x.d[3], x.d[7]);
  return make_uint4(blk_index(x.d[5], A.bd), x.d[4], x.d[3], (x.d[2] & 0x000FFFFFu) | (x.d[7] & 0xFF000000u));
}
__device__ __forceinline__ uint4 blk_load(const walk_args &A, const uint4 &r) {
#ifdef KH_TIMING_NO_PROBE_LOADS
  // timing-only build: no HBM reads (outputs are wrong); isolates the probe's compute
  return make_uint4(r.x, r.x * 3u, r.x * 5u, r.x * 7u);
#elif defined(KH_TIMING_PROBE_REGION_LOG2)
  // timing-only build: every probe reads a block of the layer's first 2^LOG2 blocks, a region
  // that stays on die (Infinity Cache / L2) -- the loads without their HBM traffic (outputs wrong)
  return ld_nt16(reinterpret_cast<const uint4 *>(A.bloom) + (r.x & ((1u << KH_TIMING_PROBE_REGION_LOG2) - 1u)));
#elif defined(KH_PROBE_PLAIN_LOAD)
  const uint8_t *shard = A.bloom + (uint64_t)(r.w >> 24) * A.bstride32;
  return reinterpret_cast<const uint4 *>(shard)[r.x];
#else
  const uint8_t *shard = A.bloom + (uint64_t)(r.w >> 24) * A.bstride32;
  return ld_nt16(reinterpret_cast<const uint4 *>(shard) + r.x);
#endif
}
__device__ __forceinline__ bool blk_match_rec(const uint4 &v, const uint4 &r) { return blk_match(v, r.y, r.z, r.w); }
// {target-filter block, w1, w2, w3} of X[0..20), w_j = bswap32(limb 7 - j) as in probe_xpoint /
// tblk_probe: the -m xpoint probe record that crosses the loop edge in k_walk<KM_XPOINTB>
__device__ __forceinline__ uint4 tblk_record(const walk_args &A, const fe &x) {
  return make_uint4((uint32_t)(((uint64_t)bswap32(x.d[7]) * A.tblocks) >> 32), bswap32(x.d[6]), bswap32(x.d[5]),
                    KH_PK_MASKS ? 0u : bswap32(x.d[4]));  // w3 feeds only the 5-bit-field masks
}
// one blocked probe, in place (the group centre)
__device__ __forceinline__ void blk_probe(const walk_args &A, const fe &x, uint64_t idx) {
  const uint4 r = blk_record(A, x);
  if (idx < A.n_points && blk_match_rec(blk_load(A, r), r)) record_hit(A, idx, 4);
}

// Reference-layout layer-1 probes of two giant-step points in lockstep (keyhunt.cpp:4819-4822
// for each): both chains issue their byte loads before either result is consumed, so every lane
// keeps two independent HBM reads in flight.  Same result as two bloom_probe_lazy calls.
__device__ __forceinline__ void probe_pair_bsgs(const walk_args &A, const fe &x1, uint64_t idx1, const fe &x2,
                                                uint64_t idx2, bool valid2) {
  uint64_t in1[4], in2[4];
  x_bytes_u64(x1, in1);
  x_bytes_u64(x2, in2);
  bool alive1 = idx1 < A.n_points;
  bool alive2 = valid2 && idx2 < A.n_points;
  uint64_t h1 = xxh64_32(in1, KH_BLOOM_SEED), h2 = xxh64_32(in2, KH_BLOOM_SEED);
  const uint64_t a1 = h1, a2 = h2;
  uint64_t b1 = 0, b2 = 0;
  const uint8_t *bf1 = A.bloom + (size_t)(x1.d[7] >> 24) * A.bd.stride;
  const uint8_t *bf2 = A.bloom + (size_t)(x2.d[7] >> 24) * A.bd.stride;
  for (uint32_t i = 0; i < A.bd.hashes && (alive1 || alive2); i++) {
    uint64_t p1 = mod_bits(h1, A.bd.bits, A.bd.recip);
    uint64_t p2 = mod_bits(h2, A.bd.bits, A.bd.recip);
#ifdef KH_TIMING_NO_PROBE_LOADS
    // timing-only build: no HBM reads (outputs are wrong); isolates the compute cost
    uint32_t v1 = (uint32_t)(p1 * 0x9E3779B1u) & (0xFFu >> (i + 1));
    uint32_t v2 = (uint32_t)(p2 * 0x9E3779B1u) & (0xFFu >> (i + 1));
#else
    uint32_t v1 = alive1 ? bf1[p1 >> 3] : 0u;
    uint32_t v2 = alive2 ? bf2[p2 >> 3] : 0u;
#endif
    if (alive1) {
      if (!((v1 >> (p1 & 7)) & 1)) {
        alive1 = false;
      } else {
        if (i == 0) b1 = xxh64_32(in1, a1);
        h1 += b1;
      }
    }
    if (alive2) {
      if (!((v2 >> (p2 & 7)) & 1)) {
        alive2 = false;
      } else {
        if (i == 0) b2 = xxh64_32(in2, a2);
        h2 += b2;
      }
    }
  }
  if (alive1) record_hit(A, idx1, 4);
  if (alive2) record_hit(A, idx2, 4);
}

template <int MODE>
constexpr bool needs_y() {
  return (MODE & 15) == KM_H160U || (MODE & 15) == KM_H160B || MODE == KM_DUMP || (MODE & 15) == KM_ETH;
}

}  // namespace

// ------------------------------------------------------------------------------------------
// The walk.  Every lane runs A.groups groups of 2H points from its saved centre.
// ------------------------------------------------------------------------------------------
// Minimum waves per SIMD per mode (VGPR cap 512/(2*LB)... measured: the probe-light modes gain from
// 4 waves/SIMD even with a few spills; the hash160 modes prefer 3).
template <int MODE>
constexpr int walk_lb() {
  return MODE == KM_H160CB ? KH_WALK_LB_H160CB
         : ((MODE & 15) == KM_H160C || (MODE & 15) == KM_H160U || (MODE & 15) == KM_H160B || (MODE & 15) == KM_ETH)
             ? KH_WALK_LB_HASH
         : MODE == KM_DUMP                                          ? 2
                                                                    : KH_WALK_LB;
}

// KH_TAB_LDS: the giant walk's table in LDS, one 1024-thread workgroup per CU
template <int MODE, int H>
constexpr bool tab_lds() {
  return KH_TAB_LDS && MODE == KM_BSGSB && H == KH_WALK_HB;
}
template <int MODE, int H>
constexpr int walk_threads() {
  return tab_lds<MODE, H>() ? 1024 : 256;
}
template <int MODE, int H>
constexpr int walk_blocks_per_cu() {
  return tab_lds<MODE, H>() ? 1 : walk_lb<MODE>();  // either way walk_lb waves per SIMD
}
// a uniform 32-bit value copied into a VGPR (KH_TAB_VCOPY): later carry chains then read it there
__device__ __forceinline__ uint32_t to_vgpr(uint32_t s) {
  uint32_t v;
  asm("v_mov_b32 %0, %1" : "=v"(v) : "s"(s));
  return v;
}
__device__ __forceinline__ void fe_to_vgpr(fe &a) {
#pragma unroll
  for (int i = 0; i < 8; i++) a.d[i] = to_vgpr(a.d[i]);
}

template <int MODE, int H = KH_WALK_H>
__global__ void __launch_bounds__((walk_threads<MODE, H>()), (walk_blocks_per_cu<MODE, H>())) k_walk(walk_args A) {
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  constexpr bool LDS = tab_lds<MODE, H>();
  // table entry i: x in words [0,8), y in [8,16); LDS: uint4 [i*4 .. i*4+3]
  __shared__ uint4 tabl[LDS ? (H + 1) * 4 : 1];
  if constexpr (LDS) {
    const uint4 *src = reinterpret_cast<const uint4 *>(A.tab);
    for (uint32_t k = threadIdx.x; k < (uint32_t)(H + 1) * 4; k += blockDim.x) tabl[k] = src[k];
    __syncthreads();
  }
  if (g >= A.L) return;
  kconst_ptr T = (kconst_ptr)A.tab;  // (H+1) x {x[8], y[8]}, wave-uniform reads
  auto ld_tx = [&](fe &x, int i) {
    if constexpr (LDS) {
      const uint4 a = tabl[i * 4], b = tabl[i * 4 + 1];
      x.d[0] = a.x; x.d[1] = a.y; x.d[2] = a.z; x.d[3] = a.w;
      x.d[4] = b.x; x.d[5] = b.y; x.d[6] = b.z; x.d[7] = b.w;
    } else {
      load_fe_k(x, T + i * 16);
    }
  };
  auto ld_ty = [&](fe &y, int i) {
    if constexpr (LDS) {
      const uint4 a = tabl[i * 4 + 2], b = tabl[i * 4 + 3];
      y.d[0] = a.x; y.d[1] = a.y; y.d[2] = a.z; y.d[3] = a.w;
      y.d[4] = b.x; y.d[5] = b.y; y.d[6] = b.z; y.d[7] = b.w;
    } else {
      load_fe_k(y, T + i * 16 + 8);
    }
  };
  uint4 *__restrict__ scr = A.scratch;
  const size_t L = A.L;
  // the pad's row stride in lane entries; the row-skew and column-swizzle A/B knobs (KH_PAD_SKEW,
  // KH_PAD_SWZ: no effect on the rate, DESIGN.md §2 "Placement") cost ~1 VALU per point, so they are
  // compiled in only with -DKH_PAD_KNOBS=1
  const size_t LS = KH_PAD_KNOBS ? L + A.pad_skew : L;
  fe cx, cy;
  load_soa(cx, A.cx, A.L, g);
  load_soa(cy, A.cy, A.L, g);

  // BSGS and xpoint walks keep only the even prefix products in the pad and rebuild each odd one
  // with one multiplication in the backward pass: half the pad traffic for +1/2 multiplication per pair
  constexpr bool SPARSE = KH_SPARSE_ALL || (KH_SPARSE_BSGS && (MODE == KM_BSGSB || MODE == KM_BSGS)) ||
                          (KH_SPARSE_XPOINT && MODE == KM_XPOINTB);
#ifdef KH_TIMING_PAD_ROWS_LOG2
  // timing-only build: the pad's stores (KH_TIMING_PAD_FOLD & 1) and/or loads (& 2) folded onto its
  // first 2^LOG2 rows (8 MB each at 2^18 lanes), which stay on die -- those accesses without their
  // HBM traffic (outputs wrong)
  auto fold = [&](int m, int which) {
    const int r = SPARSE ? (m >> 1) : m;
    return (size_t)((KH_TIMING_PAD_FOLD & which) ? (r & ((1 << KH_TIMING_PAD_ROWS_LOG2) - 1)) : r) * LS + g;
  };
  auto slot_w = [&](int m) { return fold(m, 1); };
  auto slot = [&](int m) { return fold(m, 2); };
#else
  auto slot = [&](int m) {
    const uint32_t r = SPARSE ? (uint32_t)(m >> 1) : (uint32_t)m;
    return (size_t)r * LS + (KH_PAD_KNOBS && A.pad_swz ? (g ^ ((r & 7u) << 8)) : g);
  };
  auto slot_w = slot;
#endif
  // Deferred-probe walks (one 16-B split-block load per point, issued a step ahead): the BSGS giant
  // walk against the blocked layer 1 (kind 4) and -m xpoint against the blocked target filter (kind 3)
  constexpr bool DEFER = MODE == KM_BSGSB || MODE == KM_XPOINTB;
  constexpr uint32_t DKIND = MODE == KM_BSGSB ? 4u : 3u;
  auto drec = [&](const fe &x) -> uint4 {
    if constexpr (MODE == KM_BSGSB) return blk_record(A, x);
    else return tblk_record(A, x);
  };
  auto dload = [&](const uint4 &r) -> uint4 {
    if constexpr (MODE == KM_BSGSB) return blk_load(A, r);
    else return A.tblk[r.x];
  };
  for (uint32_t j = 0; j < A.groups; j++) {
    const uint64_t cidx = A.interleave ? ((A.group_base + j) * (uint64_t)A.L + g) * (2 * H) + H
                                       : (uint64_t)g * A.lane_stride + (uint64_t)(A.group_base + j) * (2 * H) + H;
    // forward: prefix products of dx_i = T[i].x - C.x
    fe acc;
    if constexpr (DEFER) {
      // two prefix products per trip: their two differences share one interleaved carry chain
#pragma unroll 1
      for (int i = 0; i < H; i += 2) {
        fe tx0, tx1, dx0, dx1;
        ld_tx(tx0, i);
        ld_tx(tx1, i + 1);
        fe_addsub2<true, true>(dx0, tx0, cx, dx1, tx1, cx);
        if (i == 0)
          acc = dx0;
        else
          fe_mul(acc, acc, dx0);
        scr_store(scr, slot_w(i), acc, g, L);
        fe_mul(acc, acc, dx1);
        if (!SPARSE) scr_store(scr, slot_w(i + 1), acc, g, L);
      }
    } else {
#pragma unroll 1
      for (int i = 0; i < H; i++) {
        fe tx, dx;
        ld_tx(tx, i);
        fe_sub(dx, tx, cx);
        if (i == 0)
          acc = dx;
        else
          fe_mul(acc, acc, dx);
        if (!SPARSE || (i & 1) == 0) scr_store(scr, slot_w(i), acc, g, L);
      }
    }
    fe t2x, t2y, dxn;
    ld_tx(t2x, H);
    ld_ty(t2y, H);
    fe_sub(dxn, t2x, cx);
    fe inv, inv_n;
    fe_mul(inv, acc, dxn);
    fe_inv(inv, inv);
    fe_mul(inv_n, inv, acc);  // 1 / dxn
    fe_mul(inv, inv, dxn);    // 1 / prefix[H-1]

    // the centre itself (offset 0)
    if constexpr (MODE == KM_BSGSB)
      blk_probe(A, cx, cidx);
    else if constexpr (MODE == KM_XPOINTB) {
      if (cidx < A.n_points) probe_xpoint(A, cx, cidx, 0);
    } else
      probe_point<MODE>(A, cx, cy, cidx);

    // backward: recover 1/dx_i and emit C - T[i] (offset -(i+1)) and C + T[i] (offset i+1).
    // Both points use the second operand (T.x, +-T.y): x3 = s^2 - C.x - T.x, y3 = s(T.x - x3) -+ T.y.
    // prefix[i-1] is fetched one iteration ahead so its HBM latency overlaps the previous pair
    uint4 pm = make_uint4(0u, 0u, 0u, 0u), pp = make_uint4(0u, 0u, 0u, 0u);  // DEFER: previous pair's probe records
    uint64_t poff = 0;
    // liveness of the previous pair's points as two lane masks (bools across the loop edge):
    // C - off lies inside the job iff off > lm, C + off iff off < hp (off = i + 1 <= H, so 32-bit
    // compares against per-group thresholds replace the 64-bit index compares)
    bool plm = false, plp = false;
    const uint64_t nm = cidx < A.n_points ? 0u : cidx - A.n_points;   // (no min(): no u64 overload)
    const uint64_t np = A.n_points > cidx ? A.n_points - cidx : 0u;
    const uint32_t lm = nm < (uint64_t)H ? (uint32_t)nm : (uint32_t)H;
    const uint32_t hp = np < (uint64_t)H ? (uint32_t)np : (uint32_t)H;
    // every point of this group, for every lane of the wave, lies inside the job (all but a job's
    // last groups): the per-pair liveness test then needs no 64-bit compares (xpoint +0.9 %; the BSGS
    // walk measured 0.2 % slower with it, so it keeps the compares)
    bool wfull = false;
#if defined(__HIP_DEVICE_COMPILE__)
    if constexpr (MODE == KM_XPOINTB && KH_FULL_GROUPS) wfull = !kh_any(cidx + H > A.n_points);
#endif
    // KEEP (sparse pad): the even prefix row last loaded, as its two loaded halves; otherwise `pre`
    constexpr bool KEEP = SPARSE && KH_SPARSE_KEEP;
    static_assert(!KEEP || (H % 2) == 0, "the sparse pad pairs odd and even steps");
    fe pre;
    pad4 ru, rv;
    if constexpr (KEEP)
      scr_load_raw(ru, rv, scr, slot(H - 2), g, L);
    else
      scr_load(pre, scr, slot(H - 2), g, L);
    // one backward step; `par` is the parity of i when the caller knows it (1 odd, 2 even, 0 unknown)
    auto step = [&](const int i, const int par) __attribute__((always_inline)) {
      fe tx, ty, di;
#if KH_PROBE_EARLY
      // the previous pair's block loads issued before this step's inverse too (they fly during it)
      uint4 vm, vp;
      if constexpr (DEFER) {
        vm = dload(pm);
        vp = dload(pp);
      }
#endif
      ld_tx(tx, i);
      ld_ty(ty, i);
      if constexpr (KH_TAB_VCOPY && MODE == KM_BSGSB && !LDS) {
        fe_to_vgpr(tx);  // used by dx and C.x + T.x
        fe_to_vgpr(ty);  // used by both dy
      }
      if (i > 0) {
        fe dx;
        if constexpr (KEEP) {
          // An odd step i needs the even prefix[i-1], the row R itself, and then loads the next row,
          // prefix[i-3], which serves the two steps after it; an even step rebuilds the odd
          // prefix[i-1] = R * dx[i-1].  R is written by its loads only, so they land in place and
          // fly for a whole step, and each row is read once.
          fe r;
          pad_unpack(r, ru, rv);
          if (par == 1 || (par == 0 && (i & 1))) {
            fe_mul(di, inv, r);
            if (i > 1) scr_load_raw(ru, rv, scr, slot(i - 3), g, L);
          } else {
            fe tpx, d1, p;
            ld_tx(tpx, i - 1);
            fe_sub(d1, tpx, cx);
            fe_mul(p, r, d1);
            fe_mul(di, inv, p);
          }
        } else {
          if (SPARSE && ((i - 1) & 1)) {  // prefix[i-1] = prefix[i-2] * dx[i-1] (pre holds prefix[i-2])
            fe tpx, d1;
            ld_tx(tpx, i - 1);
            fe_sub(d1, tpx, cx);
            fe_mul(pre, pre, d1);
          }
          fe_mul(di, inv, pre);
          // refill `pre` for the next step right after its last use
          if (i > 1) scr_load(pre, scr, slot(i - 2), g, L);
        }
        fe_sub(dx, tx, cx);
        fe_mul(inv, inv, dx);
      } else {
        di = inv;
      }
      if constexpr (DEFER) {
        // The previous pair's block loads are issued first and tested after this pair's field
        // math: the loads fly during it.  Only their addresses cross the loop edge (ALU values),
        // never an in-flight load destination.
#if !KH_PROBE_EARLY
        const uint4 vm = dload(pm), vp = dload(pp);
#endif
        fe xm, xp, s, dy, sx;
        // x3 = s^2 - (C.x + T.x) for both points; dy = -(dy of C - T[i]): only s^2 is needed, so
        // the sign drops out.  Adjacent independent add/sub pairs share one interleaved chain.
        fe_addsub2<false, false>(sx, cx, tx, dy, ty, cy);
        fe_mul(s, dy, di);
        fe_sqr(xm, s);
        fe_addsub2<true, true>(xm, xm, sx, dy, ty, cy);
        fe_mul(s, dy, di);
        fe_sqr(xp, s);
        fe_sub(xp, xp, sx);
        if (plm && blk_match_rec(vm, pm)) record_hit(A, cidx - poff, DKIND);
        if (plp && blk_match_rec(vp, pp)) record_hit(A, cidx + poff, DKIND);
        const uint32_t off = (uint32_t)(i + 1);
        pm = drec(xm);
        pp = drec(xp);
        poff = off;
        if (wfull) {
          plm = true;
          plp = i < H - 1;
        } else {
          plm = off > lm;
          plp = off < hp;  // also false at i = H - 1 (off = H >= hp): C + H is the next group's
        }
        return;
      }
      if constexpr (MODE == KM_BSGS) {
        // both points first, then one lockstep probe of the pair (two loads in flight per lane)
        fe xm, xp, s, dy, sx;
        fe_add(sx, cx, tx);
        fe_add(dy, ty, cy);  // -(dy) of C - T[i]: only x is needed, s^2 is the same
        fe_mul(s, dy, di);
        fe_sqr(xm, s);
        fe_sub(xm, xm, sx);
        fe_sub(dy, ty, cy);
        fe_mul(s, dy, di);
        fe_sqr(xp, s);
        fe_sub(xp, xp, sx);
        const uint64_t off = (uint64_t)(i + 1);
        probe_pair_bsgs(A, xm, cidx - off, xp, cidx + off, i < H - 1);
        return;
      }
      fe sx;
      fe_add(sx, cx, tx);  // x3 = s^2 - (C.x + T.x) on both sides
      fe nty;
      fe_neg(nty, ty);
#pragma unroll 1
      for (int side = 0; side < 2; side++) {
        if (side == 1 && i == H - 1) break;
        fe tys, dy, s, x, y;
#pragma unroll
        for (int w = 0; w < 8; w++) tys.d[w] = side ? ty.d[w] : nty.d[w];
        fe_sub(dy, tys, cy);
        fe_mul(s, dy, di);
        fe_sqr(x, s);
        fe_sub(x, x, sx);
        if constexpr (needs_y<MODE>()) {
          fe t;
          fe_sub(t, tx, x);
          fe_mul(y, s, t);
          fe_sub(y, y, tys);
        }
        const uint64_t off = (uint64_t)(i + 1);
        probe_point<MODE>(A, x, y, side ? cidx + off : cidx - off);
      }
    };
    if constexpr (KEEP) {
      // two steps per trip, odd then even: the kept row's loads land in place (no copy to wait on)
#pragma unroll 1
      for (int i = H - 1; i > 0; i -= 2) {
        step(i, 1);
        step(i - 1, 2);
      }
    } else {
#pragma unroll 1
      for (int i = H - 1; i >= 0; i--) step(i, 0);
    }
    if constexpr (DEFER) {  // the last pair of the group
      if (plm && blk_match_rec(dload(pm), pm)) record_hit(A, cidx - poff, DKIND);
      if (plp && blk_match_rec(dload(pp), pp)) record_hit(A, cidx + poff, DKIND);
    }
    // next centre C += T[H]  (keyhunt.cpp:3840-3855)
    {
      fe dy, s, s2, nx, ny, t;
      fe_sub(dy, t2y, cy);
      fe_mul(s, dy, inv_n);
      fe_sqr(s2, s);
      fe_sub(nx, s2, cx);
      fe_sub(nx, nx, t2x);
      fe_sub(t, t2x, nx);
      fe_mul(ny, s, t);
      fe_sub(ny, ny, t2y);
      cx = nx;
      cy = ny;
    }
  }
  store_soa(A.cx, A.L, g, cx);
  store_soa(A.cy, A.L, g, cy);
}

// ------------------------------------------------------------------------------------------
// -m rmd160 --rmd-batch-size G < 1024 (keyhunt.cpp:815-829, 3274, 3301-3307, 3349-3461): the
// reference's batch inversion then runs over its first G/2 + 1 slots and leaves the rest of its
// 513-entry IntGroup zero, so the product, its inverse and every derived inverse are 0
// (IntGroup.cpp:36-58).  With s = 0 each non-centre point of a group degenerates to
// x = -(C.x + T[i].x), y = -T[i].y (slot H + i + 1) or +T[i].y (slot H - i - 1), slot 0 using
// T[H - 1]; only the centre C is a real point.  The next group's centre is recomputed from its key
// (3350-3354): C += T[H] with its own inversion here.  One lane walks its groups of 2H = G slots.
// ------------------------------------------------------------------------------------------
template <int MODE>
__global__ void __launch_bounds__(256, KH_WALK_LB_HASH) k_walk_zinv(walk_args A) {
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= A.L) return;
  kconst_ptr T = (kconst_ptr)A.tab;  // (H+1) x {x[8], y[8]}
  const int H = (int)A.zhalf;
  fe cx, cy;
  load_soa(cx, A.cx, A.L, g);
  load_soa(cy, A.cy, A.L, g);
  for (uint32_t j = 0; j < A.groups; j++) {
    const uint64_t cidx = (uint64_t)g * A.lane_stride + (uint64_t)(A.group_base + j) * (2 * H) + H;
    probe_point<MODE>(A, cx, cy, cidx);
#pragma unroll 1
    for (int i = 0; i < H; i++) {
      fe tx, ty, x, s;
      load_fe_k(tx, T + i * 16);
      load_fe_k(ty, T + i * 16 + 8);
      fe_add(s, cx, tx);
      fe_neg(x, s);
      probe_point<MODE>(A, x, ty, cidx - (uint64_t)(i + 1));  // C - T[i] side: y = +T[i].y
      if (i < H - 1) {
        fe nty;
        fe_neg(nty, ty);
        probe_point<MODE>(A, x, nty, cidx + (uint64_t)(i + 1));  // C + T[i] side: y = -T[i].y
      }
    }
    fe t2x, t2y, dx, dy, s, s2, nx, ny, t;
    load_fe_k(t2x, T + H * 16);
    load_fe_k(t2y, T + H * 16 + 8);
    fe_sub(dx, t2x, cx);
    // rare: C = +-T[H].  The reference computes the next centre from its key (3350-3354), so
    // C = T[H] -- a group centred on key G*stride, e.g. -r 100: with G = 512 -- doubles instead.
    // C = -T[H] (the next centre is the point at infinity) lies at the group order, which kh_scan
    // keeps away from this kernel (reaches_order).
    const bool dbl = fe_is_zero(dx);
    ge c2;
    if (dbl) {  // the wave skips this block unless one of its lanes needs it
      const ge c{cx, cy};
      ge_double(c2, c);
      dx.d[0] = 1;  // any non-zero value: this lane's common-path result is replaced
    }
    fe_inv(dx, dx);
    fe_sub(dy, t2y, cy);
    fe_mul(s, dy, dx);
    fe_sqr(s2, s);
    fe_sub(nx, s2, cx);
    fe_sub(nx, nx, t2x);
    fe_sub(t, t2x, nx);
    fe_mul(ny, s, t);
    fe_sub(ny, ny, t2y);
    cx = dbl ? c2.x : nx;
    cy = dbl ? c2.y : ny;
  }
  store_soa(A.cx, A.L, g, cx);
  store_soa(A.cy, A.L, g, cy);
}

// ------------------------------------------------------------------------------------------
// Lane setup: C_g = [Q +] s_g * G with a fixed-base byte comb, comb[j][v] = v * 2^(8j) * G.
// Bytes are added from least to most significant, so the accumulator is always (partial
// scalar)*G with partial < 2^(8j) while comb[j][v] >= 2^(8j): the mixed addition never meets
// the doubling or inverse case (scalars are < n).  One Fermat inversion per lane to go affine;
// Q (the BSGS target) is added in Jacobian coordinates before it.
// ------------------------------------------------------------------------------------------
// s*G for a scalar s != 0 given as 8 LE u32 limbs, left in Jacobian coordinates
__device__ __forceinline__ void comb_mult_jac(gej &acc, const uint32_t s[8], const uint32_t *__restrict__ comb) {
  acc.inf = true;
  for (int j = 0; j < 32; j++) {
    uint32_t v = (s[j >> 2] >> ((j & 3) * 8)) & 0xFFu;
    if (v) {
      ge q;
      const uint32_t *c = comb + ((size_t)j * 256 + v) * 16;
      load_fe(q.x, c);
      load_fe(q.y, c + 8);
      gej_add_ge(acc, q);
    }
  }
}
__device__ __forceinline__ void comb_mult(ge &r, const uint32_t s[8], const uint32_t *__restrict__ comb) {
  gej acc;
  comb_mult_jac(acc, s, comb);
  gej_to_ge(r, acc);
}

namespace {
// secp256k1 group order n, LE u32 limbs
__device__ __forceinline__ uint32_t order_limb(int i) {
  const uint32_t N[8] = {0xD0364141u, 0xBFD25E8Cu, 0xAF48A03Bu, 0xBAAEDCE6u,
                         0xFFFFFFFEu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
  return N[i];
}
// r = (a + v) mod n for a < n and v = v0 + v1*2^64 + v2*2^128 < n (v2 <= 1)
__device__ void sc_add_small(uint32_t r[8], const uint32_t a[8], uint64_t v0, uint64_t v1, uint32_t v2) {
  const uint32_t v[8] = {(uint32_t)v0, (uint32_t)(v0 >> 32), (uint32_t)v1, (uint32_t)(v1 >> 32), v2, 0, 0, 0};
  uint32_t c = 0;
  for (int i = 0; i < 8; i++) r[i] = addc(a[i], v[i], c, c);
  bool ge_n = c != 0;
  if (!ge_n) {  // r >= n ?
    ge_n = true;
    for (int i = 7; i >= 0; i--) {
      if (r[i] != order_limb(i)) {
        ge_n = r[i] > order_limb(i);
        break;
      }
    }
  }
  if (ge_n) {
    uint32_t bo = 0;
    for (int i = 0; i < 8; i++) r[i] = subb(r[i], order_limb(i), bo, bo);
  }
}
}  // namespace

namespace {
// r = (a + b) mod n for a, b < n (LE u32 limbs)
__device__ __forceinline__ void sc_addmod(uint32_t r[8], const uint32_t a[8], const uint32_t b[8]) {
  const uint32_t N[8] = {0xD0364141u, 0xBFD25E8Cu, 0xAF48A03Bu, 0xBAAEDCE6u,
                         0xFFFFFFFEu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
  uint32_t t[8], u[8], c = 0, bo = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) t[i] = addc(a[i], b[i], c, c);
#pragma unroll
  for (int i = 0; i < 8; i++) u[i] = subb(t[i], N[i], bo, bo);
  // a + b >= n exactly when the sum carried out of 2^256 or the subtraction did not borrow
  const bool ge = c != 0 || bo == 0;
#pragma unroll
  for (int i = 0; i < 8; i++) r[i] = ge ? u[i] : t[i];
}
}  // namespace

__global__ void __launch_bounds__(256) k_setup(setup_args A) {
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= A.L) return;
  uint32_t s[8];  // 8 LE u32 limbs
  if (A.prog == 1) {
    // s = s0 + g * step (mod n) by double-and-add over the bits of g, without lane-dependent branches
    uint32_t acc[8], d[8], t[8];
#pragma unroll
    for (int i = 0; i < 8; i++) {
      acc[i] = A.s0[i];
      d[i] = A.step[i];
    }
#pragma unroll 1
    for (uint32_t m = g, b = 0; b < 32 && (A.L >> b) != 0; b++, m >>= 1) {
      sc_addmod(t, acc, d);
#pragma unroll
      for (int i = 0; i < 8; i++) acc[i] = (m & 1) ? t[i] : acc[i];
      sc_addmod(d, d, d);
    }
    uint32_t z = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
      s[i] = acc[i];
      z |= acc[i];
    }
    if (z == 0) atomicOr(A.zero_flag, 1u);
  } else if (A.prog == 2) {
    // BSGS per-base rounds: s = -(key of the centre of the group starting at giant index t0), key =
    // base(b) + M + 2M*(a0 + H) with b = t0 / a_pts, a0 = t0 % a_pts (the host's centre_scalar); the
    // host takes this path only when no centre key can be 0 mod n
    const uint64_t t0 = A.t_round + (uint64_t)g * A.lane_pts;
    const uint64_t b = t0 / A.a_pts, a0 = t0 % A.a_pts;
    uint32_t base[8];
    uint64_t v0 = 0, v1 = 0;
    if (A.list) {
#pragma unroll
      for (int i = 0; i < 8; i++) base[i] = A.list[b * 8 + i];
    } else {
#pragma unroll
      for (int i = 0; i < 8; i++) base[i] = A.start[i];
      v0 = b * A.two_n;  // b*2N as 128 bits
      v1 = __umul64hi(b, A.two_n);
    }
    const uint64_t f = 2 * (a0 + A.h) + 1;  // M + 2M*(a0 + H) = M*f
    const uint64_t w0 = A.m * f, w1 = __umul64hi(A.m, f);
    const uint64_t s0 = v0 + w0;
    const uint64_t c0 = s0 < v0 ? 1 : 0;
    const uint64_t s1 = v1 + w1 + c0;
    const uint32_t s2 = (s1 < v1 || (s1 == v1 && (w1 | c0) != 0)) ? 1u : 0u;
    uint32_t kb[8];
    sc_add_small(kb, base, s0, s1, s2);
    uint32_t bo = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) s[i] = subb(order_limb(i), kb[i], bo, bo);  // n - kb, kb != 0
  } else {
#pragma unroll
    for (int i = 0; i < 8; i++) s[i] = A.scalars[(size_t)g * 8 + i];
  }
  gej acc;
  comb_mult_jac(acc, s, A.comb);
  ge r;
  if (A.has_q) {  // Q + s*G in Jacobian coordinates: one inversion per lane instead of two
    ge q;
    load_fe(q.x, A.q);
    load_fe(q.y, A.q + 8);
    fe z2, u2, h;  // h = Q.x*Z^2 - X: zero iff Q = +-s*G (AddDirect's dx = 0 case)
    fe_sqr(z2, acc.z);
    fe_mul(u2, q.x, z2);
    fe_sub(h, u2, acc.x);
    if (fe_is_zero(h)) {  // the affine AddDirect value, inverse of 0 taken as 0 (rare)
      gej_to_ge(r, acc);
      ge_add(r, q, r);
      store_soa(A.cx, A.L, g, r.x);
      store_soa(A.cy, A.L, g, r.y);
      return;
    }
    gej_add_ge(acc, q);
  }
  gej_to_ge(r, acc);
  store_soa(A.cx, A.L, g, r.x);
  store_soa(A.cy, A.L, g, r.y);
}

// ------------------------------------------------------------------------------------------
// BSGS second check (bsgs_secondcheck, keyhunt.cpp:5151-5184), one candidate per lane.
// ------------------------------------------------------------------------------------------

__global__ void __launch_bounds__(64) k_refine(refine_args A) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t n = min(*A.count, A.cap);
  if (j >= n) return;
  const uint64_t t = A.t_round + A.cands[j].idx;
  const uint64_t b = t / A.a_pts, a = t % A.a_pts;
  uint32_t base[8];
  uint64_t v0 = 0, v1 = 0;
  if (A.list_mode) {
    for (int i = 0; i < 8; i++) base[i] = A.list[b * 8 + i];
  } else {
    for (int i = 0; i < 8; i++) base[i] = A.start[i];
    v0 = b * A.two_n;  // b*2N as 128 bits
    v1 = __umul64hi(b, A.two_n);
  }
  const uint64_t w0 = a * A.two_m, w1 = __umul64hi(a, A.two_m);  // a*2M
  const uint64_t s0 = v0 + w0;
  const uint64_t c0 = s0 < v0 ? 1 : 0;
  const uint64_t s1 = v1 + w1 + c0;
  const uint32_t s2 = (s1 < v1 || (s1 == v1 && (w1 | c0) != 0)) ? 1u : 0u;
  uint32_t sk[8];
  sc_add_small(sk, base, s0, s1, s2);  // base_key (keyhunt.cpp:5159-5161)
  uint32_t nz = 0;
  for (int i = 0; i < 8; i++) nz |= sk[i];
  if (!nz) {  // base_key == 0: no point (the host's comb mult refuses it the same way)
    A.cands[j].aux = 0;
    return;
  }
  ge Q;
  load_fe(Q.x, A.q);
  load_fe(Q.y, A.q + 8);
  // S = Q - base_key*G (AddDirect, keyhunt.cpp:5172) kept in Jacobian coordinates (X, Y, Z): one
  // batched inversion then serves Z and the 32 differences S - AMP2[i] (three inversions before)
  gej S;
  comb_mult_jac(S, sk, A.comb);
  fe_neg(S.y, S.y);
  {
    fe z2, u2, h;  // h = Q.x*Z^2 - X: zero iff Q = +-base_key*G, the AddDirect dx = 0 case
    fe_sqr(z2, S.z);
    fe_mul(u2, Q.x, z2);
    fe_sub(h, u2, S.x);
    if (fe_is_zero(h)) {  // reproduce AddDirect's inverse-0 value on the affine path (rare)
      ge bp, Sa;
      gej_to_ge(bp, S);
      ge_add(Sa, Q, bp);
      S.x = Sa.x;
      S.y = Sa.y;
      fe_set_u32(S.z, 1);
    } else {
      gej_add_ge(S, Q);
    }
  }
  // e_i = AMP2[i].x * Z^2 - X = (AMP2[i].x - S.x) * Z^2: zero exactly when the reference's dx is,
  // and then (as there) its inverse counts as 0.  Prefix products over Z, e_0, ..., e_31.
  fe z2, pre[32], acc;
  fe_sqr(z2, S.z);
  acc = S.z;
  for (int i = 0; i < 32; i++) {
    fe ax, e;
    load_fe(ax, A.amp2 + i * 16);
    fe_mul(e, ax, z2);
    fe_sub(e, e, S.x);
    if (!fe_is_zero(e)) fe_mul(acc, acc, e);
    pre[i] = acc;
  }
  fe inv;
  fe_inv(inv, acc);
  // backward: 1/e_i for i = 31..0 (into pre[i], whose prefix is no longer needed), then 1/Z
  for (int i = 31; i >= 0; i--) {
    fe ax, e, d;
    load_fe(ax, A.amp2 + i * 16);
    fe_mul(e, ax, z2);
    fe_sub(e, e, S.x);
    if (fe_is_zero(e)) {
      fe_set_u32(d, 0);
    } else {
      d = i == 0 ? S.z : pre[i - 1];
      fe_mul(d, d, inv);
      fe_mul(inv, inv, e);
    }
    pre[i] = d;
  }
  // inv = 1/Z now: affine S
  fe zi2, zi3, sx, sy;
  fe_sqr(zi2, inv);
  fe_mul(zi3, zi2, inv);
  fe_mul(sx, S.x, zi2);
  fe_mul(sy, S.y, zi3);
  uint32_t mask = 0;
  for (int i = 31; i >= 0; i--) {
    fe ax, ay, di, dy, s, x;
    load_fe(ax, A.amp2 + i * 16);
    load_fe(ay, A.amp2 + i * 16 + 8);
    fe_mul(di, pre[i], z2);  // 1/dx = Z^2/e (0 stays 0)
    fe_sub(dy, ay, sy);
    fe_mul(s, dy, di);
    fe_sqr(x, s);
    fe_sub(x, x, sx);
    fe_sub(x, x, ax);
    uint64_t in[4];
    x_bytes_u64(x, in);
    const uint64_t ha = xxh64_32(in, KH_BLOOM_SEED), hb = xxh64_32(in, ha);
    if (bloom_probe(A.bloom2 + (size_t)(x.d[7] >> 24) * A.bd2.stride, A.bd2, ha, hb)) mask |= 1u << i;
  }
  A.cands[j].aux = mask;
}

// ------------------------------------------------------------------------------------------
// Parity-test kernels (exercised by tests/ through the C-ABI): hash160 and bloom probes of
// given inputs, field ops.
// ------------------------------------------------------------------------------------------
__global__ void k_test_hash160(const uint32_t *xs, const uint32_t *ys, uint32_t n, uint32_t *out) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  fe x, y;
  load_fe(x, xs + (size_t)i * 8);
  load_fe(y, ys + (size_t)i * 8);
  uint32_t *o = out + (size_t)i * 15;
  hash160_comp(x, 2, o);
  hash160_comp(x, 3, o + 5);
  hash160_uncomp(x, y, o + 10);
}

__global__ void k_test_field(const uint32_t *a, const uint32_t *b, uint32_t n, uint32_t *out) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  fe x, y, r;
  load_fe(x, a + (size_t)i * 8);
  load_fe(y, b + (size_t)i * 8);
  uint32_t *o = out + (size_t)i * 40;
  fe_mul(r, x, y);
#pragma unroll
  for (int k = 0; k < 8; k++) o[k] = r.d[k];
  fe_sqr(r, x);
#pragma unroll
  for (int k = 0; k < 8; k++) o[8 + k] = r.d[k];
  fe_inv(r, x);
#pragma unroll
  for (int k = 0; k < 8; k++) o[16 + k] = r.d[k];
  // add and sub: even inputs through the single forms, odd ones through the paired-chain form
  // (fe_addsub2, both operand orders), so every wave runs both and their rare fix-ups side by side
  fe q;
  if ((i & 1) == 0) {
    fe_add(r, x, y);
    fe_sub(q, x, y);
  } else if ((i & 3) == 1) {
    fe_addsub2<false, true>(r, x, y, q, x, y);
  } else {
    fe_addsub2<true, false>(q, x, y, r, x, y);
  }
#pragma unroll
  for (int k = 0; k < 8; k++) o[24 + k] = r.d[k];
#pragma unroll
  for (int k = 0; k < 8; k++) o[32 + k] = q.d[k];
}

// bloom_check of n items of `len` bytes (20 or 32); shard = first byte when sharded.
__global__ void k_test_bloom(const uint8_t *items, uint32_t n, uint32_t len, const uint8_t *bloom, bloom_desc bd,
                             uint32_t sharded, uint32_t blocked, uint32_t *out) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint8_t *p = items + (size_t)i * len;
  uint64_t a, b;
  if (len == 32) {
    uint64_t in[4];
    for (int k = 0; k < 4; k++) {
      uint64_t v = 0;
      for (int q = 7; q >= 0; q--) v = (v << 8) | p[8 * k + q];
      in[k] = v;
    }
    a = xxh64_32(in, KH_BLOOM_SEED);
    b = xxh64_32(in, a);
  } else {
    uint32_t w[5];
    for (int k = 0; k < 5; k++)
      w[k] = (uint32_t)p[4 * k] | ((uint32_t)p[4 * k + 1] << 8) | ((uint32_t)p[4 * k + 2] << 16) |
             ((uint32_t)p[4 * k + 3] << 24);
    a = xxh64_20(w, KH_BLOOM_SEED);
    b = xxh64_20(w, a);
  }
  const uint8_t *bf = bloom + (sharded ? (size_t)p[0] * bd.stride : 0);
  if (blocked) {
    // X[8..12), X[12..16), X[16..20), X[20..24) as big-endian u32s (limbs 5, 4, 3, 2)
    uint32_t w[4];
    for (int k = 0; k < 4; k++)
      w[k] = ((uint32_t)p[8 + 4 * k] << 24) | ((uint32_t)p[9 + 4 * k] << 16) | ((uint32_t)p[10 + 4 * k] << 8) |
             p[11 + 4 * k];
    out[i] = blk_match(reinterpret_cast<const uint4 *>(bf)[blk_index(w[0], bd)], w[1], w[2], w[3]) ? 1u : 0u;
    return;
  }
  out[i] = bloom_probe(bf, bd, a, b) ? 1u : 0u;
}

// ------------------------------------------------------------------------------------------
// launch helpers (host side)
// ------------------------------------------------------------------------------------------
namespace kh {

#if defined(KH_ISA_ONLY_BSGSB) && !defined(KH_ISA_ONLY_MODE)
#define KH_ISA_ONLY_MODE KM_BSGSB
#endif
hipError_t launch_walk(int mode, const walk_args &A, hipStream_t st, int H) {
#ifdef KH_ISA_ONLY_MODE
  // analysis builds (tools/isa_hot.py, tools/valu_mix.py): one large-group walk alone (KH_ISA_ONLY_BSGSB:
  // the BSGS giant walk; KH_ISA_ONLY_MODE=<kh_walk_mode>: any other), compiled in seconds
  constexpr int TB1 = walk_threads<KH_ISA_ONLY_MODE, KH_WALK_HB>();
  hipLaunchKernelGGL((k_walk<KH_ISA_ONLY_MODE, KH_WALK_HB>), dim3((A.L + TB1 - 1) / TB1), dim3(TB1), 0, st, A);
  (void)mode;
  (void)H;
  return hipGetLastError();
#else
  if (A.zhalf) return launch_walk_zinv(mode, A, st);
  dim3 block(256), grid((A.L + 255) / 256);
  if (KH_XPOINT_DEFER && mode == KM_XPOINT && A.tblk) mode = KM_XPOINTB;
  if (KH_H160_BLK && mode == KM_H160C && A.tblk) mode = KM_H160CB;
  if (H == KH_WALK_HB) {
    constexpr int TB = walk_threads<KM_BSGSB, KH_WALK_HB>();
    switch (mode) {
      case KM_BSGS: hipLaunchKernelGGL((k_walk<KM_BSGS, KH_WALK_HB>), grid, block, 0, st, A); break;
      case KM_BSGSB:
        hipLaunchKernelGGL((k_walk<KM_BSGSB, KH_WALK_HB>), dim3((A.L + TB - 1) / TB), dim3(TB), 0, st, A);
        break;
      case KM_XPOINT: hipLaunchKernelGGL((k_walk<KM_XPOINT, KH_WALK_HB>), grid, block, 0, st, A); break;
      case KM_XPOINTB: hipLaunchKernelGGL((k_walk<KM_XPOINTB, KH_WALK_HB>), grid, block, 0, st, A); break;
      case KM_H160C: hipLaunchKernelGGL((k_walk<KM_H160C, KH_WALK_HB>), grid, block, 0, st, A); break;
      case KM_H160CB: hipLaunchKernelGGL((k_walk<KM_H160CB, KH_WALK_HB>), grid, block, 0, st, A); break;
      default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
  }
  if (H != KH_WALK_H) return hipErrorInvalidValue;
#ifdef KH_ONLY_MODE
  if (mode != KH_ONLY_MODE) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_walk<KH_ONLY_MODE>, grid, block, 0, st, A);
  return hipGetLastError();
#endif
  switch (mode) {
    case KM_H160C: hipLaunchKernelGGL(k_walk<KM_H160C>, grid, block, 0, st, A); break;
    case KM_H160CB: hipLaunchKernelGGL(k_walk<KM_H160CB>, grid, block, 0, st, A); break;
    case KM_H160U: hipLaunchKernelGGL(k_walk<KM_H160U>, grid, block, 0, st, A); break;
    case KM_H160B: hipLaunchKernelGGL(k_walk<KM_H160B>, grid, block, 0, st, A); break;
    case KM_XPOINT: hipLaunchKernelGGL(k_walk<KM_XPOINT>, grid, block, 0, st, A); break;
    case KM_XPOINTB: hipLaunchKernelGGL(k_walk<KM_XPOINTB>, grid, block, 0, st, A); break;
    case KM_BSGS: hipLaunchKernelGGL(k_walk<KM_BSGS>, grid, block, 0, st, A); break;
    case KM_BUILD: hipLaunchKernelGGL(k_walk<KM_BUILD>, grid, block, 0, st, A); break;
    case KM_DUMP: hipLaunchKernelGGL(k_walk<KM_DUMP>, grid, block, 0, st, A); break;
    case KM_BSGSB: hipLaunchKernelGGL(k_walk<KM_BSGSB>, grid, block, 0, st, A); break;
    case KM_BUILDB: hipLaunchKernelGGL(k_walk<KM_BUILDB>, grid, block, 0, st, A); break;
    case KM_ETH: hipLaunchKernelGGL(k_walk<KM_ETH>, grid, block, 0, st, A); break;
    case KM_H160C | KM_ENDO: hipLaunchKernelGGL(k_walk<KM_H160C | KM_ENDO>, grid, block, 0, st, A); break;
    case KM_H160U | KM_ENDO: hipLaunchKernelGGL(k_walk<KM_H160U | KM_ENDO>, grid, block, 0, st, A); break;
    case KM_H160B | KM_ENDO: hipLaunchKernelGGL(k_walk<KM_H160B | KM_ENDO>, grid, block, 0, st, A); break;
    case KM_XPOINT | KM_ENDO: hipLaunchKernelGGL(k_walk<KM_XPOINT | KM_ENDO>, grid, block, 0, st, A); break;
    case KM_ETH | KM_ENDO: hipLaunchKernelGGL(k_walk<KM_ETH | KM_ENDO>, grid, block, 0, st, A); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
#endif
}

hipError_t launch_walk_zinv(int mode, const walk_args &A, hipStream_t st) {
#ifdef KH_ISA_ONLY_MODE
  (void)mode;
  (void)A;
  (void)st;
  return hipErrorInvalidValue;
#else
  dim3 block(256), grid((A.L + 255) / 256);
  if (A.zhalf < 2 || A.zhalf > KH_WALK_H) return hipErrorInvalidValue;
  switch (mode) {
    case KM_H160C: hipLaunchKernelGGL(k_walk_zinv<KM_H160C>, grid, block, 0, st, A); break;
    case KM_H160U: hipLaunchKernelGGL(k_walk_zinv<KM_H160U>, grid, block, 0, st, A); break;
    case KM_H160B: hipLaunchKernelGGL(k_walk_zinv<KM_H160B>, grid, block, 0, st, A); break;
    case KM_H160C | KM_ENDO: hipLaunchKernelGGL(k_walk_zinv<KM_H160C | KM_ENDO>, grid, block, 0, st, A); break;
    case KM_H160U | KM_ENDO: hipLaunchKernelGGL(k_walk_zinv<KM_H160U | KM_ENDO>, grid, block, 0, st, A); break;
    case KM_H160B | KM_ENDO: hipLaunchKernelGGL(k_walk_zinv<KM_H160B | KM_ENDO>, grid, block, 0, st, A); break;
    case KM_ETH: hipLaunchKernelGGL(k_walk_zinv<KM_ETH>, grid, block, 0, st, A); break;
    case KM_ETH | KM_ENDO: hipLaunchKernelGGL(k_walk_zinv<KM_ETH | KM_ENDO>, grid, block, 0, st, A); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
#endif
}

// A VALU-dense load (multiply-add chains, no memory traffic) run right before a BSGS job's first walk
// launch (KH_BURN_MS, kh_capi.cpp): it drives the board's clock down to its power cap before the walk
// starts, so the walk settles into the low-clock operating point (DESIGN.md §2 "Placement")
__global__ void __launch_bounds__(256) k_burn(uint32_t iters, uint32_t *sink) {
  uint64_t a[8];
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
#pragma unroll
  for (int k = 0; k < 8; k++) a[k] = (uint64_t)(g * 2654435761u + k) | 1;
  for (uint32_t i = 0; i < iters; i++) {
#pragma unroll
    for (int k = 0; k < 8; k++) a[k] = (uint64_t)(uint32_t)a[k] * (uint32_t)(a[k] >> 17) + a[(k + 1) & 7];
  }
  uint64_t x = 0;
#pragma unroll
  for (int k = 0; k < 8; k++) x ^= a[k];
  if (x == 0x0123456789ABCDEFull) sink[0] = g;  // never in practice: keeps the chains live
}

hipError_t launch_burn(uint32_t iters, uint32_t *sink, hipStream_t st) {
  hipLaunchKernelGGL(k_burn, dim3(256 * 8), dim3(256), 0, st, iters, sink);
  return hipGetLastError();
}

hipError_t launch_refine(const refine_args &A, hipStream_t st) {
  hipLaunchKernelGGL(k_refine, dim3((A.cap + 63) / 64), dim3(64), 0, st, A);
  return hipGetLastError();
}

hipError_t launch_setup(const setup_args &A, hipStream_t st) {
  hipLaunchKernelGGL(k_setup, dim3((A.L + 255) / 256), dim3(256), 0, st, A);
  return hipGetLastError();
}

hipError_t launch_test_hash160(const uint32_t *xs, const uint32_t *ys, uint32_t n, uint32_t *out, hipStream_t st) {
  hipLaunchKernelGGL(k_test_hash160, dim3((n + 127) / 128), dim3(128), 0, st, xs, ys, n, out);
  return hipGetLastError();
}

hipError_t launch_test_field(const uint32_t *a, const uint32_t *b, uint32_t n, uint32_t *out, hipStream_t st) {
  hipLaunchKernelGGL(k_test_field, dim3((n + 127) / 128), dim3(128), 0, st, a, b, n, out);
  return hipGetLastError();
}

hipError_t launch_test_bloom(const uint8_t *items, uint32_t n, uint32_t len, const uint8_t *bloom,
                             const bloom_desc &bd, uint32_t sharded, uint32_t blocked, uint32_t *out, hipStream_t st) {
  hipLaunchKernelGGL(k_test_bloom, dim3((n + 127) / 128), dim3(128), 0, st, items, n, len, bloom, bd, sharded, blocked,
                     out);
  return hipGetLastError();
}

}  // namespace kh
