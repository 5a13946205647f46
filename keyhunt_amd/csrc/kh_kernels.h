// kh_kernels.h -- kernel argument blocks and launch helpers shared by kh_kernels.hip and the
// C-ABI implementation (kh_capi.cpp).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "kh_math.h"

// Group half-size H: a group is 2H points around one centre (the reference uses 512,
// keyhunt.cpp:299 CPU_GRP_SIZE/2).  Scratch per lane = H * 32 bytes.
#ifndef KH_WALK_H
#define KH_WALK_H 512
#endif
static_assert(KH_WALK_H >= 64 && KH_WALK_H <= 512 && (512 % KH_WALK_H) == 0,
              "2H must divide the reference's 1024-point group so lanes never straddle a BSGS base");

// Large group half-size for the continuous BSGS giant walk (KM_BSGS / KM_BSGSB): lanes there own
// long runs, so a group may span 4096 points and its one Fermat inversion is shared 4x wider.
// Scratch per lane = KH_WALK_HB * 32 bytes; the delta table holds KH_WALK_HB + 1 points.
#ifndef KH_WALK_HB
#define KH_WALK_HB 2048
#endif
// Lanes of the address family's 4096-point-group walks (xpoint, compressed address/rmd160): 2^20, so
// one 2^32-key chunk is one launch of 16384 waves -- four per wave slot of the xpoint walk (128 VGPRs,
// 4 waves/SIMD) and 5.3 per slot of the hash walk (168 VGPRs, 3 waves/SIMD).  Waves that start as
// others end run out of phase with them, so the pad and inversion phases of some overlap the field
// math of others; with 2^18 lanes (one wave per slot, all in phase) xpoint ran 50.5 vs 57.9 G points/s
// and rmd160 7.66 vs 8.00 (profiles/r04a_geom_ab.json).  Pad: 2^20 x 4096 x 32 B / 2 = 64 GB.
#ifndef KH_LANES_HB
#define KH_LANES_HB (1u << 20)
#endif
// Lanes of the BSGS giant walk's large calls: 2^21, eight waves per wave slot in turn.  The walk
// waits on its random probes (0.76 of the quad model), and the more batches of waves a launch
// holds, the further their phases drift apart: in bench.py's BSGS leg, interleaved on one box, 2^21
// lanes ran 41.9 G giant points/s (spread 0.2 %) against 38.5-40.3 at 2^20 and ~39.7 at 2^18
// (profiles/r05x_bench_lanes_2m.json).  Pad: 2^21 x 1024 rows x 32 B = 64 GB.
#ifndef KH_BSGS_LANES
#define KH_BSGS_LANES (1u << 21)
#endif

// minimum waves per SIMD requested for the walk kernel: XPOINT/BSGS/BUILD modes (KH_WALK_LB) and
// the hash160 modes (KH_WALK_LB_HASH).  256 / LB VGPRs per lane at most; see DESIGN.md.
#ifndef KH_WALK_LB
#define KH_WALK_LB 4
#endif
// compute hash160(02||X) and hash160(03||X) with interleaved SHA-256 chains
#ifndef KH_HASH_PAIR
#define KH_HASH_PAIR 1
#endif
// KH_WALK_LB_H160CB: the compressed exact-target hash walk (the bench's rmd160 leg) at 4 waves/SIMD.  Since
// the hash IVs fold (round 5) it fits 128 VGPRs with no spill in its per-point loop: +0.3 % in an
// interleaved A/B, spreads disjoint (profiles/r05g_ab_hash_4waves.json); round 4 measured -1.1 % with the
// constants still in VGPRs.  The other hash modes (Y, uncompressed, eth) keep KH_WALK_LB_HASH.
#ifndef KH_WALK_LB_H160CB
#define KH_WALK_LB_H160CB 4
#endif
#ifndef KH_WALK_LB_HASH
#define KH_WALK_LB_HASH 3
#endif

// Blocked layer-1 bloom (KH_LAYER1_BLOCKED), a split-block filter: per shard X[0], `blocks` 16-byte
// blocks, blocks = ceil(KH_BLK_BITS_MUL x reference bits / 128).  An item X (an x-coordinate, so
// already uniform) uses its own bits instead of a hash: with u = big-endian u32 of X[8..12), the
// block is (u * blocks) >> 32; its 16 bit positions come from X[12..20) (kh_blk_masks below).  An
// item is present iff every little-endian u32 word of the block covers its mask.  3x the
// reference's bits: FP 6.6e-7 (Poisson block load) vs the reference's 1e-6; one 16-byte load per
// probe, no hashing.
#define KH_BLK_BITS_MUL 3

// Bit positions of the split-block filters (blocked layer 1 above, and the exact-target filter of
// kh_kernels.hip tblk_probe), from an item's position words s0, s1 (layer 1: the big-endian u32s of
// X[12..16), X[16..20); targets: w1, w2).  KH_PK_MASKS (default): block word w (< 4) gets 4 bits, 2 in
// each 16-bit half: with s = s_{w/2}, a = s >> 8*(w%2) and b = a >> 4, the bits
//   a & 15,  16 + ((a >> 16) & 15),  b & 15,  16 + ((b >> 16) & 15)
// -- each pair is one v_pk_lshlrev_b16 of 0x00010001, so the 16 positions cost 6 shifts and 8 packed
// shifts (the 5-bit-field form below, KH_PK_MASKS=0, costs two 32-bit shifts per position).  Every
// bit of s0 and s1 is used once; per 16-bit half the FP model is the same as per 32-bit word.
// KH_PK_MASKS=0: fields f < 16 of X[12..24) (s0, s1, s2 = X[20..24)), (s_{f/6} >> 5*(f%6)) & 31, bits
// 4w..4w+3 in word w.
#ifndef KH_PK_MASKS
#define KH_PK_MASKS 1
#endif
// (1 << (a & 15)) | (1 << (16 + ((a >> 16) & 15)))
KH_HD uint32_t kh_pk_bits(uint32_t a) {
#if defined(__HIP_DEVICE_COMPILE__)
  uint32_t r;
  asm("v_pk_lshlrev_b16 %0, %1, %2" : "=v"(r) : "v"(a), "s"(0x00010001u));
  return r;
#else
  return (1u << (a & 15u)) | (1u << (16u + ((a >> 16) & 15u)));
#endif
}
KH_HD void kh_blk_masks(uint32_t s0, uint32_t s1, uint32_t s2, uint32_t m[4]) {
  if (KH_PK_MASKS) {
    (void)s2;
    m[0] = kh_pk_bits(s0) | kh_pk_bits(s0 >> 4);
    m[1] = kh_pk_bits(s0 >> 8) | kh_pk_bits(s0 >> 12);
    m[2] = kh_pk_bits(s1) | kh_pk_bits(s1 >> 4);
    m[3] = kh_pk_bits(s1 >> 8) | kh_pk_bits(s1 >> 12);
    return;
  }
  uint32_t f[16];
  for (int t = 0; t < 16; t++) {
    const uint32_t s = t < 6 ? s0 : t < 12 ? s1 : s2;
    f[t] = 1u << ((s >> (5 * (t % 6))) & 31u);
  }
  for (int w = 0; w < 4; w++) m[w] = f[4 * w] | f[4 * w + 1] | f[4 * w + 2] | f[4 * w + 3];
}

// Variant switches of the BSGS giant walk (k_walk<KM_BSGSB, KH_WALK_HB>), A/B-measured:
//   KH_TAB_LDS   the delta table staged in LDS (one 1024-thread workgroup per CU, ds_read_b128
//                broadcasts) instead of scalar-cache reads into SGPRs
//   KH_TAB_VCOPY the table values a step uses twice copied to VGPRs once (a carry chain with an SGPR
//                operand and a carry-in reads two scalars, over gfx9's constant-bus limit of one, so
//                the compiler copies the SGPR in every such instruction)
//   KH_SPARSE_ALL the half-size inversion pad (even prefix products only) in every mode, not only BSGS
//   KH_SPARSE_BSGS the half-size pad in the BSGS walks (default on)
#ifndef KH_TAB_LDS
#define KH_TAB_LDS 0
#endif
#ifndef KH_TAB_VCOPY
#define KH_TAB_VCOPY 0
#endif
#ifndef KH_SPARSE_BSGS
#define KH_SPARSE_BSGS 1
#endif
//   KH_SPARSE_XPOINT the sparse pad (even prefix products only) for -m xpoint's blocked walk too
//                  (round 4, with KH_SPARSE_KEEP: +1.5 %, profiles/r04o_sparse_xpoint_ab.json)
#ifndef KH_SPARSE_XPOINT
#define KH_SPARSE_XPOINT 1
#endif
#ifndef KH_SPARSE_ALL
#define KH_SPARSE_ALL 0
#endif
//   KH_SPARSE_KEEP the sparse pad's backward pass keeps the loaded even row as loaded for the two
//                  steps it serves (one read per row; the load lands in place and flies for a step)
#ifndef KH_SPARSE_KEEP
#define KH_SPARSE_KEEP 1
#endif
//   KH_PAD_PLANES  the two 16-B halves of every inversion-pad entry in separate planes (kh_kernels.hip
//                  pad_idx): one wave access covers 1 KB contiguously instead of 2 KB with holes
#ifndef KH_PAD_PLANES
#define KH_PAD_PLANES 0
#endif
#ifndef KH_PAD_KNOBS
#define KH_PAD_KNOBS 0  // kernel side of the KH_PAD_SKEW / KH_PAD_SWZ pad-layout A/B knobs
#endif
//   KH_PAD_NT      the inversion pad's stores (bit 0) / loads (bit 1) with the nontemporal hint
#ifndef KH_PAD_NT
#define KH_PAD_NT 0
#endif
//   KH_PROBE_EARLY the deferred walks issue the previous pair's block loads at the top of a step,
//                  before its inverse, instead of after it
#ifndef KH_PROBE_EARLY
#define KH_PROBE_EARLY 0
#endif
//   KH_XPOINT_DEFER -m xpoint against the blocked target filter walks like the BSGS giant walk: a
//                pair's two 16-B filter loads are issued one step later and tested after that
//                step's field math (k_walk<KM_XPOINTB>), and -(dy) = T.y + C.y replaces the negation
#ifndef KH_XPOINT_DEFER
#define KH_XPOINT_DEFER 1
#endif
//   KH_FULL_GROUPS the xpoint deferred-probe walk skips the per-pair index-vs-job-end compares in
//                groups that lie wholly inside the job for every lane of the wave (a uniform test)
#ifndef KH_FULL_GROUPS
#define KH_FULL_GROUPS 1
#endif
//   KH_H160_BLK  -l compress hash160 scans with exact targets compile the blocked-filter probe alone
//                (k_walk<KM_H160CB>), so the RIPEMD-160 steps that feed digest words 3..4 drop out
#ifndef KH_H160_BLK
#define KH_H160_BLK 1
#endif

enum kh_walk_mode {
  KM_H160C = 0,   // hash160(02||X), hash160(03||X)          -l compress
  KM_H160U = 1,   // hash160(04||X||Y)                       -l uncompress
  KM_H160B = 2,   // both                                    -l both (default)
  KM_XPOINT = 3,  // X[0..20)                                -m xpoint
  KM_BSGS = 4,    // 32-byte X into the 256-shard layer-1 bloom
  KM_BUILD = 5,   // BSGS baby-step table build
  KM_DUMP = 6,    // X/Y dump (parity tests)
  KM_BSGSB = 7,   // giant steps against the blocked layer-1 bloom (one 16-B block per probe)
  KM_BUILDB = 8,  // baby-step build with the blocked layer-1 bloom
  KM_ETH = 9,     // Keccak-256(X||Y)[12..32): Ethereum address -> target bloom (-c eth)
  KM_XPOINTB = 10,  // KM_XPOINT with the blocked target filter, deferred probes (launch_walk picks it)
  KM_H160CB = 11,   // KM_H160C with the blocked target filter only (launch_walk picks it)
  // flag on KM_H160C/U/B and KM_XPOINT: also probe the endomorphism images (beta*x, y) and
  // (beta^2*x, y), i.e. keys lambda*k and lambda^2*k (-e, keyhunt.cpp:3408-3440, 3476-3830)
  KM_ENDO = 16,
};
// device hit kinds: base kind (0: 02||X, 1: 03||X, 2: 04||X||Y, 3: xpoint, 4: bsgs, 5: eth) plus, with
// KM_ENDO, the image e (0: X, 1: beta*X, 2: beta^2*X) << 4 and, for 04 hashes, the Y sign << 6
#define KH_DKIND_ENDO_SHIFT 4
#define KH_DKIND_NEG 0x40u

struct kh_dev_hit {
  uint64_t idx;   // point index within the job
  uint32_t kind;  // 0: 02||X, 1: 03||X, 2: 04||X||Y, 3: xpoint, 4: bsgs candidate
  uint32_t aux;
};

struct walk_args {
  const uint32_t *tab;   // (H+1) entries of {x[8], y[8]} (LE u32 limbs)
  uint32_t *cx, *cy;     // lane centres, SoA: word w of lane g at [w*L + g]
  uint4 *scratch;        // H * L * 32 bytes
  uint32_t L;            // lanes
  uint32_t groups;       // groups per lane in this launch
  uint64_t lane_stride;  // points per lane in the job
  uint64_t group_base;   // groups each lane already walked in this job
  uint64_t n_points;     // points in the job (indices >= n_points are not probed)
  uint32_t interleave;   // 0: lane g owns groups [g*gpl, (g+1)*gpl); 1: groups g, g+L, g+2L, ...
                         // (the table's last entry is then the L*2H*D jump)
  // probe target (target bloom, or BSGS layer 1 / build layer 1)
  const uint8_t *bloom;
  kh::bloom_desc bd;
  uint32_t *hit_count;
  kh_dev_hit *hits;
  uint32_t hit_cap;
  uint32_t probe_len;  // hash160 modes: bytes of the hash the bloom keys on (20; vanity: the prefix length)
  // exact targets: the blocked target filter probed instead of the reference-layout bloom (see
  // kh_kernels.hip tblk_probe); null for vanity prefixes
  const uint4 *tblk;
  uint32_t tblocks;
  uint32_t bstride32;  // BSGS blocked layer 1: shard stride in bytes (< 2^32, kh_bsgs_setup checks)
  // BSGS build
  uint8_t *bl1, *bl2, *bl3;
  kh::bloom_desc bd2, bd3;
  uint64_t m2, m3;
  uint64_t *rows_key;
  uint32_t *rows_val;
  // dump
  uint32_t *dump_x, *dump_y;
  // k_walk_zinv: half of the --rmd-batch-size group (groups of 2 * zhalf slots)
  uint32_t zhalf;
  // inversion pad: lanes of gap after each row (row stride L + pad_skew entries; KH_PAD_SKEW A/B knob)
  uint32_t pad_skew;
  // inversion pad: row r keeps lane g's entry in column g ^ ((r & 7) << 8) (L a multiple of 2048), so
  // the columns of one 256-lane workgroup -- one XCD's -- rotate over the 8 KB chunk classes row by row
  uint32_t pad_swz;
};

struct setup_args {
  const uint32_t *scalars;  // L x 8 LE u32 limbs (unless prog)
  const uint32_t *comb;     // 32 x 256 x 16 words
  const uint32_t *q;        // optional point added to every lane: {x[8], y[8]}
  uint32_t has_q;
  uint32_t L;
  uint32_t *cx, *cy;
  // prog == 1: the lane scalars are the progression s_g = s0 + g * step (mod n), derived on the device (no
  // host loop, no upload); a lane whose scalar is 0 sets *zero_flag
  uint32_t prog;
  uint32_t s0[8], step[8];  // LE u32 limbs, both < n
  uint32_t *zero_flag;
  // prog == 2, BSGS per-base rounds: lane g starts at giant index t0 = t_round + g*lane_pts of the call
  // (base b = t0 / a_pts, a0 = t0 % a_pts) and its scalar is -(base(b) + m*(2*(a0 + h) + 1)) mod n,
  // base(b) = list[b] (list != null) or start + b*two_n
  const uint32_t *list, *start;  // 8 LE u32 limbs per base, < n
  uint64_t t_round, lane_pts, a_pts, two_n, m;
  uint32_t h;
};

// BSGS second check on the GPU (bsgs_secondcheck, keyhunt.cpp:5151-5184).  Per first-level
// candidate (giant index t = t_round + idx, base b = t / a_pts, a = t % a_pts):
// base_key = base(b) + a*2M (mod n), S = Q - base_key*G, and the 32 points S + AMP2[i] are probed
// against layer 2 (reference layout); the candidate's aux receives the mask of layer-2 hits.
// The host then runs bsgs_thirdcheck for the set bits only, in bit order.
struct refine_args {
  kh_dev_hit *cands;       // in: idx; out: aux = layer-2 mask
  const uint32_t *count;   // candidates recorded in the round (device)
  uint32_t cap;            // entries in cands
  uint32_t list_mode;      // 0: base(b) = start + b*2N; 1: base(b) = list[b]
  uint64_t t_round;        // giant index of the round's point 0
  uint64_t a_pts;          // giant points walked per base
  uint64_t two_n, two_m;
  const uint32_t *start;   // 8 LE u32 limbs, < n
  const uint32_t *list;    // list mode: bases x 8 LE u32 limbs, each < n
  const uint32_t *comb;    // 32 x 256 x 16 words
  const uint32_t *q;       // target {x[8], y[8]}
  const uint32_t *amp2;    // 32 x {x[8], y[8]}: BSGS_AMP2 (keyhunt.cpp:1818-1842)
  const uint8_t *bloom2;   // layer 2, 256 shards at bd2.stride
  kh::bloom_desc bd2;
};

namespace kh {
hipError_t launch_walk(int mode, const walk_args &A, hipStream_t st, int H = KH_WALK_H);
// Inversion-pad rows per lane the walk launch_walk runs for (mode, blocked target filter) touches: the
// sparse-pad walks (k_walk's SPARSE: the BSGS giant walks, -m xpoint against the blocked filter) keep
// only the even prefix products, rows [0, H/2); the others all H
inline int walk_pad_rows(int mode, bool tblk, int H) {
  if (KH_XPOINT_DEFER && mode == KM_XPOINT && tblk) mode = KM_XPOINTB;
  const bool sparse = KH_SPARSE_ALL || (KH_SPARSE_BSGS && (mode == KM_BSGSB || mode == KM_BSGS)) ||
                      (KH_SPARSE_XPOINT && mode == KM_XPOINTB);
  return sparse ? H / 2 : H;
}
hipError_t launch_walk_zinv(int mode, const walk_args &A, hipStream_t st);
hipError_t launch_refine(const refine_args &A, hipStream_t st);
hipError_t launch_burn(uint32_t iters, uint32_t *sink, hipStream_t st);
hipError_t launch_setup(const setup_args &A, hipStream_t st);
hipError_t launch_test_hash160(const uint32_t *xs, const uint32_t *ys, uint32_t n, uint32_t *out, hipStream_t st);
hipError_t launch_test_field(const uint32_t *a, const uint32_t *b, uint32_t n, uint32_t *out, hipStream_t st);
hipError_t launch_test_bloom(const uint8_t *items, uint32_t n, uint32_t len, const uint8_t *bloom,
                             const bloom_desc &bd, uint32_t sharded, uint32_t blocked, uint32_t *out, hipStream_t st);
}  // namespace kh
