// kh_capi.cpp -- implementation of include/kh_gpu.h.
//
// Host side of the MI355X engine: device memory layout, lane partitioning, launches, the
// reference-exact host steps around the kernels (bloom sizing, table sort + searchbinary,
// compressed-key parity fix-up, BSGS second/third check), and event timing.  Every scan and
// build runs on the GPU kernels in kh_kernels.hip; there is no CPU fallback.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdlib.h>
#include <stdio.h>
#include <string.h>
#include <algorithm>
#include <array>
#include <atomic>
#include <mutex>
#include <thread>
#include <string>
#include <vector>

#include "kh_gpu.h"
#include "kh_kernels.h"
#include "kh_math.h"

using namespace kh;

// ==============================================================================================
// 256-bit scalars (mod n) on the host
// ==============================================================================================
namespace {

typedef unsigned __int128 u128;
struct u256 {
  uint64_t v[4];
};
const u256 ORDER_N = {{0xBFD25E8CD0364141ULL, 0xBAAEDCE6AF48A03BULL, 0xFFFFFFFFFFFFFFFEULL, 0xFFFFFFFFFFFFFFFFULL}};

u256 u256_from_be(const uint8_t b[32]) {
  u256 r;
  for (int i = 0; i < 4; i++) {
    uint64_t w = 0;
    for (int j = 0; j < 8; j++) w = (w << 8) | b[(3 - i) * 8 + j];
    r.v[i] = w;
  }
  return r;
}
void u256_to_be(uint8_t b[32], const u256 &a) {
  for (int i = 0; i < 4; i++)
    for (int j = 0; j < 8; j++) b[(3 - i) * 8 + j] = (uint8_t)(a.v[i] >> (56 - 8 * j));
}
u256 u256_from_u128(u128 x) { return u256{{(uint64_t)x, (uint64_t)(x >> 64), 0, 0}}; }
u256 u256_u64(uint64_t x) { return u256{{x, 0, 0, 0}}; }
int u256_cmp(const u256 &a, const u256 &b);
// st + count*stride >= n as plain integers (a key span that reaches the group order)
bool reaches_order(const u256 &st, const u256 &stride, uint64_t count) {
  u256 r;
  unsigned __int128 c = 0;
  for (int i = 0; i < 4; i++) {
    c += (unsigned __int128)stride.v[i] * count + st.v[i];
    r.v[i] = (uint64_t)c;
    c >>= 64;
  }
  return c != 0 || u256_cmp(r, ORDER_N) >= 0;
}
int u256_cmp(const u256 &a, const u256 &b) {
  for (int i = 3; i >= 0; i--) {
    if (a.v[i] < b.v[i]) return -1;
    if (a.v[i] > b.v[i]) return 1;
  }
  return 0;
}
bool u256_is_zero(const u256 &a) { return (a.v[0] | a.v[1] | a.v[2] | a.v[3]) == 0; }
uint64_t u256_add_raw(u256 &r, const u256 &a, const u256 &b) {
  u128 c = 0;
  for (int i = 0; i < 4; i++) {
    c += (u128)a.v[i] + b.v[i];
    r.v[i] = (uint64_t)c;
    c >>= 64;
  }
  return (uint64_t)c;
}
uint64_t u256_sub_raw(u256 &r, const u256 &a, const u256 &b) {
  uint64_t br = 0;
  for (int i = 0; i < 4; i++) {
    u128 t = (u128)a.v[i] - b.v[i] - br;
    r.v[i] = (uint64_t)t;
    br = (uint64_t)(t >> 64) & 1;
  }
  return br;
}
u256 sc_reduce(u256 a) {
  while (u256_cmp(a, ORDER_N) >= 0) u256_sub_raw(a, a, ORDER_N);
  return a;
}
u256 sc_add(const u256 &a, const u256 &b) {
  u256 r;
  uint64_t c = u256_add_raw(r, a, b);
  if (c || u256_cmp(r, ORDER_N) >= 0) u256_sub_raw(r, r, ORDER_N);
  return r;
}
u256 sc_neg(const u256 &a) {
  if (u256_is_zero(a)) return a;
  u256 r;
  u256_sub_raw(r, ORDER_N, a);
  return r;
}
u256 sc_sub(const u256 &a, const u256 &b) { return sc_add(a, sc_neg(b)); }
// a * m mod n for a < n, m < 2^64
u256 sc_mul_u64(const u256 &a, uint64_t m) {
  u256 r = u256_u64(0), x = a;
  while (m) {
    if (m & 1) r = sc_add(r, x);
    x = sc_add(x, x);
    m >>= 1;
  }
  return r;
}
// a * b mod n (double-and-add; only used per confirmed hit)
u256 sc_mul(const u256 &a, const u256 &b) {
  u256 r = u256_u64(0), x = a;
  for (int i = 0; i < 4; i++)
    for (int j = 0; j < 64; j++) {
      if ((b.v[i] >> j) & 1) r = sc_add(r, x);
      x = sc_add(x, x);
    }
  return r;
}
// a^-1 mod n (Fermat, a^(n-2); a != 0).  Host only, per chunk at most
u256 sc_inv(const u256 &a) {
  u256 e;
  u256_sub_raw(e, ORDER_N, u256_u64(2));
  u256 r = u256_u64(1), x = a;
  for (int i = 0; i < 4; i++)
    for (int j = 0; j < 64; j++) {
      if ((e.v[i] >> j) & 1) r = sc_mul(r, x);
      x = sc_mul(x, x);
    }
  return r;
}
void u256_to_limbs(uint32_t out[8], const u256 &a) {
  for (int i = 0; i < 4; i++) {
    out[2 * i] = (uint32_t)a.v[i];
    out[2 * i + 1] = (uint32_t)(a.v[i] >> 32);
  }
}
fe fe_of(const u256 &a) {
  fe r;
  u256_to_limbs(r.d, a);
  return r;
}
u256 u256_of(const fe &a) {
  u256 r;
  for (int i = 0; i < 4; i++) r.v[i] = (uint64_t)a.d[2 * i] | ((uint64_t)a.d[2 * i + 1] << 32);
  return r;
}

// ==============================================================================================
// libbloom2 sizing, exactly as bloom/bloom.cpp:154-187 computes it (long double, bpe as double)
// ==============================================================================================
bloom_desc bloom_size(uint64_t entries) {
  long double num = -logl((long double)0.000001);
  long double denom = 0.480453013918201;
  double bpe = (double)(num / denom);
  long double allbits = (long double)entries * bpe;
  bloom_desc d;
  memset(&d, 0, sizeof d);
  d.bits = (uint64_t)allbits;
  d.bytes = d.bits / 8 + ((d.bits % 8) ? 1 : 0);
  d.hashes = (uint32_t)(uint8_t)ceil(0.693147180559945 * bpe);
  d.recip = ~0ULL / d.bits;
  d.stride = d.bytes;
  return d;
}
// keyhunt's entry count rule: initBloomFilter uses max(10000, items) (keyhunt.cpp:7608)
uint64_t bloom_entries(uint64_t items) { return items <= 10000 ? 10000 : items; }

void host_bloom_hash(const uint8_t *buf, int len, uint64_t &a, uint64_t &b) {
  if (len == 32) {
    uint64_t in[4];
    for (int k = 0; k < 4; k++) {
      uint64_t v = 0;
      for (int q = 7; q >= 0; q--) v = (v << 8) | buf[8 * k + q];
      in[k] = v;
    }
    a = xxh64_32(in, KH_BLOOM_SEED);
    b = xxh64_32(in, a);
  } else {  // 20 bytes, or a shorter hash160 prefix (vanity)
    uint8_t p[20] = {0};
    memcpy(p, buf, (size_t)std::min(len, 20));
    uint32_t w[5];
    for (int k = 0; k < 5; k++)
      w[k] = (uint32_t)p[4 * k] | ((uint32_t)p[4 * k + 1] << 8) | ((uint32_t)p[4 * k + 2] << 16) |
             ((uint32_t)p[4 * k + 3] << 24);
    if (len == 20) {
      a = xxh64_20(w, KH_BLOOM_SEED);
      b = xxh64_20(w, a);
    } else {
      a = xxh64_prefix(w, (uint32_t)len, KH_BLOOM_SEED);
      b = xxh64_prefix(w, (uint32_t)len, a);
    }
  }
}
void host_bloom_add(uint8_t *bf, const bloom_desc &d, const uint8_t *buf, int len) {
  uint64_t a, b;
  host_bloom_hash(buf, len, a, b);
  uint64_t h = a;
  for (uint32_t i = 0; i < d.hashes; i++) {
    uint64_t x = h % d.bits;
    bf[x >> 3] |= (uint8_t)(1u << (x & 7));
    h += b;
  }
}
bool host_bloom_check(const uint8_t *bf, const bloom_desc &d, const uint8_t *buf, int len) {
  uint64_t a, b;
  host_bloom_hash(buf, len, a, b);
  uint64_t h = a;
  for (uint32_t i = 0; i < d.hashes; i++) {
    uint64_t x = h % d.bits;
    if (!((bf[x >> 3] >> (x & 7)) & 1)) return false;
    h += b;
  }
  return true;
}

// searchbinary (keyhunt.cpp:3065-3089): the reference's own midpoint loop
bool searchbinary(const uint8_t *rows, int64_t n, const uint8_t *key, int width, int key_off) {
  int64_t half = n, min = 0, max = n, cur = 0;
  while (half >= 1) {
    half = (max - min) / 2;
    int c = memcmp(key + key_off, rows + (cur + half) * width, width);
    if (c == 0) return true;
    if (c < 0)
      max = max - half;
    else
      min = min + half;
    cur = min;
  }
  return false;
}

// ==============================================================================================
// host EC with the comb table (the same table the setup kernel reads)
// ==============================================================================================
ge G_POINT() {
  ge g;
  const uint64_t gx[4] = {0x59F2815B16F81798ULL, 0x029BFCDB2DCE28D9ULL, 0x55A06295CE870B07ULL, 0x79BE667EF9DCBBACULL};
  const uint64_t gy[4] = {0x9C47D08FFB10D4B8ULL, 0xFD17B448A6855419ULL, 0x5DA4FBFC0E1108A8ULL, 0x483ADA7726A3C465ULL};
  fe_from_u64(g.x, gx);
  fe_from_u64(g.y, gy);
  return g;
}

struct comb_table {
  std::vector<ge> t;  // 32 * 256 (entry v = 0 unused)
  void build() {
    t.assign(32 * 256, ge{});
    ge base = G_POINT();
    for (int j = 0; j < 32; j++) {
      t[j * 256 + 1] = base;
      ge_double(t[j * 256 + 2], base);
      for (int v = 3; v < 256; v++) ge_add(t[j * 256 + v], t[j * 256 + v - 1], base);
      if (j < 31) {
        ge b = base;
        for (int k = 0; k < 8; k++) ge_double(b, b);
        base = b;
      }
    }
  }
  // k*G (k reduced mod n, k != 0); returns false for k == 0
  bool mult(ge &r, const u256 &k_in) const {
    u256 k = sc_reduce(k_in);
    if (u256_is_zero(k)) return false;
    gej acc;
    acc.inf = true;
    for (int j = 0; j < 32; j++) {
      uint32_t v = (uint32_t)(k.v[j >> 3] >> ((j & 7) * 8)) & 0xFF;
      if (v) gej_add_ge(acc, t[j * 256 + v]);
    }
    gej_to_ge(r, acc);
    return true;
  }
};

// Montgomery-trick batch inversion (IntGroup::ModInv); zero elements are skipped (left 0)
void batch_inv(std::vector<fe> &a) {
  size_t n = a.size();
  std::vector<fe> pre(n);
  fe acc;
  fe_set_u32(acc, 1);
  for (size_t i = 0; i < n; i++) {
    if (!fe_is_zero(a[i])) fe_mul(acc, acc, a[i]);
    pre[i] = acc;
  }
  fe inv;
  fe_inv(inv, acc);
  for (size_t i = n; i-- > 0;) {
    if (fe_is_zero(a[i])) continue;
    fe prev;
    if (i == 0)
      fe_set_u32(prev, 1);
    else
      prev = pre[i - 1];
    fe t;
    fe_mul(t, inv, prev);
    fe_mul(inv, inv, a[i]);
    a[i] = t;
  }
}

struct timing {
  uint64_t launches = 0, points = 0;
  double ms = 0;
};

}  // namespace

// ==============================================================================================
// context
// ==============================================================================================
struct kh_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  // BSGS rounds: the second check and the candidate copies of round r run on this high-priority
  // stream, so they start alongside round r+1's walk instead of in front of it
  hipStream_t side = nullptr;
  std::string err;
  comb_table comb;
  uint32_t *d_comb = nullptr;

  // lanes: lanes_max for the 1024-point-group walks and the BSGS giant walk; lanes_hb for the
  // address family's 4096-point groups (several waves per SIMD slot in one launch, DESIGN.md §2
  // "Launch geometry").  kh_set_geometry(lanes != 0) sets both.
  uint32_t lanes_max = 1u << 18;
  uint32_t lanes_hb = KH_LANES_HB;
  uint32_t lanes_bsgs = KH_BSGS_LANES;  // the BSGS walk's large calls
  // lanes the BSGS walk's large calls use once the context's first large call has timed the two
  // candidates against each other (bsgs_calibrated); lanes_force: one call's forced count
  uint32_t lanes_pick = 0, lanes_force = 0;
  uint32_t lanes_used = 0;  // lanes the last large-group BSGS call walked (the calibration checks it)
  bool bsgs_calibrated = false;
  // giant points/s of the placement calibration's candidates (stage 0: the pad, 1: layer 1):
  // [2s] the one kept, [2s + 1] the best other one; cal_stage: stages decided so far
  double cal_rate[4] = {0, 0, 0, 0};
  int cal_stage = 0;
  uint64_t cal_moved_bases = 0;  // bases the last KH_CAL_MOVE stage walked
  uint32_t cal_deferred = 0;      // eligible calls walked uncalibrated (KH_CAL_DEFER)
  bool burned = false;            // KH_BURN_MS ran before this context's first large BSGS call
  double burn_ms = 0;
  uint32_t groups_per_launch = 0;
  uint32_t lanes_alloc = 0;
  int scratch_h = 0;  // inversion-pad entries per lane in d_scratch
  uint32_t pad_skew = 0;  // lanes of gap after each pad row (KH_PAD_SKEW, read when the pad is allocated)
  // continuous BSGS lanes kept across kh_bsgs_scan calls: valid while the lane centres sit at the
  // first group of the call that would start at cont_next (same target, lanes and group size)
  bool cont_valid = false;
  int cont_kind = 0;        // 0: BSGS giant walk (target cont_tgt), 1: kh_scan (walk mode cont_km, stride)
  u256 cont_next{};
  u256 cont_stride{};
  uint32_t cont_L = 0, cont_tgt = 0;
  int cont_H = 0, cont_km = 0;
  uint32_t *d_q = nullptr;  // the current BSGS target {x[8], y[8]}
  uint32_t *d_cx = nullptr, *d_cy = nullptr, *d_scalars = nullptr;
  uint4 *d_scratch = nullptr;
  void *d_scratch_base = nullptr;  // the pad's allocation (d_scratch sits KH_PAD_OFFSET bytes into it)
  uint64_t pad_offset = 0;
  std::vector<uint32_t> h_scalars;

  // walk delta tables: key -> device table ((H+1) x 16 words)
  std::vector<std::pair<std::string, uint32_t *>> tables;

  // hits
  uint32_t hit_cap = 1u << 16;
  uint32_t *d_hit_count = nullptr;
  uint32_t *d_zero_flag = nullptr;  // k_setup's progression mode: a lane scalar was 0 mod n
  kh_dev_hit *d_hits = nullptr;
  std::vector<kh_dev_hit> h_hits;

  // address targets
  std::vector<uint8_t> rows;  // sorted, 20 B each
  uint64_t n_rows = 0;
  // vanity targets (kh_set_vanity): hash160 ranges [A, B] (40 B each), bloom keyed on A's prefix
  bool vanity = false;
  std::vector<uint8_t> v_ranges;
  uint32_t probe_len = 20;
  uint32_t rmd_batch = 0;  // kh_set_rmd_batch: 0 = the ordinary walk, else the reference's group < 1024
  bloom_desc tbd{};
  uint64_t t_entries = 0;  // the target bloom's struct bloom `entries`
  std::vector<uint8_t> h_tbloom;
  uint8_t *d_tbloom = nullptr;
  uint4 *d_tblk = nullptr;  // blocked target filter (exact targets only)
  uint32_t tblocks = 0;

  // bsgs
  uint32_t l1_layout = KH_LAYER1_BLOCKED;
  uint32_t bloom_mult = 1;   // -z (FLAGBLOOMMULTIPLIER) for the BSGS shards, kh_bsgs_set_bloom_multiplier
  bool bsgs_ready = false, bsgs_built = false;
  kh_bsgs_info info{};
  bloom_desc bd[3]{};
  bloom_desc bd_ref1{};      // layer 1 in the reference layout (what its files hold)
  uint64_t entries[3]{};     // bloom_init2 entries per layer (file headers)
  uint8_t *d_bl[3] = {nullptr, nullptr, nullptr};
  std::vector<uint8_t> h_bl[3];  // layers 2 and 3 on the host for refinement (index 1, 2)
  std::vector<uint8_t> h_rows;   // sorted 16-byte bsgs_xvalue rows
  std::vector<ge> amp2, amp3;
  std::vector<ge> targets;
  std::vector<uint8_t> found;
  uint64_t candidates = 0;
  // parity hook (kh_bsgs_log_candidates): every first-level candidate of the scans that follow
  bool log_cands = false;
  bool base_check = false;  // kh_bsgs_set_base_check: the daemon's per-base Q == base*G test
  std::vector<uint64_t> cand_log_base;
  std::vector<uint32_t> cand_log_a, cand_log_mask;
  uint64_t second_hits = 0;          // layer-2 positives of the second check (all candidates)
  // second check on the GPU (k_refine) unless KH_REFINE=host
  bool refine_host = false;
  uint32_t *d_amp2 = nullptr;        // 32 x {x[8], y[8]}
  uint32_t *d_ref_start = nullptr;   // 8 limbs
  uint32_t *d_ref_list = nullptr;    // list mode bases
  uint32_t *h_ref_list = nullptr;    // their pinned staging copy
  uint64_t ref_list_cap = 0;

  // timing
  hipEvent_t ev_a = nullptr, ev_b = nullptr;
  timing tm[5];

  // pipelined BSGS rounds: double-buffered hit buffers, pinned host mirrors, host scalar arrays
  uint32_t *d_cnt2[2] = {nullptr, nullptr};
  kh_dev_hit *d_hits2[2] = {nullptr, nullptr};
  uint32_t *h_cnt2[2] = {nullptr, nullptr};
  kh_dev_hit *h_hits2[2] = {nullptr, nullptr};
  uint32_t cand_cap = 1u << 16;  // candidates per round; grown (and the round redone) on overflow
  uint32_t *h_scal2[2] = {nullptr, nullptr};
  uint32_t h_scal_cap = 0;
  hipEvent_t ev_round[2][4] = {{nullptr, nullptr, nullptr, nullptr}, {nullptr, nullptr, nullptr, nullptr}};
  unsigned refine_threads = 0;

  ~kh_ctx();
};

#define HIPCHK(ctx, call)                                                                    \
  do {                                                                                       \
    hipError_t e_ = (call);                                                                  \
    if (e_ != hipSuccess) {                                                                  \
      (ctx)->err = std::string(#call) + ": " + hipGetErrorString(e_);                        \
      return KH_E_HIP;                                                                       \
    }                                                                                        \
  } while (0)

kh_ctx::~kh_ctx() {
  (void)hipSetDevice(device);
  if (stream) (void)hipStreamSynchronize(stream);
  (void)hipFree(d_comb);
  (void)hipFree(d_cx);
  (void)hipFree(d_cy);
  (void)hipFree(d_scalars);
  (void)hipFree(d_scratch_base);
  (void)hipFree(d_q);
  for (auto &t : tables) (void)hipFree(t.second);
  (void)hipFree(d_hit_count);
  (void)hipFree(d_zero_flag);
  (void)hipFree(d_hits);
  (void)hipFree(d_tbloom);
  (void)hipFree(d_tblk);
  for (int i = 0; i < 3; i++) (void)hipFree(d_bl[i]);
  (void)hipFree(d_amp2);
  (void)hipFree(d_ref_start);
  (void)hipFree(d_ref_list);
  if (h_ref_list) (void)hipHostFree(h_ref_list);
  for (int i = 0; i < 2; i++) {
    (void)hipFree(d_cnt2[i]);
    (void)hipFree(d_hits2[i]);
    if (h_cnt2[i]) (void)hipHostFree(h_cnt2[i]);
    if (h_hits2[i]) (void)hipHostFree(h_hits2[i]);
    if (h_scal2[i]) (void)hipHostFree(h_scal2[i]);
    for (int j = 0; j < 4; j++)
      if (ev_round[i][j]) (void)hipEventDestroy(ev_round[i][j]);
  }
  if (ev_a) (void)hipEventDestroy(ev_a);
  if (ev_b) (void)hipEventDestroy(ev_b);
  if (side) {
    (void)hipStreamSynchronize(side);
    (void)hipStreamDestroy(side);
  }
  if (stream) (void)hipStreamDestroy(stream);
}

namespace {

// lane centres for L lanes and an inversion pad of H rows per lane (walk_pad_rows: half the group for
// the sparse-pad walks)
// Device memory for the randomly probed layer-1 filter (which = 1) and the giant walk's inversion pad
// (which = 2).  KH_CONTIG=<mask> asks for physically contiguous memory (hipDeviceMallocContiguous)
// for an A/B; the default is an ordinary allocation: contiguous layer 1 + pad walked 35.7 / 34.5 /
// 36.0 G giant points/s against 40.0 / 39.7 / 37.4 ordinary, interleaved in the bench's BSGS leg
// (profiles/r05an_bench_contig_ab.json)
hipError_t dev_alloc(void **p, size_t bytes, int which) {
  static const int mask = [] {
    const char *e = getenv("KH_CONTIG");
    return e ? atoi(e) : 0;
  }();
  static const bool log = getenv("KH_DEBUG_ALLOC") != nullptr;  // diagnostics only: stderr
  if (mask & which) {
    if (hipExtMallocWithFlags(p, bytes, hipDeviceMallocContiguous) == hipSuccess) {
      if (log) fprintf(stderr, "[kh] %zu bytes (kind %d): contiguous\n", bytes, which);
      return hipSuccess;
    }
    (void)hipGetLastError();
    *p = nullptr;
    if (log) fprintf(stderr, "[kh] %zu bytes (kind %d): contiguous refused\n", bytes, which);
  }
  return hipMalloc(p, bytes);
}

// KH_PAD_SKEW=<lanes>: a gap of that many lane entries after every pad row, so rows sit L + skew
// entries apart instead of a power of two (A/B knob; 0 by default)
static uint32_t env_pad_skew() {
  const char *e = getenv("KH_PAD_SKEW");
  return e ? (uint32_t)strtoul(e, nullptr, 0) : 0u;
}

// KH_PAD_SWZ=1: rotate each pad row's columns by workgroup (walk_args::pad_swz), when the lanes allow
static uint32_t pad_swizzle(uint32_t L) {
  const char *e = getenv("KH_PAD_SWZ");  // read per launch: A/B tools switch it inside one process
  return e && atoi(e) && L % 2048 == 0 ? 1u : 0u;
}

// KH_PAD_OFFSET=<bytes>: the pad starts that far (rounded down to 256 B) into its allocation (A/B knob)
static uint64_t env_pad_offset() {
  const char *e = getenv("KH_PAD_OFFSET");
  return e ? strtoull(e, nullptr, 0) & ~255ull : 0ull;
}

int ensure_lanes(kh_ctx *c, uint32_t L, int H = KH_WALK_H) {
  if (L <= c->lanes_alloc && H <= c->scratch_h && c->pad_skew == env_pad_skew() && c->pad_offset == env_pad_offset())
    return KH_OK;
  L = std::max(L, c->lanes_alloc);
  H = std::max(H, c->scratch_h);
  c->cont_valid = false;
  (void)hipFree(c->d_cx);
  (void)hipFree(c->d_cy);
  (void)hipFree(c->d_scalars);
  (void)hipFree(c->d_scratch_base);
  c->d_cx = c->d_cy = c->d_scalars = nullptr;
  c->d_scratch = nullptr;
  c->d_scratch_base = nullptr;
  c->lanes_alloc = 0;
  c->scratch_h = 0;
  c->pad_skew = env_pad_skew();
  HIPCHK(c, hipMalloc(&c->d_cx, (size_t)L * 32));
  HIPCHK(c, hipMalloc(&c->d_cy, (size_t)L * 32));
  HIPCHK(c, hipMalloc(&c->d_scalars, (size_t)L * 32));
  c->pad_offset = env_pad_offset();
  HIPCHK(c, dev_alloc(&c->d_scratch_base, ((size_t)L + c->pad_skew) * H * 32 + c->pad_offset, 2));
  c->d_scratch = reinterpret_cast<uint4 *>(static_cast<uint8_t *>(c->d_scratch_base) + c->pad_offset);
  c->lanes_alloc = L;
  c->scratch_h = H;
  return KH_OK;
}

// delta table T[i] = (i+1)*D, i < H, and T[H] = 2H*D, for D = d*G (d a scalar, may be "negative")
// jump > 1 (interleaved lanes): the last entry is the jump between a lane's groups, jump*2H*D
int get_table(kh_ctx *c, const u256 &d, const uint32_t **out, const int H = KH_WALK_H, uint64_t jump = 1) {
  uint8_t be[32];
  u256_to_be(be, d);
  std::string key((const char *)be, 32);
  key += std::to_string(H) + "/" + std::to_string(jump);
  for (auto &t : c->tables)
    if (t.first == key) {
      *out = t.second;
      return KH_OK;
    }
  std::vector<uint32_t> h((size_t)(H + 1) * 16);
  ge D;
  if (!c->comb.mult(D, d)) {
    c->err = "delta scalar is 0";
    return KH_E_ARG;
  }
  ge cur = D;
  for (int i = 0; i < H; i++) {
    if (i == 1) ge_double(cur, D);
    if (i >= 2) ge_add(cur, cur, D);
    memcpy(&h[(size_t)i * 16], cur.x.d, 32);
    memcpy(&h[(size_t)i * 16 + 8], cur.y.d, 32);
  }
  ge d2;
  if (jump == 1) {
    ge_double(d2, cur);  // 2H * D
  } else {
    u256 e = u256_u64(0), x = d;  // (jump * 2H) * d mod n by double-and-add
    for (uint64_t k = jump * 2 * (uint64_t)H; k; k >>= 1) {
      if (k & 1) e = sc_add(e, x);
      x = sc_add(x, x);
    }
    if (!c->comb.mult(d2, e)) {
      c->err = "group jump scalar is 0";
      return KH_E_ARG;
    }
  }
  memcpy(&h[(size_t)H * 16], d2.x.d, 32);
  memcpy(&h[(size_t)H * 16 + 8], d2.y.d, 32);
  uint32_t *dev = nullptr;
  HIPCHK(c, hipMalloc(&dev, h.size() * 4));
  HIPCHK(c, hipMemcpy(dev, h.data(), h.size() * 4, hipMemcpyHostToDevice));
  c->tables.push_back({key, dev});
  *out = dev;
  return KH_OK;
}

// Lane centres: C_g = [Q +] s_g*G.  s: L scalars (already reduced, non-zero)
int run_setup(kh_ctx *c, const std::vector<u256> &s, const ge *q) {
  uint32_t L = (uint32_t)s.size();
  c->cont_valid = false;  // the lane centres are about to be replaced
  int r = ensure_lanes(c, L);
  if (r) return r;
  c->h_scalars.resize((size_t)L * 8);
  for (uint32_t g = 0; g < L; g++) u256_to_limbs(&c->h_scalars[(size_t)g * 8], s[g]);
  HIPCHK(c, hipMemcpyAsync(c->d_scalars, c->h_scalars.data(), (size_t)L * 32, hipMemcpyHostToDevice, c->stream));
  setup_args A;
  memset(&A, 0, sizeof A);
  A.scalars = c->d_scalars;
  A.comb = c->d_comb;
  A.L = L;
  A.cx = c->d_cx;
  A.cy = c->d_cy;
  uint32_t *dq = nullptr;
  if (q) {
    HIPCHK(c, hipMalloc(&dq, 64));
    HIPCHK(c, hipMemcpyAsync(dq, q->x.d, 32, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(dq + 8, q->y.d, 32, hipMemcpyHostToDevice, c->stream));
    A.q = dq;
    A.has_q = 1;
  }
  HIPCHK(c, hipEventRecord(c->ev_a, c->stream));
  HIPCHK(c, launch_setup(A, c->stream));
  HIPCHK(c, hipEventRecord(c->ev_b, c->stream));
  HIPCHK(c, hipEventSynchronize(c->ev_b));
  float ms = 0;
  (void)hipEventElapsedTime(&ms, c->ev_a, c->ev_b);
  c->tm[4].launches++;
  c->tm[4].ms += ms;
  c->tm[4].points += L;
  if (dq) (void)hipFree(dq);
  return KH_OK;
}

// Lane centres C_g = s_g * G for the progression s_g = s0 + g * step (mod n), g < L: the scalars are
// derived on the device (k_setup's prog mode), so a chunk whose lanes restart (-R, the first chunk)
// costs no host loop over 2^20 lanes and no 32 MB upload.  A lane scalar of 0 (its centre would be the
// point at infinity) fails the call, as the host check did.
int run_setup_prog(kh_ctx *c, const u256 &s0, const u256 &step, uint32_t L) {
  c->cont_valid = false;
  int r = ensure_lanes(c, L);
  if (r) return r;
  setup_args A;
  memset(&A, 0, sizeof A);
  A.comb = c->d_comb;
  A.L = L;
  A.cx = c->d_cx;
  A.cy = c->d_cy;
  A.prog = 1;
  u256_to_limbs(A.s0, s0);
  u256_to_limbs(A.step, step);
  A.zero_flag = c->d_zero_flag;
  HIPCHK(c, hipMemsetAsync(c->d_zero_flag, 0, 4, c->stream));
  HIPCHK(c, hipEventRecord(c->ev_a, c->stream));
  HIPCHK(c, launch_setup(A, c->stream));
  HIPCHK(c, hipEventRecord(c->ev_b, c->stream));
  uint32_t zero = 0;
  HIPCHK(c, hipMemcpyAsync(&zero, c->d_zero_flag, 4, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  float ms = 0;
  (void)hipEventElapsedTime(&ms, c->ev_a, c->ev_b);
  c->tm[4].launches++;
  c->tm[4].ms += ms;
  c->tm[4].points += L;
  if (zero) {
    c->err = "lane centre scalar is 0 mod n";
    return KH_E_ARG;
  }
  return KH_OK;
}

struct job_geom {
  uint32_t L;
  uint64_t gpl;  // groups per lane in the job
};
// lanes cover total_groups groups; gpl must divide `gpl_divides` when non-zero
job_geom plan(kh_ctx *c, uint64_t total_groups, uint64_t gpl_divides, uint32_t lanes = 0) {
  job_geom g;
  if (!lanes) lanes = c->lanes_max;
  uint64_t gpl = (total_groups + lanes - 1) / lanes;
  if (gpl == 0) gpl = 1;
  if (gpl_divides) {
    while (gpl < gpl_divides && gpl_divides % gpl) gpl++;
    if (gpl > gpl_divides) gpl = gpl_divides;
  }
  g.gpl = gpl;
  g.L = (uint32_t)((total_groups + gpl - 1) / gpl);
  return g;
}

// walk all lanes through `gpl` groups in launches of groups_per_launch; kind = timing slot
int run_walk(kh_ctx *c, int mode, int kind, walk_args A, uint64_t gpl, uint32_t default_gpl_launch,
             int H = KH_WALK_H) {
  uint32_t per = c->groups_per_launch ? c->groups_per_launch : default_gpl_launch;
  for (uint64_t gb = 0; gb < gpl; gb += per) {
    A.group_base = gb;
    A.groups = (uint32_t)std::min<uint64_t>(per, gpl - gb);
    HIPCHK(c, hipEventRecord(c->ev_a, c->stream));
    HIPCHK(c, launch_walk(mode, A, c->stream, H));
    HIPCHK(c, hipEventRecord(c->ev_b, c->stream));
    HIPCHK(c, hipEventSynchronize(c->ev_b));
    float ms = 0;
    (void)hipEventElapsedTime(&ms, c->ev_a, c->ev_b);
    c->tm[kind].launches++;
    c->tm[kind].ms += ms;
    c->tm[kind].points += (uint64_t)A.L * A.groups * 2 * H;
  }
  return KH_OK;
}

int fetch_hits(kh_ctx *c, uint32_t &n) {
  uint32_t cnt = 0;
  HIPCHK(c, hipMemcpyAsync(&cnt, c->d_hit_count, 4, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  if (cnt > c->hit_cap) {
    c->err = "device hit buffer overflow";
    return KH_E_OVERFLOW;
  }
  c->h_hits.resize(cnt);
  if (cnt) {
    HIPCHK(c, hipMemcpyAsync(c->h_hits.data(), c->d_hits, (size_t)cnt * sizeof(kh_dev_hit), hipMemcpyDeviceToHost,
                             c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
  }
  n = cnt;
  return KH_OK;
}

}  // namespace

// ==============================================================================================
// C ABI
// ==============================================================================================
// f(lo, hi) over [0, n) split across up to `threads` host threads (serial below 2^16 items)
template <class F>
void parallel_for(uint64_t n, unsigned threads, F f) {
  if (n < (1u << 16) || threads <= 1) {
    f(0, n);
    return;
  }
  const uint64_t per = (n + threads - 1) / threads;
  std::vector<std::thread> th;
  for (unsigned t = 0; t < threads; t++) {
    const uint64_t lo = t * per, hi = std::min<uint64_t>(n, lo + per);
    if (lo >= hi) break;
    th.emplace_back(f, lo, hi);
  }
  for (auto &x : th) x.join();
}

extern "C" {

int kh_abi_version(void) { return KH_ABI_VERSION; }

const char *kh_strerror(int code) {
  switch (code) {
    case KH_OK: return "ok";
    case KH_E_ARG: return "invalid argument";
    case KH_E_HIP: return "HIP runtime error";
    case KH_E_NOMEM: return "out of memory";
    case KH_E_STATE: return "call out of order";
    case KH_E_OVERFLOW: return "output buffer too small";
    case KH_E_BSGS_N: return "BSGS n has no exact square root or sqrt(n) is not a multiple of 1024";
    case KH_E_RANGE: return "the given range is small";
    case KH_E_IO: return "file missing, short or not writable";
    case KH_E_FORMAT: return "file does not match the BSGS geometry or its checksum";
    default: return "unknown error";
  }
}

const char *kh_last_error(kh_ctx *ctx) { return ctx ? ctx->err.c_str() : "no context"; }

int kh_device_count(int *count) {
  if (!count) return KH_E_ARG;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
  *count = n;
  return KH_OK;
}

int kh_device_memory(int device, uint64_t *free_bytes, uint64_t *total_bytes) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n) return KH_E_HIP;
  if (hipSetDevice(device) != hipSuccess) return KH_E_HIP;
  size_t f = 0, t = 0;
  if (hipMemGetInfo(&f, &t) != hipSuccess) return KH_E_HIP;
  if (free_bytes) *free_bytes = f;
  if (total_bytes) *total_bytes = t;
  return KH_OK;
}

int kh_open(int device, kh_ctx **out) {
  if (!out) return KH_E_ARG;
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n) return KH_E_HIP;
  kh_ctx *c = new kh_ctx();
  c->device = device;
  auto fail = [&](int r) {
    delete c;
    return r;
  };
  if (hipSetDevice(device) != hipSuccess) return fail(KH_E_HIP);
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) return fail(KH_E_HIP);
  {
    int lo = 0, hi = 0;
    if (hipDeviceGetStreamPriorityRange(&lo, &hi) != hipSuccess) lo = hi = 0;
    if (hipStreamCreateWithPriority(&c->side, hipStreamNonBlocking, hi) != hipSuccess) return fail(KH_E_HIP);
  }
  if (hipEventCreate(&c->ev_a) != hipSuccess || hipEventCreate(&c->ev_b) != hipSuccess) return fail(KH_E_HIP);
  c->comb.build();
  std::vector<uint32_t> h((size_t)32 * 256 * 16, 0);
  for (int i = 0; i < 32 * 256; i++) {
    if (i % 256 == 0) continue;
    memcpy(&h[(size_t)i * 16], c->comb.t[i].x.d, 32);
    memcpy(&h[(size_t)i * 16 + 8], c->comb.t[i].y.d, 32);
  }
  if (hipMalloc(&c->d_comb, h.size() * 4) != hipSuccess) return fail(KH_E_NOMEM);
  if (hipMemcpy(c->d_comb, h.data(), h.size() * 4, hipMemcpyHostToDevice) != hipSuccess) return fail(KH_E_HIP);
  // test hook: a small initial BSGS candidate buffer exercises the grow-and-redo path
  if (const char *e = getenv("KH_CAND_CAP")) c->cand_cap = std::max<uint32_t>(1, (uint32_t)strtoul(e, nullptr, 0));
  // A/B and parity hook: KH_REFINE=host runs the second check on host threads instead of k_refine
  if (const char *e = getenv("KH_REFINE")) c->refine_host = strcmp(e, "host") == 0;
  if (hipMalloc(&c->d_hit_count, 4) != hipSuccess) return fail(KH_E_NOMEM);
  if (hipMalloc(&c->d_zero_flag, 4) != hipSuccess) return fail(KH_E_NOMEM);
  if (hipMalloc(&c->d_hits, (size_t)c->hit_cap * sizeof(kh_dev_hit)) != hipSuccess) return fail(KH_E_NOMEM);
  *out = c;
  return KH_OK;
}

int kh_close(kh_ctx *ctx) {
  delete ctx;
  return KH_OK;
}

int kh_release_walk(kh_ctx *ctx) {
  if (!ctx) return KH_E_ARG;
  (void)hipSetDevice(ctx->device);
  (void)hipDeviceSynchronize();
  (void)hipFree(ctx->d_cx);
  (void)hipFree(ctx->d_cy);
  (void)hipFree(ctx->d_scalars);
  (void)hipFree(ctx->d_scratch_base);
  ctx->d_cx = ctx->d_cy = ctx->d_scalars = nullptr;
  ctx->d_scratch = nullptr;
  ctx->d_scratch_base = nullptr;
  ctx->lanes_alloc = 0;
  ctx->scratch_h = 0;
  ctx->cont_valid = false;
  return KH_OK;
}

int kh_bsgs_geometry(kh_ctx *ctx, uint32_t *lanes, double rates[2]) {
  if (!ctx) return KH_E_ARG;
  if (lanes) *lanes = ctx->cal_stage >= 1 ? ctx->lanes_pick : 0;
  if (rates) {
    rates[0] = ctx->cal_rate[0];
    rates[1] = ctx->cal_rate[1];
  }
  return KH_OK;
}

int kh_bsgs_placement(kh_ctx *ctx, double rates[4]) {
  if (!ctx || !rates) return KH_E_ARG;
  for (int k = 0; k < 4; k++) rates[k] = ctx->cal_rate[k];
  return ctx->bsgs_calibrated ? 1 : 0;
}

// a fresh allocation for one device buffer: the new one is taken while the old is held, the contents
// copied, then the old one freed
static int move_buffer(kh_ctx *ctx, void **p, size_t bytes, int which) {
  if (!*p) return KH_OK;
  void *nb = nullptr;
  HIPCHK(ctx, which ? dev_alloc(&nb, bytes, which) : hipMalloc(&nb, bytes));
  HIPCHK(ctx, hipMemcpy(nb, *p, bytes, hipMemcpyDeviceToDevice));
  (void)hipFree(*p);
  *p = nb;
  return KH_OK;
}

int kh_debug_replace(kh_ctx *ctx, uint32_t which) {
  if (!ctx) return KH_E_ARG;
  (void)hipSetDevice(ctx->device);
  HIPCHK(ctx, hipDeviceSynchronize());
  int r = KH_OK;
  if ((which & 1) && ctx->d_bl[0])
    r = move_buffer(ctx, reinterpret_cast<void **>(&ctx->d_bl[0]), 256 * ctx->bd[0].stride + 4, 1);
  if (!r && (which & 2) && ctx->d_scratch_base) {  // the pad (no contents to keep)
    const size_t bytes = ((size_t)ctx->lanes_alloc + ctx->pad_skew) * ctx->scratch_h * 32 + ctx->pad_offset;
    void *nb = nullptr;
    HIPCHK(ctx, dev_alloc(&nb, bytes, 2));
    (void)hipFree(ctx->d_scratch_base);
    ctx->d_scratch_base = nb;
    ctx->d_scratch = reinterpret_cast<uint4 *>(static_cast<uint8_t *>(nb) + ctx->pad_offset);
  }
  if (!r && (which & 4)) {  // lane centres and scalars (the centres are kept: lanes may continue)
    const size_t bytes = (size_t)ctx->lanes_alloc * 32;
    r = move_buffer(ctx, reinterpret_cast<void **>(&ctx->d_cx), bytes, 0);
    if (!r) r = move_buffer(ctx, reinterpret_cast<void **>(&ctx->d_cy), bytes, 0);
    if (!r) r = move_buffer(ctx, reinterpret_cast<void **>(&ctx->d_scalars), bytes, 0);
  }
  if (!r && (which & 8)) {  // the walks' delta tables
    for (auto &t : ctx->tables) {
      const size_t H = (size_t)atoi(t.first.c_str() + 32);  // key: 32 scalar bytes, then "H/jump"
      void *q = t.second;
      r = move_buffer(ctx, &q, (H + 1) * 16 * 4, 0);
      if (r) break;
      t.second = static_cast<uint32_t *>(q);
    }
  }
  if (!r && (which & 32)) {  // the walk's stream: a new one (another hardware queue), then the old one destroyed
    hipStream_t ns = nullptr;
    HIPCHK(ctx, hipStreamCreateWithFlags(&ns, hipStreamNonBlocking));
    (void)hipStreamDestroy(ctx->stream);
    ctx->stream = ns;
  }
  if (!r && (which & 16)) {  // layers 2 and 3
    for (int l = 1; l < 3 && !r; l++)
      r = move_buffer(ctx, reinterpret_cast<void **>(&ctx->d_bl[l]), 256 * ctx->bd[l].stride + 4, 0);
  }
  return r;
}

int kh_debug_burn(kh_ctx *ctx, double ms) {
  if (!ctx || !(ms > 0)) return KH_E_ARG;
  (void)hipSetDevice(ctx->device);
  uint32_t *sink = ctx->d_zero_flag;
  const uint32_t iters = 1u << 16;
  HIPCHK(ctx, hipEventRecord(ctx->ev_a, ctx->stream));
  HIPCHK(ctx, launch_burn(iters, sink, ctx->stream));
  HIPCHK(ctx, hipEventRecord(ctx->ev_b, ctx->stream));
  HIPCHK(ctx, hipEventSynchronize(ctx->ev_b));
  float one = 0;
  (void)hipEventElapsedTime(&one, ctx->ev_a, ctx->ev_b);
  const int more = one > 0 ? (int)std::min(10000.0, ms / one) : 0;
  for (int k = 1; k < more; k++) HIPCHK(ctx, launch_burn(iters, sink, ctx->stream));  // left in flight
  ctx->burn_ms = one * std::max(1, more);
  return KH_OK;
}

int kh_debug_layout(kh_ctx *ctx, uint64_t out[8]) {
  if (!ctx || !out) return KH_E_ARG;
  out[0] = (uint64_t)(uintptr_t)ctx->d_bl[0];
  out[1] = ctx->d_bl[0] ? 256 * ctx->bd[0].stride + 4 : 0;
  out[2] = (uint64_t)(uintptr_t)ctx->d_scratch;
  out[3] = (uint64_t)ctx->lanes_alloc * ctx->scratch_h * 32;
  out[4] = (uint64_t)(uintptr_t)ctx->d_bl[1];
  out[5] = ctx->d_bl[1] ? 256 * ctx->bd[1].stride + 4 : 0;
  out[6] = ctx->lanes_alloc;
  out[7] = (uint64_t)ctx->scratch_h;
  return KH_OK;
}

int kh_set_geometry(kh_ctx *ctx, uint32_t lanes, uint32_t groups_per_launch) {
  if (!ctx) return KH_E_ARG;
  ctx->lanes_max = lanes ? lanes : (1u << 18);
  ctx->lanes_hb = lanes ? lanes : KH_LANES_HB;
  ctx->lanes_bsgs = lanes ? lanes : KH_BSGS_LANES;
  ctx->groups_per_launch = groups_per_launch;
  // an explicit geometry overrides an earlier calibration's pick (and a default one calibrates again)
  ctx->lanes_pick = 0;
  ctx->bsgs_calibrated = false;
  ctx->cal_stage = 0;
  for (double &x : ctx->cal_rate) x = 0;
  return KH_OK;
}

int kh_set_rmd_batch(kh_ctx *ctx, uint32_t group) {
  if (!ctx) return KH_E_ARG;
  if (group == 0 || group == 2 * KH_WALK_H) {
    ctx->rmd_batch = 0;
    return KH_OK;
  }
  if (group < 4 || group > 2 * KH_WALK_H || group % 4) {
    ctx->err = "rmd batch size: a multiple of 4 in [4, 1024] (keyhunt.cpp:815-829 clamps to that)";
    return KH_E_ARG;
  }
  ctx->rmd_batch = group;
  ctx->cont_valid = false;
  return KH_OK;
}

int kh_synchronize(kh_ctx *ctx) {
  if (!ctx) return KH_E_ARG;
  (void)hipSetDevice(ctx->device);
  HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
  HIPCHK(ctx, hipStreamSynchronize(ctx->side));
  return KH_OK;
}

// ---------------------------------------------------------------------------------------------
// address / rmd160 / xpoint
// ---------------------------------------------------------------------------------------------
// The blocked target filter the walk probes for exact targets (kh_kernels.hip tblk_probe): 16-byte
// blocks, KH_BLK_BITS_MUL x the reference bloom's bits; row words w = little-endian u32s of the
// 20 bytes: block (w0 * blocks) >> 32, bits from w1, w2 (, w3) as kh_blk_masks (kh_kernels.h).
static int upload_tblk(kh_ctx *c) {
  const uint64_t blocks = (c->tbd.bits * KH_BLK_BITS_MUL + 127) / 128;
  std::vector<uint32_t> words(blocks * 4, 0);
  for (uint64_t r = 0; r < c->n_rows; r++) {
    const uint8_t *p = &c->rows[r * 20];
    uint32_t w[4];
    for (int k = 0; k < 4; k++)
      w[k] = (uint32_t)p[4 * k] | ((uint32_t)p[4 * k + 1] << 8) | ((uint32_t)p[4 * k + 2] << 16) |
             ((uint32_t)p[4 * k + 3] << 24);
    const uint64_t blk = ((uint64_t)w[0] * blocks) >> 32;
    uint32_t m[4];
    kh_blk_masks(w[1], w[2], w[3], m);
    for (int k = 0; k < 4; k++) words[blk * 4 + k] |= m[k];
  }
  (void)hipFree(c->d_tblk);
  c->d_tblk = nullptr;
  c->tblocks = (uint32_t)blocks;
  HIPCHK(c, hipMalloc(&c->d_tblk, words.size() * 4));
  HIPCHK(c, hipMemcpy(c->d_tblk, words.data(), words.size() * 4, hipMemcpyHostToDevice));
  return KH_OK;
}

int kh_set_targets(kh_ctx *ctx, const uint8_t *rows, uint64_t n, uint64_t bloom_items) {
  if (!ctx || (!rows && n)) return KH_E_ARG;
  (void)hipSetDevice(ctx->device);
  std::vector<std::array<uint8_t, 20>> v(n);
  for (uint64_t i = 0; i < n; i++) memcpy(v[i].data(), rows + i * 20, 20);
  std::sort(v.begin(), v.end(), [](const std::array<uint8_t, 20> &a, const std::array<uint8_t, 20> &b) {
    return memcmp(a.data(), b.data(), 20) < 0;
  });
  ctx->rows.resize(n * 20);
  for (uint64_t i = 0; i < n; i++) memcpy(&ctx->rows[i * 20], v[i].data(), 20);
  ctx->n_rows = n;
  ctx->vanity = false;
  ctx->cont_valid = false;  // the next walk may need another pad (dense vs sparse): start its lanes again
  ctx->probe_len = 20;
  ctx->v_ranges.clear();
  ctx->t_entries = bloom_entries(bloom_items ? bloom_items : n);
  ctx->tbd = bloom_size(ctx->t_entries);
  ctx->h_tbloom.assign(ctx->tbd.bytes, 0);
  for (uint64_t i = 0; i < n; i++) host_bloom_add(ctx->h_tbloom.data(), ctx->tbd, &ctx->rows[i * 20], 20);
  (void)hipFree(ctx->d_tbloom);
  ctx->d_tbloom = nullptr;
  HIPCHK(ctx, hipMalloc(&ctx->d_tbloom, ctx->tbd.bytes + 4));
  HIPCHK(ctx, hipMemcpy(ctx->d_tbloom, ctx->h_tbloom.data(), ctx->tbd.bytes, hipMemcpyHostToDevice));
  return upload_tblk(ctx);
}

int kh_set_vanity(kh_ctx *ctx, const uint8_t *ranges, uint64_t n, uint32_t probe_len, uint64_t bloom_items) {
  if (!ctx || (!ranges && n) || probe_len == 0 || probe_len > 20) return KH_E_ARG;
  (void)hipSetDevice(ctx->device);
  ctx->v_ranges.assign(ranges, ranges + n * 40);
  ctx->rows.clear();
  ctx->n_rows = 0;
  ctx->vanity = true;
  ctx->cont_valid = false;  // a vanity walk writes the dense pad: never resume an exact-target walk's lanes
  ctx->probe_len = probe_len;
  (void)hipFree(ctx->d_tblk);  // prefixes probe the reference-layout bloom
  ctx->d_tblk = nullptr;
  // processOneVanity / readFileVanity (keyhunt.cpp:6970-7035): bloom over A's first probe_len bytes
  ctx->t_entries = bloom_entries(bloom_items ? bloom_items : n);
  ctx->tbd = bloom_size(ctx->t_entries);
  ctx->h_tbloom.assign(ctx->tbd.bytes, 0);
  for (uint64_t i = 0; i < n; i++) host_bloom_add(ctx->h_tbloom.data(), ctx->tbd, &ctx->v_ranges[i * 40], (int)probe_len);
  (void)hipFree(ctx->d_tbloom);
  ctx->d_tbloom = nullptr;
  HIPCHK(ctx, hipMalloc(&ctx->d_tbloom, ctx->tbd.bytes + 4));
  HIPCHK(ctx, hipMemcpy(ctx->d_tbloom, ctx->h_tbloom.data(), ctx->tbd.bytes, hipMemcpyHostToDevice));
  return upload_tblk(ctx);
}

int kh_scan_memory(uint64_t n_keys, uint32_t mode, uint32_t search, uint64_t *needed_bytes) {
  if (!needed_bytes || n_keys == 0) return KH_E_ARG;
  const bool endo = (mode & KH_MODE_ENDO) != 0;
  mode &= ~(uint32_t)KH_MODE_ENDO;
  if (mode > KH_MODE_ETH || search > KH_SEARCH_BOTH) return KH_E_ARG;
  int km = mode == KH_MODE_XPOINT ? KM_XPOINT
         : mode == KH_MODE_ETH ? KM_ETH
         : search == KH_SEARCH_COMPRESS ? KM_H160C
         : search == KH_SEARCH_UNCOMPRESS ? KM_H160U
                                          : KM_H160B;
  if (endo) km |= KM_ENDO;
  // kh_scan's choice at the default geometry (a chunk that reaches the order keeps the small groups,
  // which need less): exact targets, so -m xpoint probes the blocked filter with the sparse pad
  const int H = (km == KM_XPOINT || km == KM_H160C) && n_keys % (2 * KH_WALK_HB) == 0 ? KH_WALK_HB : KH_WALK_H;
  const uint64_t lanes = H == KH_WALK_HB ? KH_LANES_HB : (1u << 18);
  const uint64_t groups = (n_keys + 2 * H - 1) / (2 * H);
  const uint64_t gpl = (groups + lanes - 1) / lanes, L = (groups + gpl - 1) / gpl;
  *needed_bytes = L * (uint64_t)walk_pad_rows(km, true, H) * 32 + L * 32 * 3 + (512u << 10) +
                  (uint64_t)65536 * sizeof(kh_dev_hit);
  return KH_OK;
}

int kh_scan(kh_ctx *ctx, const uint8_t start[32], const uint8_t stride_be[32], uint64_t n_keys, uint32_t mode,
            uint32_t search, kh_hit *hits, uint32_t cap, uint32_t *n_hits) {
  if (!ctx || !start || !n_hits || n_keys == 0) return KH_E_ARG;
  // --rmd-batch-size below 1024: groups of zg slots (kh_set_rmd_batch, k_walk_zinv)
  const uint32_t zg = ctx->rmd_batch;
  if (!zg && n_keys % (2 * KH_WALK_H)) return KH_E_ARG;
  const bool endo = (mode & KH_MODE_ENDO) != 0;
  mode &= ~(uint32_t)KH_MODE_ENDO;
  if (mode > KH_MODE_ETH || search > KH_SEARCH_BOTH) return KH_E_ARG;
  if (zg && (mode == KH_MODE_XPOINT || ctx->vanity)) {
    ctx->err = "--rmd-batch-size applies to -m rmd160 (hash160 or -c eth) with exact targets only";
    return KH_E_ARG;
  }
  if (!ctx->d_tbloom) return KH_E_STATE;
  (void)hipSetDevice(ctx->device);
  if (zg) {
    // k_walk_zinv centres group m on offset zg/2 + m*zg and reaches it by C += T[H] from the previous
    // centre (or, a lane's first, by a scalar multiplication).  A centre whose key is 0 mod n -- offset
    // k0 = -start * stride^-1 mod n -- is the point at infinity, from which the reference builds its
    // group out of its own infinity representation; this engine does not restate that group.  The
    // groups before it are scanned (and their hits returned), then the call reports KH_E_RANGE.
    const u256 st0 = sc_reduce(u256_from_be(start));
    const u256 sd0 = stride_be ? sc_reduce(u256_from_be(stride_be)) : u256_u64(1);
    if (u256_is_zero(sd0)) return KH_E_ARG;
    const u256 k0 = u256_cmp(sd0, u256_u64(1)) == 0 ? sc_neg(st0) : sc_mul(sc_neg(st0), sc_inv(sd0));
    const uint64_t half = zg / 2, groups = (n_keys + zg - 1) / zg;
    if (k0.v[1] == 0 && k0.v[2] == 0 && k0.v[3] == 0 && k0.v[0] >= half && (k0.v[0] - half) % zg == 0 &&
        (k0.v[0] - half) / zg < groups) {
      const uint64_t m_bad = (k0.v[0] - half) / zg;
      uint32_t nh = 0;
      int r0 = KH_OK;
      if (m_bad) {
        r0 = kh_scan(ctx, start, stride_be, m_bad * zg, mode | (endo ? KH_MODE_ENDO : 0), search, hits, cap, &nh);
        if (r0 && r0 != KH_E_OVERFLOW) return r0;
      }
      *n_hits = nh;
      ctx->err = "--rmd-batch-size below 1024: a group centred on the key 0 mod n (the reference builds it "
                 "from its point at infinity); the groups before it were scanned";
      return r0 == KH_E_OVERFLOW ? r0 : KH_E_RANGE;
    }
  }
  int km = mode == KH_MODE_XPOINT ? KM_XPOINT
         : mode == KH_MODE_ETH ? KM_ETH
         : search == KH_SEARCH_COMPRESS ? KM_H160C
         : search == KH_SEARCH_UNCOMPRESS ? KM_H160U
                                          : KM_H160B;
  if (endo) km |= KM_ENDO;
  u256 st = sc_reduce(u256_from_be(start));
  u256 stride = stride_be ? sc_reduce(u256_from_be(stride_be)) : u256_u64(1);
  if (u256_is_zero(stride)) return KH_E_ARG;
  // xpoint and compressed rmd160/address (configs 2-3) walk 4096-point groups when the chunk holds
  // whole ones (the default 2^32-key chunk does): one inversion per 4096 points.  A chunk that
  // reaches the group order keeps the reference's 1024-key groups: there a centre can equal
  // -(i+1)*stride*G, whose zero difference collapses the group's batch inversion (parity note 4),
  // and only the reference's own geometry collapses the same groups (fixtures *_near_order)
  const int H = zg ? (int)(zg / 2)
                : ((km == KM_XPOINT || km == KM_H160C) && n_keys % (2 * KH_WALK_HB) == 0 &&
                   !reaches_order(st, stride, n_keys + 4 * KH_WALK_HB) && !getenv("KH_NO_BIG_GROUPS"))
                    ? KH_WALK_HB
                    : KH_WALK_H;
  const uint32_t *tab = nullptr;
  int r;

  // m * stride mod n (m < 2^128): double-and-add over the bits of m
  auto mul_stride = [&](u128 m) {
    if (u256_cmp(stride, u256_u64(1)) == 0) return sc_reduce(u256_from_u128(m));
    u256 acc = u256_u64(0), x = stride;
    for (int b = 0; b < 128; b++) {
      if ((m >> b) & 1) acc = sc_add(acc, x);
      x = sc_add(x, x);
    }
    return acc;
  };
  // the reference's do-while runs whole groups (keyhunt.cpp:3350, 3836): a chunk that is no
  // multiple of the group overshoots its end
  uint64_t total_groups = (n_keys + 2 * H - 1) / (2 * H);
  const uint64_t n_points = total_groups * 2 * H;
  job_geom jg = plan(ctx, total_groups, 0, H == KH_WALK_HB ? ctx->lanes_hb : 0);
  // large-group modes interleave lanes (lane g walks groups g, g + L, ...) when the lanes divide
  // the chunk: after the call every lane sits on its group of the chunk that follows, so a call
  // starting there continues them without a lane setup
  const bool inter = H == KH_WALK_HB && (uint64_t)jg.L * jg.gpl == total_groups;
  r = get_table(ctx, stride, &tab, H, inter ? jg.L : 1);
  if (r) return r;
  // the pad's rows per lane (the walk below probes the blocked target filter exactly when A.tblk is
  // set): a resumed walk must find at least that many rows, since the exact-target (sparse) pad is half
  // the dense one a vanity or reference-bloom walk writes
  const bool tblk = !(ctx->vanity || getenv("KH_REF_TARGET_BLOOM")) && ctx->d_tblk;
  const int pad_rows = zg ? H : walk_pad_rows(km, tblk, H);  // km keeps KM_ENDO: as launch_walk sees it
  const bool resume = inter && ctx->cont_valid && ctx->cont_kind == 1 && ctx->cont_km == km &&
                      ctx->cont_L == jg.L && ctx->cont_H == H && ctx->scratch_h >= pad_rows &&
                      ctx->lanes_alloc >= jg.L && u256_cmp(ctx->cont_next, st) == 0 &&
                      u256_cmp(ctx->cont_stride, stride) == 0;
  ctx->cont_valid = false;
  // lane g's first centre: offset H + g * lane_step, lane_step = 2H (interleaved) or gpl * 2H; the
  // scalars s0 + g * (lane_step * stride) are derived on the device (run_setup_prog: a -R chunk
  // restarts 2^20 lanes)
  const u256 lane_step = mul_stride(inter ? (u128)(2 * H) : (u128)jg.gpl * (2 * H));
  const u256 s0 = sc_add(st, mul_stride((u128)H));
  if (!resume) {
    r = ensure_lanes(ctx, jg.L, pad_rows);  // before the centres are set
    if (r) return r;
    r = run_setup_prog(ctx, s0, lane_step, jg.L);
    if (r) return r;
  }

  walk_args A;
  memset(&A, 0, sizeof A);
  A.tab = tab;
  A.cx = ctx->d_cx;
  A.cy = ctx->d_cy;
  A.scratch = ctx->d_scratch;
  A.L = jg.L;
  A.pad_skew = ctx->pad_skew;
  A.pad_swz = pad_swizzle(A.L);
  A.lane_stride = jg.gpl * 2 * H;
  A.interleave = inter ? 1 : 0;
  A.n_points = n_points;
  A.zhalf = zg ? (uint32_t)H : 0;
  A.bloom = ctx->d_tbloom;
  A.bd = ctx->tbd;
  A.tblk = tblk ? ctx->d_tblk : nullptr;
  A.tblocks = ctx->tblocks;
  A.hit_count = ctx->d_hit_count;
  A.hits = ctx->d_hits;
  A.hit_cap = ctx->hit_cap;
  A.probe_len = mode == KH_MODE_XPOINT || mode == KH_MODE_ETH ? 20 : ctx->probe_len;
  uint32_t nd = 0;
  for (;;) {
    HIPCHK(ctx, hipMemsetAsync(ctx->d_hit_count, 0, 4, ctx->stream));
    r = run_walk(ctx, km, mode == KH_MODE_XPOINT ? 1 : 0, A, jg.gpl, 2, H);
    if (r) return r;
    r = fetch_hits(ctx, nd);
    if (r != KH_E_OVERFLOW) break;
    // more bloom hits than the buffer holds (short vanity prefixes): grow it, redo the chunk
    uint32_t need = 0;
    HIPCHK(ctx, hipMemcpy(&need, ctx->d_hit_count, 4, hipMemcpyDeviceToHost));
    uint64_t cap2 = ctx->hit_cap;
    while (cap2 < need) cap2 *= 2;
    if (cap2 > (1u << 26)) return KH_E_OVERFLOW;
    (void)hipFree(ctx->d_hits);
    ctx->d_hits = nullptr;
    HIPCHK(ctx, hipMalloc(&ctx->d_hits, cap2 * sizeof(kh_dev_hit)));
    ctx->hit_cap = (uint32_t)cap2;
    A.hits = ctx->d_hits;
    A.hit_cap = ctx->hit_cap;
    r = run_setup_prog(ctx, s0, lane_step, jg.L);  // the walk moved the lane centres on: start them again
    if (r) return r;
  }
  if (r) return r;
  if (inter) {  // the lanes now sit on the chunk that starts at st + n_keys * stride
    u256 adv = u256_u64(0), x = stride;
    for (uint64_t k = n_keys; k; k >>= 1) {
      if (k & 1) adv = sc_add(adv, x);
      x = sc_add(x, x);
    }
    ctx->cont_valid = true;
    ctx->cont_kind = 1;
    ctx->cont_km = km;
    ctx->cont_L = jg.L;
    ctx->cont_H = H;
    ctx->cont_stride = stride;
    ctx->cont_next = sc_add(st, adv);
  }

  // Confirm each bloom hit against the sorted table and resolve the key: parity fix-up
  // (keyhunt.cpp:3619-3636); with -e the image e gives key * lambda^e, and the 04 variants with
  // -Y the negated key (keyhunt.cpp:3525-3700, 3765-3800).  Hits come out in the order one
  // reference thread prints them: per point, compressed variants (image-major), then
  // uncompressed, then xpoint.
  auto order = [](uint32_t kind) {
    uint32_t base = kind & 15u, e = (kind >> KH_DKIND_ENDO_SHIFT) & 3u, neg = (kind & KH_DKIND_NEG) ? 1u : 0u;
    return base < 2 ? 2 * e + base : base == 2 || base == KH_KIND_ETH ? 6 + 2 * e + neg : 12 + e;
  };
  std::vector<kh_dev_hit> dh(ctx->h_hits.begin(), ctx->h_hits.begin() + nd);
  // -e -c eth: a hit on (beta X, Y) is also the reference's slot-4 hit (keyhunt.cpp:3533), whose key
  // it derives as lambda^2 k, checks against the image, and so negates (3736-3744): added as kind
  // ETH | ENDO2 (an image the GPU never probes in this mode) before the sort, whose order puts it
  // between the point's slot-3 eth(-beta P) and slot-5 eth(-beta^2 P) hits (3706-3745)
  if (endo && mode == KH_MODE_ETH) {
    for (size_t i = 0, n = dh.size(); i < n; i++)
      if (dh[i].kind == (KH_KIND_ETH | (1u << KH_DKIND_ENDO_SHIFT))) {
        kh_dev_hit t = dh[i];
        t.kind = KH_KIND_ETH | (2u << KH_DKIND_ENDO_SHIFT);
        dh.push_back(t);
      }
  }
  std::sort(dh.begin(), dh.end(), [&](const kh_dev_hit &a, const kh_dev_hit &b) {
    return a.idx != b.idx ? a.idx < b.idx : order(a.kind) < order(b.kind);
  });
  static const u256 LAMBDA[3] = {
      u256_u64(1),
      u256{{0xdf02967c1b23bd72ULL, 0x122e22ea20816678ULL, 0xa5261c028812645aULL, 0x5363ad4cc05c30e0ULL}},
      u256{{0xe0cfc810b51283ceULL, 0xa880b9fc8ec739c2ULL, 0x5ad9e3fd77ed9ba4ULL, 0xac9c52b33fa3cf1fULL}}};
  static const fe BETA[3] = {
      fe{{1, 0, 0, 0, 0, 0, 0, 0}},
      fe{{0x719501eeu, 0xc1396c28u, 0x12f58995u, 0x9cf04975u, 0xac3434e9u, 0x6e64479eu, 0x657c0710u, 0x7ae96a2bu}},
      fe{{0x8e6afa40u, 0x3ec693d6u, 0xed0a766au, 0x630fb68au, 0x53cbcb16u, 0x919bb861u, 0x9a83f8efu, 0x851695d4u}}};
  std::vector<kh_hit> out;
  for (auto &h : dh) {
    const u256 k = sc_add(st, mul_stride((u128)h.idx));
    ge P;
    if (!ctx->comb.mult(P, k)) continue;
    const uint32_t base = h.kind & 15u, e = (h.kind >> KH_DKIND_ENDO_SHIFT) & 3u;
    const bool neg = (h.kind & KH_DKIND_NEG) != 0;
    if (e > 2) continue;
    // the point the walk produced at this slot: k*G, or with --rmd-batch-size < 1024 and a slot
    // other than its group's centre, x = -(C.x + (i+1)D.x), y = -+(i+1)D.y (k_walk_zinv)
    ge S = P;
    bool garbage = false;
    if (zg && h.idx % zg != (uint64_t)H) {
      const uint64_t grp = h.idx / zg, t = h.idx % zg;
      const uint64_t i = t > (uint64_t)H ? t - H - 1 : H - t - 1;
      ge C, Di;
      if (!ctx->comb.mult(C, sc_add(st, mul_stride((u128)grp * zg + H))) ||
          !ctx->comb.mult(Di, mul_stride((u128)(i + 1))))
        continue;
      fe sx;
      fe_add(sx, C.x, Di.x);
      fe_neg(S.x, sx);
      S.y = Di.y;
      if (t > (uint64_t)H) fe_neg(S.y, Di.y);
      garbage = true;
    }
    fe xe = S.x, ye = S.y;
    if (e) fe_mul(xe, S.x, BETA[e]);
    if (neg) fe_neg(ye, S.y);
    uint8_t probe[20];
    uint32_t w[5];
    bool compressed = false;
    if (base == KH_KIND_02 || base == KH_KIND_03) {
      hash160_comp(xe, 2 + base, w);
      compressed = true;
    } else if (base == KH_KIND_04) {
      hash160_uncomp(xe, ye, w);
    } else if (base == KH_KIND_ETH) {
      if (endo && e == 2 && !neg)  // the slot-4 twin: its image is eth(beta P)
        fe_mul(xe, S.x, BETA[1]);
      eth_address(xe, ye, w);
    } else {
      for (int j = 0; j < 5; j++) w[j] = bswap32(xe.d[7 - j]);
    }
    memcpy(probe, w, 20);
    if (ctx->vanity && base != KH_KIND_XPOINT && base != KH_KIND_ETH) {
      // vanityrmdmatch (keyhunt.cpp:6677-6703): inside any [A, B] range
      bool in = false;
      for (size_t j = 0; j < ctx->v_ranges.size() && !in; j += 40)
        in = memcmp(&ctx->v_ranges[j], probe, 20) <= 0 && memcmp(&ctx->v_ranges[j + 20], probe, 20) >= 0;
      if (!in) continue;
    } else if (!searchbinary(ctx->rows.data(), (int64_t)ctx->n_rows, probe, 20, 0)) {
      continue;
    }
    kh_hit o;
    memset(&o, 0, sizeof o);
    u256 kr = e ? sc_mul(k, LAMBDA[e]) : k;  // (beta^e x, y) = lambda^e * (x, y)
    if (base == KH_KIND_ETH && endo && e == 2 && !neg) {
      kr = sc_neg(kr);  // the slot-4 twin: lambda^2 k gives (beta^2 X, Y), not the image: negated
    } else if (garbage && (compressed ? !endo : endo)) {
      // where the reference checks the found key's own image against the hit -- compressed without
      // -e (keyhunt.cpp:3619-3636), 04 and eth with -e (3652-3680, 3714-3744) -- a point that is no
      // multiple of G never matches it: negated
      kr = sc_neg(kr);
    } else if (compressed) {
      uint32_t odd = P.y.d[0] & 1;  // the image keeps Y; -e: the slot key's parity (3565-3600)
      if (odd != (base == KH_KIND_03 ? 1u : 0u)) kr = sc_neg(kr);
    } else if (neg) {
      kr = sc_neg(kr);
    }
    u256_to_be(o.key, kr);
    o.offset = h.idx;
    o.kind = h.kind;
    o.compressed = compressed ? 1 : 0;
    out.push_back(o);
  }
  *n_hits = (uint32_t)out.size();
  if (hits)
    for (uint32_t i = 0; i < out.size() && i < cap; i++) hits[i] = out[i];
  return out.size() > cap ? KH_E_OVERFLOW : KH_OK;
}

// ---------------------------------------------------------------------------------------------
// BSGS
// ---------------------------------------------------------------------------------------------
int kh_bsgs_setup(kh_ctx *ctx, uint64_t n, uint64_t k, kh_bsgs_info *info) {
  if (ctx) ctx->cont_valid = false;
  if (!ctx || !k) return KH_E_ARG;
  (void)hipSetDevice(ctx->device);
  // keyhunt.cpp:1454-1661
  uint64_t m = (uint64_t)sqrtl((long double)n);
  while (m * m > n) m--;
  while ((m + 1) * (m + 1) <= n) m++;
  if (m * m != n || m % 1024) return KH_E_BSGS_N;
  m *= k;
  uint64_t m2 = m / 32 + (m % 32 ? 1 : 0);
  uint64_t m3 = m2 / 32 + (m2 % 32 ? 1 : 0);
  uint64_t aux = n / m;
  if (n % m) n = m * aux;
  kh_bsgs_info &I = ctx->info;
  memset(&I, 0, sizeof I);
  ctx->entries[0] = ctx->entries[1] = ctx->entries[2] = 0;
  I.n = n;
  I.m = m;
  I.m2 = m2;
  I.m3 = m3;
  I.aux = aux;
  I.cycles = aux / 1024 + (aux % 1024 ? 1 : 0);
  uint64_t it[3];
  it[0] = (m / 256 > 10000) ? (m / 256 + (m % 256 ? 1 : 0)) : 1000;
  it[1] = (m2 / 256 > 1000) ? (m2 / 256 + (m2 % 256 ? 1 : 0)) : 1000;
  it[2] = (m3 / 256 > 1000) ? (m3 / 256 + (m3 % 256 ? 1 : 0)) : 1000;
  for (int l = 0; l < 3; l++) {
    // initBloomFilter's entry count (keyhunt.cpp:7608): the 10000 floor, else -z x items
    ctx->entries[l] = it[l] <= 10000 ? 10000 : (uint64_t)ctx->bloom_mult * it[l];
    ctx->bd[l] = bloom_size(ctx->entries[l]);
    ctx->bd_ref1 = l == 0 ? ctx->bd[0] : ctx->bd_ref1;
    ctx->bd_ref1.stride = (ctx->bd_ref1.bytes + 255) & ~255ULL;
    if (l == 0 && ctx->l1_layout == KH_LAYER1_BLOCKED) {
      // 3x the reference's bits per shard in whole 128-bit blocks (kh_kernels.h); desc.bits = blocks
      uint64_t blocks = (ctx->bd[0].bits * KH_BLK_BITS_MUL + 127) / 128;
      // the probe record carries the block index within a shard and the shard byte, and addresses a
      // shard by a 32-bit stride (k_walk blk_record / blk_load): shards must stay below 4 GB
      if (((blocks * 16 + 255) & ~255ULL) >> 32) {
        ctx->err = "blocked layer 1 needs shards below 4 GB (M < ~2^36.6; the reference layout's shards reach the "
                   "2^32-bit probe limit below that, at M ~2^35.1)";
        return KH_E_ARG;
      }
      ctx->bd[0].bits = blocks;
      ctx->bd[0].recip = ~0ULL / blocks;
      ctx->bd[0].bytes = blocks * 16;
    }
    ctx->bd[l].stride = (ctx->bd[l].bytes + 255) & ~255ULL;
    if (ctx->bd[l].bits >> 32) {  // shards of 2^32 bits or more (M >= ~2^35.1 in layer 1) are refused
      ctx->err = "a bloom shard of 2^32 bits or more (M >= ~2^35.1) is outside the engine's tested probe range";
      return KH_E_ARG;
    }
    I.bloom_bits[l] = (l == 0 && ctx->l1_layout == KH_LAYER1_BLOCKED) ? ctx->bd[0].bits * 128 : ctx->bd[l].bits;
    I.bloom_bytes[l] = ctx->bd[l].bytes;
    I.bloom_hashes[l] = (l == 0 && ctx->l1_layout == KH_LAYER1_BLOCKED) ? 16u : ctx->bd[l].hashes;
  }
  I.layer1_layout = ctx->l1_layout;
  for (int l = 0; l < 3; l++) {
    (void)hipFree(ctx->d_bl[l]);
    ctx->d_bl[l] = nullptr;
    size_t bytes = 256 * ctx->bd[l].stride + 4;
    // (fine-grained and uncached memory types for layer 1 were measured in round 4: no gain, the
    // probes still cost the same power, profiles/r04e_alloc_ab.json)
    if (l == 0)
      HIPCHK(ctx, dev_alloc(reinterpret_cast<void **>(&ctx->d_bl[l]), bytes, 1));
    else
      HIPCHK(ctx, hipMalloc(&ctx->d_bl[l], bytes));
    HIPCHK(ctx, hipMemset(ctx->d_bl[l], 0, bytes));
  }
  // AMP2[i] = -(M2 + 2i*M2)G, AMP3[i] = -(M3 + 2i*M3)G  (keyhunt.cpp:1818-1842)
  ctx->amp2.resize(32);
  ctx->amp3.resize(32);
  for (int i = 0; i < 32; i++) {
    ge a;
    ctx->comb.mult(a, u256_u64(m2 * (2 * (uint64_t)i + 1)));
    fe_neg(a.y, a.y);
    ctx->amp2[i] = a;
    ctx->comb.mult(a, u256_u64(m3 * (2 * (uint64_t)i + 1)));
    fe_neg(a.y, a.y);
    ctx->amp3[i] = a;
  }
  {
    std::vector<uint32_t> w(32 * 16);
    for (int i = 0; i < 32; i++) {
      memcpy(&w[i * 16], ctx->amp2[i].x.d, 32);
      memcpy(&w[i * 16 + 8], ctx->amp2[i].y.d, 32);
    }
    if (!ctx->d_amp2) HIPCHK(ctx, hipMalloc(&ctx->d_amp2, w.size() * 4));
    if (!ctx->d_ref_start) HIPCHK(ctx, hipMalloc(&ctx->d_ref_start, 32));
    HIPCHK(ctx, hipMemcpy(ctx->d_amp2, w.data(), w.size() * 4, hipMemcpyHostToDevice));
  }
  ctx->second_hits = 0;
  ctx->bsgs_ready = true;
  ctx->bsgs_built = false;
  ctx->candidates = 0;
  ctx->second_hits = 0;
  if (info) *info = I;
  return KH_OK;
}

int kh_bsgs_set_layer1(kh_ctx *ctx, uint32_t layout) {
  if (!ctx || layout > KH_LAYER1_BLOCKED) return KH_E_ARG;
  ctx->l1_layout = layout;
  return KH_OK;
}

int kh_bsgs_set_bloom_multiplier(kh_ctx *ctx, uint32_t mult) {
  if (!ctx || !mult) return KH_E_ARG;
  ctx->bloom_mult = mult;
  return KH_OK;
}

namespace {
// the baby-step walk (thread_bPload, keyhunt.cpp:5284-5472): babies (i+1)G, i < M, into layer 1
// (bl1/bd1, reference or blocked layout by `mode`), layers 2/3 (the context's) and the bP rows
// baby steps 1..count (count = M unless a single layer is rebuilt) into bl1 with bd1 and, for the
// first M2 / M3 of them, into layers 2 / 3 and the bP rows (m2 = m3 = 0: layer bl1 alone)
int build_walk(kh_ctx *ctx, int mode, uint8_t *bl1, const bloom_desc &bd1, uint64_t *d_key, uint32_t *d_val,
               uint64_t count = 0, bool one_layer = false) {
  const int H = KH_WALK_H;
  ctx->cont_valid = false;
  const kh_bsgs_info &I = ctx->info;
  if (!count) count = I.m;
  const uint32_t *tab = nullptr;
  int r = get_table(ctx, u256_u64(1), &tab);
  if (r) return r;
  uint64_t total_groups = (count + 2 * H - 1) / (2 * H);
  job_geom jg = plan(ctx, total_groups, 0);
  std::vector<u256> s(jg.L);
  for (uint32_t g = 0; g < jg.L; g++) s[g] = u256_u64(1 + (uint64_t)g * jg.gpl * 2 * H + H);  // baby i <-> key i+1
  r = run_setup(ctx, s, nullptr);
  if (r) return r;
  walk_args A;
  memset(&A, 0, sizeof A);
  A.tab = tab;
  A.cx = ctx->d_cx;
  A.cy = ctx->d_cy;
  A.scratch = ctx->d_scratch;
  A.L = jg.L;
  A.pad_skew = ctx->pad_skew;
  A.pad_swz = pad_swizzle(A.L);
  A.lane_stride = jg.gpl * 2 * H;
  A.n_points = count;
  A.bl1 = bl1;
  A.bl2 = ctx->d_bl[1];
  A.bl3 = ctx->d_bl[2];
  A.bd = bd1;
  A.bd2 = ctx->bd[1];
  A.bd3 = ctx->bd[2];
  A.m2 = one_layer ? 0 : I.m2;
  A.m3 = one_layer ? 0 : I.m3;
  A.rows_key = d_key;
  A.rows_val = d_val;
  return run_walk(ctx, mode, 3, A, jg.gpl, 4);
}
}  // namespace

int kh_bsgs_memory(kh_ctx *ctx, uint64_t *needed_bytes, uint64_t *held_bytes) {
  if (!ctx) return KH_E_ARG;
  if (!ctx->bsgs_ready) return KH_E_STATE;
  uint64_t layers = 0;
  for (int l = 0; l < 3; l++) layers += 256 * ctx->bd[l].stride + 4;
  const uint64_t L = ctx->lanes_max;
  // the giant walk's pad (L x KH_WALK_HB entries of 32 B), lane centres and scalars, the comb, the two
  // rounds' candidate buffers at their current size (16 B per entry, plus the first list's copy), the
  // base list of a kh_bsgs_scan_list call of up to 2^16 bases (32 B each: bsgsd's batch; a longer
  // list adds 32 B per base), and the build's transient row keys (m3 x 12 B).  A round whose
  // candidates overflow doubles its buffers on demand (up to 2^28 entries), which this figure cannot
  // foresee.
  const uint64_t walk = L * (uint64_t)walk_pad_rows(KM_BSGSB, false, KH_WALK_HB) * 32 + L * 32 * 3 + (512u << 10) + 4ull * ctx->cand_cap * 16 +
                        (1ull << 16) * 32 + ctx->info.m3 * 12;
  if (needed_bytes) *needed_bytes = layers + walk;
  if (held_bytes)
    *held_bytes = layers + (uint64_t)ctx->lanes_alloc * ctx->scratch_h * 32 + (uint64_t)ctx->lanes_alloc * 32 * 3;
  return KH_OK;
}

int kh_bsgs_build(kh_ctx *ctx) {
  if (!ctx) return KH_E_ARG;
  if (!ctx->bsgs_ready) return KH_E_STATE;
  (void)hipSetDevice(ctx->device);
  const kh_bsgs_info &I = ctx->info;
  int r;
  uint64_t *d_key = nullptr;
  uint32_t *d_val = nullptr;
  HIPCHK(ctx, hipMalloc(&d_key, I.m3 * 8));
  HIPCHK(ctx, hipMalloc(&d_val, I.m3 * 4));
  r = build_walk(ctx, ctx->l1_layout == KH_LAYER1_BLOCKED ? KM_BUILDB : KM_BUILD, ctx->d_bl[0], ctx->bd[0], d_key, d_val);
  if (r) {
    (void)hipFree(d_key);
    (void)hipFree(d_val);
    return r;
  }
  // bsgs_sort (keyhunt.cpp:4412-4508): order rows by the 6 value bytes (ties by index)
  std::vector<uint64_t> keys(I.m3);
  std::vector<uint32_t> vals(I.m3);
  HIPCHK(ctx, hipMemcpy(keys.data(), d_key, I.m3 * 8, hipMemcpyDeviceToHost));
  HIPCHK(ctx, hipMemcpy(vals.data(), d_val, I.m3 * 4, hipMemcpyDeviceToHost));
  (void)hipFree(d_key);
  (void)hipFree(d_val);
  std::vector<uint64_t> order(I.m3);
  for (uint64_t i = 0; i < I.m3; i++) order[i] = i;
  std::sort(order.begin(), order.end(), [&](uint64_t a, uint64_t b) {
    return keys[a] != keys[b] ? keys[a] < keys[b] : vals[a] < vals[b];
  });
  ctx->h_rows.assign(I.m3 * 16, 0);
  for (uint64_t i = 0; i < I.m3; i++) {
    uint64_t kk = keys[order[i]];
    uint8_t *row = &ctx->h_rows[i * 16];
    for (int b = 0; b < 6; b++) row[b] = (uint8_t)(kk >> (40 - 8 * b));
    uint64_t idx = vals[order[i]];
    memcpy(row + 8, &idx, 8);
  }
  // layers 2 and 3 on the host for the refinement steps
  for (int l = 1; l < 3; l++) {
    ctx->h_bl[l].resize(256 * ctx->bd[l].stride);
    HIPCHK(ctx, hipMemcpy(ctx->h_bl[l].data(), ctx->d_bl[l], ctx->h_bl[l].size(), hipMemcpyDeviceToHost));
  }
  ctx->bsgs_built = true;
  return KH_OK;
}

// ==============================================================================================
// BSGS table files (-S, keyhunt.cpp:1983-2230 read, 2504-2652 write): per layer 256 records of
// {struct bloom (112 B), bit array, checksumsha256 {sha256(bits), same again}} in
// keyhunt_bsgs_4_<M>.blm / _6_<M2>.blm / _7_<M3>.blm, and the sorted bP rows + sha256 in
// keyhunt_bsgs_2_<M3>.tbl.
// ==============================================================================================
namespace {

// SHA-256 of a byte string (the reference's sha256(), hash/sha256.cpp), on kh_math.h's compression
void sha256_bytes(const uint8_t *p, size_t n, uint8_t out[32]) {
  uint32_t st[8], w[16];
  sha256_init(st);
  uint8_t blk[64];
  size_t off = 0;
  auto compress = [&](const uint8_t *b) {
    for (int i = 0; i < 16; i++)
      w[i] = ((uint32_t)b[4 * i] << 24) | ((uint32_t)b[4 * i + 1] << 16) | ((uint32_t)b[4 * i + 2] << 8) | b[4 * i + 3];
    sha256_transform(st, w);
  };
  for (; off + 64 <= n; off += 64) compress(p + off);
  size_t rem = n - off;
  memset(blk, 0, 64);
  memcpy(blk, p + off, rem);
  blk[rem] = 0x80;
  if (rem >= 56) {
    compress(blk);
    memset(blk, 0, 64);
  }
  const uint64_t bits = (uint64_t)n * 8;
  for (int i = 0; i < 8; i++) blk[56 + i] = (uint8_t)(bits >> (56 - 8 * i));
  compress(blk);
  for (int i = 0; i < 8; i++) {
    out[4 * i] = (uint8_t)(st[i] >> 24);
    out[4 * i + 1] = (uint8_t)(st[i] >> 16);
    out[4 * i + 2] = (uint8_t)(st[i] >> 8);
    out[4 * i + 3] = (uint8_t)st[i];
  }
}

constexpr size_t KH_BLOOM_STRUCT = 112;  // sizeof(struct bloom) on x86-64 (bloom/bloom.h:26-49)

// struct bloom as bloom_init2 leaves it (bloom/bloom.cpp:154-187): entries, bits, bytes, hashes,
// error (x87 long double), ready = 1, version 2.201, bpe; the pointers and chunk fields are 0 here
// (the reference writes its own heap pointer into `bf` and replaces it on reading)
void bloom_header(uint8_t h[KH_BLOOM_STRUCT], uint64_t entries, const bloom_desc &d) {
  memset(h, 0, KH_BLOOM_STRUCT);
  memcpy(h + 0, &entries, 8);
  memcpy(h + 8, &d.bits, 8);
  memcpy(h + 16, &d.bytes, 8);
  h[24] = (uint8_t)d.hashes;
  const long double err = 0.000001;
  memcpy(h + 32, &err, 10);
  h[48] = 1;
  h[49] = 2;
  h[50] = 201;
  const long double num = -logl(err), denom = 0.480453013918201;
  const double bpe = (double)(num / denom);
  memcpy(h + 56, &bpe, 8);
}

struct table_path {
  std::string s;
  table_path(const char *dir, int kind, uint64_t m, const char *ext) {
    char name[96];
    snprintf(name, sizeof name, "keyhunt_bsgs_%d_%llu.%s", kind, (unsigned long long)m, ext);
    s = std::string((dir && *dir) ? dir : ".") + "/" + name;
  }
};

// one layer (256 shards at d.stride in `bits`) -> .blm
int write_blm(kh_ctx *c, const std::string &path, const uint8_t *bits, const bloom_desc &d, uint64_t entries) {
  FILE *f = fopen(path.c_str(), "wb");
  if (!f) {
    c->err = "can't create the file " + path;
    return KH_E_IO;
  }
  uint8_t h[KH_BLOOM_STRUCT], ck[64];
  bloom_header(h, entries, d);
  bool ok = true;
  for (int i = 0; i < 256 && ok; i++) {
    const uint8_t *bf = bits + (size_t)i * d.stride;
    sha256_bytes(bf, d.bytes, ck);
    memcpy(ck + 32, ck, 32);
    ok = fwrite(h, KH_BLOOM_STRUCT, 1, f) == 1 && fwrite(bf, d.bytes, 1, f) == 1 && fwrite(ck, 64, 1, f) == 1;
  }
  ok = (fclose(f) == 0) && ok;
  if (!ok) {
    c->err = "error writing the file " + path;
    return KH_E_IO;
  }
  return KH_OK;
}

// .blm -> one layer (256 shards at d.stride in `bits`); headers must carry this geometry
int read_blm(kh_ctx *c, const std::string &path, uint8_t *bits, const bloom_desc &d, uint64_t entries, bool verify) {
  FILE *f = fopen(path.c_str(), "rb");
  if (!f) {
    c->err = "missing file " + path;
    return KH_E_IO;
  }
  uint8_t h[KH_BLOOM_STRUCT], ck[64], sum[32];
  int rc = KH_OK;
  for (int i = 0; i < 256 && rc == KH_OK; i++) {
    uint8_t *bf = bits + (size_t)i * d.stride;
    if (fread(h, KH_BLOOM_STRUCT, 1, f) != 1) {
      rc = KH_E_IO;
      break;
    }
    uint64_t fe_, fb, fy;
    memcpy(&fe_, h, 8);
    memcpy(&fb, h + 8, 8);
    memcpy(&fy, h + 16, 8);
    if (fe_ != entries || fb != d.bits || fy != d.bytes || h[24] != (uint8_t)d.hashes || h[48] != 1) {
      c->err = "bloom geometry in " + path + " does not match this N/k";
      rc = KH_E_FORMAT;
      break;
    }
    if (fread(bf, d.bytes, 1, f) != 1 || fread(ck, 64, 1, f) != 1) {
      rc = KH_E_IO;
      break;
    }
    if (verify) {
      sha256_bytes(bf, d.bytes, sum);
      if (memcmp(ck, sum, 32) != 0 || memcmp(ck + 32, sum, 32) != 0) {
        c->err = "checksum file mismatch! " + path;
        rc = KH_E_FORMAT;
      }
    }
  }
  if (rc == KH_E_IO) c->err = "error reading the file " + path;
  fclose(f);
  return rc;
}

// layer 1 in the reference layout on the host: the device layer itself, or (blocked layout) a
// reference-layout baby walk into a temporary buffer
int ref_layer1(kh_ctx *c, std::vector<uint8_t> &out) {
  const bloom_desc &d = c->bd_ref1;
  out.assign(256 * d.stride, 0);
  if (c->l1_layout == KH_LAYER1_REFERENCE) {
    HIPCHK(c, hipMemcpy(out.data(), c->d_bl[0], out.size(), hipMemcpyDeviceToHost));
    return KH_OK;
  }
  uint8_t *tmp = nullptr;
  uint64_t *d_key = nullptr;
  uint32_t *d_val = nullptr;
  int r = KH_OK;
  if (hipMalloc(&tmp, out.size() + 4) != hipSuccess || hipMalloc(&d_key, c->info.m3 * 8) != hipSuccess ||
      hipMalloc(&d_val, c->info.m3 * 4) != hipSuccess || hipMemset(tmp, 0, out.size() + 4) != hipSuccess) {
    c->err = "no device memory for the reference-layout layer 1";
    r = KH_E_NOMEM;
  }
  if (r == KH_OK) r = build_walk(c, KM_BUILD, tmp, d, d_key, d_val);
  if (r == KH_OK && hipMemcpy(out.data(), tmp, out.size(), hipMemcpyDeviceToHost) != hipSuccess) r = KH_E_HIP;
  (void)hipFree(tmp);
  (void)hipFree(d_key);
  (void)hipFree(d_val);
  return r;
}

}  // namespace

int kh_bsgs_save(kh_ctx *ctx, const char *dir) {
  if (!ctx) return KH_E_ARG;
  if (!ctx->bsgs_built) return KH_E_STATE;
  (void)hipSetDevice(ctx->device);
  const kh_bsgs_info &I = ctx->info;
  std::vector<uint8_t> l1;
  int r = ref_layer1(ctx, l1);
  if (r) return r;
  r = write_blm(ctx, table_path(dir, 4, I.m, "blm").s, l1.data(), ctx->bd_ref1, ctx->entries[0]);
  if (r) return r;
  l1.clear();
  l1.shrink_to_fit();
  r = write_blm(ctx, table_path(dir, 6, I.m2, "blm").s, ctx->h_bl[1].data(), ctx->bd[1], ctx->entries[1]);
  if (r) return r;
  r = write_blm(ctx, table_path(dir, 7, I.m3, "blm").s, ctx->h_bl[2].data(), ctx->bd[2], ctx->entries[2]);
  if (r) return r;
  const std::string tp = table_path(dir, 2, I.m3, "tbl").s;
  FILE *f = fopen(tp.c_str(), "wb");
  if (!f) {
    ctx->err = "can't create the file " + tp;
    return KH_E_IO;
  }
  uint8_t ck[32];
  sha256_bytes(ctx->h_rows.data(), ctx->h_rows.size(), ck);
  bool ok = fwrite(ctx->h_rows.data(), ctx->h_rows.size(), 1, f) == 1 && fwrite(ck, 32, 1, f) == 1;
  ok = (fclose(f) == 0) && ok;
  if (!ok) {
    ctx->err = "error writing the file " + tp;
    return KH_E_IO;
  }
  return KH_OK;
}

int kh_bsgs_load(kh_ctx *ctx, const char *dir, uint32_t flags) {
  if (!ctx) return KH_E_ARG;
  if (!ctx->bsgs_ready) return KH_E_STATE;
  (void)hipSetDevice(ctx->device);
  const kh_bsgs_info &I = ctx->info;
  const bool verify = !(flags & KH_LOAD_SKIP_CHECKSUM);
  ctx->bsgs_built = false;
  // bP table
  const std::string tp = table_path(dir, 2, I.m3, "tbl").s;
  std::vector<uint8_t> rows(I.m3 * 16);
  {
    FILE *f = fopen(tp.c_str(), "rb");
    if (!f) {
      ctx->err = "missing file " + tp;
      return KH_E_IO;
    }
    uint8_t ck[32], sum[32];
    bool ok = fread(rows.data(), rows.size(), 1, f) == 1 && fread(ck, 32, 1, f) == 1;
    fclose(f);
    if (!ok) {
      ctx->err = "error reading the file " + tp;
      return KH_E_IO;
    }
    if (verify) {
      sha256_bytes(rows.data(), rows.size(), sum);
      if (memcmp(ck, sum, 32) != 0) {
        ctx->err = "checksum file mismatch! " + tp;
        return KH_E_FORMAT;
      }
    }
  }
  // layers 2 and 3 (host copies serve the refinement)
  for (int l = 1; l < 3; l++) {
    std::vector<uint8_t> &h = ctx->h_bl[l];
    h.assign(256 * ctx->bd[l].stride, 0);
    int r = read_blm(ctx, table_path(dir, l == 1 ? 6 : 7, l == 1 ? I.m2 : I.m3, "blm").s, h.data(), ctx->bd[l],
                     ctx->entries[l], verify);
    if (r) return r;
    HIPCHK(ctx, hipMemcpy(ctx->d_bl[l], h.data(), h.size(), hipMemcpyHostToDevice));
  }
  // layer 1: the file's bits for the reference layout; the blocked layout is rebuilt on the GPU
  // (its bits are not in any reference file), after checking the file all the same
  {
    std::vector<uint8_t> l1(256 * ctx->bd_ref1.stride, 0);
    int r = read_blm(ctx, table_path(dir, 4, I.m, "blm").s, l1.data(), ctx->bd_ref1, ctx->entries[0], verify);
    if (r) return r;
    if (ctx->l1_layout == KH_LAYER1_REFERENCE) {
      HIPCHK(ctx, hipMemcpy(ctx->d_bl[0], l1.data(), l1.size(), hipMemcpyHostToDevice));
    } else {
      uint64_t *d_key = nullptr;
      uint32_t *d_val = nullptr;
      HIPCHK(ctx, hipMalloc(&d_key, I.m3 * 8));
      HIPCHK(ctx, hipMalloc(&d_val, I.m3 * 4));
      HIPCHK(ctx, hipMemset(ctx->d_bl[0], 0, 256 * ctx->bd[0].stride + 4));
      r = build_walk(ctx, KM_BUILDB, ctx->d_bl[0], ctx->bd[0], d_key, d_val);
      (void)hipFree(d_key);
      (void)hipFree(d_val);
      if (r) return r;
    }
  }
  ctx->h_rows.swap(rows);
  ctx->bsgs_built = true;
  return KH_OK;
}

// ==============================================================================================
// Target files (-S for address/rmd160/xpoint): data_<hex>.dat as readFileAddress reads it
// (keyhunt.cpp:7033-7210) and writeFileIfNeeded writes it (7756-7855):
//   sha256(bloom bits) | struct bloom (112 B) | bloom bits | sha256(table) | u64 table bytes |
//   the sorted 20-byte rows (struct address_value).
// ==============================================================================================
int kh_targets_save(kh_ctx *ctx, const char *path) {
  if (!ctx || !path) return KH_E_ARG;
  if (!ctx->d_tbloom || ctx->vanity) return KH_E_STATE;
  FILE *f = fopen(path, "wb");
  if (!f) {
    ctx->err = std::string("can't create the file ") + path;
    return KH_E_IO;
  }
  uint8_t ckb[32], ckd[32], h[KH_BLOOM_STRUCT];
  sha256_bytes(ctx->h_tbloom.data(), ctx->tbd.bytes, ckb);
  bloom_header(h, ctx->t_entries, ctx->tbd);
  const uint64_t data_size = ctx->n_rows * 20;
  sha256_bytes(ctx->rows.data(), data_size, ckd);
  bool ok = fwrite(ckb, 1, 32, f) == 32 && fwrite(h, 1, KH_BLOOM_STRUCT, f) == KH_BLOOM_STRUCT &&
            fwrite(ctx->h_tbloom.data(), 1, ctx->tbd.bytes, f) == ctx->tbd.bytes && fwrite(ckd, 1, 32, f) == 32 &&
            fwrite(&data_size, 1, 8, f) == 8 && fwrite(ctx->rows.data(), 1, data_size, f) == data_size;
  ok = (fclose(f) == 0) && ok;
  if (!ok) {
    ctx->err = std::string("error writing the file ") + path;
    return KH_E_IO;
  }
  return KH_OK;
}

int kh_targets_load(kh_ctx *ctx, const char *path, uint32_t flags) {
  if (!ctx || !path) return KH_E_ARG;
  (void)hipSetDevice(ctx->device);
  FILE *f = fopen(path, "rb");
  if (!f) {
    ctx->err = std::string("can't open the file ") + path;
    return KH_E_IO;
  }
  uint8_t ckb[32], ckd[32], h[KH_BLOOM_STRUCT], ck[32];
  std::vector<uint8_t> bits, rows;
  uint64_t entries = 0, nbits = 0, nbytes = 0, data_size = 0;
  int rc = KH_OK;
  if (fread(ckb, 1, 32, f) != 32 || fread(h, 1, KH_BLOOM_STRUCT, f) != KH_BLOOM_STRUCT) rc = KH_E_IO;
  if (!rc) {
    memcpy(&entries, h + 0, 8);
    memcpy(&nbits, h + 8, 8);
    memcpy(&nbytes, h + 16, 8);
    // the reader trusts bits/bytes/hashes of the stored struct (keyhunt.cpp:7076-7081)
    if (nbits == 0 || h[24] == 0 || nbytes != nbits / 8 + ((nbits % 8) ? 1 : 0)) rc = KH_E_FORMAT;
  }
  if (!rc) {
    bits.resize(nbytes);
    if (fread(bits.data(), 1, nbytes, f) != nbytes || fread(ckd, 1, 32, f) != 32 || fread(&data_size, 1, 8, f) != 8)
      rc = KH_E_IO;
  }
  if (!rc && data_size % 20) rc = KH_E_FORMAT;
  if (!rc) {
    rows.resize(data_size);
    if (fread(rows.data(), 1, data_size, f) != data_size) rc = KH_E_IO;
  }
  fclose(f);
  if (!rc && !(flags & KH_LOAD_SKIP_CHECKSUM)) {  // FLAGSKIPCHECKSUM (keyhunt.cpp:7129-7146, 7193-7200)
    sha256_bytes(bits.data(), nbytes, ck);
    if (memcmp(ck, ckb, 32)) rc = KH_E_FORMAT;
    sha256_bytes(rows.data(), data_size, ck);
    if (!rc && memcmp(ck, ckd, 32)) rc = KH_E_FORMAT;
  }
  if (rc) {
    ctx->err = std::string(rc == KH_E_IO ? "error reading the file " : "checksum or format mismatch in ") + path;
    return rc;
  }
  bloom_desc d;
  memset(&d, 0, sizeof d);
  d.bits = nbits;
  d.bytes = nbytes;
  d.hashes = h[24];
  d.recip = ~0ULL / d.bits;
  d.stride = d.bytes;
  ctx->rows.swap(rows);
  ctx->n_rows = data_size / 20;
  ctx->vanity = false;
  ctx->probe_len = 20;
  ctx->v_ranges.clear();
  ctx->t_entries = entries;
  ctx->tbd = d;
  ctx->h_tbloom.swap(bits);
  (void)hipFree(ctx->d_tbloom);
  ctx->d_tbloom = nullptr;
  HIPCHK(ctx, hipMalloc(&ctx->d_tbloom, ctx->tbd.bytes + 4));
  HIPCHK(ctx, hipMemcpy(ctx->d_tbloom, ctx->h_tbloom.data(), ctx->tbd.bytes, hipMemcpyHostToDevice));
  return KH_OK;
}

int kh_bsgs_set_targets(kh_ctx *ctx, const uint8_t *xy, uint32_t n) {
  if (!ctx || (!xy && n)) return KH_E_ARG;
  ctx->cont_valid = false;
  ctx->targets.resize(n);
  for (uint32_t i = 0; i < n; i++) {
    fe_from_be(ctx->targets[i].x, xy + 64 * i);
    fe_from_be(ctx->targets[i].y, xy + 64 * i + 32);
  }
  ctx->found.assign(n, 0);
  return KH_OK;
}

int kh_bsgs_reset_found(kh_ctx *ctx) {
  if (!ctx) return KH_E_ARG;
  std::fill(ctx->found.begin(), ctx->found.end(), 0);
  return KH_OK;
}

int kh_bsgs_refine_stats(kh_ctx *ctx, uint64_t *first_level, uint64_t *second_level) {
  if (!ctx || !first_level || !second_level) return KH_E_ARG;
  *first_level = ctx->candidates;
  *second_level = ctx->second_hits;
  return KH_OK;
}

int kh_bsgs_candidates(kh_ctx *ctx, uint64_t *count) {
  if (!ctx || !count) return KH_E_ARG;
  *count = ctx->candidates;
  return KH_OK;
}

namespace {

bool rows_search(const kh_ctx *c, const uint8_t x32[32], uint64_t &idx) {
  // bsgs_searchbinary (keyhunt.cpp:4510-4544), no bucket cache
  const uint8_t *rows = c->h_rows.data();
  int64_t n = (int64_t)c->info.m3, min = 0, max = n, cur = 0, half = n;
  while (half >= 1) {
    half = (max - min) / 2;
    const uint8_t *row = rows + (cur + half) * 16;
    int cmp = memcmp(x32 + 16, row, 6);
    if (cmp == 0) {
      memcpy(&idx, row + 8, 8);
      return true;
    }
    if (cmp < 0)
      max = max - half;
    else
      min = min + half;
    cur = min;
  }
  return false;
}

// S + A[i] for i < 32, X only, one batched inversion.  AddDirect with dx == 0 yields
// x = -S.x - A.x in the reference (inverse of 0 is 0); reproduced.
void add32_x(const ge &S, const std::vector<ge> &A, fe out[32]) {
  std::vector<fe> dx(32);
  for (int i = 0; i < 32; i++) fe_sub(dx[i], A[i].x, S.x);
  batch_inv(dx);
  for (int i = 0; i < 32; i++) {
    fe dy, s, x;
    fe_sub(dy, A[i].y, S.y);
    fe_mul(s, dy, dx[i]);
    fe_sqr(x, s);
    fe_sub(x, x, S.x);
    fe_sub(x, x, A[i].x);
    out[i] = x;
  }
}

// bsgs_thirdcheck (keyhunt.cpp:5186-5248)
bool third_check(const kh_ctx *c, const u256 &base_key, uint32_t a, const ge &Q, u256 &key) {
  const kh_bsgs_info &I = c->info;
  u256 base3 = sc_add(base_key, sc_reduce(u256_from_u128((u128)a * 2 * I.m2)));
  ge bp;
  if (!c->comb.mult(bp, base3)) return false;
  fe_neg(bp.y, bp.y);
  ge S;
  ge_add(S, Q, bp);
  fe xs[32];
  add32_x(S, c->amp3, xs);
  for (int i = 0; i < 32; i++) {
    uint8_t xr[32];
    fe_to_be(xr, xs[i]);
    u256 calc = u256_u64(i == 0 ? I.m3 : (uint64_t)i * 2 * I.m3 + I.m3);
    if (host_bloom_check(c->h_bl[2].data() + (size_t)xr[0] * c->bd[2].stride, c->bd[2], xr, 32)) {
      uint64_t j;
      if (rows_search(c, xr, j)) {
        for (int sgn = 0; sgn < 2; sgn++) {
          u256 jj = u256_u64(j + 1);
          u256 k = sgn == 0 ? sc_add(calc, jj) : sc_sub(calc, jj);
          k = sc_add(k, base3);
          ge chk;
          if (c->comb.mult(chk, k) && fe_eq(chk.x, Q.x)) {
            key = k;
            return true;
          }
        }
      }
    } else if (fe_eq(S.x, c->amp3[i].x)) {
      key = sc_add(calc, base3);
      return true;
    }
  }
  return false;
}

// bsgs_secondcheck (keyhunt.cpp:5151-5184) in two halves.  second_mask: the layer-2 hits of the
// 32 points S + AMP2[i] (S = Q - base_key*G) as a bit mask -- the host twin of k_refine;
// second_finish: the reference's loop over those hits, calling bsgs_thirdcheck in order.
u256 second_base_key(const kh_ctx *c, const u256 &base, uint64_t a) {
  return sc_add(base, sc_reduce(u256_from_u128((u128)a * 2 * c->info.m)));
}
uint32_t second_mask(const kh_ctx *c, const u256 &base_key, const ge &Q) {
  ge bp;
  if (!c->comb.mult(bp, base_key)) return 0;
  fe_neg(bp.y, bp.y);
  ge S;
  ge_add(S, Q, bp);
  fe xs[32];
  add32_x(S, c->amp2, xs);
  uint32_t mask = 0;
  for (int i = 0; i < 32; i++) {
    uint8_t xr[32];
    fe_to_be(xr, xs[i]);
    if (host_bloom_check(c->h_bl[1].data() + (size_t)xr[0] * c->bd[1].stride, c->bd[1], xr, 32)) mask |= 1u << i;
  }
  return mask;
}
bool second_finish(const kh_ctx *c, const u256 &base_key, uint32_t mask, const ge &Q, u256 &key) {
  for (int i = 0; i < 32; i++)
    if (((mask >> i) & 1) && third_check(c, base_key, (uint32_t)i, Q, key)) return true;
  return false;
}

}  // namespace

namespace {

int ensure_pipeline(kh_ctx *c, uint32_t L, int H) {
  for (int i = 0; i < 2; i++) {
    if (!c->d_cnt2[i]) {
      HIPCHK(c, hipMalloc(&c->d_cnt2[i], 4));
      HIPCHK(c, hipMalloc(&c->d_hits2[i], (size_t)c->cand_cap * sizeof(kh_dev_hit)));
      HIPCHK(c, hipHostMalloc(&c->h_cnt2[i], 4, hipHostMallocDefault));
      HIPCHK(c, hipHostMalloc(&c->h_hits2[i], (size_t)c->cand_cap * sizeof(kh_dev_hit), hipHostMallocDefault));
      for (int j = 0; j < 4; j++) HIPCHK(c, hipEventCreate(&c->ev_round[i][j]));
    }
  }
  if (L > c->h_scal_cap) {
    for (int i = 0; i < 2; i++) {
      if (c->h_scal2[i]) (void)hipHostFree(c->h_scal2[i]);
      c->h_scal2[i] = nullptr;
      HIPCHK(c, hipHostMalloc(&c->h_scal2[i], (size_t)L * 32, hipHostMallocDefault));
    }
    c->h_scal_cap = L;
  }
  return ensure_lanes(c, L, walk_pad_rows(KM_BSGSB, false, H));  // the giant walks' sparse pad
}

// grow the per-round candidate buffers to hold `need` entries (stream must be idle)
int grow_candidates(kh_ctx *c, uint64_t need) {
  uint64_t cap = c->cand_cap;
  while (cap < need) cap *= 2;
  if (cap > (1u << 28)) {
    c->err = "first-level candidates per round exceed 2^28";
    return KH_E_OVERFLOW;
  }
  for (int i = 0; i < 2; i++) {
    (void)hipFree(c->d_hits2[i]);
    if (c->h_hits2[i]) (void)hipHostFree(c->h_hits2[i]);
    c->d_hits2[i] = nullptr;
    c->h_hits2[i] = nullptr;
  }
  c->cand_cap = (uint32_t)cap;
  for (int i = 0; i < 2; i++) {
    HIPCHK(c, hipMalloc(&c->d_hits2[i], (size_t)cap * sizeof(kh_dev_hit)));
    HIPCHK(c, hipHostMalloc(&c->h_hits2[i], (size_t)cap * sizeof(kh_dev_hit), hipHostMallocDefault));
  }
  return KH_OK;
}

// candidates copied back with each round's count; more are fetched on demand
constexpr uint32_t KH_CAND_EAGER = 4096;

struct bsgs_round {
  uint64_t g0, rg;   // rounds over bases: walk groups [g0, g0 + rg) of this call;
                     // continuous mode: groups [g0, g0 + rg) of every lane
  uint64_t t_round;  // giant index of the round's point 0 (continuous mode: 0, indices are global)
  uint32_t L;
  uint64_t gpl;
  uint32_t launches;
  uint64_t points;
  bool setup;        // the round (re)started its lanes
};

// giant points per pipelined round of continuous mode: 2^34 (2^21 lanes x 2 groups of 4096, one
// launch).  Every launch starts its first batch of waves in phase; two groups per lane per launch
// walked 41.1 G giant points/s against 40.05 at one (2^33) and 40.7 at four (2^35), three repeats each,
// spread 0.05 % (profiles/r05ae_round_ab.json); in the bench's BSGS leg four groups ran 43.0 vs 40.1
// at one on another box (r05ab_bench_round_points.json); eight groups per launch lost 1-14 %
constexpr uint64_t KH_BSGS_ROUND_POINTS = 1ULL << 34;

}  // namespace

// The giant-step scan behind kh_bsgs_scan (bases start + b*2N) and kh_bsgs_scan_list (any bases).
static int bsgs_scan_one(kh_ctx *ctx, const u256 &st, const std::vector<u256> *list, uint64_t n_bases,
                         kh_bsgs_found *found, uint32_t cap, uint32_t *n_found) {
  if (!ctx->bsgs_built) return KH_E_STATE;
  (void)hipSetDevice(ctx->device);
  *n_found = 0;
  if (n_bases == 0) return KH_OK;
  const kh_bsgs_info &I = ctx->info;
  const uint64_t A_pts = I.cycles * 1024;  // giant points walked per base (cycles x 1024)
  // Continuous mode: when a base's walk ends exactly where the next base's starts (cycles*1024 ==
  // aux, every power-of-two k), P_t = Q - (start + M + 2M t)G is ONE progression over the whole
  // call.  Lanes then own long runs of t, start once, and every round just continues them.
  // Otherwise (bases overlap, SURVEY parity note 13) rounds restart lanes per base run.
  const bool cont = !list && A_pts == I.aux;
  // group half-size: the large groups (one inversion per 2*KH_WALK_HB points) whenever a base holds
  // whole ones (every power-of-two k >= 16); otherwise the reference's 1024-point group
  const int H = (A_pts % (2 * KH_WALK_HB) == 0 && !getenv("KH_NO_BIG_GROUPS")) ? KH_WALK_HB : KH_WALK_H;
  auto base_of = [&](uint64_t b) {
    return list ? (*list)[b] : sc_add(st, sc_reduce(u256_from_u128((u128)b * 2 * I.n)));
  };
  // GSn[i] = -(i+1)*2M*G  (keyhunt.cpp:1797-1816)
  const uint32_t *tab = nullptr;
  int r = get_table(ctx, sc_neg(u256_u64(2 * I.m)), &tab, H);
  if (r) return r;
  if (!ctx->refine_threads) {
    unsigned hw = std::thread::hardware_concurrency();
    ctx->refine_threads = std::max(1u, std::min(16u, hw ? hw : 4u));
  }
  uint32_t nf = 0;
  // two groups per lane per launch (KH_BSGS_ROUND_POINTS below): per-base rounds too
  uint32_t per_launch = ctx->groups_per_launch ? ctx->groups_per_launch : 2;
  if (const char *e = getenv("KH_BSGS_GROUPS_PER_LAUNCH")) per_launch = std::max(1u, (uint32_t)strtoul(e, nullptr, 0));  // A/B knob
  // giant points of this call: t in [0, n_bases*A); t -> base b = t / A, a = t % A; the centre
  // of a group whose first point is t sits at key base_b + M + 2M*(a + H).
  const uint64_t gpb = A_pts / (2 * H);  // walk groups per base
  const uint64_t total_groups = n_bases * gpb;
  // lanes per launch: lanes_bsgs (2^21: eight waves per wave slot in turn, kh_kernels.h) for the
  // large groups when the call holds that many groups and the device has room for their pad, else
  // the largest power of two below it that fits (down to lanes_max, 2^18: one wave per slot).  The
  // count must tile the call (below): plan()'s balanced count for a 7274496-base call (1039214
  // lanes) walked 6 % slower than 2^20 (profiles/r05q_geom_lanes_count.json)
  uint32_t lanes = ctx->lanes_max, wide = ctx->lanes_force ? ctx->lanes_force : ctx->lanes_pick ? ctx->lanes_pick : ctx->lanes_bsgs;
  if (const char *e = getenv("KH_BSGS_LANES")) wide = (uint32_t)strtoul(e, nullptr, 0);  // A/B knob
  if (getenv("KH_BSGS_NARROW")) wide = lanes;
  if (H == KH_WALK_HB) {
    // a wider geometry is taken only if it leaves 32 GB of the device free for other contexts (their
    // tables are built while this one walks: `-g N` on one GPU)
    const uint64_t rows = (uint64_t)walk_pad_rows(KM_BSGSB, false, H);
    const uint64_t have = ctx->lanes_alloc >= lanes ? (uint64_t)ctx->lanes_alloc * ((uint64_t)ctx->scratch_h * 32 + 96) : 0;
    size_t fr = 0, tot = 0;
    const bool known = hipMemGetInfo(&fr, &tot) == hipSuccess;
    for (uint32_t w = wide; w > lanes; w >>= 1) {
      if (total_groups < w) continue;
      const uint64_t need = (uint64_t)w * (rows * 32 + 96);
      if (known && need > have && fr + have < need + (32ull << 30)) continue;
      if (ensure_pipeline(ctx, w, H) == KH_OK) {
        lanes = w;
        break;
      }
      (void)hipGetLastError();  // out of device memory (other contexts): a smaller geometry
      ctx->err.clear();
    }
  }
  ctx->lanes_used = H == KH_WALK_HB ? lanes : 0;
  job_geom jc{};
  uint64_t gpr = 0;  // continuous mode: groups per lane per round
  if (cont) {
    // interleaved lanes: lane g walks groups g, g + L, g + 2L, ... of the call, so after the call
    // it sits on group g of the call that starts where this one ends (kept across calls)
    jc = plan(ctx, total_groups, 0, lanes);
    // keep the power-of-two lane count when the ragged last round (lanes past the call's end walk
    // unprobed) costs at most 1/32 of the call: the balanced count plan() picks otherwise (e.g.
    // 1039214 lanes for a 7274496-base call) walked 6 % slower than 2^20 lanes, interleaved on one
    // box (profiles/r05q_geom_lanes_count.json)
    if (total_groups >= lanes) {
      const uint64_t gpl = (total_groups + lanes - 1) / lanes;
      if ((gpl * lanes - total_groups) * 32 <= total_groups) {
        jc.L = lanes;
        jc.gpl = gpl;
      }
    }
    uint64_t round_pts = KH_BSGS_ROUND_POINTS;
    if (const char *e = getenv("KH_BSGS_ROUND_POINTS")) round_pts = strtoull(e, nullptr, 0);  // A/B knob
    gpr = std::max<uint64_t>(1, round_pts / ((uint64_t)jc.L * 2 * H));
    gpr = std::min<uint64_t>(gpr, jc.gpl);
    r = get_table(ctx, sc_neg(u256_u64(2 * I.m)), &tab, H, jc.L);
    if (r) return r;
  } else if (!list) {
    ctx->cont_valid = false;
  }
  if (list) ctx->cont_valid = false;
  // lane g ends the call on group g + gpl*L of it: the first group of the next call only when the
  // lanes tile the call exactly (else a following call starts its lanes again)
  const bool keep_lanes = cont && ctx->targets.size() == 1 && (uint64_t)jc.L * jc.gpl == total_groups;
  // second check on the GPU: the kernel derives base_key from the candidate's giant index
  const bool gpu_refine = !ctx->refine_host;
  // per-base rounds derive their lane scalars on the device (k_setup prog 2) unless a centre key can
  // reach n (key = base + M + 2M*(a0 + H) <= base + vmax; 0 mod n only at base + v = n) or
  // KH_HOST_CENTRES is set; the host loop cost ~50 ns per lane, 2^18 lanes a round
  bool dev_centres = !cont && !getenv("KH_HOST_CENTRES");
  const u256 vmax = u256_from_u128((u128)I.m * (2 * (A_pts + H) + 1));
  if (dev_centres && !list) {
    u256 top;
    dev_centres = !u256_add_raw(top, st, vmax) && !reaches_order(top, u256_from_u128((u128)2 * I.n), n_bases - 1);
  }
  if (list) {
    // the bases as device limbs, packed on the host threads into a pinned buffer (a serial pass over
    // 2^20 bases and a pageable copy took ~15 ms of each CLI call), with the centre-key check
    if (n_bases > ctx->ref_list_cap) {
      (void)hipFree(ctx->d_ref_list);
      if (ctx->h_ref_list) (void)hipHostFree(ctx->h_ref_list);
      ctx->d_ref_list = ctx->h_ref_list = nullptr;
      ctx->ref_list_cap = 0;
      HIPCHK(ctx, hipMalloc(&ctx->d_ref_list, (size_t)n_bases * 32));
      HIPCHK(ctx, hipHostMalloc(&ctx->h_ref_list, (size_t)n_bases * 32, hipHostMallocDefault));
      ctx->ref_list_cap = n_bases;
    }
    u256 thr;
    u256_sub_raw(thr, ORDER_N, vmax);
    std::atomic<bool> risky{false};
    uint32_t *hl = ctx->h_ref_list;
    parallel_for(n_bases, ctx->refine_threads, [&](uint64_t lo, uint64_t hi) {
      bool r = false;
      for (uint64_t b = lo; b < hi; b++) {
        u256_to_limbs(hl + b * 8, (*list)[b]);
        r |= u256_cmp((*list)[b], thr) >= 0;
      }
      if (r) risky = true;
    });
    if (risky) dev_centres = false;
  }
  if (gpu_refine || dev_centres) {
    uint32_t sl[8];
    u256_to_limbs(sl, st);
    HIPCHK(ctx, hipMemcpyAsync(ctx->d_ref_start, sl, 32, hipMemcpyHostToDevice, ctx->stream));
    if (list)
      HIPCHK(ctx, hipMemcpyAsync(ctx->d_ref_list, ctx->h_ref_list, (size_t)n_bases * 32, hipMemcpyHostToDevice,
                                 ctx->stream));
  }
  auto centre_scalar = [&](uint64_t t0) {  // -(key of the centre of the group starting at t0)
    uint64_t b = t0 / A_pts, a0 = t0 % A_pts;
    u256 kb = sc_add(base_of(b), sc_reduce(u256_from_u128((u128)I.m + (u128)2 * I.m * (a0 + H))));
    return sc_neg(kb);
  };
  for (uint32_t tgt = 0; tgt < ctx->targets.size(); tgt++) {
    if (ctx->found[tgt]) continue;
    const ge Q = ctx->targets[tgt];
    // rounds are pipelined: the GPU walks round r+1 while the host refines round r's
    // first-level candidates
    // per-base rounds (list mode, overlapping bases): up to `lanes` bases per round, each lane
    // walking a divisor of gpb groups (plan), so large calls start one lane per base and small
    // ones still fill ~lanes_max lanes
    const uint64_t round_max = (uint64_t)lanes * gpb;
    const uint64_t g_end = cont ? jc.gpl : total_groups;
    uint64_t g0 = 0;
    // continuous mode: (re)start the lanes at group g0, unless the previous call left them here
    bool need_setup = !(keep_lanes && ctx->cont_valid && ctx->cont_kind == 0 && ctx->cont_tgt == tgt &&
                        ctx->cont_L == jc.L && ctx->cont_H == H && u256_cmp(ctx->cont_next, st) == 0);
    ctx->cont_valid = false;
    int cur = 0, pending = -1;
    bsgs_round rounds[2];
    bool done = false;
    uint32_t Qw[16];
    memcpy(Qw, Q.x.d, 32);
    memcpy(Qw + 8, Q.y.d, 32);
    if (!ctx->d_q) HIPCHK(ctx, hipMalloc(&ctx->d_q, 64));
    uint32_t *dq = ctx->d_q;
    HIPCHK(ctx, hipMemcpyAsync(dq, Qw, 64, hipMemcpyHostToDevice, ctx->stream));
    auto enqueue = [&](int slot) -> int {
      bsgs_round &R = rounds[slot];
      uint64_t rg;
      job_geom jg;
      if (cont) {
        rg = std::min<uint64_t>(g_end - g0, gpr);
        jg = jc;
        R.t_round = 0;
      } else {
        rg = std::min<uint64_t>(g_end - g0, round_max);
        jg = plan(ctx, rg, gpb, lanes);  // a lane's run never crosses a base
        R.t_round = g0 * 2 * H;
      }
      R.g0 = g0;
      R.rg = rg;
      R.L = jg.L;
      R.gpl = jg.gpl;
      int rr = ensure_pipeline(ctx, jg.L, H);
      if (rr) return rr;
      if (!cont || need_setup) {
        setup_args S;
        memset(&S, 0, sizeof S);
        if (dev_centres) {
          S.prog = 2;
          S.list = list ? ctx->d_ref_list : nullptr;
          S.start = ctx->d_ref_start;
          S.t_round = R.t_round;
          S.lane_pts = jg.gpl * 2 * H;
          S.a_pts = A_pts;
          S.two_n = 2 * I.n;
          S.m = I.m;
          S.h = (uint32_t)H;
        } else {
          uint32_t *hs = ctx->h_scal2[slot];
          for (uint32_t g = 0; g < jg.L; g++) {
            uint64_t t0 = cont ? (g0 * jc.L + g) * 2 * H : R.t_round + (uint64_t)g * jg.gpl * 2 * H;
            u256_to_limbs(hs + (size_t)g * 8, centre_scalar(t0));
          }
          HIPCHK(ctx, hipMemcpyAsync(ctx->d_scalars, hs, (size_t)jg.L * 32, hipMemcpyHostToDevice, ctx->stream));
        }
        S.scalars = ctx->d_scalars;
        S.comb = ctx->d_comb;
        S.q = dq;
        S.has_q = 1;
        S.L = jg.L;
        S.cx = ctx->d_cx;
        S.cy = ctx->d_cy;
        HIPCHK(ctx, hipEventRecord(ctx->ev_round[slot][0], ctx->stream));
        HIPCHK(ctx, launch_setup(S, ctx->stream));
        need_setup = false;
        R.setup = true;
      } else {
        R.setup = false;
        HIPCHK(ctx, hipEventRecord(ctx->ev_round[slot][0], ctx->stream));
      }
      HIPCHK(ctx, hipEventRecord(ctx->ev_round[slot][1], ctx->stream));
      HIPCHK(ctx, hipMemsetAsync(ctx->d_cnt2[slot], 0, 4, ctx->stream));
      walk_args Aw;
      memset(&Aw, 0, sizeof Aw);
      Aw.tab = tab;
      Aw.cx = ctx->d_cx;
      Aw.cy = ctx->d_cy;
      Aw.scratch = ctx->d_scratch;
      Aw.L = jg.L;
      Aw.pad_skew = ctx->pad_skew;
      Aw.pad_swz = pad_swizzle(Aw.L);
      Aw.lane_stride = jg.gpl * 2 * H;
      Aw.interleave = cont ? 1 : 0;
      Aw.n_points = cont ? total_groups * 2 * H : rg * 2 * H;
      Aw.bloom = ctx->d_bl[0];
      Aw.bd = ctx->bd[0];
      Aw.bstride32 = (uint32_t)ctx->bd[0].stride;  // < 2^32: checked by kh_bsgs_setup
      Aw.hit_count = ctx->d_cnt2[slot];
      Aw.hits = ctx->d_hits2[slot];
      Aw.hit_cap = ctx->cand_cap;
      R.launches = 0;
      R.points = 0;
      const uint64_t gb0 = cont ? g0 : 0, gb1 = cont ? g0 + rg : jg.gpl;
      for (uint64_t gb = gb0; gb < gb1; gb += per_launch) {
        Aw.group_base = gb;
        Aw.groups = (uint32_t)std::min<uint64_t>(per_launch, gb1 - gb);
        HIPCHK(ctx, launch_walk(ctx->info.layer1_layout == KH_LAYER1_BLOCKED ? KM_BSGSB : KM_BSGS, Aw, ctx->stream, H));
        R.launches++;
        // probed points: continuous mode's ragged last round walks lanes past the call unprobed
        uint64_t real = (uint64_t)jg.L * Aw.groups;
        if (cont) {
          const uint64_t lo = gb * jg.L, hi = std::min<uint64_t>((gb + Aw.groups) * jg.L, total_groups);
          real = hi > lo ? hi - lo : 0;
        }
        R.points += real * 2 * H;
      }
      HIPCHK(ctx, hipEventRecord(ctx->ev_round[slot][2], ctx->stream));
      HIPCHK(ctx, hipStreamWaitEvent(ctx->side, ctx->ev_round[slot][2], 0));
      if (gpu_refine) {  // second check of this round's candidates, in place (aux = layer-2 mask)
        refine_args Ra;
        memset(&Ra, 0, sizeof Ra);
        Ra.cands = ctx->d_hits2[slot];
        Ra.count = ctx->d_cnt2[slot];
        Ra.cap = ctx->cand_cap;
        Ra.list_mode = list ? 1 : 0;
        Ra.t_round = R.t_round;
        Ra.a_pts = A_pts;
        Ra.two_n = 2 * I.n;
        Ra.two_m = 2 * I.m;
        Ra.start = ctx->d_ref_start;
        Ra.list = ctx->d_ref_list;
        Ra.comb = ctx->d_comb;
        Ra.q = dq;
        Ra.amp2 = ctx->d_amp2;
        Ra.bloom2 = ctx->d_bl[1];
        Ra.bd2 = ctx->bd[1];
        HIPCHK(ctx, launch_refine(Ra, ctx->side));
      }
      HIPCHK(ctx, hipMemcpyAsync(ctx->h_cnt2[slot], ctx->d_cnt2[slot], 4, hipMemcpyDeviceToHost, ctx->side));
      HIPCHK(ctx, hipMemcpyAsync(ctx->h_hits2[slot], ctx->d_hits2[slot],
                                 (size_t)std::min(ctx->cand_cap, KH_CAND_EAGER) * sizeof(kh_dev_hit),
                                 hipMemcpyDeviceToHost, ctx->side));
      HIPCHK(ctx, hipEventRecord(ctx->ev_round[slot][3], ctx->side));
      g0 += rg;
      return KH_OK;
    };
    // wait for round `slot`, account its time, refine its candidates in parallel.  Returns 1 when
    // the round overflowed the candidate buffer: the buffers were grown and the caller redoes it.
    auto finish = [&](int slot) -> int {
      bsgs_round &R = rounds[slot];
      // ev[3] follows the walk and the candidate copies of this round only
      HIPCHK(ctx, hipEventSynchronize(ctx->ev_round[slot][3]));
      float ms_setup = 0, ms_walk = 0;
      (void)hipEventElapsedTime(&ms_setup, ctx->ev_round[slot][0], ctx->ev_round[slot][1]);
      (void)hipEventElapsedTime(&ms_walk, ctx->ev_round[slot][1], ctx->ev_round[slot][2]);
      if (R.setup) {
        ctx->tm[4].launches++;
        ctx->tm[4].ms += ms_setup;
        ctx->tm[4].points += R.L;
      }
      ctx->tm[2].launches += R.launches;
      ctx->tm[2].ms += ms_walk;
      ctx->tm[2].points += R.points;
      uint32_t cnt = *ctx->h_cnt2[slot];
      if (cnt > ctx->cand_cap) {
        HIPCHK(ctx, hipStreamSynchronize(ctx->stream));  // drain the speculative next round
        HIPCHK(ctx, hipStreamSynchronize(ctx->side));
        int rr = grow_candidates(ctx, (uint64_t)cnt * 2);
        return rr ? rr : 1;
      }
      if (cnt > KH_CAND_EAGER)
        HIPCHK(ctx, hipMemcpy(ctx->h_hits2[slot] + KH_CAND_EAGER, ctx->d_hits2[slot] + KH_CAND_EAGER,
                              (size_t)(cnt - KH_CAND_EAGER) * sizeof(kh_dev_hit), hipMemcpyDeviceToHost));
      std::vector<kh_dev_hit> dh(ctx->h_hits2[slot], ctx->h_hits2[slot] + cnt);
      std::sort(dh.begin(), dh.end(), [](const kh_dev_hit &x, const kh_dev_hit &y) { return x.idx < y.idx; });
      ctx->candidates += cnt;
      std::vector<uint8_t> ok(dh.size(), 0);
      std::vector<u256> keys(dh.size());
      auto key_of = [&](size_t i) {
        uint64_t t = R.t_round + dh[i].idx;
        return second_base_key(ctx, base_of(t / A_pts), t % A_pts);
      };
      if (!gpu_refine) {  // layer-2 masks on host threads (KH_REFINE=host)
        std::atomic<size_t> next{0};
        auto work = [&]() {
          for (;;) {
            size_t i = next++;
            if (i >= dh.size()) break;
            dh[i].aux = second_mask(ctx, key_of(i), Q);
          }
        };
        unsigned nt = std::min<unsigned>(ctx->refine_threads, (unsigned)dh.size());
        if (nt <= 1) {
          work();
        } else {
          std::vector<std::thread> th;
          for (unsigned k = 0; k < nt; k++) th.emplace_back(work);
          for (auto &x : th) x.join();
        }
      }
      if (ctx->log_cands)
        for (auto &h : dh) {
          const uint64_t t = R.t_round + h.idx;
          ctx->cand_log_base.push_back(t / A_pts);
          ctx->cand_log_a.push_back((uint32_t)(t % A_pts));
          ctx->cand_log_mask.push_back(h.aux);
        }
      // third checks for the (rare) layer-2 hits, in giant-step order; stop at the first key
      for (size_t i = 0; i < dh.size(); i++) {
        const uint64_t t = R.t_round + dh[i].idx;
        if (ctx->base_check && t % A_pts == 0) {
          // bsgsd's test of each base point against the target (bsgsd.cpp:2544-2561): a key at the
          // very start of a base is a candidate at a = 0 whose S = Q - base*G is the point at
          // infinity, which no second check can refine (the CLI misses it, bsgsd reports it)
          const u256 b = base_of(t / A_pts);
          ge bp;
          if (ctx->comb.mult(bp, b) && fe_eq(bp.x, Q.x) && fe_eq(bp.y, Q.y)) {
            keys[i] = b;
            ok[i] = 1;
            break;
          }
        }
        if (!dh[i].aux) continue;
        ctx->second_hits += (uint64_t)__builtin_popcount(dh[i].aux);
        const u256 bk = key_of(i);
        if (second_finish(ctx, bk, dh[i].aux, Q, keys[i])) {
          ok[i] = 1;
          break;
        }
      }
      for (size_t i = 0; i < dh.size(); i++)
        if (ok[i]) {  // the first candidate (in giant-step order) that refines to a key
          ctx->found[tgt] = 1;
          if (found && nf < cap) {
            found[nf].target = tgt;
            found[nf].pad = 0;
            u256_to_be(found[nf].key, keys[i]);
          }
          nf++;
          done = true;
          break;
        }
      return KH_OK;
    };
    while ((g0 < g_end || pending >= 0) && !done) {
      int nxt = -1;
      if (g0 < g_end) {
        r = enqueue(cur);
        if (r) return r;
        nxt = cur;
        cur ^= 1;
      }
      if (pending >= 0) {
        const uint64_t redo = rounds[pending].g0;
        r = finish(pending);
        if (r == 1) {  // overflowed: walk again from that round with the larger buffers
          g0 = redo;
          need_setup = true;  // continuous mode: the lanes already moved past it
          pending = -1;
          continue;
        }
        if (r) return r;
      }
      pending = nxt;
    }
    if (pending >= 0 && done) {  // drain the speculative round
      (void)hipStreamSynchronize(ctx->stream);
      (void)hipStreamSynchronize(ctx->side);
    }
    if (keep_lanes && !done && g0 == g_end) {  // every lane walked all its groups of this call
      ctx->cont_valid = true;
      ctx->cont_kind = 0;
      ctx->cont_next = sc_add(st, sc_reduce(u256_from_u128((u128)n_bases * 2 * I.n)));
      ctx->cont_tgt = tgt;
      ctx->cont_L = jc.L;
      ctx->cont_H = H;
    }
  }
  *n_found = nf;
  return nf > cap ? KH_E_OVERFLOW : KH_OK;
}

// The giant walk's rate depends on where its 64-GB inversion pad (and on some boxes its layer 1) land in
// physical memory and on the box: the same process walks 1-8 % faster on one allocation of the pad than
// on another, with identical instruction and request counts; the slow placements show only longer L2
// request latencies in cycles at a higher clock (DESIGN.md §2 "Placement", profiles/r06f_state_counters.json,
// r06j_buffer_replacement.json).  A context's first continuous call of at least 2^23 walk groups therefore
// calibrates: it walks the call's parts on candidate placements in the order A B B A (A B C C B A, ...),
// so a linear drift of clock or power cancels, times each part on the walk's events and keeps the faster.
// The default candidates are 2^21 and 2^20 lanes on the one pad (2^20 lanes walk its first half: other
// physical pages) -- the form that measured best over five boxes (profiles/r06n..r06q_calibration_ab.json:
// 41.2 G giant points/s mean against 40.7 uncalibrated, never below 39.4).  Opt-in stages, measured no
// better: KH_PAD_CANDIDATES=N (N pads of the same size held at once, each at 2^21 lanes; with
// KH_CAL_LANES=1 the primary at 2^20 lanes too), KH_CAL_STAGES=2 (then a stage over layer 1: a copy in a
// new allocation), KH_CAL_MOVE=1 (the pad moved once or twice instead), KH_CAL_DEFER=N (the first N calls
// uncalibrated).  Neither buffer holds state across launches that a swap could break: the pad is
// rewritten by every group and the layer-1 copies are identical, so the lanes run on through the swaps.
// KH_BSGS_CALIBRATE=0, KH_BSGS_LANES or kh_set_geometry's lanes switch the calibration off.  Every base
// is walked once either way, so keys and candidates are those of an uncalibrated call.
static constexpr int KH_CAL_SKIP = 1000;  // cal_stage: nothing walked, no candidate fits
struct cal_slot {
  void *base;  // the allocation (freed when the slot loses)
  void *ptr;   // what the walk reads (the pad: base + KH_PAD_OFFSET)
};
static void cal_swap(kh_ctx *ctx, int stage, cal_slot &c) {
  if (stage == 0) {
    std::swap(ctx->d_scratch_base, c.base);
    void *p = ctx->d_scratch;
    ctx->d_scratch = static_cast<uint4 *>(c.ptr);
    c.ptr = p;
  } else {
    void *p = ctx->d_bl[0];
    ctx->d_bl[0] = static_cast<uint8_t *>(c.ptr);
    c.ptr = p;
    c.base = p;
  }
}
// one calibration stage over the n_bases bases from st; returns the walk's status, hits in found
static int cal_stage(kh_ctx *ctx, int stage, const u256 &st, uint64_t n_bases, kh_bsgs_found *found, uint32_t cap,
                     uint32_t *n_found) {
  const kh_bsgs_info &I = ctx->info;
  const uint32_t hi = ctx->lanes_bsgs, lo = ctx->lanes_bsgs / 2;
  const uint64_t gpb = I.cycles * 1024 / (2 * KH_WALK_HB);
  const uint64_t rows = walk_pad_rows(KM_BSGSB, false, KH_WALK_HB);
  struct cand {
    int slot;  // 0: the primary (in ctx), k: slots[k]
    uint32_t lanes;
    double ms, pts;
  };
  std::vector<cand> cands{{0, hi, 0, 0}};
  std::vector<cal_slot> slots(1, cal_slot{nullptr, nullptr});
  size_t fr = 0, tot = 0;
  if (stage == 0) {
    const char *ncand = getenv("KH_PAD_CANDIDATES");
    const int want = std::max(1, std::min(4, ncand ? atoi(ncand) : 1));
    const uint64_t pad_bytes = ((uint64_t)hi + ctx->pad_skew) * rows * 32 + ctx->pad_offset;
    for (int k = 1; k < want; k++) {
      void *b = nullptr;
      if (hipMemGetInfo(&fr, &tot) != hipSuccess || fr < pad_bytes + (32ull << 30) ||
          dev_alloc(&b, pad_bytes, 2) != hipSuccess) {
        (void)hipGetLastError();
        break;
      }
      slots.push_back({b, static_cast<uint8_t *>(b) + ctx->pad_offset});
      cands.push_back({(int)slots.size() - 1, hi, 0, 0});
    }
    // one pad (or KH_CAL_LANES=1): 2^20 lanes, which walk the first half of the primary pad
    const char *cl = getenv("KH_CAL_LANES");
    if (cands.size() == 1 || (cl && atoi(cl))) cands.push_back({0, lo, 0, 0});
  } else {
    const size_t bytes = 256 * ctx->bd[0].stride + 4;
    void *b = nullptr;
    if (hipMemGetInfo(&fr, &tot) == hipSuccess && fr >= bytes + (32ull << 30) && dev_alloc(&b, bytes, 1) == hipSuccess &&
        hipMemcpy(b, ctx->d_bl[0], bytes, hipMemcpyDeviceToDevice) == hipSuccess) {
      slots.push_back({b, b});
      cands.push_back({1, hi, 0, 0});
    } else {
      (void)hipGetLastError();
      if (b) (void)hipFree(b);
      return KH_CAL_SKIP;  // no room for a copy: the stage is skipped
    }
  }
  const int nc = (int)cands.size();
  std::vector<int> order;
  for (int k = 0; k < nc; k++) order.push_back(k);
  for (int k = nc - 1; k >= 0; k--) order.push_back(k);
  const uint64_t tile = std::max<uint64_t>(1, hi / std::max<uint64_t>(1, gpb));
  const uint64_t nbq = std::max<uint64_t>(tile, (n_bases / order.size()) / tile * tile);
  uint32_t nf_all = 0;
  bool exact = true;
  int r = KH_OK, cur = 0;
  uint64_t done_b = 0;
  for (size_t q = 0; q < order.size() && done_b < n_bases; q++) {
    cand &c = cands[order[q]];
    const uint64_t nb = q + 1 == order.size() ? n_bases - done_b : std::min(nbq, n_bases - done_b);
    const u256 s = sc_add(st, sc_reduce(u256_from_u128((u128)done_b * 2 * I.n)));
    if (c.slot != cur) {  // swap the buffer under the running lanes (the walk is idle between calls)
      (void)hipStreamSynchronize(ctx->stream);
      (void)hipStreamSynchronize(ctx->side);
      if (cur) cal_swap(ctx, stage, slots[cur]);  // the primary back
      if (c.slot) cal_swap(ctx, stage, slots[c.slot]);
      cur = c.slot;
    }
    ctx->lanes_force = c.lanes;
    const timing t0 = ctx->tm[2];
    uint32_t nf = 0;
    const uint32_t off = std::min(nf_all, cap);
    r = bsgs_scan_one(ctx, s, nullptr, nb, found ? found + off : nullptr, cap - off, &nf);
    ctx->lanes_force = 0;
    if (ctx->lanes_used != c.lanes) exact = false;
    c.ms += ctx->tm[2].ms - t0.ms;
    c.pts += (double)(ctx->tm[2].points - t0.points);
    nf_all += nf;
    done_b += nb;
    if ((r && r != KH_E_OVERFLOW) || ctx->found[0]) break;  // an error, or the key ended the call
  }
  (void)hipStreamSynchronize(ctx->stream);
  (void)hipStreamSynchronize(ctx->side);
  int best = -1, timed = 0;
  for (int k = 0; k < nc; k++) {
    if (!(cands[k].ms > 0 && cands[k].pts > 0)) continue;
    timed++;
    if (best < 0 || cands[k].pts / cands[k].ms > cands[best].pts / cands[best].ms) best = k;
  }
  const bool decided = best >= 0 && timed == nc && exact && (r == KH_OK || r == KH_E_OVERFLOW);
  const int keep = decided ? cands[best].slot : cur;
  if (cur) cal_swap(ctx, stage, slots[cur]);     // the primary back in ctx
  if (keep) cal_swap(ctx, stage, slots[keep]);   // the kept one into ctx, the primary into its slot
  for (size_t k = 1; k < slots.size(); k++) (void)hipFree(slots[k].base);
  *n_found = nf_all;
  if (decided) {
    if (stage == 0) ctx->lanes_pick = cands[best].lanes;
    ctx->cal_rate[2 * stage] = cands[best].pts / cands[best].ms * 1e3;
    ctx->cal_rate[2 * stage + 1] = 0;
    for (int k = 0; k < nc; k++)
      if (k != best) ctx->cal_rate[2 * stage + 1] = std::max(ctx->cal_rate[2 * stage + 1], cands[k].pts / cands[k].ms * 1e3);
    ctx->cal_stage = stage + 1;
  }
  return r;
}
// KH_CAL_MOVE=1 (pad stage variant): walk a part on the current pad, move the pad (a new allocation
// taken while the old one is held, then the old one freed), walk a part; if that was slower, move once
// more and keep the third placement.  Parts of n_bases / 3 (whole tiles).
static int cal_move(kh_ctx *ctx, const u256 &st, uint64_t n_bases, kh_bsgs_found *found, uint32_t cap,
                    uint32_t *n_found) {
  const kh_bsgs_info &I = ctx->info;
  const uint32_t hi = ctx->lanes_bsgs;
  const uint64_t gpb = I.cycles * 1024 / (2 * KH_WALK_HB);
  const uint64_t tile = std::max<uint64_t>(1, hi / std::max<uint64_t>(1, gpb));
  const uint64_t nbq = std::max<uint64_t>(tile, (n_bases / 3) / tile * tile);
  double rate[3] = {0, 0, 0};
  uint32_t nf_all = 0;
  uint64_t done_b = 0;
  int r = KH_OK;
  for (int q = 0; q < 3 && done_b < n_bases; q++) {
    if (q == 2 && rate[1] >= rate[0]) break;  // the moved pad is at least as fast: keep it
    if (q > 0) {
      (void)hipStreamSynchronize(ctx->stream);
      (void)hipStreamSynchronize(ctx->side);
      r = kh_debug_replace(ctx, 2);
      if (r) return r;
    }
    const uint64_t nb = std::min(nbq, n_bases - done_b);
    const u256 s = sc_add(st, sc_reduce(u256_from_u128((u128)done_b * 2 * I.n)));
    ctx->lanes_force = hi;
    const timing t0 = ctx->tm[2];
    uint32_t nf = 0;
    const uint32_t off = std::min(nf_all, cap);
    r = bsgs_scan_one(ctx, s, nullptr, nb, found ? found + off : nullptr, cap - off, &nf);
    ctx->lanes_force = 0;
    const double ms = ctx->tm[2].ms - t0.ms, pts = (double)(ctx->tm[2].points - t0.points);
    rate[q] = ms > 0 ? pts / ms * 1e3 : 0;
    nf_all += nf;
    done_b += nb;
    if ((r && r != KH_E_OVERFLOW) || ctx->found[0]) break;
  }
  *n_found = nf_all;
  if (rate[0] > 0 && rate[1] > 0) {
    ctx->lanes_pick = hi;
    ctx->cal_rate[0] = rate[2] > 0 ? rate[2] : rate[1];
    ctx->cal_rate[1] = rate[2] > 0 ? std::max(rate[0], rate[1]) : rate[0];
    ctx->cal_stage = 1;
  }
  ctx->cal_moved_bases = done_b;
  return r;
}

static int bsgs_scan_impl(kh_ctx *ctx, const u256 &st, const std::vector<u256> *list, uint64_t n_bases,
                          kh_bsgs_found *found, uint32_t cap, uint32_t *n_found) {
  if (!ctx->bsgs_built) return KH_E_STATE;
  const kh_bsgs_info &I = ctx->info;
  const uint64_t A_pts = I.cycles * 1024;
  const uint64_t gpb = A_pts / (2 * KH_WALK_HB);
  const uint32_t hi = ctx->lanes_bsgs, lo = ctx->lanes_bsgs / 2;
  const uint64_t tile = std::max<uint64_t>(1, hi / std::max<uint64_t>(1, gpb));  // bases per 2^21 groups
  // KH_BURN_MS=<ms>: before the context's first large call, that long a VALU-dense load on the walk's
  // stream, enqueued right ahead of the walk (A/B knob for the clock/latency operating point)
  if (!ctx->burned && n_bases * gpb >= hi) {
    ctx->burned = true;
    const char *bm = getenv("KH_BURN_MS");
    const double want_ms = bm ? atof(bm) : 0.0;
    if (want_ms > 0) {
      const int rb = kh_debug_burn(ctx, want_ms);
      if (rb) return rb;
    }
  }
  const char *cal = getenv("KH_BSGS_CALIBRATE");
  const bool calibrate = !ctx->bsgs_calibrated && !list && A_pts == I.aux && A_pts % (2 * KH_WALK_HB) == 0 &&
                         hi == KH_BSGS_LANES && lo > ctx->lanes_max && !(cal && atoi(cal) == 0) &&
                         !getenv("KH_BSGS_LANES") && !getenv("KH_BSGS_NARROW") && !getenv("KH_NO_BIG_GROUPS") &&
                         n_bases * gpb >= 4ull * hi && ctx->targets.size() == 1 && !ctx->found[0];
  if (!calibrate) return bsgs_scan_one(ctx, st, list, n_bases, found, cap, n_found);
  // KH_CAL_DEFER=N: the first N eligible calls walk uncalibrated (the board settles into its power-capped
  // operating point first)
  const char *dfr = getenv("KH_CAL_DEFER");
  if (dfr && ctx->cal_deferred < (uint32_t)atoi(dfr)) {
    ctx->cal_deferred++;
    return bsgs_scan_one(ctx, st, list, n_bases, found, cap, n_found);
  }
  // the primary pad at 2^21 lanes first (bsgs_scan_one would take it too): with no room, no calibration
  {
    size_t fr = 0, tot = 0;
    const uint64_t lane_bytes = (uint64_t)hi * (walk_pad_rows(KM_BSGSB, false, KH_WALK_HB) * 32 + 96);
    const uint64_t have = ctx->lanes_alloc >= hi ? lane_bytes : 0;
    if (hipMemGetInfo(&fr, &tot) != hipSuccess || fr + have < lane_bytes + (32ull << 30) ||
        ensure_pipeline(ctx, hi, KH_WALK_HB) != KH_OK) {
      (void)hipGetLastError();
      ctx->err.clear();
      return bsgs_scan_one(ctx, st, list, n_bases, found, cap, n_found);
    }
  }
  uint32_t nf_all = 0;
  uint64_t done_b = 0;
  int r = KH_OK;
  // stages while the call has 4 tiles left for one (the last stage of the call takes the rest of it);
  // KH_CAL_STAGES=1: the pad stage only
  const char *nst = getenv("KH_CAL_STAGES");
  const int stages = std::max(1, std::min(2, nst ? atoi(nst) : 1));
  if (ctx->cal_stage >= stages) ctx->cal_stage = 2;
  while (ctx->cal_stage < stages && (n_bases - done_b) >= 4 * tile && !ctx->found[0]) {
    const uint64_t left = n_bases - done_b;
    // with a second stage to come, the first takes half of a call that holds both
    const uint64_t nb = ctx->cal_stage == 0 && stages > 1 && left >= 8 * tile ? left / 2 / tile * tile : left;
    const u256 s = sc_add(st, sc_reduce(u256_from_u128((u128)done_b * 2 * I.n)));
    uint32_t nf = 0;
    const uint32_t off = std::min(nf_all, cap);
    const int stage = ctx->cal_stage;
    const char *mv = getenv("KH_CAL_MOVE");
    uint64_t walked = nb;
    if (stage == 0 && mv && atoi(mv)) {
      r = cal_move(ctx, s, nb, found ? found + off : nullptr, cap - off, &nf);
      walked = ctx->cal_moved_bases;
    } else {
      r = cal_stage(ctx, stage, s, nb, found ? found + off : nullptr, cap - off, &nf);
    }
    if (r == KH_CAL_SKIP) {  // no room for the stage's candidate: calibration ends here
      r = KH_OK;
      ctx->cal_stage = 2;
      break;
    }
    nf_all += nf;
    done_b += walked;
    if (r && r != KH_E_OVERFLOW) return r;
    if (ctx->cal_stage == stage) {  // undecided: the key ended the call (try again next call), or a
      if (!ctx->found[0]) ctx->cal_stage = 2;  // part could not take its lane count (give up)
      break;
    }
  }
  if (ctx->cal_stage >= stages) ctx->bsgs_calibrated = true;
  if (done_b < n_bases && !ctx->found[0] && (r == KH_OK || r == KH_E_OVERFLOW)) {
    const u256 s = sc_add(st, sc_reduce(u256_from_u128((u128)done_b * 2 * I.n)));
    uint32_t nf = 0;
    const uint32_t off = std::min(nf_all, cap);
    const int r2 = bsgs_scan_one(ctx, s, nullptr, n_bases - done_b, found ? found + off : nullptr, cap - off, &nf);
    nf_all += nf;
    if (r2 && r2 != KH_E_OVERFLOW) return r2;
    if (r2) r = r2;
  }
  *n_found = nf_all;
  return *n_found > cap ? KH_E_OVERFLOW : r;
}

int kh_bsgs_scan(kh_ctx *ctx, const uint8_t start[32], uint64_t n_bases, kh_bsgs_found *found, uint32_t cap,
                 uint32_t *n_found) {
  if (!ctx || !start || !n_found) return KH_E_ARG;
  return bsgs_scan_impl(ctx, sc_reduce(u256_from_be(start)), nullptr, n_bases, found, cap, n_found);
}

int kh_bsgs_scan_list(kh_ctx *ctx, const uint8_t *bases, uint64_t n_bases, kh_bsgs_found *found, uint32_t cap,
                      uint32_t *n_found) {
  if (!ctx || (!bases && n_bases) || !n_found) return KH_E_ARG;
  std::vector<u256> list(n_bases);
  if (!ctx->refine_threads) {
    unsigned hw = std::thread::hardware_concurrency();
    ctx->refine_threads = std::max(1u, std::min(16u, hw ? hw : 4u));
  }
  parallel_for(n_bases, ctx->refine_threads, [&](uint64_t lo, uint64_t hi) {
    for (uint64_t b = lo; b < hi; b++) list[b] = sc_reduce(u256_from_be(bases + 32 * b));
  });
  return bsgs_scan_impl(ctx, u256{}, &list, n_bases, found, cap, n_found);
}

// ---------------------------------------------------------------------------------------------
// measurement
// ---------------------------------------------------------------------------------------------
int kh_bloom_add(uint8_t *bf, uint64_t bits, uint32_t hashes, const uint8_t *items, uint64_t n, uint32_t len) {
  if (!bf || !bits || (!items && n) || !len || len > 32 || (len > 20 && len != 32)) return KH_E_ARG;
  bloom_desc d;
  memset(&d, 0, sizeof d);
  d.bits = bits;
  d.hashes = hashes;
  for (uint64_t i = 0; i < n; i++) host_bloom_add(bf, d, items + i * len, (int)len);
  return KH_OK;
}

int kh_bsgs_layer_bits(kh_ctx *ctx, uint32_t layer, uint64_t bits, uint32_t hashes, uint64_t bytes, uint8_t *shards) {
  if (!ctx || layer < 1 || layer > 3 || !bits || !bytes || !shards || bits > bytes * 8) return KH_E_ARG;
  if (!ctx->bsgs_built) return KH_E_STATE;
  (void)hipSetDevice(ctx->device);
  const kh_bsgs_info &I = ctx->info;
  const uint64_t count = layer == 1 ? I.m : layer == 2 ? I.m2 : I.m3;
  bloom_desc d;
  memset(&d, 0, sizeof d);
  d.bits = bits;
  d.bytes = bytes;
  d.stride = (bytes + 255) / 256 * 256;
  d.recip = ~0ULL / bits;
  d.hashes = hashes;
  std::vector<uint8_t> h(256 * d.stride, 0);
  for (int i = 0; i < 256; i++) memcpy(&h[(size_t)i * d.stride], shards + (size_t)i * bytes, bytes);
  uint8_t *dev = nullptr;
  if (hipMalloc(&dev, h.size() + 4) != hipSuccess) return KH_E_NOMEM;
  int r = hipMemcpy(dev, h.data(), h.size(), hipMemcpyHostToDevice) == hipSuccess ? KH_OK : KH_E_HIP;
  if (r == KH_OK) r = build_walk(ctx, KM_BUILD, dev, d, nullptr, nullptr, count, true);
  if (r == KH_OK && hipMemcpy(h.data(), dev, h.size(), hipMemcpyDeviceToHost) != hipSuccess) r = KH_E_HIP;
  (void)hipFree(dev);
  if (r == KH_OK)
    for (int i = 0; i < 256; i++) memcpy(shards + (size_t)i * bytes, &h[(size_t)i * d.stride], bytes);
  return r;
}

int kh_bsgs_table_rows(kh_ctx *ctx, const uint8_t **rows, uint64_t *n_rows) {
  if (!ctx || !rows || !n_rows) return KH_E_ARG;
  if (!ctx->bsgs_built) return KH_E_STATE;
  *rows = ctx->h_rows.data();
  *n_rows = ctx->h_rows.size() / 16;
  return KH_OK;
}

int kh_bsgs_set_base_check(kh_ctx *ctx, int enable) {
  if (!ctx) return KH_E_ARG;
  ctx->base_check = enable != 0;
  return KH_OK;
}

int kh_bsgs_log_candidates(kh_ctx *ctx, int enable) {
  if (!ctx) return KH_E_ARG;
  ctx->log_cands = enable != 0;
  ctx->cand_log_base.clear();
  ctx->cand_log_a.clear();
  ctx->cand_log_mask.clear();
  return KH_OK;
}

int kh_bsgs_get_candidates(kh_ctx *ctx, uint64_t *base_index, uint32_t *a, uint32_t *mask, uint64_t cap,
                           uint64_t *n) {
  if (!ctx || !n) return KH_E_ARG;
  *n = ctx->cand_log_base.size();
  for (uint64_t i = 0; i < *n && i < cap; i++) {
    if (base_index) base_index[i] = ctx->cand_log_base[i];
    if (a) a[i] = ctx->cand_log_a[i];
    if (mask) mask[i] = ctx->cand_log_mask[i];
  }
  return *n > cap ? KH_E_OVERFLOW : KH_OK;
}

int kh_bsgs_second_masks(kh_ctx *ctx, uint32_t target, const uint8_t *base_keys, uint32_t n, uint32_t *gpu_mask,
                         uint32_t *host_mask) {
  if (!ctx || !base_keys || !gpu_mask || !host_mask) return KH_E_ARG;
  if (!ctx->bsgs_built || target >= ctx->targets.size()) return KH_E_STATE;
  (void)hipSetDevice(ctx->device);
  if (n == 0) return KH_OK;
  const ge &Q = ctx->targets[target];
  std::vector<uint32_t> lw((size_t)n * 8);
  std::vector<kh_dev_hit> c(n);
  for (uint32_t j = 0; j < n; j++) {
    u256 k = sc_reduce(u256_from_be(base_keys + (size_t)j * 32));
    u256_to_limbs(&lw[(size_t)j * 8], k);
    c[j].idx = j;  // list mode with one point per base: t = j -> base j, a = 0
    c[j].kind = 4;
    c[j].aux = 0xFFFFFFFFu;
    host_mask[j] = second_mask(ctx, k, Q);
  }
  uint32_t Qw[16];
  memcpy(Qw, Q.x.d, 32);
  memcpy(Qw + 8, Q.y.d, 32);
  uint32_t *d_list = nullptr, *d_q = nullptr, *d_cnt = nullptr;
  kh_dev_hit *d_c = nullptr;
  int rc = KH_OK;
  auto chk = [&](hipError_t e, const char *what) {
    if (e != hipSuccess && rc == KH_OK) {
      ctx->err = std::string(what) + ": " + hipGetErrorString(e);
      rc = KH_E_HIP;
    }
  };
  chk(hipMalloc(&d_list, lw.size() * 4), "hipMalloc");
  chk(hipMalloc(&d_q, 64), "hipMalloc");
  chk(hipMalloc(&d_cnt, 4), "hipMalloc");
  chk(hipMalloc(&d_c, (size_t)n * sizeof(kh_dev_hit)), "hipMalloc");
  if (rc == KH_OK) {
    chk(hipMemcpy(d_list, lw.data(), lw.size() * 4, hipMemcpyHostToDevice), "hipMemcpy");
    chk(hipMemcpy(d_q, Qw, 64, hipMemcpyHostToDevice), "hipMemcpy");
    chk(hipMemcpy(d_cnt, &n, 4, hipMemcpyHostToDevice), "hipMemcpy");
    chk(hipMemcpy(d_c, c.data(), (size_t)n * sizeof(kh_dev_hit), hipMemcpyHostToDevice), "hipMemcpy");
  }
  if (rc == KH_OK) {
    refine_args Ra;
    memset(&Ra, 0, sizeof Ra);
    Ra.cands = d_c;
    Ra.count = d_cnt;
    Ra.cap = n;
    Ra.list_mode = 1;
    Ra.a_pts = 1;
    Ra.two_n = 2 * ctx->info.n;
    Ra.two_m = 2 * ctx->info.m;
    Ra.start = ctx->d_ref_start;
    Ra.list = d_list;
    Ra.comb = ctx->d_comb;
    Ra.q = d_q;
    Ra.amp2 = ctx->d_amp2;
    Ra.bloom2 = ctx->d_bl[1];
    Ra.bd2 = ctx->bd[1];
    chk(launch_refine(Ra, ctx->stream), "k_refine");
    chk(hipStreamSynchronize(ctx->stream), "hipStreamSynchronize");
    chk(hipMemcpy(c.data(), d_c, (size_t)n * sizeof(kh_dev_hit), hipMemcpyDeviceToHost), "hipMemcpy");
    for (uint32_t j = 0; j < n; j++) gpu_mask[j] = c[j].aux;
  }
  (void)hipFree(d_list);
  (void)hipFree(d_q);
  (void)hipFree(d_cnt);
  (void)hipFree(d_c);
  return rc;
}

int kh_kernel_time(kh_ctx *ctx, uint32_t kind, uint64_t *launches, double *ms, uint64_t *points) {
  if (!ctx || kind > 4) return KH_E_ARG;
  if (launches) *launches = ctx->tm[kind].launches;
  if (ms) *ms = ctx->tm[kind].ms;
  if (points) *points = ctx->tm[kind].points;
  return KH_OK;
}

int kh_kernel_time_reset(kh_ctx *ctx) {
  if (!ctx) return KH_E_ARG;
  for (auto &t : ctx->tm) t = timing();
  return KH_OK;
}

// ---------------------------------------------------------------------------------------------
// parity hooks
// ---------------------------------------------------------------------------------------------
int kh_pubkeys(kh_ctx *ctx, const uint8_t *scalars, uint32_t n, uint8_t *xy) {
  if (!ctx || !scalars || !xy || !n) return KH_E_ARG;
  (void)hipSetDevice(ctx->device);
  std::vector<u256> s(n);
  for (uint32_t i = 0; i < n; i++) {
    s[i] = sc_reduce(u256_from_be(scalars + 32 * i));
    if (u256_is_zero(s[i])) return KH_E_ARG;
  }
  int r = run_setup(ctx, s, nullptr);
  if (r) return r;
  std::vector<uint32_t> cx((size_t)n * 8), cy((size_t)n * 8);
  for (int w = 0; w < 8; w++) {
    HIPCHK(ctx, hipMemcpy(&cx[(size_t)w * n], ctx->d_cx + (size_t)w * n, (size_t)n * 4, hipMemcpyDeviceToHost));
    HIPCHK(ctx, hipMemcpy(&cy[(size_t)w * n], ctx->d_cy + (size_t)w * n, (size_t)n * 4, hipMemcpyDeviceToHost));
  }
  for (uint32_t i = 0; i < n; i++) {
    fe x, y;
    for (int w = 0; w < 8; w++) {
      x.d[w] = cx[(size_t)w * n + i];
      y.d[w] = cy[(size_t)w * n + i];
    }
    fe_to_be(xy + 64 * i, x);
    fe_to_be(xy + 64 * i + 32, y);
  }
  return KH_OK;
}

int kh_walk_points(kh_ctx *ctx, const uint8_t start[32], const uint8_t stride_be[32], uint64_t n_points,
                   uint8_t *out_x, uint8_t *out_y) {
  if (!ctx || !start || !out_x || !n_points || n_points % (2 * KH_WALK_H)) return KH_E_ARG;
  (void)hipSetDevice(ctx->device);
  const int H = KH_WALK_H;
  u256 st = sc_reduce(u256_from_be(start));
  u256 stride = stride_be ? sc_reduce(u256_from_be(stride_be)) : u256_u64(1);
  const uint32_t *tab = nullptr;
  int r = get_table(ctx, stride, &tab);
  if (r) return r;
  job_geom jg = plan(ctx, n_points / (2 * H), 0);
  std::vector<u256> s(jg.L);
  for (uint32_t g = 0; g < jg.L; g++) {
    u128 off = (u128)g * jg.gpl * 2 * H + H;
    u256 acc = u256_u64(0), x = stride;
    for (int b = 0; b < 128; b++) {
      if ((off >> b) & 1) acc = sc_add(acc, x);
      x = sc_add(x, x);
    }
    s[g] = sc_add(st, acc);
  }
  r = run_setup(ctx, s, nullptr);
  if (r) return r;
  uint32_t *dx = nullptr, *dy = nullptr;
  HIPCHK(ctx, hipMalloc(&dx, n_points * 32));
  if (out_y) HIPCHK(ctx, hipMalloc(&dy, n_points * 32));
  walk_args A;
  memset(&A, 0, sizeof A);
  A.tab = tab;
  A.cx = ctx->d_cx;
  A.cy = ctx->d_cy;
  A.scratch = ctx->d_scratch;
  A.L = jg.L;
  A.pad_skew = ctx->pad_skew;
  A.pad_swz = pad_swizzle(A.L);
  A.lane_stride = jg.gpl * 2 * H;
  A.n_points = n_points;
  A.dump_x = dx;
  A.dump_y = dy;
  r = run_walk(ctx, KM_DUMP, 0, A, jg.gpl, 4);
  if (r) {
    (void)hipFree(dx);
    (void)hipFree(dy);
    return r;
  }
  std::vector<uint32_t> hx(n_points * 8), hy(out_y ? n_points * 8 : 0);
  HIPCHK(ctx, hipMemcpy(hx.data(), dx, n_points * 32, hipMemcpyDeviceToHost));
  if (out_y) HIPCHK(ctx, hipMemcpy(hy.data(), dy, n_points * 32, hipMemcpyDeviceToHost));
  (void)hipFree(dx);
  (void)hipFree(dy);
  for (uint64_t i = 0; i < n_points; i++) {
    fe x;
    memcpy(x.d, &hx[i * 8], 32);
    fe_to_be(out_x + 32 * i, x);
    if (out_y) {
      fe y;
      memcpy(y.d, &hy[i * 8], 32);
      fe_to_be(out_y + 32 * i, y);
    }
  }
  return KH_OK;
}

int kh_hash160(kh_ctx *ctx, const uint8_t *xy, uint32_t n, uint8_t *out60) {
  if (!ctx || !xy || !out60 || !n) return KH_E_ARG;
  (void)hipSetDevice(ctx->device);
  std::vector<uint32_t> hx((size_t)n * 8), hy((size_t)n * 8), ho((size_t)n * 15);
  for (uint32_t i = 0; i < n; i++) {
    fe x, y;
    fe_from_be(x, xy + 64 * i);
    fe_from_be(y, xy + 64 * i + 32);
    memcpy(&hx[(size_t)i * 8], x.d, 32);
    memcpy(&hy[(size_t)i * 8], y.d, 32);
  }
  uint32_t *dx, *dy, *dout;
  HIPCHK(ctx, hipMalloc(&dx, hx.size() * 4));
  HIPCHK(ctx, hipMalloc(&dy, hy.size() * 4));
  HIPCHK(ctx, hipMalloc(&dout, ho.size() * 4));
  HIPCHK(ctx, hipMemcpy(dx, hx.data(), hx.size() * 4, hipMemcpyHostToDevice));
  HIPCHK(ctx, hipMemcpy(dy, hy.data(), hy.size() * 4, hipMemcpyHostToDevice));
  HIPCHK(ctx, launch_test_hash160(dx, dy, n, dout, ctx->stream));
  HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
  HIPCHK(ctx, hipMemcpy(ho.data(), dout, ho.size() * 4, hipMemcpyDeviceToHost));
  (void)hipFree(dx);
  (void)hipFree(dy);
  (void)hipFree(dout);
  memcpy(out60, ho.data(), (size_t)n * 60);
  return KH_OK;
}

int kh_field_ops(kh_ctx *ctx, const uint8_t *a, const uint8_t *b, uint32_t n, uint8_t *out160) {
  if (!ctx || !a || !b || !out160 || !n) return KH_E_ARG;
  (void)hipSetDevice(ctx->device);
  std::vector<uint32_t> ha((size_t)n * 8), hb((size_t)n * 8), ho((size_t)n * 40);
  for (uint32_t i = 0; i < n; i++) {
    fe x, y;
    fe_from_be(x, a + 32 * i);
    fe_from_be(y, b + 32 * i);
    memcpy(&ha[(size_t)i * 8], x.d, 32);
    memcpy(&hb[(size_t)i * 8], y.d, 32);
  }
  uint32_t *da, *db, *dout;
  HIPCHK(ctx, hipMalloc(&da, ha.size() * 4));
  HIPCHK(ctx, hipMalloc(&db, hb.size() * 4));
  HIPCHK(ctx, hipMalloc(&dout, ho.size() * 4));
  HIPCHK(ctx, hipMemcpy(da, ha.data(), ha.size() * 4, hipMemcpyHostToDevice));
  HIPCHK(ctx, hipMemcpy(db, hb.data(), hb.size() * 4, hipMemcpyHostToDevice));
  HIPCHK(ctx, launch_test_field(da, db, n, dout, ctx->stream));
  HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
  HIPCHK(ctx, hipMemcpy(ho.data(), dout, ho.size() * 4, hipMemcpyDeviceToHost));
  (void)hipFree(da);
  (void)hipFree(db);
  (void)hipFree(dout);
  for (uint32_t i = 0; i < n; i++)
    for (int k = 0; k < 5; k++) {
      fe r;
      memcpy(r.d, &ho[(size_t)i * 40 + 8 * k], 32);
      fe_to_be(out160 + 160 * i + 32 * k, r);
    }
  return KH_OK;
}

int kh_bloom_check(kh_ctx *ctx, uint32_t layer, const uint8_t *items, uint32_t n, uint32_t len, uint8_t *out) {
  if (!ctx || !items || !out || !n || (len != 20 && len != 32) || layer > 3) return KH_E_ARG;
  (void)hipSetDevice(ctx->device);
  const uint8_t *bl;
  bloom_desc d;
  if (layer == 0) {
    if (!ctx->d_tbloom) return KH_E_STATE;
    bl = ctx->d_tbloom;
    d = ctx->tbd;
  } else {
    if (!ctx->bsgs_ready) return KH_E_STATE;
    bl = ctx->d_bl[layer - 1];
    d = ctx->bd[layer - 1];
  }
  uint8_t *ditems;
  uint32_t *dout;
  HIPCHK(ctx, hipMalloc(&ditems, (size_t)n * len));
  HIPCHK(ctx, hipMalloc(&dout, (size_t)n * 4));
  HIPCHK(ctx, hipMemcpy(ditems, items, (size_t)n * len, hipMemcpyHostToDevice));
  uint32_t blocked = (layer == 1 && ctx->info.layer1_layout == KH_LAYER1_BLOCKED) ? 1 : 0;
  HIPCHK(ctx, launch_test_bloom(ditems, n, len, bl, d, layer ? 1 : 0, blocked, dout, ctx->stream));
  HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
  std::vector<uint32_t> ho(n);
  HIPCHK(ctx, hipMemcpy(ho.data(), dout, (size_t)n * 4, hipMemcpyDeviceToHost));
  (void)hipFree(ditems);
  (void)hipFree(dout);
  for (uint32_t i = 0; i < n; i++) out[i] = (uint8_t)ho[i];
  return KH_OK;
}

int kh_get_bloom(kh_ctx *ctx, uint32_t layer, uint8_t *buf, uint64_t cap, uint64_t *bytes) {
  if (!ctx || layer > 3 || !bytes) return KH_E_ARG;
  (void)hipSetDevice(ctx->device);
  if (layer == 0) {
    if (!ctx->d_tbloom) return KH_E_STATE;
    *bytes = ctx->tbd.bytes;
    if (!buf) return KH_OK;
    if (cap < ctx->tbd.bytes) return KH_E_OVERFLOW;
    HIPCHK(ctx, hipMemcpy(buf, ctx->d_tbloom, ctx->tbd.bytes, hipMemcpyDeviceToHost));
    return KH_OK;
  }
  if (!ctx->bsgs_ready) return KH_E_STATE;
  const bloom_desc &d = ctx->bd[layer - 1];
  *bytes = 256 * d.bytes;
  if (!buf) return KH_OK;
  if (cap < 256 * d.bytes) return KH_E_OVERFLOW;
  HIPCHK(ctx, hipMemcpy2D(buf, d.bytes, ctx->d_bl[layer - 1], d.stride, d.bytes, 256, hipMemcpyDeviceToHost));
  return KH_OK;
}

int kh_get_bsgs_table(kh_ctx *ctx, uint8_t *buf, uint64_t cap_rows, uint64_t *rows) {
  if (!ctx || !rows) return KH_E_ARG;
  if (!ctx->bsgs_built) return KH_E_STATE;
  *rows = ctx->info.m3;
  if (!buf) return KH_OK;
  if (cap_rows < ctx->info.m3) return KH_E_OVERFLOW;
  memcpy(buf, ctx->h_rows.data(), ctx->h_rows.size());
  return KH_OK;
}

// --load-ptable (keyhunt.cpp:1871-1892): the rows come from the caller's file, as the reference's
// mapping of that file replaces the table thread_bPload would have written (5404, 5587).  Like
// the reference, the rows are taken as they are: neither checked nor re-sorted.
int kh_bsgs_set_table(kh_ctx *ctx, const uint8_t *rows, uint64_t n_rows) {
  if (!ctx || !rows) return KH_E_ARG;
  if (!ctx->bsgs_built) return KH_E_STATE;
  if (n_rows != ctx->info.m3) {
    ctx->err = "bP table rows " + std::to_string(n_rows) + " != M3 " + std::to_string(ctx->info.m3);
    return KH_E_ARG;
  }
  ctx->h_rows.assign(rows, rows + n_rows * 16);
  return KH_OK;
}

}  // extern "C"
