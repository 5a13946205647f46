/*
 * kh_oracle.c -- CPU restatement of keyhunt's hot path.  TEST INFRASTRUCTURE ONLY.
 *
 * This file is the parity oracle for the MI355X engine in keyhunt_amd/.  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it, and only as a checker
 * (or as the timed CPU baseline).  The product path (libkh_gpu.so, keyhunt-amd) never links,
 * loads or calls anything in oracle/.
 *
 * Written from scratch in plain C (gcc, unsigned __int128) from the published algorithms; every
 * function names the reference file:line whose behaviour it restates (paths relative to the
 * reference checkout, naanprofit/keyhunt @ 0.2.230519):
 *   - secp256k1 field / group arithmetic ....... secp256k1/IntMod.cpp, secp256k1/SECP256K1.cpp
 *   - batched (Montgomery-trick) inversion ...... secp256k1/IntGroup.cpp:36-58
 *   - 1024-point group walk ..................... keyhunt.cpp:3349-3461, 3840-3855
 *   - hash160 of 02/03||X and 04||X||Y ......... secp256k1/SECP256K1.cpp:974-1250, hash/ (sha256, ripemd160)
 *   - XXH64 (xxHash 0.8.0) ...................... xxhash/xxhash.h:2290-2529
 *   - libbloom2 sizing / add / check ............ bloom/bloom.cpp:122-218
 *   - sorted 20-byte table + searchbinary ....... keyhunt.cpp:3065-3089
 *   - BSGS params / baby build / giant walk /
 *     second & third check ..................... keyhunt.cpp:1454-1842, 4549-4888, 5151-5248,
 *                                                5284-5472, 4510-4544, 7859-7868
 *
 * Parity of this restatement is pinned by (a) the reference's own fixture data (puzzle
 * addresses / hash160s / pubkeys with known private keys: tests/golden/data, README known
 * answers) and (b) golden vectors produced by the reference itself compiled from its sources
 * by oracle/Makefile.ref into oracle/_ref/ (tests/golden/ref_vectors.json, generator
 * oracle/ref_golden.cpp + oracle/make_golden.py).
 *
 * Conventions: field elements / scalars are 4 x uint64 little-endian limbs internally and
 * 32-byte BIG-endian at the API (Int::Get32Bytes, secp256k1/Int.cpp:308-316).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <math.h>
#include <pthread.h>

typedef unsigned __int128 u128;
typedef struct { uint64_t v[4]; } fe;          /* field element / 256-bit scalar */
typedef struct { fe x, y; int inf; } ge;        /* affine point */
typedef struct { fe x, y, z; int inf; } gej;    /* jacobian point */

/* p = 2^256 - 2^32 - 977 (SECP256K1.cpp Init) */
static const fe FE_P = {{0xFFFFFFFEFFFFFC2FULL, 0xFFFFFFFFFFFFFFFFULL, 0xFFFFFFFFFFFFFFFFULL, 0xFFFFFFFFFFFFFFFFULL}};
/* group order n */
static const fe SC_N = {{0xBFD25E8CD0364141ULL, 0xBAAEDCE6AF48A03BULL, 0xFFFFFFFFFFFFFFFEULL, 0xFFFFFFFFFFFFFFFFULL}};
static const fe GX = {{0x59F2815B16F81798ULL, 0x029BFCDB2DCE28D9ULL, 0x55A06295CE870B07ULL, 0x79BE667EF9DCBBACULL}};
static const fe GY = {{0x9C47D08FFB10D4B8ULL, 0xFD17B448A6855419ULL, 0x5DA4FBFC0E1108A8ULL, 0x483ADA7726A3C465ULL}};

/* ------------------------------------------------------------------------------------------ */
/* 256-bit helpers                                                                             */
/* ------------------------------------------------------------------------------------------ */
static void fe_from_be(fe *r, const uint8_t b[32]) {
  for (int i = 0; i < 4; i++) {
    uint64_t w = 0;
    for (int j = 0; j < 8; j++) w = (w << 8) | b[(3 - i) * 8 + j];
    r->v[i] = w;
  }
}
static void fe_to_be(uint8_t b[32], const fe *a) {
  for (int i = 0; i < 4; i++)
    for (int j = 0; j < 8; j++) b[(3 - i) * 8 + j] = (uint8_t)(a->v[i] >> (56 - 8 * j));
}
static int u256_cmp(const fe *a, const fe *b) {
  for (int i = 3; i >= 0; i--) {
    if (a->v[i] < b->v[i]) return -1;
    if (a->v[i] > b->v[i]) return 1;
  }
  return 0;
}
static int u256_is_zero(const fe *a) { return (a->v[0] | a->v[1] | a->v[2] | a->v[3]) == 0; }
/* r = a + b, returns carry */
static uint64_t u256_add(fe *r, const fe *a, const fe *b) {
  u128 c = 0;
  for (int i = 0; i < 4; i++) { c += (u128)a->v[i] + b->v[i]; r->v[i] = (uint64_t)c; c >>= 64; }
  return (uint64_t)c;
}
/* r = a - b, returns borrow */
static uint64_t u256_sub(fe *r, const fe *a, const fe *b) {
  uint64_t br = 0;
  for (int i = 0; i < 4; i++) {
    u128 t = (u128)a->v[i] - b->v[i] - br;
    r->v[i] = (uint64_t)t;
    br = (uint64_t)(t >> 64) & 1;
  }
  return br;
}
static void u256_add_u64(fe *r, const fe *a, uint64_t b) {
  fe t = {{b, 0, 0, 0}};
  u256_add(r, a, &t);
}

/* ------------------------------------------------------------------------------------------ */
/* Field arithmetic mod p.  IntMod.cpp:41-108 (ModAdd/ModSub/ModNeg), 855-915 (ModMulK1:       */
/* 512-bit product folded with 0x1000003D1), 977-1093 (ModSquareK1).  Results here are always  */
/* canonical (< p); the reference skips the last conditional subtraction (IntMod.cpp:912),     */
/* which only matters with probability ~2^-224 (SURVEY 8a parity note 5).                       */
/* ------------------------------------------------------------------------------------------ */
static void fe_norm(fe *a) {
  if (u256_cmp(a, &FE_P) >= 0) u256_sub(a, a, &FE_P);
}
static void fe_add(fe *r, const fe *a, const fe *b) {
  uint64_t c = u256_add(r, a, b);
  if (c || u256_cmp(r, &FE_P) >= 0) u256_sub(r, r, &FE_P);
}
static void fe_sub(fe *r, const fe *a, const fe *b) {
  if (u256_sub(r, a, b)) u256_add(r, r, &FE_P);
}
static void fe_neg(fe *r, const fe *a) {
  fe z = {{0, 0, 0, 0}};
  fe_sub(r, &z, a);
}
static void fe_mul(fe *r, const fe *a, const fe *b) {
  uint64_t t[8] = {0};
  for (int i = 0; i < 4; i++) {
    u128 c = 0;
    for (int j = 0; j < 4; j++) {
      c += (u128)a->v[i] * b->v[j] + t[i + j];
      t[i + j] = (uint64_t)c;
      c >>= 64;
    }
    t[i + 4] = (uint64_t)c;
  }
  /* fold: lo + hi * 0x1000003D1 */
  const uint64_t K = 0x1000003D1ULL;
  u128 c = 0;
  uint64_t r5[5];
  for (int i = 0; i < 4; i++) {
    c += (u128)t[i + 4] * K + t[i];
    r5[i] = (uint64_t)c;
    c >>= 64;
  }
  r5[4] = (uint64_t)c;
  c = (u128)r5[4] * K + r5[0];
  r->v[0] = (uint64_t)c; c >>= 64;
  for (int i = 1; i < 4; i++) { c += r5[i]; r->v[i] = (uint64_t)c; c >>= 64; }
  if (c) { /* wrapped past 2^256: add K once more (cannot carry again) */
    u128 d = (u128)r->v[0] + K;
    r->v[0] = (uint64_t)d; d >>= 64;
    for (int i = 1; i < 4 && d; i++) { d += r->v[i]; r->v[i] = (uint64_t)d; d >>= 64; }
  }
  fe_norm(r);
}
static void fe_sqr(fe *r, const fe *a) { fe_mul(r, a, a); }
/* a^(p-2) (Fermat).  The reference uses DRS62 xgcd (IntMod.cpp:382-511); both are the
 * unique inverse.  0 maps to 0 as in IntMod.cpp:497-500. */
static void fe_inv(fe *r, const fe *a) {
  fe e = FE_P;
  e.v[0] -= 2;
  fe res = {{1, 0, 0, 0}}, base = *a;
  for (int i = 255; i >= 0; i--) {
    fe_sqr(&res, &res);
    if ((e.v[i >> 6] >> (i & 63)) & 1) fe_mul(&res, &res, &base);
  }
  *r = res;
}
/* square root (p = 3 mod 4): a^((p+1)/4) */
static int fe_sqrt(fe *r, const fe *a) {
  fe e = FE_P;
  u256_add_u64(&e, &e, 1);
  /* e >>= 2 */
  for (int i = 0; i < 4; i++) e.v[i] = (e.v[i] >> 2) | (i < 3 ? e.v[i + 1] << 62 : 0);
  fe res = {{1, 0, 0, 0}};
  for (int i = 255; i >= 0; i--) {
    fe_sqr(&res, &res);
    if ((e.v[i >> 6] >> (i & 63)) & 1) fe_mul(&res, &res, a);
  }
  fe chk;
  fe_sqr(&chk, &res);
  *r = res;
  return u256_cmp(&chk, a) == 0;
}

/* ------------------------------------------------------------------------------------------ */
/* Group arithmetic.  SECP256K1.cpp:455-478 (AddDirect), 589-614 (DoubleDirect), 316-324        */
/* (Negation), 702-747 (ScalarBaseMultiplication; here plain double-and-add in Jacobian).      */
/* ------------------------------------------------------------------------------------------ */
static void ge_add(ge *r, const ge *p, const ge *q) {
  if (p->inf) { *r = *q; return; }
  if (q->inf) { *r = *p; return; }
  fe dx, dy, s, s2, t;
  fe_sub(&dx, &q->x, &p->x);
  fe_sub(&dy, &q->y, &p->y);
  if (u256_is_zero(&dx)) {
    if (u256_is_zero(&dy)) { /* doubling */
      fe x2, n3, d2, inv;
      fe_sqr(&x2, &p->x);
      fe_add(&n3, &x2, &x2); fe_add(&n3, &n3, &x2);
      fe_add(&d2, &p->y, &p->y);
      fe_inv(&inv, &d2);
      fe_mul(&s, &n3, &inv);
    } else { r->inf = 1; memset(&r->x, 0, sizeof(fe)); memset(&r->y, 0, sizeof(fe)); return; }
  } else {
    fe inv;
    fe_inv(&inv, &dx);
    fe_mul(&s, &dy, &inv);
  }
  fe_sqr(&s2, &s);
  fe rx, ry;
  fe_sub(&rx, &s2, &p->x);
  fe_sub(&rx, &rx, &q->x);
  fe_sub(&t, &p->x, &rx);
  fe_mul(&ry, &s, &t);
  fe_sub(&ry, &ry, &p->y);
  r->x = rx; r->y = ry; r->inf = 0;
}
static void ge_neg(ge *r, const ge *p) { *r = *p; if (!p->inf) fe_neg(&r->y, &p->y); }
/* Secp256K1::AddDirect (secp256k1/SECP256K1.cpp:455-478): the chord formula with no special cases;
 * ModInv of dx = 0 leaves 0 (IntMod.cpp:497-500), so then s = 0 and x = -p1.x - p2.x.  Fermat's
 * 0^(p-2) is 0 as well. */
static void ge_add_direct(ge *r, const ge *p1, const ge *p2) {
  fe dx, dy, inv, s, s2, rx, ry, t;
  fe_sub(&dy, &p2->y, &p1->y);
  fe_sub(&dx, &p2->x, &p1->x);
  fe_inv(&inv, &dx);
  fe_mul(&s, &dy, &inv);
  fe_sqr(&s2, &s);
  fe_sub(&rx, &s2, &p1->x);
  fe_sub(&rx, &rx, &p2->x);
  fe_sub(&t, &p2->x, &rx);
  fe_mul(&ry, &t, &s);
  fe_sub(&ry, &ry, &p2->y);
  r->x = rx; r->y = ry; r->inf = 0;
}

static void gej_double(gej *r, const gej *p) {
  if (p->inf || u256_is_zero(&p->y)) { r->inf = 1; return; }
  fe a, b, c, d, e, f, t;
  fe_sqr(&a, &p->x);                 /* A = X^2 */
  fe_sqr(&b, &p->y);                 /* B = Y^2 */
  fe_sqr(&c, &b);                    /* C = B^2 */
  fe_add(&t, &p->x, &b); fe_sqr(&t, &t); fe_sub(&t, &t, &a); fe_sub(&t, &t, &c);
  fe_add(&d, &t, &t);                /* D = 2((X+B)^2 - A - C) */
  fe_add(&e, &a, &a); fe_add(&e, &e, &a);   /* E = 3A */
  fe_sqr(&f, &e);                    /* F = E^2 */
  gej o;
  fe_sub(&o.x, &f, &d); fe_sub(&o.x, &o.x, &d);
  fe c8; fe_add(&c8, &c, &c); fe_add(&c8, &c8, &c8); fe_add(&c8, &c8, &c8);
  fe_sub(&t, &d, &o.x); fe_mul(&o.y, &e, &t); fe_sub(&o.y, &o.y, &c8);
  fe_mul(&o.z, &p->y, &p->z); fe_add(&o.z, &o.z, &o.z);
  o.inf = 0;
  *r = o;
}
static void gej_add_ge(gej *r, const gej *p, const ge *q) {
  if (q->inf) { *r = *p; return; }
  if (p->inf) { r->x = q->x; r->y = q->y; r->z = (fe){{1, 0, 0, 0}}; r->inf = 0; return; }
  fe z2, u2, s2, h, rr, h2, h3, t;
  fe_sqr(&z2, &p->z);
  fe_mul(&u2, &q->x, &z2);
  fe_mul(&s2, &q->y, &z2); fe_mul(&s2, &s2, &p->z);
  fe_sub(&h, &u2, &p->x);
  fe_sub(&rr, &s2, &p->y);
  if (u256_is_zero(&h)) {
    if (u256_is_zero(&rr)) { gej_double(r, p); return; }
    r->inf = 1; return;
  }
  fe_sqr(&h2, &h); fe_mul(&h3, &h2, &h);
  fe v; fe_mul(&v, &p->x, &h2);
  gej o;
  fe_sqr(&o.x, &rr); fe_sub(&o.x, &o.x, &h3); fe_sub(&o.x, &o.x, &v); fe_sub(&o.x, &o.x, &v);
  fe_sub(&t, &v, &o.x); fe_mul(&o.y, &rr, &t); fe_mul(&t, &p->y, &h3); fe_sub(&o.y, &o.y, &t);
  fe_mul(&o.z, &p->z, &h);
  o.inf = 0;
  *r = o;
}
static void gej_to_ge(ge *r, const gej *p) {
  if (p->inf) { r->inf = 1; memset(&r->x, 0, sizeof(fe)); memset(&r->y, 0, sizeof(fe)); return; }
  fe zi, zi2, zi3;
  fe_inv(&zi, &p->z);
  fe_sqr(&zi2, &zi); fe_mul(&zi3, &zi2, &zi);
  fe_mul(&r->x, &p->x, &zi2);
  fe_mul(&r->y, &p->y, &zi3);
  r->inf = 0;
}
/* k*G for k a 256-bit scalar (ComputePublicKey, SECP256K1.cpp:205-207). k is reduced mod n. */
static void scalar_mult_g(ge *r, const fe *k_in) {
  fe k = *k_in;
  while (u256_cmp(&k, &SC_N) >= 0) u256_sub(&k, &k, &SC_N);
  ge g = {GX, GY, 0};
  gej acc; acc.inf = 1;
  for (int i = 255; i >= 0; i--) {
    gej_double(&acc, &acc);
    if ((k.v[i >> 6] >> (i & 63)) & 1) gej_add_ge(&acc, &acc, &g);
  }
  gej_to_ge(r, &acc);
}
/* scalar arithmetic mod n: r = a - b mod n, r = a + b mod n */
static void sc_add(fe *r, const fe *a, const fe *b) {
  uint64_t c = u256_add(r, a, b);
  if (c || u256_cmp(r, &SC_N) >= 0) u256_sub(r, r, &SC_N);
}
static void sc_neg(fe *r, const fe *a) {
  if (u256_is_zero(a)) { *r = *a; return; }
  u256_sub(r, &SC_N, a);
}
/* r = a * b mod n (Int::ModMulK1order, used with lambda for -e) by double-and-add */
static void sc_mul(fe *r, const fe *a, const fe *b) {
  fe acc = {{0, 0, 0, 0}}, x = *a;
  for (int i = 0; i < 256; i++) {
    if ((b->v[i >> 6] >> (i & 63)) & 1) sc_add(&acc, &acc, &x);
    sc_add(&x, &x, &x);
  }
  *r = acc;
}

/* ------------------------------------------------------------------------------------------ */
/* SHA-256 (FIPS 180-4), RIPEMD-160 (Dobbertin/Bosselaers/Preneel).  Reference: hash/sha256.cpp */
/* 431-527, hash/ripemd160.cpp:292-318 (scalar) and their 4-lane SSE forms.                     */
/* ------------------------------------------------------------------------------------------ */
static const uint32_t SHA_K[64] = {
  0x428a2f98,0x71374491,0xb5c0fbcf,0xe9b5dba5,0x3956c25b,0x59f111f1,0x923f82a4,0xab1c5ed5,
  0xd807aa98,0x12835b01,0x243185be,0x550c7dc3,0x72be5d74,0x80deb1fe,0x9bdc06a7,0xc19bf174,
  0xe49b69c1,0xefbe4786,0x0fc19dc6,0x240ca1cc,0x2de92c6f,0x4a7484aa,0x5cb0a9dc,0x76f988da,
  0x983e5152,0xa831c66d,0xb00327c8,0xbf597fc7,0xc6e00bf3,0xd5a79147,0x06ca6351,0x14292967,
  0x27b70a85,0x2e1b2138,0x4d2c6dfc,0x53380d13,0x650a7354,0x766a0abb,0x81c2c92e,0x92722c85,
  0xa2bfe8a1,0xa81a664b,0xc24b8b70,0xc76c51a3,0xd192e819,0xd6990624,0xf40e3585,0x106aa070,
  0x19a4c116,0x1e376c08,0x2748774c,0x34b0bcb5,0x391c0cb3,0x4ed8aa4a,0x5b9cca4f,0x682e6ff3,
  0x748f82ee,0x78a5636f,0x84c87814,0x8cc70208,0x90befffa,0xa4506ceb,0xbef9a3f7,0xc67178f2};
#define ROR32(x, n) (((x) >> (n)) | ((x) << (32 - (n))))
#define ROL32(x, n) (((x) << (n)) | ((x) >> (32 - (n))))
static void sha256_block(uint32_t st[8], const uint8_t blk[64]) {
  uint32_t w[64];
  for (int i = 0; i < 16; i++)
    w[i] = ((uint32_t)blk[4 * i] << 24) | ((uint32_t)blk[4 * i + 1] << 16) | ((uint32_t)blk[4 * i + 2] << 8) | blk[4 * i + 3];
  for (int i = 16; i < 64; i++) {
    uint32_t s0 = ROR32(w[i - 15], 7) ^ ROR32(w[i - 15], 18) ^ (w[i - 15] >> 3);
    uint32_t s1 = ROR32(w[i - 2], 17) ^ ROR32(w[i - 2], 19) ^ (w[i - 2] >> 10);
    w[i] = w[i - 16] + s0 + w[i - 7] + s1;
  }
  uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
  for (int i = 0; i < 64; i++) {
    uint32_t t1 = h + (ROR32(e, 6) ^ ROR32(e, 11) ^ ROR32(e, 25)) + ((e & f) ^ (~e & g)) + SHA_K[i] + w[i];
    uint32_t t2 = (ROR32(a, 2) ^ ROR32(a, 13) ^ ROR32(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
    h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
  }
  st[0] += a; st[1] += b; st[2] += c; st[3] += d; st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}
void or_sha256(const uint8_t *msg, uint64_t len, uint8_t out[32]) {
  uint32_t st[8] = {0x6a09e667,0xbb67ae85,0x3c6ef372,0xa54ff53a,0x510e527f,0x9b05688c,0x1f83d9ab,0x5be0cd19};
  uint8_t blk[64];
  uint64_t off = 0;
  while (len - off >= 64) { sha256_block(st, msg + off); off += 64; }
  uint64_t rem = len - off;
  memset(blk, 0, 64);
  memcpy(blk, msg + off, rem);
  blk[rem] = 0x80;
  if (rem >= 56) { sha256_block(st, blk); memset(blk, 0, 64); }
  uint64_t bits = len * 8;
  for (int i = 0; i < 8; i++) blk[63 - i] = (uint8_t)(bits >> (8 * i));
  sha256_block(st, blk);
  for (int i = 0; i < 8; i++) {
    out[4 * i] = st[i] >> 24; out[4 * i + 1] = st[i] >> 16; out[4 * i + 2] = st[i] >> 8; out[4 * i + 3] = st[i];
  }
}

static const uint8_t RMD_RL[80] = {
  0,1,2,3,4,5,6,7,8,9,10,11,12,13,14,15, 7,4,13,1,10,6,15,3,12,0,9,5,2,14,11,8,
  3,10,14,4,9,15,8,1,2,7,0,6,13,11,5,12, 1,9,11,10,0,8,12,4,13,3,7,15,14,5,6,2,
  4,0,5,9,7,12,2,10,14,1,3,8,11,6,15,13};
static const uint8_t RMD_RR[80] = {
  5,14,7,0,9,2,11,4,13,6,15,8,1,10,3,12, 6,11,3,7,0,13,5,10,14,15,8,12,4,9,1,2,
  15,5,1,3,7,14,6,9,11,8,12,2,10,0,4,13, 8,6,4,1,3,11,15,0,5,12,2,13,9,7,10,14,
  12,15,10,4,1,5,8,7,6,2,13,14,0,3,9,11};
static const uint8_t RMD_SL[80] = {
  11,14,15,12,5,8,7,9,11,13,14,15,6,7,9,8, 7,6,8,13,11,9,7,15,7,12,15,9,11,7,13,12,
  11,13,6,7,14,9,13,15,14,8,13,6,5,12,7,5, 11,12,14,15,14,15,9,8,9,14,5,6,8,6,5,12,
  9,15,5,11,6,8,13,12,5,12,13,14,11,8,5,6};
static const uint8_t RMD_SR[80] = {
  8,9,9,11,13,15,15,5,7,7,8,11,14,14,12,6, 9,13,15,7,12,8,9,11,7,7,12,7,6,15,13,11,
  9,7,15,11,8,6,6,14,12,13,5,14,13,13,7,5, 15,5,8,11,14,14,6,14,6,9,12,9,12,5,15,8,
  8,5,12,9,12,5,14,6,8,13,6,5,15,13,11,11};
static uint32_t rmd_f(int j, uint32_t x, uint32_t y, uint32_t z) {
  switch (j / 16) {
    case 0: return x ^ y ^ z;
    case 1: return (x & y) | (~x & z);
    case 2: return (x | ~y) ^ z;
    case 3: return (x & z) | (y & ~z);
    default: return x ^ (y | ~z);
  }
}
static void rmd160_block(uint32_t st[5], const uint8_t blk[64]) {
  static const uint32_t KL[5] = {0x00000000, 0x5A827999, 0x6ED9EBA1, 0x8F1BBCDC, 0xA953FD4E};
  static const uint32_t KR[5] = {0x50A28BE6, 0x5C4DD124, 0x6D703EF3, 0x7A6D76E9, 0x00000000};
  uint32_t x[16];
  for (int i = 0; i < 16; i++)
    x[i] = (uint32_t)blk[4 * i] | ((uint32_t)blk[4 * i + 1] << 8) | ((uint32_t)blk[4 * i + 2] << 16) | ((uint32_t)blk[4 * i + 3] << 24);
  uint32_t al = st[0], bl = st[1], cl = st[2], dl = st[3], el = st[4];
  uint32_t ar = al, br = bl, cr = cl, dr = dl, er = el;
  for (int j = 0; j < 80; j++) {
    uint32_t t = ROL32(al + rmd_f(j, bl, cl, dl) + x[RMD_RL[j]] + KL[j / 16], RMD_SL[j]) + el;
    al = el; el = dl; dl = ROL32(cl, 10); cl = bl; bl = t;
    t = ROL32(ar + rmd_f(79 - j, br, cr, dr) + x[RMD_RR[j]] + KR[j / 16], RMD_SR[j]) + er;
    ar = er; er = dr; dr = ROL32(cr, 10); cr = br; br = t;
  }
  uint32_t t = st[1] + cl + dr;
  st[1] = st[2] + dl + er; st[2] = st[3] + el + ar; st[3] = st[4] + al + br; st[4] = st[0] + bl + cr; st[0] = t;
}
void or_ripemd160(const uint8_t *msg, uint64_t len, uint8_t out[20]) {
  uint32_t st[5] = {0x67452301, 0xEFCDAB89, 0x98BADCFE, 0x10325476, 0xC3D2E1F0};
  uint8_t blk[64];
  uint64_t off = 0;
  while (len - off >= 64) { rmd160_block(st, msg + off); off += 64; }
  uint64_t rem = len - off;
  memset(blk, 0, 64);
  memcpy(blk, msg + off, rem);
  blk[rem] = 0x80;
  if (rem >= 56) { rmd160_block(st, blk); memset(blk, 0, 64); }
  uint64_t bits = len * 8;
  for (int i = 0; i < 8; i++) blk[56 + i] = (uint8_t)(bits >> (8 * i));
  rmd160_block(st, blk);
  for (int i = 0; i < 5; i++) {
    out[4 * i] = st[i]; out[4 * i + 1] = st[i] >> 8; out[4 * i + 2] = st[i] >> 16; out[4 * i + 3] = st[i] >> 24;
  }
}
/* hash160 of the SEC1 compressed key prefix||X (GetHash160_fromX, SECP256K1.cpp:1207-1250) */
void or_hash160_comp(const uint8_t x[32], uint8_t prefix, uint8_t out[20]) {
  uint8_t m[33], d[32];
  m[0] = prefix;
  memcpy(m + 1, x, 32);
  or_sha256(m, 33, d);
  or_ripemd160(d, 32, out);
}
/* hash160 of 04||X||Y (GetHash160 uncompressed, SECP256K1.cpp:1045-1130) */
void or_hash160_uncomp(const uint8_t x[32], const uint8_t y[32], uint8_t out[20]) {
  uint8_t m[65], d[32];
  m[0] = 4;
  memcpy(m + 1, x, 32);
  memcpy(m + 33, y, 32);
  or_sha256(m, 65, d);
  or_ripemd160(d, 32, out);
}

/* ------------------------------------------------------------------------------------------ */
/* XXH64 (xxHash 0.8.0: xxhash/xxhash.h:2290-2294 primes, 2304 round, 2468-2529 XXH64).       */
/* ------------------------------------------------------------------------------------------ */
#define XP1 0x9E3779B185EBCA87ULL
#define XP2 0xC2B2AE3D27D4EB4FULL
#define XP3 0x165667B19E3779F9ULL
#define XP4 0x85EBCA77C2B2AE63ULL
#define XP5 0x27D4EB2F165667C5ULL
static uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
static uint64_t rd64(const uint8_t *p) { uint64_t v = 0; for (int i = 7; i >= 0; i--) v = (v << 8) | p[i]; return v; }
static uint32_t rd32(const uint8_t *p) { return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24); }
static uint64_t xxr(uint64_t acc, uint64_t in) { acc += in * XP2; acc = rotl64(acc, 31); return acc * XP1; }
static uint64_t xxm(uint64_t acc, uint64_t v) { v = xxr(0, v); acc ^= v; return acc * XP1 + XP4; }
uint64_t or_xxh64(const uint8_t *p, uint64_t len, uint64_t seed) {
  const uint8_t *end = p + len;
  uint64_t h;
  if (len >= 32) {
    uint64_t v1 = seed + XP1 + XP2, v2 = seed + XP2, v3 = seed, v4 = seed - XP1;
    const uint8_t *lim = end - 32;
    do {
      v1 = xxr(v1, rd64(p)); v2 = xxr(v2, rd64(p + 8)); v3 = xxr(v3, rd64(p + 16)); v4 = xxr(v4, rd64(p + 24));
      p += 32;
    } while (p <= lim);
    h = rotl64(v1, 1) + rotl64(v2, 7) + rotl64(v3, 12) + rotl64(v4, 18);
    h = xxm(h, v1); h = xxm(h, v2); h = xxm(h, v3); h = xxm(h, v4);
  } else {
    h = seed + XP5;
  }
  h += len;
  while (end - p >= 8) { h ^= xxr(0, rd64(p)); h = rotl64(h, 27) * XP1 + XP4; p += 8; }
  if (end - p >= 4) { h ^= (uint64_t)rd32(p) * XP1; h = rotl64(h, 23) * XP2 + XP3; p += 4; }
  while (p < end) { h ^= (*p) * XP5; h = rotl64(h, 11) * XP1; p++; }
  h ^= h >> 33; h *= XP2; h ^= h >> 29; h *= XP3; h ^= h >> 32;
  return h;
}

/* ------------------------------------------------------------------------------------------ */
/* libbloom2 (bloom/bloom.cpp:154-187 bloom_init2 sizing, 122-146 bloom_check_add, 189-212     */
/* bloom_check).  The sizing is done in long double exactly like the reference (bpe is stored  */
/* as double, bloom.h:43).                                                                     */
/* ------------------------------------------------------------------------------------------ */
#define BLOOM_SEED 0x59f2815b16f81798ULL
/* Keccak-256, original 0x01 padding (sha3/sha3.c:229 KECCAK_256_Final; keyhunt.cpp:5647-5653) */
static const uint64_t KEC_RC[24] = {
    0x0000000000000001ULL, 0x0000000000008082ULL, 0x800000000000808aULL, 0x8000000080008000ULL,
    0x000000000000808bULL, 0x0000000080000001ULL, 0x8000000080008081ULL, 0x8000000000008009ULL,
    0x000000000000008aULL, 0x0000000000000088ULL, 0x0000000080008009ULL, 0x000000008000000aULL,
    0x000000008000808bULL, 0x800000000000008bULL, 0x8000000000008089ULL, 0x8000000000008003ULL,
    0x8000000000008002ULL, 0x8000000000000080ULL, 0x000000000000800aULL, 0x800000008000000aULL,
    0x8000000080008081ULL, 0x8000000000008080ULL, 0x0000000080000001ULL, 0x8000000080008008ULL};
/* the state as a 5x5 array a[x + 5y]; rho offsets r[x][y] and pi (x, y) -> (y, 2x + 3y) written out */
static void keccak_f(uint64_t a[25]) {
  static const int R[25] = {0, 1, 62, 28, 27, 36, 44, 6, 55, 20, 3, 10, 43, 25, 39, 41, 45, 15, 21, 8, 18, 2, 61, 56, 14};
  for (int r = 0; r < 24; r++) {
    uint64_t c[5], b[25];
    for (int x = 0; x < 5; x++) c[x] = a[x] ^ a[x + 5] ^ a[x + 10] ^ a[x + 15] ^ a[x + 20];
    for (int x = 0; x < 5; x++)
      for (int y = 0; y < 5; y++) a[x + 5 * y] ^= c[(x + 4) % 5] ^ rotl64(c[(x + 1) % 5], 1);
    for (int x = 0; x < 5; x++)
      for (int y = 0; y < 5; y++) {
        uint64_t v = a[x + 5 * y];
        int rr = R[x + 5 * y];
        b[y + 5 * ((2 * x + 3 * y) % 5)] = rr ? rotl64(v, rr) : v;
      }
    for (int x = 0; x < 5; x++)
      for (int y = 0; y < 5; y++) a[x + 5 * y] = b[x + 5 * y] ^ (~b[(x + 1) % 5 + 5 * y] & b[(x + 2) % 5 + 5 * y]);
    a[0] ^= KEC_RC[r];
  }
}
void or_keccak256(const uint8_t *msg, uint64_t len, uint8_t out[32]) {
  uint64_t a[25] = {0};
  uint8_t blk[136];
  uint64_t off = 0;
  for (;;) {
    uint64_t n = len - off < 136 ? len - off : 136;
    memset(blk, 0, 136);
    memcpy(blk, msg + off, n);
    if (n < 136) {  /* last block: pad 0x01 ... 0x80 */
      blk[n] ^= 0x01;
      blk[135] ^= 0x80;
    }
    for (int i = 0; i < 17; i++) a[i] ^= rd64(blk + 8 * i);
    keccak_f(a);
    off += n;
    if (n < 136) break;
  }
  for (int i = 0; i < 32; i++) out[i] = (uint8_t)(a[i / 8] >> (8 * (i % 8)));
}
/* generate_binaddress_eth (keyhunt.cpp:5663-5669): Keccak-256(X||Y) bytes 12..31 */
void or_eth_address(const uint8_t x[32], const uint8_t y[32], uint8_t out[20]) {
  uint8_t m[64], d[32];
  memcpy(m, x, 32);
  memcpy(m + 32, y, 32);
  or_keccak256(m, 64, d);
  memcpy(out, d + 12, 20);
}

int or_bloom_params(uint64_t entries, double error, uint64_t *bits, uint64_t *bytes, uint32_t *hashes) {
  if (entries < 1000 || error <= 0 || error >= 1) return 1;
  long double err = (long double)error;
  long double num = -logl(err);
  long double denom = 0.480453013918201;
  double bpe = (double)(num / denom);
  long double allbits = (long double)entries * bpe;
  *bits = (uint64_t)allbits;
  *bytes = *bits / 8 + ((*bits % 8) ? 1 : 0);
  *hashes = (uint32_t)(uint8_t)ceil(0.693147180559945 * bpe);
  return 0;
}
/* keyhunt's entries rule for a target table (initBloomFilter, keyhunt.cpp:7605-7626) and for
 * the BSGS shards (keyhunt.cpp:1633-1661 then initBloomFilter's max(10000, items)). */
uint64_t or_bloom_entries(uint64_t items) { return items <= 10000 ? 10000 : items; }

int or_bloom_add(uint8_t *bf, uint64_t bits, uint32_t hashes, const uint8_t *buf, int len) {
  uint64_t a = or_xxh64(buf, len, BLOOM_SEED);
  uint64_t b = or_xxh64(buf, len, a);
  int hits = 0;
  for (uint32_t i = 0; i < hashes; i++) {
    uint64_t x = (a + b * i) % bits;
    uint8_t m = (uint8_t)(1u << (x & 7));
    if (bf[x >> 3] & m) hits++; else bf[x >> 3] |= m;
  }
  return hits == (int)hashes;
}
int or_bloom_check(const uint8_t *bf, uint64_t bits, uint32_t hashes, const uint8_t *buf, int len) {
  uint64_t a = or_xxh64(buf, len, BLOOM_SEED);
  uint64_t b = or_xxh64(buf, len, a);
  for (uint32_t i = 0; i < hashes; i++) {
    uint64_t x = (a + b * i) % bits;
    if (!(bf[x >> 3] & (1u << (x & 7)))) return 0;
  }
  return 1;
}
/* bit positions a bloom probe would test (all `hashes`, no early exit) */
void or_bloom_positions(uint64_t bits, uint32_t hashes, const uint8_t *buf, int len, uint64_t *out) {
  uint64_t a = or_xxh64(buf, len, BLOOM_SEED);
  uint64_t b = or_xxh64(buf, len, a);
  for (uint32_t i = 0; i < hashes; i++) out[i] = (a + b * i) % bits;
}

/* ------------------------------------------------------------------------------------------ */
/* searchbinary (keyhunt.cpp:3065-3089): the reference's own midpoint loop, restated literally  */
/* because its exact probing is what decides a hit.                                            */
/* ------------------------------------------------------------------------------------------ */
int or_searchbinary(const uint8_t *rows, int64_t n, const uint8_t *key, int width, int key_off) {
  int64_t half = n, min = 0, max = n, cur = 0;
  while (half >= 1) {
    half = (max - min) / 2;
    int c = memcmp(key + key_off, rows + (cur + half) * width, width);
    if (c == 0) return 1;
    if (c < 0) max = max - half; else min = min + half;
    cur = min;
  }
  return 0;
}

/* ------------------------------------------------------------------------------------------ */
/* Public EC helpers                                                                           */
/* ------------------------------------------------------------------------------------------ */
void or_fe_mul(const uint8_t a[32], const uint8_t b[32], uint8_t out[32]) {
  fe x, y, r; fe_from_be(&x, a); fe_from_be(&y, b); fe_norm(&x); fe_norm(&y); fe_mul(&r, &x, &y); fe_to_be(out, &r);
}
void or_fe_inv(const uint8_t a[32], uint8_t out[32]) {
  fe x, r; fe_from_be(&x, a); fe_norm(&x); fe_inv(&r, &x); fe_to_be(out, &r);
}
/* returns 1 if k*G is the point at infinity */
int or_pubkey(const uint8_t k[32], uint8_t x[32], uint8_t y[32]) {
  fe kk; ge r;
  fe_from_be(&kk, k);
  scalar_mult_g(&r, &kk);
  fe_to_be(x, &r.x); fe_to_be(y, &r.y);
  return r.inf;
}
/* ParsePublicKeyHex for 02/03 compressed keys: recover y of the requested parity. */
int or_decompress(const uint8_t x[32], int odd, uint8_t y[32]) {
  fe X, r, t, s;
  fe_from_be(&X, x);
  fe_sqr(&t, &X); fe_mul(&t, &t, &X);
  fe seven = {{7, 0, 0, 0}};
  fe_add(&t, &t, &seven);
  if (!fe_sqrt(&s, &t)) return 0;
  if ((int)(s.v[0] & 1) != odd) fe_neg(&s, &s);
  r = s;
  fe_to_be(y, &r);
  return 1;
}
/* generic affine add of two points given as big-endian coordinate pairs */
int or_point_add(const uint8_t ax[32], const uint8_t ay[32], const uint8_t bx[32], const uint8_t by[32],
                 uint8_t rx[32], uint8_t ry[32]) {
  ge a, b, r;
  fe_from_be(&a.x, ax); fe_from_be(&a.y, ay); a.inf = 0;
  fe_from_be(&b.x, bx); fe_from_be(&b.y, by); b.inf = 0;
  ge_add(&r, &a, &b);
  fe_to_be(rx, &r.x); fe_to_be(ry, &r.y);
  return r.inf;
}

/* ------------------------------------------------------------------------------------------ */
/* The reference's 1024-point group walk (keyhunt.cpp:3349-3461 + IntGroup.cpp:36-58).         */
/* Gn[i] = (i+1)*stride*G, i < 512.  For a group starting at key K the centre is C = (K +      */
/* 512*stride)G and pts[t] = (K + t*stride)G for t in [0, 1024).  X only; Y when need_y.       */
/* Batch inversion collapses to all-zero when any dx is 0 (SURVEY parity note 4) -- restated.  */
/* ------------------------------------------------------------------------------------------ */
#define GRP 1024
#define HALF 512
typedef struct { ge gn[HALF]; ge g2n; } walk_tab;

static void build_walk_tab(walk_tab *t, const fe *stride) {
  ge g; scalar_mult_g(&g, stride);
  t->gn[0] = g;
  ge d; ge_add(&d, &g, &g);
  t->gn[1] = d;
  for (int i = 2; i < HALF; i++) ge_add(&t->gn[i], &t->gn[i - 1], &g);
  ge_add(&t->g2n, &t->gn[HALF - 1], &t->gn[HALF - 1]);
}
/* IntGroup::ModInv: Montgomery trick over n elements, in place */
static void batch_inv(fe *a, int n) {
  fe *sub = (fe *)malloc(sizeof(fe) * n);
  sub[0] = a[0];
  for (int i = 1; i < n; i++) fe_mul(&sub[i], &sub[i - 1], &a[i]);
  fe inv; fe_inv(&inv, &sub[n - 1]);
  for (int i = n - 1; i > 0; i--) {
    fe newv; fe_mul(&newv, &sub[i - 1], &inv);
    fe_mul(&inv, &inv, &a[i]);
    a[i] = newv;
  }
  a[0] = inv;
  free(sub);
}
/* one group of 2*half points from centre C (affine, with y): pts[0..2*half), next centre written
 * to *next.  half = HALF is the reference's 1024-key group.  A smaller half is -m rmd160
 * --rmd-batch-size 2*half (keyhunt.cpp:3301-3307, 3349-3461): the reference still inverts its
 * whole IntGroup of HALF + 1 elements (3274), of which only dx[0..half] are ever set -- the rest
 * keep Int's zero -- so the product and every inverse are 0 (IntGroup.cpp:36-58, ModInv(0) = 0),
 * as they are here: the same formulas then give the reference's points. */
static void walk_group_n(const walk_tab *t, const ge *c, ge *pts, int need_y, ge *next, int half) {
  fe dx[HALF + 1];
  int i;
  memset(dx, 0, sizeof dx);
  for (i = 0; i < half; i++) fe_sub(&dx[i], &t->gn[i].x, &c->x);
  fe_sub(&dx[half], &t->g2n.x, &c->x);
  batch_inv(dx, HALF + 1);
  pts[half] = *c;
  for (i = 0; i < half; i++) {
    fe dy, s, p2, tmp;
    /* c + Gn[i] */
    if (i < half - 1) {
      ge pp;
      fe_sub(&dy, &t->gn[i].y, &c->y);
      fe_mul(&s, &dy, &dx[i]);
      fe_sqr(&p2, &s);
      fe_sub(&pp.x, &p2, &c->x); fe_sub(&pp.x, &pp.x, &t->gn[i].x);
      if (need_y) { fe_sub(&tmp, &t->gn[i].x, &pp.x); fe_mul(&pp.y, &tmp, &s); fe_sub(&pp.y, &pp.y, &t->gn[i].y); }
      else memset(&pp.y, 0, sizeof(fe));
      pp.inf = 0;
      pts[half + i + 1] = pp;
    }
    /* c - Gn[i] */
    ge pn; fe ny;
    fe_neg(&ny, &t->gn[i].y);
    fe_sub(&dy, &ny, &c->y);
    fe_mul(&s, &dy, &dx[i]);
    fe_sqr(&p2, &s);
    fe_sub(&pn.x, &p2, &c->x); fe_sub(&pn.x, &pn.x, &t->gn[i].x);
    if (need_y) { fe_sub(&tmp, &t->gn[i].x, &pn.x); fe_mul(&pn.y, &tmp, &s); fe_add(&pn.y, &pn.y, &t->gn[i].y); }
    else memset(&pn.y, 0, sizeof(fe));
    pn.inf = 0;
    pts[half - i - 1] = pn;
  }
  if (next) {
    fe dy, s, p2, tmp;
    fe_sub(&dy, &t->g2n.y, &c->y);
    fe_mul(&s, &dy, &dx[half]);
    fe_sqr(&p2, &s);
    fe_sub(&next->x, &p2, &c->x); fe_sub(&next->x, &next->x, &t->g2n.x);
    fe_sub(&tmp, &t->g2n.x, &next->x); fe_mul(&next->y, &tmp, &s); fe_sub(&next->y, &next->y, &t->g2n.y);
    next->inf = 0;
  }
}
static void walk_group(const walk_tab *t, const ge *c, ge *pts, int need_y, ge *next) {
  walk_group_n(t, c, pts, need_y, next, HALF);
}

/* X coordinates (and optionally Y) of keys K + t*stride for t in [0, n_groups*1024), computed by
 * the group walk.  Like the reference, each group's centre comes from a fresh scalar mult
 * (keyhunt.cpp:3349-3353).  out_x/out_y: n*32 bytes big-endian. */
void or_walk_points(const uint8_t start_be[32], const uint8_t stride_be[32], uint64_t n_groups,
                    uint8_t *out_x, uint8_t *out_y) {
  fe key, stride, half;
  fe_from_be(&key, start_be);
  fe_from_be(&stride, stride_be);
  walk_tab *t = (walk_tab *)malloc(sizeof(walk_tab));
  build_walk_tab(t, &stride);
  ge *pts = (ge *)malloc(sizeof(ge) * GRP);
  /* half = 512*stride (mod n) */
  fe_from_be(&half, stride_be);
  { fe s = half; for (int i = 0; i < 9; i++) sc_add(&s, &s, &s); half = s; }
  for (uint64_t g = 0; g < n_groups; g++) {
    fe ck; ge c;
    sc_add(&ck, &key, &half);
    scalar_mult_g(&c, &ck);
    walk_group(t, &c, pts, out_y != 0, 0);
    for (int i = 0; i < GRP; i++) {
      fe_to_be(out_x + (g * GRP + i) * 32, &pts[i].x);
      if (out_y) fe_to_be(out_y + (g * GRP + i) * 32, &pts[i].y);
    }
    /* key += 1024*stride */
    fe s1024 = half; sc_add(&s1024, &s1024, &half);
    sc_add(&key, &key, &s1024);
  }
  free(pts);
  free(t);
}

/* ------------------------------------------------------------------------------------------ */
/* Sequential scan over one chunk (thread_process, keyhunt.cpp:3265-3861), restated for the     */
/* modes on the hot path.  mode: 0 = rmd160/address (BTC), 1 = xpoint.  search: 0 = compress,  */
/* 1 = uncompress, 2 = both (FLAGSEARCH).  rows: sorted n x 20-byte table.  bloom: reference    */
/* layout.  Every hit is reported as (32-byte key, compressed flag) in the order the reference */
/* would print it (within one thread).                                                          */
/* ------------------------------------------------------------------------------------------ */
typedef struct {
  uint8_t key[32];
  int32_t compressed;
  int32_t kind;   /* 0 = 02||X, 1 = 03||X, 2 = 04||X||Y, 3 = xpoint */
} or_hit;

/* -e constants (keyhunt.cpp:926-930): lambda*(x, y) = (beta*x, y) */
static const fe END_BETA[3] = {{{1, 0, 0, 0}},
                               {{0xc1396c28719501eeULL, 0x9cf0497512f58995ULL, 0x6e64479eac3434e9ULL, 0x7ae96a2b657c0710ULL}},
                               {{0x3ec693d68e6afa40ULL, 0x630fb68aed0a766aULL, 0x919bb86153cbcb16ULL, 0x851695d49a83f8efULL}}};
static const fe END_LAMBDA[3] = {{{1, 0, 0, 0}},
                                 {{0xdf02967c1b23bd72ULL, 0x122e22ea20816678ULL, 0xa5261c028812645aULL, 0x5363ad4cc05c30e0ULL}},
                                 {{0xe0cfc810b51283ceULL, 0xa880b9fc8ec739c2ULL, 0x5ad9e3fd77ed9ba4ULL, 0xac9c52b33fa3cf1fULL}}};

static void push_hit(or_hit *hits, int cap, int *nh, const fe *k, int compressed, int kind) {
  if (*nh < cap) { fe_to_be(hits[*nh].key, k); hits[*nh].compressed = compressed; hits[*nh].kind = kind; }
  (*nh)++;
}

/* thread_process for one chunk (keyhunt.cpp:3349-3830): per point, the compressed variants, then
 * the uncompressed ones; with endo (-e) each over the images e = 0, 1, 2 (beta^e * X), the 04
 * variants also over (X, -Y).  Kinds: base (0: 02, 1: 03, 2: 04, 3: xpoint) | e << 4 | neg << 6.
 * scan_groups does groups [g0, g1) of the chunk into its own hit list. */
typedef struct {
  int mode, search, endo, grp;  /* grp: keys per group (1024, or --rmd-batch-size) */
  fe start;
  uint64_t g0, g1;
  const uint8_t *rows; int64_t n_rows; const uint8_t *bf; uint64_t bits; uint32_t hashes;
  or_hit *hits; int cap, nh;
} scan_job;

static void *scan_groups(void *arg) {
  scan_job *J = (scan_job *)arg;
  const int mode = J->mode, search = J->search, endo = J->endo;
  const uint8_t *rows = J->rows, *bf = J->bf;
  const int64_t n_rows = J->n_rows;
  const uint64_t bits = J->bits;
  const uint32_t hashes = J->hashes;
  or_hit *hits = J->hits;
  const int cap = J->cap;
  int nh = 0;
  int need_y = (search == 1 || search == 2 || mode == 2);
  int ne = endo ? 3 : 1;
  const int grp = J->grp;
  fe key, one = {{1, 0, 0, 0}};
  u256_add_u64(&key, &J->start, J->g0 * (uint64_t)grp);
  walk_tab *wt = (walk_tab *)malloc(sizeof(walk_tab));
  build_walk_tab(wt, &one);
  ge *pts = (ge *)malloc(sizeof(ge) * GRP);
  uint8_t *xs = (uint8_t *)malloc(GRP * 32), *ys = (uint8_t *)malloc(GRP * 32);
  for (uint64_t g = J->g0; g < J->g1; g++) {
    /* the centre from its key (keyhunt.cpp:3349-3353), then the group's points */
    fe ck; ge c;
    u256_add_u64(&ck, &key, (uint64_t)(grp / 2));
    scalar_mult_g(&c, &ck);
    walk_group_n(wt, &c, pts, need_y, 0, grp / 2);
    for (int t = 0; t < grp; t++) {
      fe_to_be(xs + t * 32, &pts[t].x);
      fe_to_be(ys + t * 32, &pts[t].y);
    }
    for (int t = 0; t < grp; t++) {
      fe kf; u256_add_u64(&kf, &key, (uint64_t)t);
      fe x0; fe_from_be(&x0, xs + t * 32);
      uint8_t xe[3][32];
      for (int e = 0; e < ne; e++) { fe v; fe_mul(&v, &x0, &END_BETA[e]); fe_to_be(xe[e], &v); }
      if (mode == 2) {  /* -c eth (keyhunt.cpp:3524-3548, 3703-3760): the uncompressed point */
        uint8_t ya[32], h[20];
        memcpy(ya, ys + t * 32, 32);
        or_eth_address(xs + t * 32, ya, h);
        if (or_bloom_check(bf, bits, hashes, h, 20) && or_searchbinary(rows, n_rows, h, 20, 0))
          push_hit(hits, cap, &nh, &kf, 0, 5);
        continue;
      }
      if (mode == 1) {  /* xpoint (keyhunt.cpp:3801-3824) */
        for (int e = 0; e < ne; e++)
          if (or_bloom_check(bf, bits, hashes, xe[e], 20) && or_searchbinary(rows, n_rows, xe[e], 20, 0)) {
            fe kr; sc_mul(&kr, &kf, &END_LAMBDA[e]);
            push_hit(hits, cap, &nh, &kr, 0, 3 | (e << 4));
          }
        continue;
      }
      if (search == 0 || search == 2) {
        for (int l = 0; l < 2 * ne; l++) {
          int e = l / 2, pfx = l % 2;
          uint8_t h[20];
          or_hash160_comp(xe[e], (uint8_t)(2 + pfx), h);
          if (or_bloom_check(bf, bits, hashes, h, 20) && or_searchbinary(rows, n_rows, h, 20, 0)) {
            /* -e (keyhunt.cpp:3565-3600): the image keeps Y; negate when the slot key's parity
               disagrees with the matched prefix.  Without -e (3619-3636): negate unless the slot
               key's own compressed hash is the match */
            ge P; scalar_mult_g(&P, &kf);
            fe kr; sc_mul(&kr, &kf, &END_LAMBDA[e]);
            if (endo) {
              int odd = (int)(P.y.v[0] & 1);
              if (odd != pfx) sc_neg(&kr, &kr);
            } else {
              uint8_t px[32], h2[20];
              fe_to_be(px, &P.x);
              or_hash160_comp(px, (uint8_t)(2 + (P.y.v[0] & 1)), h2);
              if (memcmp(h2, h, 20) != 0) sc_neg(&kr, &kr);
            }
            push_hit(hits, cap, &nh, &kr, 1, pfx | (e << 4));
          }
        }
      }
      if (search == 1 || search == 2) {
        fe y0; fe_from_be(&y0, ys + t * 32);
        fe ny; fe_neg(&ny, &y0);
        uint8_t yb[2][32];
        fe_to_be(yb[0], &y0); fe_to_be(yb[1], &ny);
        for (int l = 0; l < (endo ? 6 : 1); l++) {
          int e = l / 2, neg = l % 2;
          uint8_t h[20];
          or_hash160_uncomp(xe[e], yb[neg], h);
          if (or_bloom_check(bf, bits, hashes, h, 20) && or_searchbinary(rows, n_rows, h, 20, 0)) {
            fe kr; sc_mul(&kr, &kf, &END_LAMBDA[e]);
            if (endo) {  /* keyhunt.cpp:3643-3680: keep the key whose 04-hash is the match */
              ge P; scalar_mult_g(&P, &kr);
              uint8_t px[32], py[32], h2[20];
              fe_to_be(px, &P.x); fe_to_be(py, &P.y);
              or_hash160_uncomp(px, py, h2);
              if (memcmp(h2, h, 20) != 0) sc_neg(&kr, &kr);
            }
            push_hit(hits, cap, &nh, &kr, 0, 2 | (e << 4) | (neg << 6));
          }
        }
      }
    }
    u256_add_u64(&key, &key, (uint64_t)grp);
  }
  free(xs); free(ys); free(pts); free(wt);
  J->nh = nh;
  return 0;
}

/* the chunk on up to 16 threads (contiguous group ranges, hits concatenated in key order) */
/* grp: keys per group -- 1024, or -m rmd160 --rmd-batch-size (a multiple of 4 below 1024): the
 * chunk is then ceil(n_keys / grp) whole groups (the reference's do-while, keyhunt.cpp:3350-3836) */
int or_scan_chunk3(int mode, int search, int endo, int grp, const uint8_t start_be[32], uint64_t n_keys,
                   const uint8_t *rows, int64_t n_rows, const uint8_t *bf, uint64_t bits, uint32_t hashes,
                   or_hit *hits, int cap) {
  if (grp < 4 || grp > GRP || grp % 4) return -1;
  uint64_t groups = (n_keys + grp - 1) / grp;
  int nt = (int)(groups < 16 ? (groups ? groups : 1) : 16);
  scan_job *jobs = (scan_job *)calloc(nt, sizeof(scan_job));
  pthread_t *th = (pthread_t *)calloc(nt, sizeof(pthread_t));
  for (int i = 0; i < nt; i++) {
    scan_job *J = &jobs[i];
    J->mode = mode; J->search = search; J->endo = endo; J->grp = grp;
    fe_from_be(&J->start, start_be);
    J->g0 = groups * i / nt; J->g1 = groups * (i + 1) / nt;
    J->rows = rows; J->n_rows = n_rows; J->bf = bf; J->bits = bits; J->hashes = hashes;
    J->cap = cap; J->hits = (or_hit *)calloc(cap > 0 ? cap : 1, sizeof(or_hit));
    pthread_create(&th[i], 0, scan_groups, J);
  }
  int nh = 0;
  for (int i = 0; i < nt; i++) {
    pthread_join(th[i], 0);
    for (int j = 0; j < jobs[i].nh; j++) {
      if (nh < cap && j < jobs[i].cap) hits[nh] = jobs[i].hits[j];
      nh++;
    }
    free(jobs[i].hits);
  }
  free(jobs); free(th);
  return nh;
}

int or_scan_chunk2(int mode, int search, int endo, const uint8_t start_be[32], uint64_t n_keys,
                   const uint8_t *rows, int64_t n_rows, const uint8_t *bf, uint64_t bits, uint32_t hashes,
                   or_hit *hits, int cap) {
  return or_scan_chunk3(mode, search, endo, GRP, start_be, n_keys, rows, n_rows, bf, bits, hashes, hits, cap);
}

int or_scan_chunk(int mode, int search, const uint8_t start_be[32], uint64_t n_keys,
                  const uint8_t *rows, int64_t n_rows, const uint8_t *bf, uint64_t bits, uint32_t hashes,
                  or_hit *hits, int cap) {
  return or_scan_chunk2(mode, search, 0, start_be, n_keys, rows, n_rows, bf, bits, hashes, hits, cap);
}

/* ------------------------------------------------------------------------------------------ */
/* BSGS (keyhunt.cpp:1454-1661 parameters, 5284-5472 baby build, 4549-4888 giant walk,         */
/* 5151-5248 second/third check, 7859-7868 calcualteindex, 4412-4544 table sort/search).       */
/* ------------------------------------------------------------------------------------------ */
typedef struct {
  uint64_t n, m, m2, m3, aux, cycles;
  uint64_t items1, items2, items3;       /* per-shard bloom item counts (before max(10000,.)) */
  uint64_t bits[3], bytes[3];
  uint32_t hashes[3];
} or_bsgs_params;

/* n: -n (power of two, exact sqrt, sqrt multiple of 1024), k: -k.  Returns 0 on success. */
int or_bsgs_params_compute(uint64_t n, uint64_t k, or_bsgs_params *p) {
  uint64_t m = (uint64_t)sqrtl((long double)n);
  while (m * m > n) m--;
  while ((m + 1) * (m + 1) <= n) m++;
  if (m * m != n) return 1;
  if (m % 1024) return 2;
  m *= k;
  uint64_t m2 = m / 32 + (m % 32 ? 1 : 0);
  uint64_t m3 = m2 / 32 + (m2 % 32 ? 1 : 0);
  uint64_t aux = n / m;
  if (n % m) n = m * aux;
  p->n = n; p->m = m; p->m2 = m2; p->m3 = m3; p->aux = aux;
  p->cycles = aux / 1024 + (aux % 1024 ? 1 : 0);
  p->items1 = (m / 256 > 10000) ? (m / 256 + (m % 256 ? 1 : 0)) : 1000;
  p->items2 = (m2 / 256 > 1000) ? (m2 / 256 + (m2 % 256 ? 1 : 0)) : 1000;
  p->items3 = (m3 / 256 > 1000) ? (m3 / 256 + (m3 % 256 ? 1 : 0)) : 1000;
  uint64_t it[3] = {p->items1, p->items2, p->items3};
  for (int l = 0; l < 3; l++)
    if (or_bloom_params(or_bloom_entries(it[l]), 0.000001, &p->bits[l], &p->bytes[l], &p->hashes[l])) return 3;
  return 0;
}

/* bsgs_xvalue row: {u8 value[6] = X[16..22); u64 index} -- laid out here as 16 bytes: 6 value
 * bytes, 2 pad bytes, 8 index bytes (LE) like the reference's struct on x86-64. */
typedef struct { uint8_t value[6]; uint8_t pad[2]; uint64_t index; } or_bxrow;

static int bxrow_cmp(const void *a, const void *b) {
  int c = memcmp(((const or_bxrow *)a)->value, ((const or_bxrow *)b)->value, 6);
  if (c) return c;
  /* ties: deterministic order by index (reference introsort order is unspecified on ties) */
  uint64_t ia = ((const or_bxrow *)a)->index, ib = ((const or_bxrow *)b)->index;
  return ia < ib ? -1 : ia > ib;
}

/* Baby-step build: for i in [0, m): X((i+1)G) -> shard X[0] -> bloom layer1 (all), layer2
 * (i < m2), layer3 + table (i < m3).  bf1/bf2/bf3: 256 shards each of bytes[l], contiguous. */
void or_bsgs_build(const or_bsgs_params *p, uint8_t *bf1, uint8_t *bf2, uint8_t *bf3, or_bxrow *table) {
  fe one = {{1, 0, 0, 0}};
  uint8_t onebe[32], kb[32];
  fe_to_be(onebe, &one);
  uint8_t *xs = (uint8_t *)malloc(GRP * 32);
  uint64_t groups = p->m / GRP + (p->m % GRP ? 1 : 0);
  fe key = one;
  for (uint64_t g = 0; g < groups; g++) {
    fe_to_be(kb, &key);
    or_walk_points(kb, onebe, 1, xs, 0);
    for (int t = 0; t < GRP; t++) {
      uint64_t i = g * GRP + t;
      const uint8_t *x = xs + t * 32;
      unsigned s = x[0];
      if (i < p->m3) {
        memcpy(table[i].value, x + 16, 6); memset(table[i].pad, 0, 2); table[i].index = i;
        or_bloom_add(bf3 + s * p->bytes[2], p->bits[2], p->hashes[2], x, 32);
      }
      if (i < p->m2) or_bloom_add(bf2 + s * p->bytes[1], p->bits[1], p->hashes[1], x, 32);
      if (i < p->m) or_bloom_add(bf1 + s * p->bytes[0], p->bits[0], p->hashes[0], x, 32);
    }
    fe k1024 = {{GRP, 0, 0, 0}};
    u256_add(&key, &key, &k1024);
  }
  qsort(table, p->m3, sizeof(or_bxrow), bxrow_cmp);
  free(xs);
}

/* bsgs_searchbinary (keyhunt.cpp:4510-4544, no bucket cache): returns 1 and *idx on a match */
static int bsgs_search(const or_bxrow *t, int64_t n, const uint8_t *x32, uint64_t *idx) {
  int64_t min = 0, max = n, cur = 0, half = n;
  while (half >= 1) {
    half = (max - min) / 2;
    int c = memcmp(x32 + 16, t[cur + half].value, 6);
    if (c == 0) { *idx = t[cur + half].index; return 1; }
    if (c < 0) max = max - half; else min = min + half;
    cur = min;
  }
  return 0;
}

typedef struct {
  const or_bsgs_params *p;
  const uint8_t *bf1, *bf2, *bf3;
  const or_bxrow *table;
  ge amp2[32], amp3[32];
} bsgs_ctx;

static void bsgs_ctx_init(bsgs_ctx *c, const or_bsgs_params *p, const uint8_t *bf1, const uint8_t *bf2,
                          const uint8_t *bf3, const or_bxrow *table) {
  c->p = p; c->bf1 = bf1; c->bf2 = bf2; c->bf3 = bf3; c->table = table;
  /* AMP2[i] = -(M2 + 2i*M2)G, AMP3[i] = -(M3 + 2i*M3)G  (keyhunt.cpp:1818-1842) */
  for (int i = 0; i < 32; i++) {
    fe k2 = {{p->m2 * (2 * (uint64_t)i + 1), 0, 0, 0}}, k3 = {{p->m3 * (2 * (uint64_t)i + 1), 0, 0, 0}};
    ge a; scalar_mult_g(&a, &k2); ge_neg(&c->amp2[i], &a);
    scalar_mult_g(&a, &k3); ge_neg(&c->amp3[i], &a);
  }
}

/* bsgs_thirdcheck (keyhunt.cpp:5186-5248) */
static int bsgs_third(const bsgs_ctx *c, const fe *start, uint32_t a, const ge *Q, fe *key) {
  const or_bsgs_params *p = c->p;
  fe base, off = {{(uint64_t)a * 2 * p->m2, 0, 0, 0}};
  sc_add(&base, start, &off);
  ge bp, nbp, S;
  scalar_mult_g(&bp, &base); ge_neg(&nbp, &bp);
  ge_add_direct(&S, Q, &nbp);
  for (int i = 0; i < 32; i++) {
    ge T; uint8_t xr[32];
    ge_add_direct(&T, &S, &c->amp3[i]);
    fe_to_be(xr, &T.x);
    fe calc = {{(i == 0) ? p->m3 : (uint64_t)i * 2 * p->m3 + p->m3, 0, 0, 0}};
    if (or_bloom_check(c->bf3 + xr[0] * p->bytes[2], p->bits[2], p->hashes[2], xr, 32)) {
      uint64_t j;
      if (bsgs_search(c->table, (int64_t)p->m3, xr, &j)) {
        fe k, jj = {{j + 1, 0, 0, 0}};
        ge chk;
        u256_add(&k, &calc, &jj); sc_add(&k, &k, &base);
        scalar_mult_g(&chk, &k);
        if (u256_cmp(&chk.x, &Q->x) == 0) { *key = k; return 1; }
        u256_sub(&k, &calc, &jj); sc_add(&k, &k, &base);
        scalar_mult_g(&chk, &k);
        if (u256_cmp(&chk.x, &Q->x) == 0) { *key = k; return 1; }
      }
    } else if (u256_cmp(&S.x, &c->amp3[i].x) == 0) {
      /* keyhunt.cpp:5238-5243 special case */
      fe k; sc_add(&k, &calc, &base);
      *key = k; return 1;
    }
  }
  return 0;
}
/* bsgs_secondcheck (keyhunt.cpp:5151-5184) */
static int bsgs_second(const bsgs_ctx *c, const fe *start, uint32_t a, const ge *Q, fe *key) {
  const or_bsgs_params *p = c->p;
  fe base;
  u128 off128 = (u128)a * 2 * p->m;
  fe off = {{(uint64_t)off128, (uint64_t)(off128 >> 64), 0, 0}};
  sc_add(&base, start, &off);
  ge bp, nbp, S;
  scalar_mult_g(&bp, &base); ge_neg(&nbp, &bp);
  ge_add_direct(&S, Q, &nbp);
  for (int i = 0; i < 32; i++) {
    ge T; uint8_t xr[32];
    ge_add_direct(&T, &S, &c->amp2[i]);
    fe_to_be(xr, &T.x);
    if (or_bloom_check(c->bf2 + xr[0] * p->bytes[1], p->bits[1], p->hashes[1], xr, 32))
      if (bsgs_third(c, &base, (uint32_t)i, Q, key)) return 1;
  }
  return 0;
}

/* The layer-2 probes of bsgs_secondcheck (keyhunt.cpp:5151-5184) for base keys given directly: bit i
 * of masks[j] is bloom_check(bloom_bPx2nd[X[0]], X) of S + AMP2[i], S = Q - base_keys[j]*G, for all
 * 32 i (the reference stops at the first i whose third check finds the key; the engine's k_refine
 * computes every bit).  A base key of 0 (no point) gives 0. */
void or_bsgs_second_masks(const or_bsgs_params *p, const uint8_t *bf2, const uint8_t *base_keys_be, uint64_t n,
                          const uint8_t qx[32], const uint8_t qy[32], uint32_t *masks) {
  bsgs_ctx c; bsgs_ctx_init(&c, p, 0, bf2, 0, 0);
  ge Q; fe_from_be(&Q.x, qx); fe_from_be(&Q.y, qy); Q.inf = 0;
  for (uint64_t j = 0; j < n; j++) {
    fe base; fe_from_be(&base, base_keys_be + 32 * j);
    while (u256_cmp(&base, &SC_N) >= 0) u256_sub(&base, &base, &SC_N);
    masks[j] = 0;
    if (u256_is_zero(&base)) continue;
    ge bp, nbp, S;
    scalar_mult_g(&bp, &base); ge_neg(&nbp, &bp);
    ge_add_direct(&S, &Q, &nbp);
    for (int i = 0; i < 32; i++) {
      ge T; uint8_t xr[32];
      ge_add_direct(&T, &S, &c.amp2[i]);
      fe_to_be(xr, &T.x);
      if (or_bloom_check(bf2 + xr[0] * p->bytes[1], p->bits[1], p->hashes[1], xr, 32)) masks[j] |= 1u << i;
    }
  }
}

/* Refine one first-level candidate (base, a) for target (qx,qy).  Returns 1 + key. */
int or_bsgs_refine(const or_bsgs_params *p, const uint8_t *bf2, const uint8_t *bf3, const or_bxrow *table,
                   const uint8_t base_be[32], uint32_t a, const uint8_t qx[32], const uint8_t qy[32], uint8_t key_out[32]) {
  bsgs_ctx c; bsgs_ctx_init(&c, p, 0, bf2, bf3, table);
  fe base, key; ge Q;
  fe_from_be(&base, base_be);
  fe_from_be(&Q.x, qx); fe_from_be(&Q.y, qy); Q.inf = 0;
  if (bsgs_second(&c, &base, a, &Q, &key)) { fe_to_be(key_out, &key); return 1; }
  return 0;
}

/* The engine's blocked layer 1 (its own layout, in place of the reference's layer-1 bloom_check
 * of keyhunt.cpp:4819-4822; specified in keyhunt_amd/csrc/kh_kernels.h, KH_PK_MASKS, restated
 * here independently of the device code): shard X[0] holds `blocks` 16-byte blocks; the item's
 * block is (u * blocks) >> 32 with u the big-endian u32 X[8..12); little-endian block word w must
 * cover, with s the big-endian u32 X[12 + 4*(w/2) ..), a = s >> 8*(w%2) and b = a >> 4, the bits
 * a & 15, 16 + ((a >> 16) & 15), b & 15 and 16 + ((b >> 16) & 15). */
static uint32_t rd_be32(const uint8_t *b) {
  return ((uint32_t)b[0] << 24) | ((uint32_t)b[1] << 16) | ((uint32_t)b[2] << 8) | b[3];
}
int or_blk_check(const uint8_t *bf1, uint64_t blocks, const uint8_t x[32]) {
  const uint8_t *blk = bf1 + (uint64_t)x[0] * blocks * 16 + ((rd_be32(x + 8) * blocks) >> 32) * 16;
  for (int w = 0; w < 4; w++) {
    uint32_t a = rd_be32(x + 12 + 4 * (w / 2)) >> (8 * (w % 2)), b = a >> 4;
    uint32_t mask = (1u << (a & 15)) | (1u << (16 + ((a >> 16) & 15))) | (1u << (b & 15)) |
                    (1u << (16 + ((b >> 16) & 15)));
    uint32_t word = (uint32_t)blk[4 * w] | ((uint32_t)blk[4 * w + 1] << 8) | ((uint32_t)blk[4 * w + 2] << 16) |
                    ((uint32_t)blk[4 * w + 3] << 24);
    if ((word & mask) != mask) return 0;
  }
  return 1;
}

/* Giant-step scan over whole bases [start, start + n_bases*2N) for ONE target, exactly as the
 * sequential worker does (keyhunt.cpp:4549-4888): per base, startP = Q - (base + 1025M)G,
 * 1024-point groups along GSn[i] = -(i+1)*2M*G, probe bloom1[X[0]] with the 32-byte X, refine
 * candidates.  Stops at the first found key (bsgs_found).  cand_out (optional): list of
 * (base index, a) first-level candidates, in order.  Returns 1 if found.  l1_blocks != 0: layer 1
 * is the engine's blocked layout with that many blocks per shard (or_blk_check), else the
 * reference's bloom. */
int or_bsgs_scan_l1(const or_bsgs_params *p, const uint8_t *bf1, uint64_t l1_blocks, const uint8_t *bf2,
                    const uint8_t *bf3, const or_bxrow *table, const uint8_t start_be[32], uint64_t n_bases,
                    const uint8_t qx[32], const uint8_t qy[32], uint8_t key_out[32],
                    uint64_t *cand_out, uint64_t cand_cap, uint64_t *n_cand);
int or_bsgs_scan(const or_bsgs_params *p, const uint8_t *bf1, const uint8_t *bf2, const uint8_t *bf3,
                 const or_bxrow *table, const uint8_t start_be[32], uint64_t n_bases,
                 const uint8_t qx[32], const uint8_t qy[32], uint8_t key_out[32],
                 uint64_t *cand_out, uint64_t cand_cap, uint64_t *n_cand) {
  return or_bsgs_scan_l1(p, bf1, 0, bf2, bf3, table, start_be, n_bases, qx, qy, key_out, cand_out, cand_cap, n_cand);
}
int or_bsgs_scan_l1(const or_bsgs_params *p, const uint8_t *bf1, uint64_t l1_blocks, const uint8_t *bf2,
                    const uint8_t *bf3, const or_bxrow *table, const uint8_t start_be[32], uint64_t n_bases,
                    const uint8_t qx[32], const uint8_t qy[32], uint8_t key_out[32],
                    uint64_t *cand_out, uint64_t cand_cap, uint64_t *n_cand) {
  bsgs_ctx c; bsgs_ctx_init(&c, p, bf1, bf2, bf3, table);
  ge Q; fe_from_be(&Q.x, qx); fe_from_be(&Q.y, qy); Q.inf = 0;
  /* GSn[i] = -(i+1)*2M*G, _2GSn = 2*GSn[511] (keyhunt.cpp:1797-1816) */
  walk_tab *t = (walk_tab *)malloc(sizeof(walk_tab));
  {
    fe m2x = {{2 * p->m, 0, 0, 0}};
    ge bs, nbs; scalar_mult_g(&bs, &m2x); ge_neg(&nbs, &bs);
    t->gn[0] = nbs;
    ge_add(&t->gn[1], &nbs, &nbs);
    for (int i = 2; i < HALF; i++) ge_add(&t->gn[i], &t->gn[i - 1], &nbs);
    ge_add(&t->g2n, &t->gn[HALF - 1], &t->gn[HALF - 1]);
  }
  ge *pts = (ge *)malloc(sizeof(ge) * GRP);
  fe base; fe_from_be(&base, start_be);
  fe step2n = {{2 * p->n, 0, 0, 0}};
  fe intaux = {{2 * p->m * 512 + p->m, 0, 0, 0}};
  uint64_t nc = 0;
  int found = 0;
  for (uint64_t b = 0; b < n_bases && !found; b++) {
    fe km; ge pa, sp;
    sc_add(&km, &base, &intaux); sc_neg(&km, &km);
    scalar_mult_g(&pa, &km);
    ge_add(&sp, &Q, &pa);
    for (uint64_t j = 0; j < p->cycles && !found; j++) {
      ge nxt;
      walk_group(t, &sp, pts, 0, &nxt);
      for (int i = 0; i < GRP && !found; i++) {
        uint8_t xr[32];
        fe_to_be(xr, &pts[i].x);
        if (l1_blocks ? or_blk_check(bf1, l1_blocks, xr)
                      : or_bloom_check(bf1 + xr[0] * p->bytes[0], p->bits[0], p->hashes[0], xr, 32)) {
          uint32_t a = (uint32_t)(j * 1024 + i);
          if (cand_out && nc < cand_cap) { cand_out[2 * nc] = b; cand_out[2 * nc + 1] = a; }
          nc++;
          fe key;
          if (bsgs_second(&c, &base, a, &Q, &key)) { fe_to_be(key_out, &key); found = 1; }
        }
      }
      sp = nxt;
    }
    if (!found) sc_add(&base, &base, &step2n);
  }
  if (n_cand) *n_cand = nc;
  free(pts); free(t);
  return found;
}

/* ------------------------------------------------------------------------------------------ */
/* CPU baseline: giant-step probe rate (the BSGS inner loop of keyhunt.cpp:4644-4880 without    */
/* refinement) on `threads` pthreads, each walking its own bases for `n_groups` 1024-groups.   */
/* Returns the number of first-level bloom hits; elapsed time is measured by the caller.       */
/* ------------------------------------------------------------------------------------------ */
typedef struct {
  const or_bsgs_params *p; const uint8_t *bf1; const walk_tab *t;
  ge start; uint64_t n_groups; uint64_t hits;
} giant_job;
static void *giant_worker(void *arg) {
  giant_job *j = (giant_job *)arg;
  ge *pts = (ge *)malloc(sizeof(ge) * GRP);
  ge sp = j->start;
  uint64_t h = 0;
  for (uint64_t g = 0; g < j->n_groups; g++) {
    ge nxt;
    walk_group(j->t, &sp, pts, 0, &nxt);
    for (int i = 0; i < GRP; i++) {
      uint8_t xr[32];
      fe_to_be(xr, &pts[i].x);
      h += or_bloom_check(j->bf1 + xr[0] * j->p->bytes[0], j->p->bits[0], j->p->hashes[0], xr, 32);
    }
    sp = nxt;
  }
  j->hits = h;
  free(pts);
  return 0;
}
uint64_t or_bsgs_giant_probe(const or_bsgs_params *p, const uint8_t *bf1, const uint8_t qx[32], const uint8_t qy[32],
                             uint64_t n_groups_per_thread, int threads) {
  walk_tab *t = (walk_tab *)malloc(sizeof(walk_tab));
  fe m2x = {{2 * p->m, 0, 0, 0}};
  ge bs, nbs; scalar_mult_g(&bs, &m2x); ge_neg(&nbs, &bs);
  t->gn[0] = nbs;
  ge_add(&t->gn[1], &nbs, &nbs);
  for (int i = 2; i < HALF; i++) ge_add(&t->gn[i], &t->gn[i - 1], &nbs);
  ge_add(&t->g2n, &t->gn[HALF - 1], &t->gn[HALF - 1]);
  giant_job *jobs = (giant_job *)calloc(threads, sizeof(giant_job));
  pthread_t *th = (pthread_t *)calloc(threads, sizeof(pthread_t));
  ge Q; fe_from_be(&Q.x, qx); fe_from_be(&Q.y, qy); Q.inf = 0;
  for (int i = 0; i < threads; i++) {
    fe k = {{(uint64_t)(i + 1) * 0x1000000ULL + 12345, 0, 0, 0}};
    ge off; scalar_mult_g(&off, &k);
    jobs[i].p = p; jobs[i].bf1 = bf1; jobs[i].t = t; jobs[i].n_groups = n_groups_per_thread;
    ge_add(&jobs[i].start, &Q, &off);
    pthread_create(&th[i], 0, giant_worker, &jobs[i]);
  }
  uint64_t h = 0;
  for (int i = 0; i < threads; i++) { pthread_join(th[i], 0); h += jobs[i].hits; }
  free(jobs); free(th); free(t);
  return h;
}

/* ------------------------------------------------------------------------------------------ */
/* Base58 (libbase58 b58tobin / b58enc semantics for the address strings keyhunt parses and     */
/* prints: keyhunt.cpp:3028-3038, 7283-7292).                                                  */
/* ------------------------------------------------------------------------------------------ */
static const char B58[] = "123456789ABCDEFGHJKLMNPQRSTUVWXYZabcdefghijkmnopqrstuvwxyz";
/* P2PKH address of a hash160 (version byte 0x00) */
int or_h160_to_address(const uint8_t h[20], char *out, int cap) {
  uint8_t d[25], c1[32], c2[32];
  d[0] = 0; memcpy(d + 1, h, 20);
  or_sha256(d, 21, c1); or_sha256(c1, 32, c2);
  memcpy(d + 21, c2, 4);
  uint8_t buf[40] = {0};
  int zeros = 0;
  while (zeros < 25 && d[zeros] == 0) zeros++;
  int len = 0;
  for (int i = zeros; i < 25; i++) {
    int carry = d[i];
    for (int j = 0; j < len; j++) { carry += buf[j] * 256; buf[j] = carry % 58; carry /= 58; }
    while (carry) { buf[len++] = carry % 58; carry /= 58; }
  }
  if (zeros + len + 1 > cap) return -1;
  int o = 0;
  for (int i = 0; i < zeros; i++) out[o++] = '1';
  for (int i = len - 1; i >= 0; i--) out[o++] = B58[buf[i]];
  out[o] = 0;
  return o;
}
/* decode a Base58Check P2PKH address into its 25 raw bytes; returns byte count or -1 */
int or_address_decode(const char *s, uint8_t out[25]) {
  uint8_t buf[64] = {0};
  int len = 0, zeros = 0;
  while (s[zeros] == '1') zeros++;
  for (const char *q = s + zeros; *q; q++) {
    const char *pos = strchr(B58, *q);
    if (!pos || !*q) return -1;
    int carry = (int)(pos - B58);
    for (int j = 0; j < len; j++) { carry += buf[j] * 58; buf[j] = carry & 0xff; carry >>= 8; }
    while (carry) { buf[len++] = carry & 0xff; carry >>= 8; }
  }
  int total = zeros + len;
  if (total != 25) return -1;
  memset(out, 0, zeros);
  for (int i = 0; i < len; i++) out[zeros + i] = buf[len - 1 - i];
  return 25;
}
