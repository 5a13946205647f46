// ref_golden.cpp -- golden-vector generator (TEST INFRASTRUCTURE, our code).
//
// Linked by oracle/Makefile.ref against objects compiled from the reference's own sources
// (secp256k1/, hash/, bloom/, xxhash/ under /root/reference).  It calls the reference's
// primitives -- Int::ModMulK1 / ModSquareK1 / ModInv, IntGroup::ModInv, Secp256K1::
// ComputePublicKey / AddDirect / DoubleDirect / GetHash160_fromX / GetHash160, XXH64,
// bloom_init2 / bloom_add -- on deterministic inputs and prints one JSON document.  The output
// is committed as tests/golden/ref_vectors.json (see oracle/make_golden.py); nothing of the
// reference itself is committed.
#include <stdio.h>
#include <stdint.h>
#include <string.h>
#include <vector>
#include <string>
#include <algorithm>
#include "secp256k1/SECP256k1.h"
#include "secp256k1/Int.h"
#include "secp256k1/IntGroup.h"
#include "secp256k1/Point.h"
#include "hash/sha256.h"
#include "bloom/bloom.h"
#include "xxhash/xxhash.h"
#include "sha3/sha3.h"

static uint64_t rng_state = 0x6b657968756e7421ULL;
static uint64_t g_rnd() {  // splitmix64
  uint64_t z = (rng_state += 0x9E3779B97F4A7C15ULL);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}
static std::string hexs(const uint8_t *b, int n) {
  static const char *H = "0123456789abcdef";
  std::string s;
  for (int i = 0; i < n; i++) { s += H[b[i] >> 4]; s += H[b[i] & 15]; }
  return s;
}
static std::string ihex(Int &v) { uint8_t b[32]; v.Get32Bytes(b); return hexs(b, 32); }
static void rand_int(Int &v) { for (int i = 0; i < 4; i++) v.SetQWord(i, g_rnd()); v.SetQWord(4, 0); }
static std::string sha_hex(const uint8_t *p, size_t n) {
  uint8_t d[32];
  sha256((uint8_t *)p, n, d);
  return hexs(d, 32);
}

Secp256K1 *secp;

int main() {
  secp = new Secp256K1();
  secp->Init();
  Int P(&secp->P);
  printf("{\n");

  // ---------------- field ----------------
  printf("\"field\": [\n");
  for (int t = 0; t < 48; t++) {
    Int a, b, r;
    rand_int(a); rand_int(b);
    if (t == 0) { a.SetBase16("FFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEFFFFFC2E"); b.Set(&a); }
    if (t == 1) { a.SetInt32(1); b.SetInt32(2); }
    if (t == 2) { a.SetBase16("FFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEFFFFFC2E"); b.SetInt32(2); }
    a.Mod(&P); b.Mod(&P);
    Int m, s, inv, ad, sb;
    m.ModMulK1(&a, &b);
    s.ModSquareK1(&a);
    inv.Set(&a); inv.ModInv();
    ad.ModAdd(&a, &b);
    sb.ModSub(&a, &b);
    printf("  {\"a\":\"%s\",\"b\":\"%s\",\"mul\":\"%s\",\"sqr\":\"%s\",\"inv\":\"%s\",\"add\":\"%s\",\"sub\":\"%s\"}%s\n",
           ihex(a).c_str(), ihex(b).c_str(), ihex(m).c_str(), ihex(s).c_str(), ihex(inv).c_str(),
           ihex(ad).c_str(), ihex(sb).c_str(), t == 47 ? "" : ",");
  }
  printf("],\n");

  // ---------------- public keys + hash160 ----------------
  printf("\"pubkeys\": [\n");
  std::vector<std::string> ks = {"1", "2", "3", "7", "8", "FFFFFFFF", "100000000", "2832ED74F2B5E35EE",
                                 "7CCE5EFDACCF6808", "F7051F27B09112D4", "1C533B6BB7F0804E09960225E44877AC",
                                 "B10F22572C497A836EA187F2E1FC23", "33E7665705359F04F28B88CF897C603C9"};
  for (int t = 0; t < 12; t++) { char buf[80]; snprintf(buf, 80, "%016llX%016llX", (unsigned long long)g_rnd(), (unsigned long long)g_rnd()); ks.push_back(buf); }
  for (size_t t = 0; t < ks.size(); t++) {
    Int k; k.SetBase16((char *)ks[t].c_str());
    Point p = secp->ComputePublicKey(&k);
    uint8_t h02[4][20], h03[4][20], hu[20];
    secp->GetHash160_fromX(0, 0x02, &p.x, &p.x, &p.x, &p.x, h02[0], h02[1], h02[2], h02[3]);
    secp->GetHash160_fromX(0, 0x03, &p.x, &p.x, &p.x, &p.x, h03[0], h03[1], h03[2], h03[3]);
    secp->GetHash160(0, false, p, hu);
    printf("  {\"k\":\"%s\",\"x\":\"%s\",\"y\":\"%s\",\"h02\":\"%s\",\"h03\":\"%s\",\"h04\":\"%s\"}%s\n",
           ihex(k).c_str(), ihex(p.x).c_str(), ihex(p.y).c_str(), hexs(h02[0], 20).c_str(),
           hexs(h03[0], 20).c_str(), hexs(hu, 20).c_str(), t + 1 == ks.size() ? "" : ",");
  }
  printf("],\n");

  // ---------------- XXH64 (bloom's two chained hashes) ----------------
  printf("\"xxh64\": [\n");
  for (int t = 0; t < 32; t++) {
    uint8_t buf[32];
    int len = (t & 1) ? 32 : 20;
    for (int i = 0; i < 32; i++) buf[i] = (uint8_t)g_rnd();
    uint64_t a = XXH64(buf, len, 0x59f2815b16f81798ULL);
    uint64_t b = XXH64(buf, len, a);
    printf("  {\"buf\":\"%s\",\"a\":\"%016llx\",\"b\":\"%016llx\"}%s\n", hexs(buf, len).c_str(),
           (unsigned long long)a, (unsigned long long)b, t == 31 ? "" : ",");
  }
  printf("],\n");

  // ---------------- bloom sizing ----------------
  printf("\"bloom_params\": [\n");
  uint64_t ents[] = {1000, 10000, 10001, 65536, 235563ULL, 1048576ULL, 2097152ULL, 8388608ULL};
  for (int t = 0; t < 8; t++) {
    struct bloom bl;
    bloom_init2(&bl, ents[t], 0.000001);
    printf("  {\"entries\":%llu,\"bits\":%llu,\"bytes\":%llu,\"hashes\":%u}%s\n", (unsigned long long)ents[t],
           (unsigned long long)bl.bits, (unsigned long long)bl.bytes, (unsigned)bl.hashes, t == 7 ? "" : ",");
    bloom_free(&bl);
  }
  printf("],\n");

  // ---------------- bloom fill: 10000-entry filter with 200 x 20-byte items ----------------
  {
    struct bloom bl;
    bloom_init2(&bl, 10000, 0.000001);
    std::vector<std::string> items;
    uint8_t probe_hits = 0;
    for (int t = 0; t < 200; t++) {
      uint8_t buf[20];
      for (int i = 0; i < 20; i++) buf[i] = (uint8_t)g_rnd();
      bloom_add(&bl, buf, 20);
      items.push_back(hexs(buf, 20));
    }
    int neg = 0;
    for (int t = 0; t < 1000; t++) { uint8_t buf[20]; for (int i = 0; i < 20; i++) buf[i] = (uint8_t)g_rnd(); neg += bloom_check(&bl, buf, 20); }
    (void)probe_hits;
    printf("\"bloom_fill\": {\"entries\":10000,\"sha256\":\"%s\",\"false_pos_of_1000\":%d,\"items\":[", sha_hex(bl.bf, bl.bytes).c_str(), neg);
    for (size_t i = 0; i < items.size(); i++) printf("\"%s\"%s", items[i].c_str(), i + 1 == items.size() ? "" : ",");
    printf("]},\n");
    bloom_free(&bl);
  }

  // ---------------- group walk with the reference's own IntGroup + AddDirect ----------------
  // keyhunt.cpp:3349-3461 geometry restated on reference primitives; sha256 of the 1024 X's
  // (32-byte BE each) of two consecutive groups, next to the same X's from ComputePublicKey.
  printf("\"group_walk\": [\n");
  {
    std::vector<Point> Gn(512);
    Int one; one.SetInt32(1);
    Point G = secp->ComputePublicKey(&one);
    Gn[0] = G;
    Gn[1] = secp->DoubleDirect(G);
    for (int i = 2; i < 512; i++) Gn[i] = secp->AddDirect(Gn[i - 1], G);
    Point _2Gn = secp->DoubleDirect(Gn[511]);
    const char *starts[] = {"1", "20000000000000000", "7CCE5EFDACCF6000"};
    for (int s = 0; s < 3; s++) {
      Int key; key.SetBase16((char *)starts[s]);
      Int half; half.SetInt32(512);
      Int c; c.Set(&key); c.Add(&half);
      Point startP = secp->ComputePublicKey(&c);
      std::vector<uint8_t> xs, xr;
      for (int grp = 0; grp < 2; grp++) {
        Int dx[513];
        IntGroup g(513);
        g.Set(dx);
        for (int i = 0; i < 512; i++) dx[i].ModSub(&Gn[i].x, &startP.x);
        dx[512].ModSub(&_2Gn.x, &startP.x);
        g.ModInv();
        std::vector<Point> pts(1024);
        pts[512] = startP;
        for (int i = 0; i < 512; i++) {
          Int dy, sl, p2;
          if (i < 511) {
            Point pp = startP;
            dy.ModSub(&Gn[i].y, &pp.y);
            sl.ModMulK1(&dy, &dx[i]); p2.ModSquareK1(&sl);
            pp.x.ModNeg(); pp.x.ModAdd(&p2); pp.x.ModSub(&Gn[i].x);
            pts[512 + i + 1] = pp;
          }
          Point pn = startP;
          Int dyn; dyn.Set(&Gn[i].y); dyn.ModNeg(); dyn.ModSub(&pn.y);
          sl.ModMulK1(&dyn, &dx[i]); p2.ModSquareK1(&sl);
          pn.x.ModNeg(); pn.x.ModAdd(&p2); pn.x.ModSub(&Gn[i].x);
          pts[512 - i - 1] = pn;
        }
        for (int i = 0; i < 1024; i++) { uint8_t b[32]; pts[i].x.Get32Bytes(b); xs.insert(xs.end(), b, b + 32); }
        // next centre (keyhunt.cpp:3840-3855)
        Point pp = startP;
        Int dy, sl, p2;
        dy.ModSub(&_2Gn.y, &pp.y);
        sl.ModMulK1(&dy, &dx[512]); p2.ModSquareK1(&sl);
        pp.x.ModNeg(); pp.x.ModAdd(&p2); pp.x.ModSub(&_2Gn.x);
        pp.y.ModSub(&_2Gn.x, &pp.x); pp.y.ModMulK1(&sl); pp.y.ModSub(&_2Gn.y);
        startP = pp;
      }
      for (int i = 0; i < 2048; i++) {
        Int k; k.Set(&key); k.Add((uint64_t)i);
        Point p = secp->ComputePublicKey(&k);
        uint8_t b[32]; p.x.Get32Bytes(b); xr.insert(xr.end(), b, b + 32);
      }
      uint8_t first[32]; memcpy(first, xs.data(), 32);
      printf("  {\"start\":\"%s\",\"n\":2048,\"sha256_walk\":\"%s\",\"sha256_direct\":\"%s\",\"x0\":\"%s\"}%s\n",
             ihex(key).c_str(), sha_hex(xs.data(), xs.size()).c_str(), sha_hex(xr.data(), xr.size()).c_str(),
             hexs(first, 32).c_str(), s == 2 ? "" : ",");
    }
  }
  printf("],\n");

  // ---------------- BSGS baby tables at small M ----------------
  // thread_bPload (keyhunt.cpp:5284-5472) restated on reference primitives + reference bloom.
  printf("\"bsgs_build\": [\n");
  {
    struct { uint64_t n, k; } cfg[] = {{1ULL << 20, 1}, {1ULL << 22, 2}, {1ULL << 24, 4}};
    for (int c = 0; c < 3; c++) {
      uint64_t m = 1; while ((m + 1) * (m + 1) <= cfg[c].n) m++;
      m *= cfg[c].k;
      uint64_t m2 = m / 32 + (m % 32 ? 1 : 0), m3 = m2 / 32 + (m2 % 32 ? 1 : 0);
      uint64_t it1 = (m / 256 > 10000) ? (m / 256 + (m % 256 ? 1 : 0)) : 1000;
      uint64_t it2 = (m2 / 256 > 1000) ? (m2 / 256 + (m2 % 256 ? 1 : 0)) : 1000;
      uint64_t it3 = (m3 / 256 > 1000) ? (m3 / 256 + (m3 % 256 ? 1 : 0)) : 1000;
      uint64_t its[3] = {it1, it2, it3};
      std::vector<struct bloom> L[3];
      for (int l = 0; l < 3; l++) {
        L[l].resize(256);
        for (int s = 0; s < 256; s++) bloom_init2(&L[l][s], its[l] <= 10000 ? 10000 : its[l], 0.000001);
      }
      struct row { uint8_t v[6]; uint64_t idx; };
      std::vector<row> tab;
      for (uint64_t i = 0; i < m; i++) {
        Int k; k.SetInt64(i + 1);
        Point p = secp->ComputePublicKey(&k);
        uint8_t x[32]; p.x.Get32Bytes(x);
        int s = x[0];
        if (i < m3) { row r; memcpy(r.v, x + 16, 6); r.idx = i; tab.push_back(r); bloom_add(&L[2][s], x, 32); }
        if (i < m2) bloom_add(&L[1][s], x, 32);
        bloom_add(&L[0][s], x, 32);
      }
      std::sort(tab.begin(), tab.end(), [](const row &a, const row &b) {
        int c2 = memcmp(a.v, b.v, 6); if (c2) return c2 < 0; return a.idx < b.idx; });
      std::string sh[3];
      for (int l = 0; l < 3; l++) {
        std::vector<uint8_t> all;
        for (int s = 0; s < 256; s++) all.insert(all.end(), L[l][s].bf, L[l][s].bf + L[l][s].bytes);
        sh[l] = sha_hex(all.data(), all.size());
      }
      std::vector<uint8_t> tb;
      for (auto &r : tab) { uint8_t b[16] = {0}; memcpy(b, r.v, 6); memcpy(b + 8, &r.idx, 8); tb.insert(tb.end(), b, b + 16); }
      printf("  {\"n\":%llu,\"k\":%llu,\"m\":%llu,\"m2\":%llu,\"m3\":%llu,\"bytes\":[%llu,%llu,%llu],\"sha256_l1\":\"%s\",\"sha256_l2\":\"%s\",\"sha256_l3\":\"%s\",\"sha256_table\":\"%s\"}%s\n",
             (unsigned long long)cfg[c].n, (unsigned long long)cfg[c].k, (unsigned long long)m,
             (unsigned long long)m2, (unsigned long long)m3, (unsigned long long)L[0][0].bytes,
             (unsigned long long)L[1][0].bytes, (unsigned long long)L[2][0].bytes, sh[0].c_str(), sh[1].c_str(),
             sh[2].c_str(), sha_hex(tb.data(), tb.size()).c_str(), c == 2 ? "" : ",");
      for (int l = 0; l < 3; l++) for (int s = 0; s < 256; s++) bloom_free(&L[l][s]);
    }
  }
  printf("],\n");
  // Ethereum addresses (generate_binaddress_eth, keyhunt.cpp:5663-5669): the reference's
  // SHA3_256_Init / Update / KECCAK_256_Final (keyhunt.cpp:5647-5653) of the 64-byte X||Y
  printf("\"eth\": [\n");
  for (int i = 0; i < 40; i++) {
    Int k;
    if (i < 8) k.SetInt32((uint32_t)(i * 7919 + 1));
    else rand_int(k);
    Point P = secp->ComputePublicKey(&k);
    uint8_t xy[64], d[32];
    P.x.Get32Bytes(xy);
    P.y.Get32Bytes(xy + 32);
    SHA3_256_CTX ctx;
    SHA3_256_Init(&ctx);
    SHA3_256_Update(&ctx, xy, 64);
    KECCAK_256_Final(d, &ctx);
    printf("  {\"k\":\"%s\",\"xy\":\"%s\",\"keccak\":\"%s\",\"address\":\"%s\"}%s\n", ihex(k).c_str(),
           hexs(xy, 64).c_str(), hexs(d, 32).c_str(), hexs(d + 12, 20).c_str(), i == 39 ? "" : ",");
  }
  printf("]\n}\n");
  return 0;
}
