// kh_host_util.h -- host helpers shared by the engine's command-line programs (keyhunt-amd,
// bsgsd-amd): 256-bit range arithmetic and hex I/O (the reference's Int, secp256k1/Int.cpp),
// public-key parsing (Secp256K1::ParsePublicKeyHex, secp256k1/SECP256K1.cpp:327-380) and the
// -n/-k validation (util.c:358-389).
#pragma once
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <mutex>
#include <random>
#include <string>
#include <vector>

#include "../csrc/kh_math.h"

namespace khh {
using namespace kh;

// ---------------------------------------------------------------------------------------------
// big integers (256-bit, plus a little headroom for range arithmetic)
// ---------------------------------------------------------------------------------------------
typedef unsigned __int128 u128;
struct U {
  uint64_t v[5] = {0, 0, 0, 0, 0};
};
inline U u_from_u64(uint64_t x) {
  U r;
  r.v[0] = x;
  return r;
}
inline int u_cmp(const U &a, const U &b) {
  for (int i = 4; i >= 0; i--) {
    if (a.v[i] < b.v[i]) return -1;
    if (a.v[i] > b.v[i]) return 1;
  }
  return 0;
}
inline U u_add(const U &a, const U &b) {
  U r;
  u128 c = 0;
  for (int i = 0; i < 5; i++) {
    c += (u128)a.v[i] + b.v[i];
    r.v[i] = (uint64_t)c;
    c >>= 64;
  }
  return r;
}
inline U u_sub(const U &a, const U &b) {
  U r;
  uint64_t br = 0;
  for (int i = 0; i < 5; i++) {
    u128 t = (u128)a.v[i] - b.v[i] - br;
    r.v[i] = (uint64_t)t;
    br = (uint64_t)(t >> 64) & 1;
  }
  return r;
}
inline U u_mul_u64(const U &a, uint64_t m) {
  U r;
  u128 c = 0;
  for (int i = 0; i < 5; i++) {
    c += (u128)a.v[i] * m;
    r.v[i] = (uint64_t)c;
    c >>= 64;
  }
  return r;
}
inline bool u_is_zero(const U &a) { return !(a.v[0] | a.v[1] | a.v[2] | a.v[3] | a.v[4]); }
inline U u_shl1(int bits) {  // 1 << bits
  U r;
  r.v[bits / 64] = 1ULL << (bits % 64);
  return r;
}
// a / b for b < 2^64, and remainder
inline U u_divmod_u64(const U &a, uint64_t b, uint64_t *rem) {
  U q;
  u128 r = 0;
  for (int i = 4; i >= 0; i--) {
    r = (r << 64) | a.v[i];
    q.v[i] = (uint64_t)(r / b);
    r %= b;
  }
  if (rem) *rem = (uint64_t)r;
  return q;
}
inline int u_bitlen(const U &a) {
  for (int i = 4; i >= 0; i--)
    if (a.v[i]) return 64 * i + 64 - __builtin_clzll(a.v[i]);
  return 0;
}
// uniform in [a, b) by rejection over bitlen(b - a) bits (the reference's Int::Rand(a, b) draws
// from MT19937 seeded by getrandom, keyhunt.cpp:697-715; not reproducible there either)
inline std::mt19937_64 g_rng{std::random_device{}()};
inline std::mutex g_rng_mtx;
inline U u_rand_range(const U &a, const U &b) {
  if (u_cmp(b, a) <= 0) return a;
  U span = u_sub(b, a), r;
  int bits = u_bitlen(span);
  std::lock_guard<std::mutex> lk(g_rng_mtx);
  do {
    for (int i = 0; i < 5; i++) {
      int lo = 64 * i;
      r.v[i] = lo >= bits ? 0 : g_rng();
      if (lo < bits && bits - lo < 64) r.v[i] &= (1ULL << (bits - lo)) - 1;
    }
  } while (u_cmp(r, span) >= 0);
  return u_add(a, r);
}
inline bool u_from_hex(const char *s, U &r) {
  r = U();
  if (s[0] == '0' && (s[1] == 'x' || s[1] == 'X')) s += 2;
  size_t n = strlen(s);
  if (n == 0 || n > 64) return false;
  for (size_t i = 0; i < n; i++) {
    char c = s[i];
    int d = (c >= '0' && c <= '9') ? c - '0' : (c >= 'a' && c <= 'f') ? c - 'a' + 10 : (c >= 'A' && c <= 'F') ? c - 'A' + 10 : -1;
    if (d < 0) return false;
    // r = r*16 + d
    for (int k = 4; k > 0; k--) r.v[k] = (r.v[k] << 4) | (r.v[k - 1] >> 60);
    r.v[0] = (r.v[0] << 4) | (uint64_t)d;
  }
  return true;
}
inline bool u_from_dec(const char *s, U &r) {
  r = U();
  if (!*s) return false;
  for (; *s; s++) {
    if (*s < '0' || *s > '9') return false;
    r = u_add(u_mul_u64(r, 10), u_from_u64((uint64_t)(*s - '0')));
  }
  return true;
}
// lowercase hex without leading zeros (Int::GetBase16, secp256k1/Int.cpp:1019-1055)
inline std::string u_hex(const U &a) {
  static const char *H = "0123456789abcdef";
  std::string s;
  bool lead = true;
  for (int i = 4; i >= 0; i--)
    for (int j = 60; j >= 0; j -= 4) {
      int d = (int)((a.v[i] >> j) & 15);
      if (lead && d == 0) continue;
      lead = false;
      s += H[d];
    }
  return s.empty() ? "0" : s;
}
inline std::string u_dec(const U &a) {
  if (u_is_zero(a)) return "0";
  std::string s;
  U x = a;
  while (!u_is_zero(x)) {
    uint64_t r;
    x = u_divmod_u64(x, 10, &r);
    s += (char)('0' + r);
  }
  std::reverse(s.begin(), s.end());
  return s;
}
inline void u_to_be32(const U &a, uint8_t b[32]) {
  for (int i = 0; i < 4; i++)
    for (int j = 0; j < 8; j++) b[(3 - i) * 8 + j] = (uint8_t)(a.v[i] >> (56 - 8 * j));
}
inline U u_from_be32(const uint8_t b[32]) {
  U r;
  for (int i = 0; i < 4; i++) {
    uint64_t w = 0;
    for (int j = 0; j < 8; j++) w = (w << 8) | b[(3 - i) * 8 + j];
    r.v[i] = w;
  }
  return r;
}
inline const char *ORDER_HEX = "FFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEBAAEDCE6AF48A03BBFD25E8CD0364141";

inline std::string hex(const uint8_t *b, int n) {
  static const char *H = "0123456789abcdef";
  std::string s;
  for (int i = 0; i < n; i++) {
    s += H[b[i] >> 4];
    s += H[b[i] & 15];
  }
  return s;
}
inline bool is_hex(const char *s) {
  for (; *s; s++)
    if (!strchr("0123456789abcdefABCDEF", *s)) return false;
  return true;
}

inline bool hex2bin(const char *s, uint8_t *out, size_t n) {
  if (strlen(s) < 2 * n) return false;
  for (size_t i = 0; i < n; i++) {
    unsigned v;
    if (sscanf(s + 2 * i, "%2x", &v) != 1) return false;
    out[i] = (uint8_t)v;
  }
  return true;
}

inline void trim(char *s) {
  size_t n = strlen(s);
  while (n && strchr(" \t\r\n", s[n - 1])) s[--n] = 0;
  size_t i = 0;
  while (s[i] && strchr(" \t\r\n", s[i])) i++;
  if (i) memmove(s, s + i, n - i + 1);
}

inline bool parse_pubkey(const char *s, fe &x, fe &y, bool &compressed) {
  size_t n = strlen(s);
  uint8_t raw[65];
  if (n == 66 && (s[0] == '0' && (s[1] == '2' || s[1] == '3'))) {
    if (!hex2bin(s + 2, raw, 32)) return false;
    fe_from_be(x, raw);
    fe t, s3, seven;
    fe_sqr(t, x);
    fe_mul(t, t, x);
    fe_set_u32(seven, 7);
    fe_add(s3, t, seven);
    if (!fe_sqrt(y, s3)) return false;
    uint32_t odd = s[1] == '3';
    if ((y.d[0] & 1) != odd) fe_neg(y, y);
    compressed = true;
    return true;
  }
  if (n == 130 && s[0] == '0' && s[1] == '4') {
    if (!hex2bin(s + 2, raw, 64)) return false;
    fe_from_be(x, raw);
    fe_from_be(y, raw + 32);
    compressed = false;
    return true;
  }
  return false;
}

// Secp256K1::ParsePublicKeyHex (secp256k1/SECP256K1.cpp:303-380) with its printed messages: bytes
// read two characters at a time by sscanf("%X") (GetByte, 303-314), the prefix picks the form, and
// the point must lie on the curve.  Returns 1 on success, 0 on a refused key, -1 where the reference
// calls exit(-1) (a digit pair sscanf cannot read, a 04 key of the wrong length).
inline int parse_pubkey_hex_ref(const char *s, fe &x, fe &y, bool &compressed) {
  const size_t len = strlen(s);
  if (len < 2) {
    printf("ParsePublicKeyHex: Error invalid public key specified (66 or 130 character length)\n");
    return 0;
  }
  bool bad = false;
  auto byte = [&](size_t idx) -> uint8_t {
    char tmp[3] = {idx * 2 < len ? s[2 * idx] : '\0', idx * 2 + 1 < len ? s[2 * idx + 1] : '\0', 0};
    int val = 0;
    if (sscanf(tmp, "%X", &val) != 1) bad = true;
    return (uint8_t)val;
  };
  auto fail_digit = [&]() {
    printf("ParsePublicKeyHex: Error invalid public key specified (unexpected hexadecimal digit)\n");
    return -1;
  };
  const uint8_t type = byte(0);
  if (bad) return fail_digit();
  uint8_t raw[64];
  if (type == 0x02 || type == 0x03) {
    if (len != 66) {
      printf("ParsePublicKeyHex: Error invalid public key specified (66 character length)\n");
      return 0;
    }
    for (int i = 0; i < 32; i++) raw[i] = byte(i + 1);
    if (bad) return fail_digit();
    fe_from_be(x, raw);
    fe t, s3, seven;
    fe_sqr(t, x);
    fe_mul(t, t, x);
    fe_set_u32(seven, 7);
    fe_add(s3, t, seven);
    if (!fe_sqrt(y, s3)) {
      printf("ParsePublicKeyHex: Error invalid public key specified (Not lie on elliptic curve)\n");
      return 0;
    }
    if ((y.d[0] & 1) != (uint32_t)(type == 0x03)) fe_neg(y, y);
    compressed = true;
    return 1;
  }
  if (type == 0x04) {
    if (len != 130) {
      printf("ParsePublicKeyHex: Error invalid public key specified (130 character length)\n");
      return -1;
    }
    for (int i = 0; i < 64; i++) raw[i] = byte(i + 1);
    if (bad) return fail_digit();
    fe_from_be(x, raw);
    fe_from_be(y, raw + 32);
    fe t, r, seven;
    fe_sqr(t, x);
    fe_mul(t, t, x);
    fe_set_u32(seven, 7);
    fe_add(r, t, seven);
    fe_sqr(t, y);
    if (!fe_eq(t, r)) {
      printf("ParsePublicKeyHex: Error invalid public key specified (Not lie on elliptic curve)\n");
      return 0;
    }
    compressed = false;
    return 1;
  }
  printf("ParsePublicKeyHex: Error invalid public key specified (Unexpected prefix (only 02,03 or 04 allowed)\n");
  return 0;
}

// ---------------------------------------------------------------------------------------------
// vanity targets
// ---------------------------------------------------------------------------------------------
// b58tobin (base58/base58.c, libbase58): big-endian into *binszp bytes with 32-bit limbs, false on
// an invalid digit or overflow (then *binszp is unchanged); else *binszp = the canonical length
// (binsz - leading zero bytes + leading '1's)
inline bool b58tobin_ref(uint8_t *bin, size_t *binszp, const char *b58, size_t b58sz) {
  static const char *D = "123456789ABCDEFGHJKLMNPQRSTUVWXYZabcdefghijkmnopqrstuvwxyz";
  const size_t binsz = *binszp;
  const size_t outisz = (binsz + 3) / 4;
  std::vector<uint32_t> outi(outisz ? outisz : 1, 0);
  const unsigned bytesleft = binsz % 4;
  const uint32_t zeromask = bytesleft ? (uint32_t)(0xFFFFFFFFull << (bytesleft * 8)) : 0;
  unsigned zerocount = 0;
  size_t i = 0;
  for (; i < b58sz && b58[i] == '1'; ++i) ++zerocount;
  for (; i < b58sz; ++i) {
    const char *pos = ((unsigned char)b58[i] & 0x80) ? nullptr : strchr(D, b58[i]);
    if (!pos || !b58[i]) return false;
    uint32_t c = (uint32_t)(pos - D);
    for (size_t j = outisz; j--;) {
      const uint64_t t = (uint64_t)outi[j] * 58 + c;
      c = (uint32_t)(t >> 32);
      outi[j] = (uint32_t)t;
    }
    if (c || (outi[0] & zeromask)) return false;
  }
  uint8_t *b = bin;
  size_t j = 0;
  if (bytesleft) {
    for (unsigned q = bytesleft; q > 0; --q) *(b++) = (uint8_t)(outi[0] >> (8 * (q - 1)));
    ++j;
  }
  for (; j < outisz; ++j)
    for (int q = 4; q > 0; --q) *(b++) = (uint8_t)(outi[j] >> (8 * (q - 1)));
  for (i = 0; i < binsz; ++i) {
    if (bin[i]) break;
    --*binszp;
  }
  *binszp += zerocount;
  return true;
}

inline bool is_base58(const char *s) {
  for (; *s; s++)
    if (!strchr("123456789ABCDEFGHJKLMNPQRSTUVWXYZabcdefghijkmnopqrstuvwxyz", *s)) return false;
  return true;
}

// addvanity (keyhunt.cpp:6739-6866): the hash160 ranges [A_j, B_j] of the addresses that start
// with `target` (padded with '1' for A, 'z' for B up to each 25-byte decoding length), appended to
// `ranges` (40 bytes each); min_bytes tracks the common-prefix length the vanity bloom keys on.
struct vanity_set {
  std::vector<uint8_t> ranges;
  uint64_t total = 0;      // vanity_rmd_total
  int min_bytes = 999999;  // vanity_rmd_minimun_bytes_check_length
  int targets = 0;
};
inline int addvanity(const char *target, vanity_set &v) {
  const int targetsize = (int)strlen(target);
  if (targetsize >= 30) return 0;
  std::vector<std::vector<uint8_t>> side[2];
  for (int sd = 0; sd < 2; sd++) {
    char copy[50];
    memset(copy, 0, 50);
    memcpy(copy, target, (size_t)targetsize);
    int stringsize = targetsize;
    uint8_t raw[50];
    memset(raw, 0, 50);
    size_t len;
    do {
      len = 50;
      b58tobin_ref(raw, &len, copy, (size_t)stringsize);
      if (len < 25) copy[stringsize++] = sd ? 'z' : '1';
      if (len == 25) {
        b58tobin_ref(raw, &len, copy, (size_t)stringsize);
        side[sd].push_back(std::vector<uint8_t>(raw + 1, raw + 21));
        copy[stringsize++] = sd ? 'z' : '1';
      }
    } while (len <= 25 && stringsize < 50);
  }
  if (side[0].empty() || side[1].empty()) return 0;
  const int r = (int)std::min(side[0].size(), side[1].size());
  for (int j = 0; j < r; j++) {
    int same = 0;
    while (same < 20 && side[0][j][same] == side[1][j][same]) same++;
    v.min_bytes = std::min(v.min_bytes, same);
    v.ranges.insert(v.ranges.end(), side[0][j].begin(), side[0][j].end());
    v.ranges.insert(v.ranges.end(), side[1][j].begin(), side[1][j].end());
  }
  v.total += (uint64_t)r;
  v.targets++;
  return r;
}

// validate_nk (util.c:358-389)
inline bool validate_nk(uint64_t n, uint64_t k) {
  if (n < (1ULL << 20)) {
    fprintf(stderr, "[E] n must be at least 2^20 (0x100000)\n");
    return false;
  }
  if (n & (n - 1)) {
    fprintf(stderr, "[E] n must be a power of two\n");
    return false;
  }
  int bits = 0;
  for (uint64_t t = n; t > 1; t >>= 1) bits++;
  if (bits % 2 || bits < 20 || bits > 64) {
    fprintf(stderr, "[E] invalid n 0x%llx\n", (unsigned long long)n);
    return false;
  }
  // table: {20,1},{22,2},{24,4},... k_max doubles every 2 bits
  const uint64_t kmax = 1ULL << ((bits - 20) / 2);
  if (k > kmax) {
    fprintf(stderr, "[E] k value %llu is too large for n 0x%llx (max %llu)\n", (unsigned long long)k,
            (unsigned long long)n, (unsigned long long)kmax);
    return false;
  }
  return true;
}

// MD5 (RFC 1321) of a file, for --ptable-cache's FILE.md5 and FILE.cache (keyhunt.cpp:1958-1981,
// 2655-2700).
struct md5_ctx {
  uint32_t h[4] = {0x67452301u, 0xefcdab89u, 0x98badcfeu, 0x10325476u};
  uint8_t buf[64];
  uint64_t len = 0;
  void block(const uint8_t *p) {
    static const uint32_t K[64] = {
        0xd76aa478, 0xe8c7b756, 0x242070db, 0xc1bdceee, 0xf57c0faf, 0x4787c62a, 0xa8304613, 0xfd469501,
        0x698098d8, 0x8b44f7af, 0xffff5bb1, 0x895cd7be, 0x6b901122, 0xfd987193, 0xa679438e, 0x49b40821,
        0xf61e2562, 0xc040b340, 0x265e5a51, 0xe9b6c7aa, 0xd62f105d, 0x02441453, 0xd8a1e681, 0xe7d3fbc8,
        0x21e1cde6, 0xc33707d6, 0xf4d50d87, 0x455a14ed, 0xa9e3e905, 0xfcefa3f8, 0x676f02d9, 0x8d2a4c8a,
        0xfffa3942, 0x8771f681, 0x6d9d6122, 0xfde5380c, 0xa4beea44, 0x4bdecfa9, 0xf6bb4b60, 0xbebfbc70,
        0x289b7ec6, 0xeaa127fa, 0xd4ef3085, 0x04881d05, 0xd9d4d039, 0xe6db99e5, 0x1fa27cf8, 0xc4ac5665,
        0xf4292244, 0x432aff97, 0xab9423a7, 0xfc93a039, 0x655b59c3, 0x8f0ccc92, 0xffeff47d, 0x85845dd1,
        0x6fa87e4f, 0xfe2ce6e0, 0xa3014314, 0x4e0811a1, 0xf7537e82, 0xbd3af235, 0x2ad7d2bb, 0xeb86d391};
    static const int R[16] = {7, 12, 17, 22, 5, 9, 14, 20, 4, 11, 16, 23, 6, 10, 15, 21};
    uint32_t m[16];
    for (int i = 0; i < 16; i++)
      m[i] = p[4 * i] | p[4 * i + 1] << 8 | p[4 * i + 2] << 16 | (uint32_t)p[4 * i + 3] << 24;
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3];
    for (int i = 0; i < 64; i++) {
      uint32_t f;
      int g;
      switch (i >> 4) {
        case 0: f = (b & c) | (~b & d); g = i; break;
        case 1: f = (d & b) | (~d & c); g = (5 * i + 1) & 15; break;
        case 2: f = b ^ c ^ d; g = (3 * i + 5) & 15; break;
        default: f = c ^ (b | ~d); g = (7 * i) & 15; break;
      }
      const uint32_t t = a + f + K[i] + m[g];
      const int r = R[(i >> 4) * 4 + (i & 3)];
      a = d;
      d = c;
      c = b;
      b = b + ((t << r) | (t >> (32 - r)));
    }
    h[0] += a;
    h[1] += b;
    h[2] += c;
    h[3] += d;
  }
  void update(const uint8_t *p, size_t n) {
    size_t fill = len % 64;
    len += n;
    while (n) {
      const size_t take = std::min(n, (size_t)64 - fill);
      memcpy(buf + fill, p, take);
      fill += take;
      p += take;
      n -= take;
      if (fill == 64) {
        block(buf);
        fill = 0;
      }
    }
  }
  void final(uint8_t out[16]) {
    const uint64_t bits = len * 8;
    const uint8_t one = 0x80, zero = 0;
    update(&one, 1);
    while (len % 64 != 56) update(&zero, 1);
    uint8_t l[8];
    for (int i = 0; i < 8; i++) l[i] = (uint8_t)(bits >> (8 * i));
    update(l, 8);
    for (int i = 0; i < 16; i++) out[i] = (uint8_t)(h[i / 4] >> (8 * (i % 4)));
  }
};
inline bool md5_of_file(const char *path, uint8_t out[16]) {
  FILE *f = fopen(path, "rb");
  if (!f) return false;
  md5_ctx c;
  std::vector<uint8_t> b(1 << 20);
  size_t n;
  while ((n = fread(b.data(), 1, b.size(), f)) > 0) c.update(b.data(), n);
  const bool ok = !ferror(f);
  fclose(f);
  if (ok) c.final(out);
  return ok;
}

// FILE.md5 as keyhunt writes and reads it: the hex MD5 and a newline (keyhunt.cpp:186-241)
inline bool read_md5_file(const char *path, uint8_t out[16]) {
  char buf[64] = {0};
  FILE *f = fopen(path, "r");
  if (!f) return false;
  size_t n = fread(buf, 1, sizeof buf - 1, f);
  fclose(f);
  buf[n] = 0;
  if (char *nl = strchr(buf, '\n')) *nl = 0;
  if (strlen(buf) < 32) return false;
  buf[32] = 0;
  return hex2bin(buf, out, 16);
}
inline bool write_md5_file(const char *path, const uint8_t md5[16]) {
  FILE *f = fopen(path, "w");
  bool ok = f && fprintf(f, "%s\n", hex(md5, 16).c_str()) > 0;
  if (f) ok = fclose(f) == 0 && ok;
  return ok;
}

// FILE.cache: struct bptable_cache_file {magic 'BPTC', version 1, entries, md5, 257 bucket starts by
// value[0] of the 16-byte rows} (keyhunt.cpp:137-143, 186-241; bsgsd.cpp:255-360)
#pragma pack(push, 1)
struct bptable_cache_file {
  uint32_t magic, version;
  uint64_t entries;
  uint8_t md5[16];
  uint64_t boundaries[257];
};
#pragma pack(pop)
static_assert(sizeof(bptable_cache_file) == 2088, "struct bptable_cache_file");
// 1: a cache of this MD5 and row count, -1: another one, 0: none readable
inline int bptable_cache_status(const char *path, const uint8_t md5[16], uint64_t m3) {
  bptable_cache_file disk;
  FILE *f = fopen(path, "rb");
  if (!f) return 0;
  int st = 0;
  if (fread(&disk, sizeof disk, 1, f) == 1)
    st = disk.magic == 0x42505443u && disk.version == 1 && disk.entries == m3 && !memcmp(disk.md5, md5, 16) ? 1 : -1;
  fclose(f);
  return st;
}
inline bool bptable_cache_write(const char *path, const uint8_t md5[16], const uint8_t *rows, uint64_t m3) {
  bptable_cache_file fc;
  memset(&fc, 0, sizeof fc);
  fc.magic = 0x42505443u;
  fc.version = 1;
  fc.entries = m3;
  memcpy(fc.md5, md5, 16);
  uint64_t pos = 0;
  for (int bucket = 0; bucket < 256; bucket++) {
    while (pos < m3 && rows[pos * 16] < bucket) pos++;
    fc.boundaries[bucket] = pos;
  }
  fc.boundaries[256] = m3;
  FILE *f = fopen(path, "wb");
  bool ok = f && fwrite(&fc, sizeof fc, 1, f) == 1;
  if (f) ok = fclose(f) == 0 && ok;
  return ok;
}

}  // namespace khh
