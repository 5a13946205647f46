// keyhunt_cli.cpp -- command-line host of the MI355X engine (bin/keyhunt-amd).
//
// Keeps the reference's interface for the hot-path modes: -m address|rmd160|xpoint|bsgs, -f, -r,
// -b, -k, -n, -l, -q, -s, -I (stride), plus -g (GPUs to use; one host thread + kh_ctx each, like one
// pthread per -t in the reference, keyhunt.cpp:2717-2839).  Hit text, KEYFOUNDKEYFOUND.txt records
// and the stats line follow keyhunt.cpp:6891-6923 (writekey), 4825-4858 (BSGS) and 2850-2962.
// Sequential scans consume the range in whole N_SEQUENTIAL_MAX chunks (keyhunt.cpp:3314-3330) and
// BSGS in whole 2N bases (keyhunt.cpp:4600-4617), exactly as the reference's cursors do.
// BSGS base schedules -B sequential|backward|both|random|dance|angrygiant and random chunks (-R)
// follow the reference's cursors (see take_bases).  -e (address/rmd160/xpoint), -c eth (address/rmd160)
// -m vanity, and -S / -6 (the BSGS table files and the address/rmd160/xpoint data_<hex>.dat target
// cache, in the reference's formats) and -B ggsb / --bsgs-block-count / --bsgs-block-size are
// provided; minikeys are rejected.
#include <ctype.h>
#include <fcntl.h>
#include <getopt.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <random>
#include <atomic>
#include <condition_variable>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "kh_gpu.h"
#include "../csrc/kh_math.h"
#include "kh_host_util.h"
#include "kh_mapped.h"

using namespace kh;
using namespace khh;

namespace {

const char *VERSION = "keyhunt-amd 0.1 (MI355X engine for keyhunt 0.2.230519 hot paths)";

// ---------------------------------------------------------------------------------------------
// hashing / encoding for hit output
// ---------------------------------------------------------------------------------------------
void sha256(const uint8_t *msg, size_t len, uint8_t out[32]) {
  uint32_t st[8];
  sha256_init(st);
  size_t off = 0;
  uint32_t w[16];
  auto load = [&](const uint8_t *b) {
    for (int i = 0; i < 16; i++)
      w[i] = ((uint32_t)b[4 * i] << 24) | ((uint32_t)b[4 * i + 1] << 16) | ((uint32_t)b[4 * i + 2] << 8) | b[4 * i + 3];
  };
  while (len - off >= 64) {
    load(msg + off);
    sha256_transform(st, w);
    off += 64;
  }
  uint8_t blk[128] = {0};
  size_t rem = len - off;
  memcpy(blk, msg + off, rem);
  blk[rem] = 0x80;
  size_t nb = rem >= 56 ? 2 : 1;
  uint64_t bits = (uint64_t)len * 8;
  for (int i = 0; i < 8; i++) blk[nb * 64 - 1 - i] = (uint8_t)(bits >> (8 * i));
  for (size_t b = 0; b < nb; b++) {
    load(blk + 64 * b);
    sha256_transform(st, w);
  }
  for (int i = 0; i < 8; i++) {
    out[4 * i] = st[i] >> 24;
    out[4 * i + 1] = st[i] >> 16;
    out[4 * i + 2] = st[i] >> 8;
    out[4 * i + 3] = st[i];
  }
}
const char *B58 = "123456789ABCDEFGHJKLMNPQRSTUVWXYZabcdefghijkmnopqrstuvwxyz";
std::string b58enc(const uint8_t *d, int n) {
  std::vector<uint8_t> buf;
  int zeros = 0;
  while (zeros < n && d[zeros] == 0) zeros++;
  for (int i = zeros; i < n; i++) {
    int carry = d[i];
    for (auto &b : buf) {
      carry += b * 256;
      b = carry % 58;
      carry /= 58;
    }
    while (carry) {
      buf.push_back(carry % 58);
      carry /= 58;
    }
  }
  std::string s(zeros, '1');
  for (auto it = buf.rbegin(); it != buf.rend(); ++it) s += B58[*it];
  return s;
}
std::string rmd_to_address(const uint8_t h[20]) {
  uint8_t d[25], c1[32], c2[32];
  d[0] = 0;
  memcpy(d + 1, h, 20);
  sha256(d, 21, c1);
  sha256(c1, 32, c2);
  memcpy(d + 21, c2, 4);
  return b58enc(d, 25);
}
// ---------------------------------------------------------------------------------------------
// options and shared state
// ---------------------------------------------------------------------------------------------
enum { MODE_ADDRESS, MODE_RMD160, MODE_XPOINT, MODE_BSGS, MODE_VANITY };
struct options {
  int mode = MODE_ADDRESS;
  const char *file = nullptr;
  int search = KH_SEARCH_BOTH;
  bool have_range = false, have_bits = false;
  U start, end;
  int bits = 0;
  uint64_t kfactor = 1;
  bool flag_n = false;
  const char *str_n = nullptr;
  int gpus = 0;
  bool quiet = false;
  int seconds = 30;
  U stride = u_from_u64(1);
  bool matrix = false;
  uint32_t layer1 = KH_LAYER1_BLOCKED;
  bool random = false;  // -R
  bool endo = false;    // -e
  bool stride_set = false;
  int bsgs_mode = 0;    // -B, index into BSGS_MODES
  bool eth = false;            // -c eth (keyhunt.cpp:874-891)
  vanity_set vanity;           // -m vanity targets (-v, -f)
  bool save_read = false;      // -S: read the table files if present, else build and write them
  bool skip_checksum = false;  // -6
  int bloom_mult = 1;          // -z (FLAGBLOOMMULTIPLIER)
  // GGSB (keyhunt.cpp:1477-1499, 1617-1627): -B ggsb or --bsgs-block-count/--bsgs-block-size
  bool ggsb = false;
  uint64_t ggsb_count = 0, ggsb_size = 0;
  // --ptable FILE / --ptable-size S / --load-ptable (keyhunt.cpp:772-787, 1847-1956)
  const char *ptable = nullptr;
  uint64_t ptable_size = 0;
  bool load_ptable = false;
  bool ptable_cache = false;  // --ptable-cache: FILE.md5 + FILE.cache (keyhunt.cpp:1958-1981, 2655-2700)
  // memory-mapped bloom files (keyhunt.cpp:493-499, 724-806)
  bool mapped = false;           // FLAGMAPPED
  bool create_mapped = false;    // FLAGCREATEMAPPED
  bool load_bloom = false;       // FLAGLOADBLOOM
  const char *mapped_name = nullptr;
  uint64_t mapped_entries = 0;   // mapped_entries_override
  long double mapped_error = 0;  // mapped_error_override
  uint32_t mapped_chunks = 1;
  int rmd_batch = 1024;  // --rmd-batch-size (keyhunt.cpp:301, 815-829), -m rmd160 only
  bool crypto_given = false;      // -c (FLAGCRYPTO set): no "Setting search for btc" line
  std::string range_start_str, range_end_str;  // -r as typed (BSGS prints them so, keyhunt.cpp:1529-1531)
} opt;
// keyhunt.cpp:419; ggsb and angrygiant walk like sequential (ggsb with BSGS_STEP = 2 x block size)
const char *BSGS_MODES[7] = {"sequential", "backward", "both", "random", "dance", "ggsb", "angrygiant"};
enum { BM_SEQUENTIAL, BM_BACKWARD, BM_BOTH, BM_RANDOM, BM_DANCE, BM_GGSB, BM_ANGRYGIANT };

std::mutex g_keys_mtx, g_cursor_mtx;
std::atomic<uint64_t> g_groups_done{0};  // groups walked (address family): 1024 keys each in the stats
std::atomic<uint64_t> g_bases_done{0};   // BSGS bases
std::atomic<int> g_running{0};
U g_cursor;
U g_end;

// ---------------------------------------------------------------------------------------------
// hit output
// ---------------------------------------------------------------------------------------------
void writekey(kh_ctx *ctx, bool compressed, const uint8_t key[32]) {
  // keyhunt.cpp:6891-6923
  uint8_t xy[64];
  kh_pubkeys(ctx, key, 1, xy);
  fe x, y;
  fe_from_be(x, xy);
  fe_from_be(y, xy + 32);
  uint32_t hw[5];
  std::string pub;
  if (compressed) {
    uint8_t pfx = (y.d[0] & 1) ? 3 : 2;
    hash160_comp(x, pfx, hw);
    pub = hex(&pfx, 1) + hex(xy, 32);
  } else {
    uint8_t pfx = 4;
    hash160_uncomp(x, y, hw);
    pub = hex(&pfx, 1) + hex(xy, 64);
  }
  uint8_t rmd[20];
  memcpy(rmd, hw, 20);
  std::string addr = rmd_to_address(rmd);
  std::string k = u_hex(u_from_be32(key));
  std::lock_guard<std::mutex> lk(g_keys_mtx);
  FILE *f = fopen("KEYFOUNDKEYFOUND.txt", "a+");
  if (f) {
    fprintf(f, "Private Key: %s\npubkey: %s\nAddress %s\nrmd160 %s\n", k.c_str(), pub.c_str(), addr.c_str(),
            hex(rmd, 20).c_str());
    fclose(f);
  }
  printf("\nHit! Private Key: %s\npubkey: %s\nAddress %s\nrmd160 %s\n", k.c_str(), pub.c_str(), addr.c_str(),
         hex(rmd, 20).c_str());
  fflush(stdout);
}

// keyhunt.cpp:6925-6950: Ethereum hits
void writekeyeth(kh_ctx *ctx, const uint8_t key[32]) {
  uint8_t xy[64];
  kh_pubkeys(ctx, key, 1, xy);
  fe x, y;
  fe_from_be(x, xy);
  fe_from_be(y, xy + 32);
  uint32_t w[5];
  eth_address(x, y, w);
  uint8_t a[20];
  memcpy(a, w, 20);
  const std::string k = u_hex(u_from_be32(key)), addr = "0x" + hex(a, 20);
  std::lock_guard<std::mutex> lk(g_keys_mtx);
  FILE *f = fopen("KEYFOUNDKEYFOUND.txt", "a+");
  if (f) {
    fprintf(f, "Private Key: %s\naddress: %s\n", k.c_str(), addr.c_str());
    fclose(f);
  }
  printf("\n Hit!!!! Private Key: %s\naddress: %s\n", k.c_str(), addr.c_str());
  fflush(stdout);
}

// keyhunt.cpp:6705-6737: vanity hits
void writevanitykey(kh_ctx *ctx, bool compressed, const uint8_t key[32]) {
  uint8_t xy[64];
  kh_pubkeys(ctx, key, 1, xy);
  fe x, y;
  fe_from_be(x, xy);
  fe_from_be(y, xy + 32);
  uint32_t hw[5];
  std::string pub;
  if (compressed) {
    uint8_t pfx = (y.d[0] & 1) ? 3 : 2;
    hash160_comp(x, pfx, hw);
    pub = hex(&pfx, 1) + hex(xy, 32);
  } else {
    uint8_t pfx = 4;
    hash160_uncomp(x, y, hw);
    pub = hex(&pfx, 1) + hex(xy, 64);
  }
  uint8_t rmd[20];
  memcpy(rmd, hw, 20);
  const std::string addr = rmd_to_address(rmd), k = u_hex(u_from_be32(key));
  std::lock_guard<std::mutex> lk(g_keys_mtx);
  FILE *f = fopen("VANITYKEYFOUND.txt", "a+");
  if (f) {
    fprintf(f, "Vanity Private Key: %s\npubkey: %s\nAddress %s\nrmd160 %s\n", k.c_str(), pub.c_str(), addr.c_str(),
            hex(rmd, 20).c_str());
    fclose(f);
  }
  printf("\nVanity Private Key: %s\npubkey: %s\nAddress %s\nrmd160 %s\n", k.c_str(), pub.c_str(), addr.c_str(),
         hex(rmd, 20).c_str());
  fflush(stdout);
}

// ---------------------------------------------------------------------------------------------
// target files
// ---------------------------------------------------------------------------------------------
// readFileVanity (keyhunt.cpp:6990-7035): base58 prefixes, one per line, added to the -v ones
bool read_vanity(const char *fn) {
  FILE *f = fn ? fopen(fn, "r") : nullptr;
  if (f) {
    char line[1024];
    while (fgets(line, sizeof line, f)) {
      trim(line);
      const size_t len = strlen(line);
      if (len > 0 && len < 36) {
        if (is_base58(line))
          addvanity(line, opt.vanity);
        else
          fprintf(stderr, "[E] the string \"%s\" is not valid Base58, omiting it\n", line);
      }
    }
    fclose(f);
  }
  if (opt.vanity.targets == 0) {
    fprintf(stderr, "[E] There aren't any vanity targets\n");
    return false;
  }
  return true;
}

// initBloomFilter's lines (keyhunt.cpp:7605-7626): the item count it was given and the size of the
// filter it makes, bloom_init2(max(10000, items) (x -z above the floor), 1e-6).  The --mapped path
// prints its own (kh_mapped.h).
void print_bloom_init(uint64_t items) {
  if (opt.mapped) return;
  const uint64_t total = items <= 10000 ? 10000 : (uint64_t)opt.bloom_mult * items;
  printf("[+] Bloom filter for %llu elements.\n", (unsigned long long)items);
  printf("[+] Loading data to the bloomfilter total: %.2f MB\n", (double)mapped::bytes_for(total, 0.000001L) / 1048576.0);
}

// forceReadFileAddressEth (keyhunt.cpp:7312-7384): 40 hex digits, or 0x and 40 hex digits
bool read_targets_eth(const char *fn, std::vector<uint8_t> &rows, uint64_t &bloom_items,
                      std::vector<uint8_t> *adds = nullptr) {
  FILE *f = fopen(fn, "r");
  if (!f) {
    fprintf(stderr, "[E] Error opening the file %s\n", fn);
    return false;
  }
  char line[1024];
  std::vector<std::string> lines;
  uint64_t counted = 0;
  while (fgets(line, sizeof line, f)) {
    trim(line);
    if (strlen(line) >= 40) counted++;
    lines.push_back(line);
  }
  fclose(f);
  bloom_items = counted;
  printf("[+] Allocating memory for %llu elements: %.2f MB\n", (unsigned long long)counted,
         (double)(counted * 20) / 1048576.0);
  print_bloom_init(counted);
  for (auto &ln : lines) {
    uint8_t raw[20];
    const size_t r = ln.size();
    if (r == 40 && is_hex(ln.c_str()) && hex2bin(ln.c_str(), raw, 20)) {
      rows.insert(rows.end(), raw, raw + 20);
      if (adds) adds->insert(adds->end(), raw, raw + 20);
    } else if (r == 42 && is_hex(ln.c_str() + 2) && hex2bin(ln.c_str() + 2, raw, 20)) {
      rows.insert(rows.end(), raw, raw + 20);
      if (adds) adds->insert(adds->end(), raw, raw + 20);
    } else if (r >= 40) {
      fprintf(stderr, "[I] Ommiting invalid line %s\n", ln.c_str());
    }
  }
  return true;
}

// forceReadFileAddress (keyhunt.cpp:7239-7310) / forceReadFileXPoint (7392-7490)
// The reference's line reads: fgets(buf, cap) pieces of at most cap - 1 characters (a longer line
// is read as several pieces), trimmed of " \t\n\r" (util.c:217).
std::vector<std::string> fgets_pieces(FILE *f, size_t cap) {
  std::vector<std::string> out;
  std::vector<char> buf(cap);
  while (fgets(buf.data(), (int)cap, f)) {
    trim(buf.data());
    out.emplace_back(buf.data());
  }
  return out;
}

// -m address / rmd160 / xpoint target files, with the reference's reading quirks.
//  address, rmd160 (forceReadFileAddress, keyhunt.cpp:7239-7305): items = lines longer than 20
//    characters; then lines are consumed in order while i < items, a line that is not a 25-byte
//    base58 address or 40 hex digits printing "[I] Ommiting invalid line" and lowering items by one,
//    so valid lines after short or blank ones can go unread.  The base58 decode is b58tobin into a
//    25-byte buffer whose result length alone decides (its return value is ignored, as there).
//  xpoint (forceReadFileXPoint, keyhunt.cpp:7392-7490): items = lines of 40+ characters; the first
//    `items` lines are table rows in order, an unusable one a zero row; lines missing at the end of
//    the file lower the count.  (A blank line among them crashes the reference: strlen(NULL).)
bool read_targets(const char *fn, int mode, std::vector<uint8_t> &rows, uint64_t &bloom_items,
                  std::vector<uint8_t> *adds = nullptr) {
  FILE *f = fopen(fn, "r");
  if (!f) {
    fprintf(stderr, "[E] Error opening the file %s\n", fn);
    return false;
  }
  const bool xp = mode == MODE_XPOINT;
  std::vector<std::string> lines = fgets_pieces(f, xp ? 1000 : 100);
  fclose(f);
  uint64_t counted = 0;
  for (auto &ln : lines)
    if ((xp && ln.size() >= 40) || (!xp && ln.size() > 20)) counted++;
  bloom_items = counted;
  printf("[+] Allocating memory for %llu elements: %.2f MB\n", (unsigned long long)counted,
         (double)(counted * 20) / 1048576.0);
  print_bloom_init(counted);
  uint8_t raw[100] = {0};
  size_t next = 0;
  if (xp) {
    for (uint64_t i = 0; i < counted; i++) {
      if (next >= lines.size()) {  // fgets hit the end of the file: "Omiting line", N--
        fprintf(stderr, "[E] Omiting line : \n");
        continue;
      }
      const std::string &ln = lines[next++];
      std::string tok = ln.substr(0, ln.find_first_of(" \t:"));
      if (!is_hex(tok.c_str())) {
        fprintf(stderr, "[E] Ignoring invalid hexvalue %s\n", tok.c_str());  // aux after strtok
        rows.insert(rows.end(), 20, 0);  // the row stays zero (keyhunt.cpp:7433)
        continue;
      }
      // the bloom gets the first 20 bytes of what was decoded: 04||X[0..19) for an uncompressed key
      // while its table row is X[1..21) (keyhunt.cpp:7462-7467, SURVEY 8a parity note 9)
      if (tok.size() == 64 && hex2bin(tok.c_str(), raw, 32)) rows.insert(rows.end(), raw, raw + 20);
      else if (tok.size() == 66 && hex2bin(tok.c_str() + 2, raw, 32)) rows.insert(rows.end(), raw, raw + 20);
      else if (tok.size() == 130 && hex2bin(tok.c_str(), raw, 65)) rows.insert(rows.end(), raw + 2, raw + 22);
      else {
        fprintf(stderr, "[E] Omiting line unknow length size %zu: %s\n", tok.size(), tok.c_str());
        rows.insert(rows.end(), 20, 0);
        continue;
      }
      if (adds) adds->insert(adds->end(), raw, raw + 20);
    }
    return true;
  }
  uint64_t items = counted, i = 0;
  while (i < items) {
    const std::string ln = next < lines.size() ? lines[next++] : std::string();
    const size_t r = ln.size();
    bool ok = false;
    if (r > 0 && r <= 40) {
      if (r < 40 && is_base58(ln.c_str())) {
        size_t len = 25;
        b58tobin_ref(raw, &len, ln.c_str(), r);
        if (len == 25) {
          rows.insert(rows.end(), raw + 1, raw + 21);
          if (adds) adds->insert(adds->end(), raw + 1, raw + 21);
          ok = true;
        }
      }
      if (r == 40 && is_hex(ln.c_str()) && hex2bin(ln.c_str(), raw, 20)) {
        rows.insert(rows.end(), raw, raw + 20);
        if (adds) adds->insert(adds->end(), raw, raw + 20);
        ok = true;
      }
    }
    if (ok) {
      i++;
    } else {
      fprintf(stderr, "[I] Ommiting invalid line %s\n", ln.c_str());
      items--;
    }
  }
  return true;
}


// ---------------------------------------------------------------------------------------------
// --mapped bloom files (keyhunt.cpp:1131-1172, 1700-1785, 7630-7706; bloom/bloom.cpp:454-747).
// A mapped filter is its raw bit array in NAME (or NAME.0 .. NAME.<c-1> with --mapped-chunks c,
// flat concatenation); the reference keeps it mapped MAP_SHARED, so the bits its loaders add reach
// the file.  Here every GPU context searches with its usual tables (the hits are decided by the
// exact table / bP-table checks, which these filters only gate), and the files are written with
// exactly the bits the reference leaves in them: a fresh file gets bloom_init_mmap's geometry; an
// existing one (without a size override) is reloaded with bloom_load_mmap's, bits = bytes * 8 and
// the hash count entries_hashes_for_bytes derives from the size, and the items are added again on
// top of its bits.  With chunks, the reference's bit -> chunk map (byte / chunk_bytes) equals the
// concatenation except for bytes past c * chunk_bytes, which it indexes out of bounds.
// ---------------------------------------------------------------------------------------------
// the mapped bloom files live in kh_mapped.h (shared with bsgsd-amd); mapped::cfg is filled
// from the options once they are parsed

// ---------------------------------------------------------------------------------------------
// stats (keyhunt.cpp:2850-2962)
// ---------------------------------------------------------------------------------------------
void print_stats(uint64_t secs, const U &total) {
  static const char *pfx[7] = {"Mkeys/s", "Gkeys/s", "Tkeys/s", "Pkeys/s", "Ekeys/s", "Zkeys/s", "Ykeys/s"};
  uint64_t rem;
  U per = u_divmod_u64(total, secs ? secs : 1, &rem);
  U lim[7];
  U l = u_from_u64(1000000);
  for (int i = 0; i < 7; i++) {
    lim[i] = l;
    l = u_mul_u64(l, 1000);
  }
  // -M (FLAGMATRIX) prints the line as a line of its own; otherwise it overwrites itself in place
  const char *lead = opt.matrix ? "" : "\r", *tail = opt.matrix ? "\n" : "\r";
  if (u_cmp(per, lim[0]) < 0) {
    printf("%s[+] Total %s keys in %llu seconds: %s keys/s%s", lead, u_dec(total).c_str(), (unsigned long long)secs,
           u_dec(per).c_str(), tail);
  } else {
    int i = 0;
    while (i < 6 && u_cmp(per, lim[i + 1]) >= 0) i++;
    uint64_t div = 1;
    for (int k = 0; k < 6 + 3 * i && k < 18; k++) div *= 10;
    U d = per;
    for (int k = 0; k < i; k++) d = u_divmod_u64(d, 1000, nullptr);
    d = u_divmod_u64(d, 1000000, nullptr);
    printf("%s[+] Total %s keys in %llu seconds: ~%s %s (%s keys/s)%s", lead, u_dec(total).c_str(),
           (unsigned long long)secs, u_dec(d).c_str(), pfx[i], u_dec(per).c_str(), tail);
  }
  fflush(stdout);
}

U keys_done(const U &twoN) {
  if (opt.mode == MODE_BSGS) {
    U t = u_mul_u64(twoN, g_bases_done.load());
    return t;
  }
  U t = u_mul_u64(u_from_u64(1024), g_groups_done.load());
  if (opt.endo)  // keyhunt.cpp:2883-2891
    t = u_mul_u64(t, opt.mode == MODE_XPOINT ? 3 : 6);
  else if (opt.search == KH_SEARCH_COMPRESS)
    t = u_mul_u64(t, 2);
  return t;
}

// ---------------------------------------------------------------------------------------------
// workers
// ---------------------------------------------------------------------------------------------
struct addr_job {
  int device;
  int index = 0;  // worker number (the reference's thread_number)
  const std::vector<uint8_t> *rows;
  uint64_t bloom_items;
  uint64_t nseq;
  const char *data_file = nullptr;  // -S: data_<hex>.dat to read (or, with save_data, to write)
  bool save_data = false;
  int rc = 0;
};

// -S target cache name (readFileAddress / writeFileIfNeeded, keyhunt.cpp:7043-7049, 7765-7770):
// data_ + hex of the first 4 bytes of the target file's sha256
bool data_file_name(const char *fn, std::string &name) {
  FILE *f = fopen(fn, "rb");
  if (!f) return false;
  std::vector<uint8_t> buf;
  uint8_t chunk[1 << 16];
  size_t n;
  while ((n = fread(chunk, 1, sizeof chunk, f)) > 0) buf.insert(buf.end(), chunk, chunk + n);
  fclose(f);
  uint8_t ck[32];
  sha256(buf.data(), buf.size(), ck);
  char hex[9];
  snprintf(hex, sizeof hex, "%02x%02x%02x%02x", ck[0], ck[1], ck[2], ck[3]);
  name = std::string("data_") + hex + ".dat";
  return true;
}

// writeFileIfNeeded (keyhunt.cpp:7756-7855) when the target filter lives in a mapped file (-S with
// --mapped): sha256(bits) | that filter's struct bloom (kh_mapped.h struct_bloom) | its bits |
// sha256(rows) | u64 row bytes | the 20-byte rows sorted.  (Without --mapped the engine writes the
// file from its own filter, kh_targets_save.)
bool write_mapped_data_file(const std::string &path, const mapped::filter &F, const std::vector<uint8_t> &rows) {
  const size_t n = rows.size() / 20;
  std::vector<uint32_t> ix(n);
  for (size_t i = 0; i < n; i++) ix[i] = (uint32_t)i;
  std::sort(ix.begin(), ix.end(), [&](uint32_t a, uint32_t b) { return memcmp(&rows[20 * (size_t)a], &rows[20 * (size_t)b], 20) < 0; });
  std::vector<uint8_t> srt(rows.size());
  for (size_t i = 0; i < n; i++) memcpy(&srt[20 * i], &rows[20 * (size_t)ix[i]], 20);
  const uint64_t data_size = srt.size();
  uint8_t ckb[32], ckd[32], h[112];
  sha256(F.bf.data(), F.bytes, ckb);
  sha256(srt.data(), srt.size(), ckd);
  mapped::struct_bloom(F, h);
  FILE *f = fopen(path.c_str(), "wb");
  if (!f) return false;
  bool ok = fwrite(ckb, 1, 32, f) == 32 && fwrite(h, 1, 112, f) == 112 &&
            (F.bytes == 0 || fwrite(F.bf.data(), 1, F.bytes, f) == F.bytes) && fwrite(ckd, 1, 32, f) == 32 &&
            fwrite(&data_size, 1, 8, f) == 8 && (data_size == 0 || fwrite(srt.data(), 1, data_size, f) == data_size);
  ok = fclose(f) == 0 && ok;
  return ok;
}

void addr_worker(addr_job *j) {
  kh_ctx *ctx = nullptr;
  int r = kh_open(j->device, &ctx);
  if (r) {
    fprintf(stderr, "[E] GPU %d: %s\n", j->device, kh_strerror(r));
    j->rc = r;
    g_running--;
    return;
  }
  if (opt.mode == MODE_VANITY)
    r = kh_set_vanity(ctx, opt.vanity.ranges.data(), opt.vanity.ranges.size() / 40, (uint32_t)opt.vanity.min_bytes,
                      opt.vanity.total);
  else if (j->data_file && !j->save_data)
    r = kh_targets_load(ctx, j->data_file, opt.skip_checksum ? KH_LOAD_SKIP_CHECKSUM : 0);
  else
    r = kh_set_targets(ctx, j->rows->data(), j->rows->size() / 20, j->bloom_items);
  if (!r && j->save_data) {
    printf("[D] size data %llu\n", (unsigned long long)(j->rows->size()));  // keyhunt.cpp:7773
    printf("[+] Writing file %s ........\n", j->data_file);
    r = kh_targets_save(ctx, j->data_file);
  }
  // --rmd-batch-size below 1024: the reference's groups of that size (thread_process,
  // keyhunt.cpp:3301-3307 -- FLAGMODE == MODE_RMD160 only), each counted as 1024 keys in the stats
  // (steps[] x CPU_GRP_SIZE, 2847-2880) like every group
  const uint64_t group = opt.mode == MODE_RMD160 ? (uint64_t)opt.rmd_batch : 1024;
  if (!r && group != 1024) r = kh_set_rmd_batch(ctx, (uint32_t)group);
  if (r) fprintf(stderr, "[E] GPU %d: %s (%s)\n", j->device, kh_strerror(r), kh_last_error(ctx));
  std::vector<kh_hit> hits(1 << 16);
  uint8_t st_be[32], stride_be[32];
  u_to_be32(opt.stride, stride_be);
  const U span = u_mul_u64(opt.stride, j->nseq);
  while (!r) {
    U base;
    {
      std::lock_guard<std::mutex> lk(g_cursor_mtx);
      if (opt.random) {
        base = u_rand_range(g_cursor, g_end);  // key_mpz.Rand(start, end) per chunk (keyhunt.cpp:3309-3311)
      } else {
        if (u_cmp(g_cursor, g_end) >= 0) break;
        base = g_cursor;
        g_cursor = u_add(g_cursor, span);
      }
    }
    // the chunk's progress line (thread_process, keyhunt.cpp:3333-3346): one line per chunk with -M,
    // else (without -q) overwritten in place; "thread" is this worker's index, as the reference's
    if (opt.matrix) {
      printf("Base key: %s thread %i\n", u_hex(base).c_str(), j->index);
      fflush(stdout);
    } else if (!opt.quiet) {
      printf("\rBase key: %s     \r", u_hex(base).c_str());
      fflush(stdout);
    }
    u_to_be32(base, st_be);
    uint32_t nh = 0;
    r = kh_scan(ctx, st_be, stride_be, j->nseq,
                opt.mode == MODE_XPOINT ? (KH_MODE_XPOINT | (opt.endo ? KH_MODE_ENDO : 0))
                : (opt.eth && (opt.mode == MODE_ADDRESS || opt.mode == MODE_RMD160)) ? (KH_MODE_ETH | (opt.endo ? KH_MODE_ENDO : 0))
                      : (KH_MODE_ADDRESS | (opt.endo ? KH_MODE_ENDO : 0)),
                (uint32_t)opt.search, hits.data(), (uint32_t)hits.size(), &nh);
    if (r == KH_E_OVERFLOW && nh > hits.size()) {  // a short vanity prefix: take them all
      hits.resize(nh);
      r = kh_scan(ctx, st_be, stride_be, j->nseq, KH_MODE_ADDRESS | (opt.endo ? KH_MODE_ENDO : 0),
                  (uint32_t)opt.search, hits.data(), (uint32_t)hits.size(), &nh);
    }
    // KH_E_RANGE (--rmd-batch-size, a group centred on the key 0 mod n): the hits of the groups
    // before it are reported, then the worker stops
    if (r && r != KH_E_RANGE) {
      fprintf(stderr, "[E] kh_scan: %s (%s)\n", kh_strerror(r), kh_last_error(ctx));
      break;
    }
    for (uint32_t i = 0; i < nh && i < hits.size(); i++) {
      if ((hits[i].kind & 15u) == KH_KIND_ETH)
        writekeyeth(ctx, hits[i].key);
      else if (opt.mode == MODE_VANITY)
        writevanitykey(ctx, hits[i].compressed != 0, hits[i].key);
      else
        writekey(ctx, hits[i].compressed != 0, hits[i].key);
    }
    if (r) {
      fprintf(stderr, "[E] kh_scan: %s (%s)\n", kh_strerror(r), kh_last_error(ctx));
      break;
    }
    g_groups_done += (j->nseq + group - 1) / group;
  }
  j->rc = r;
  kh_close(ctx);
  g_running--;
}

struct bsgs_job {
  int device;
  const std::vector<fe> *tx, *ty;
  const std::vector<bool> *comp;
  uint64_t n, k;
  uint64_t bases_per_call;       // consecutive bases of 2N (one counted progression per call)
  uint64_t list_bases_per_call;  // listed bases (-B backward|both|random|dance, ggsb): the host lists,
                                 // sorts and uploads each one, so calls stay at ~2^31 giant points
  bool first = false;  // the first GPU's worker (writes the -S files)
  int rc = 0;
};
std::vector<uint8_t> g_found;  // bsgs_found[]
std::mutex g_found_mtx;

// Base schedules of -B (one call takes up to `want` bases under the cursor lock, as the
// reference's threads take one each):
//   sequential / angrygiant  BSGS_CURRENT += 2N while < end           keyhunt.cpp:4600-4617
//   backward                 end -= 2N; base = max(end, start)          keyhunt.cpp:5995-6014
//   both                     rand()%2 picks TOP (as backward, against BSGS_CURRENT) or BOTTOM
//                            (as sequential, against the moving end)    keyhunt.cpp:6257-6300
//   random                   Rand(start, end), endless                  keyhunt.cpp:4934-4952
//   dance                    rand()%3: TOP, BOTTOM or Rand(current, end) keyhunt.cpp:5706-5750
// g_cursor plays BSGS_CURRENT (and n_range_start), g_top n_range_end.
U g_top;
U g_step;  // BSGS_STEP
// step = BSGS_STEP: 2N, or 2 x the GGSB block size when the babies are split into several blocks
bool take_bases(const U &twoN, uint64_t want, std::vector<U> &out) {
  out.clear();
  std::lock_guard<std::mutex> lk(g_cursor_mtx);
  auto top = [&]() {
    if (u_cmp(g_top, g_cursor) <= 0) return false;
    g_top = u_sub(g_top, twoN);
    out.push_back(u_cmp(g_top, g_cursor) < 0 ? g_cursor : g_top);
    return true;
  };
  auto bottom = [&]() {
    if (u_cmp(g_cursor, g_top) >= 0) return false;
    out.push_back(g_cursor);
    g_cursor = u_add(g_cursor, twoN);
    return true;
  };
  int mode = opt.bsgs_mode;
  if (mode == BM_SEQUENTIAL || mode == BM_ANGRYGIANT || mode == BM_BACKWARD || mode == BM_GGSB) {
    while (out.size() < want && (mode == BM_BACKWARD ? top() : bottom())) {
    }
    return !out.empty();
  }
  if (mode == BM_RANDOM) {
    while (out.size() < want) out.push_back(u_rand_range(g_cursor, g_top));
    return true;
  }
  // both / dance: one draw per batch (the reference draws per base; the set of bases is the same)
  int pick = rand() % (mode == BM_DANCE ? 3 : 2);
  if (pick == 2) {
    while (out.size() < want) out.push_back(u_rand_range(g_cursor, g_top));
    return true;
  }
  while (out.size() < want && (pick == 0 ? top() : bottom())) {
  }
  if (out.empty()) {  // this side is exhausted; the other may not be
    while (out.size() < want && (pick == 0 ? bottom() : top())) {
    }
  }
  return !out.empty();
}

// One engine call's bases of a listed schedule: `drawn` in the reference's order (the progress
// lines); a run 2N apart, ascending or descending (backward, both), goes through kh_bsgs_scan from its
// lowest base, any other set through kh_bsgs_scan_list in drawn order (the engine needs no order)
struct list_batch {
  bool ok = false;
  std::vector<U> drawn;
  bool consecutive = false;
  uint8_t st_be[32];
  std::vector<uint8_t> be;
};

void prepare_batch(const U &twoN, uint64_t want, list_batch &B) {
  B.ok = take_bases(twoN, want, B.drawn);
  B.be.clear();
  if (!B.ok) return;
  const size_t n = B.drawn.size();
  bool up = true, down = true;
  for (size_t i = 1; i < n && (up || down); i++) {
    if (up) up = u_cmp(B.drawn[i], B.drawn[i - 1]) > 0 && u_cmp(u_sub(B.drawn[i], B.drawn[i - 1]), twoN) == 0;
    if (down) down = u_cmp(B.drawn[i - 1], B.drawn[i]) > 0 && u_cmp(u_sub(B.drawn[i - 1], B.drawn[i]), twoN) == 0;
  }
  B.consecutive = up || down;
  if (B.consecutive) {
    u_to_be32(up ? B.drawn[0] : B.drawn[n - 1], B.st_be);
    return;
  }
  B.be.resize(32 * n);
  for (size_t i = 0; i < n; i++) u_to_be32(B.drawn[i], &B.be[32 * i]);
}

// The sequential schedules (sequential, angrygiant, ggsb) as one progression: up to `want` bases
// from the cursor, step apart, while below the end -- the bases take_bases would list, counted
// instead of listed (a call of 2^20 bases spent ~9 % of the GPU's time listing, sorting and
// checking them on the host between calls)
bool take_progression(const U &step, uint64_t want, U &start, uint64_t &count) {
  std::lock_guard<std::mutex> lk(g_cursor_mtx);
  if (u_cmp(g_cursor, g_top) >= 0) return false;
  start = g_cursor;
  const U rem = u_sub(g_top, g_cursor);
  uint64_t n = want;
  if (step.v[1] == 0 && step.v[2] == 0 && step.v[3] == 0 && step.v[4] == 0 && step.v[0]) {
    uint64_t r = 0;
    const U q = u_divmod_u64(rem, step.v[0], &r);  // bases below the end: ceil(rem / step)
    if (u_bitlen(q) < 63) n = std::min<uint64_t>(want, q.v[0] + (r ? 1 : 0));
    count = n;
    g_cursor = u_add(g_cursor, u_mul_u64(step, n));
    return true;
  }
  for (count = 0; count < want && u_cmp(g_cursor, g_top) < 0; count++) g_cursor = u_add(g_cursor, step);
  return true;
}

// --ptable-cache: FILE.md5 holds the file's MD5 as hex text; FILE.cache the 257 bucket starts of
// the rows by value[0] under that MD5 (struct bptable_cache_file, keyhunt.cpp:137-143, 186-241).
// Two phases, where the reference has them: with --load-ptable, before the tables are built, an
// existing FILE.md5 is trusted, else the MD5 is computed from the file and written (1956-1981);
// after the tables (and the -S files), the MD5 is computed if it is not known yet, and the cache
// file is checked and rebuilt when it is of another MD5 or size (2655-2700).  Only the files are
// produced: the engine's third check does not need the buckets.
uint8_t g_md5[16];
bool g_md5_ready = false;

void ptable_md5_loaded() {
  if (!opt.ptable_cache || !opt.load_ptable || !opt.ptable) return;
  const std::string md5_path = std::string(opt.ptable) + ".md5";
  if (read_md5_file(md5_path.c_str(), g_md5)) {
    g_md5_ready = true;
    printf("[+] bP table MD5 loaded (%s)\n", md5_path.c_str());
  } else if (md5_of_file(opt.ptable, g_md5)) {
    g_md5_ready = true;
    uint8_t disk[16];
    if (read_md5_file(md5_path.c_str(), disk))
      printf(memcmp(disk, g_md5, 16) == 0 ? "[+] bP table MD5 verified (%s)\n" : "[W] bP table MD5 mismatch (%s); refreshing\n",
             md5_path.c_str());
    if (!write_md5_file(md5_path.c_str(), g_md5))
      fprintf(stderr, "[W] Unable to write bP table MD5 file %s\n", md5_path.c_str());
  } else {
    fprintf(stderr, "[W] Unable to compute MD5 for bP table %s\n", opt.ptable);
  }
}

void ptable_cache(const uint8_t *rows, uint64_t m3) {
  if (!opt.ptable_cache) return;
  const std::string md5_path = std::string(opt.ptable) + ".md5", cache_path = std::string(opt.ptable) + ".cache";
  if (!g_md5_ready) {
    g_md5_ready = md5_of_file(opt.ptable, g_md5);
    if (g_md5_ready) {
      if (!write_md5_file(md5_path.c_str(), g_md5))
        fprintf(stderr, "[W] Unable to write bP table MD5 file %s\n", md5_path.c_str());
    } else {
      fprintf(stderr, "[W] Unable to compute MD5 for bP table %s\n", opt.ptable);
    }
  }
  if (!g_md5_ready) return;
  const int status = bptable_cache_status(cache_path.c_str(), g_md5, m3);
  if (status == 1) {
    printf("[+] bP table cache hit (%s)\n", cache_path.c_str());
    return;
  }
  if (status < 0)
    printf("[W] bP table cache mismatch (%s); rebuilding\n", cache_path.c_str());
  else
    printf("[I] bP table cache not found (%s); creating\n", cache_path.c_str());
  if (bptable_cache_write(cache_path.c_str(), g_md5, rows, m3))
    printf("[+] bP table cache refreshed (%s)\n", cache_path.c_str());
  else
    printf("[W] Unable to write bP table cache to %s\n", cache_path.c_str());
}

// --ptable FILE (keyhunt.cpp:1847-1956): the reference maps FILE (grown to max(M3 x 16 B,
// --ptable-size), never shrunk) as its bP table, so the baby-step workers (or -S's .tbl read) leave
// the sorted rows in it.  The rows are built on the GPU here, and the first worker writes them.
// With --load-ptable the existing FILE is mapped read-only and its first M3 rows are the table.
int bsgs_ptable(kh_ctx *ctx, const kh_bsgs_info &info, bool first) {
  if (!opt.ptable) return KH_OK;
  const uint64_t bytes = info.m3 * 16;
  if (opt.load_ptable) {
    // the file is mapped read-only, as the reference maps it (keyhunt.cpp:1880-1900), and its first
    // M3 rows go straight from the mapping into the context's table
    int fd = open(opt.ptable, O_RDONLY);
    if (fd < 0) {
      fprintf(stderr, "[E] Cannot open bP table file\n");
      return KH_E_IO;
    }
    struct stat st;
    if (fstat(fd, &st) != 0) {
      close(fd);
      fprintf(stderr, "[E] Cannot stat bP table file\n");
      return KH_E_IO;
    }
    if ((uint64_t)st.st_size < bytes) {
      close(fd);
      fprintf(stderr, "[E] Existing bP table file too small\n");
      return KH_E_IO;
    }
    const uint8_t *map = nullptr;
    if (bytes) {
      void *m = mmap(nullptr, bytes, PROT_READ, MAP_SHARED, fd, 0);
      if (m == MAP_FAILED) {
        close(fd);
        fprintf(stderr, "[E] mmap failed for bP table\n");
        return KH_E_IO;
      }
      map = (const uint8_t *)m;
    }
    close(fd);
    int r = kh_bsgs_set_table(ctx, map, info.m3);
    if (!r && first) ptable_cache(map, info.m3);
    if (map) munmap((void *)map, bytes);
    if (r) fprintf(stderr, "[E] %s\n", kh_last_error(ctx));
    return r;
  }
  if (!first) return KH_OK;
  // the context's own sorted rows, written without another host copy
  const uint8_t *rows = nullptr;
  uint64_t nrows = 0;
  int r = kh_bsgs_table_rows(ctx, &rows, &nrows);
  if (r) return r;
  const uint64_t map_bytes = std::max(bytes, opt.ptable_size);
  int fd = open(opt.ptable, O_RDWR | O_CREAT, 0600);
  if (fd < 0) {
    fprintf(stderr, "[E] Cannot create bP table file\n");
    return KH_E_IO;
  }
  struct stat st;
  bool ok = fstat(fd, &st) == 0;
  if (ok && (uint64_t)st.st_size < map_bytes) ok = ftruncate(fd, (off_t)map_bytes) == 0;
  if (!ok) {
    close(fd);
    fprintf(stderr, "[E] Cannot resize bP table file\n");
    return KH_E_IO;
  }
  // mappings under 1 MiB are zeroed first (keyhunt.cpp:1941-1951); larger ones keep their bytes
  if (map_bytes < (1ull << 20)) {
    std::vector<uint8_t> zero(map_bytes, 0);
    ok = pwrite(fd, zero.data(), map_bytes, 0) == (ssize_t)map_bytes;
  }
  for (uint64_t o = 0; ok && o < bytes;) {
    ssize_t w = pwrite(fd, rows + o, bytes - o, (off_t)o);
    ok = w > 0;
    if (ok) o += (uint64_t)w;
  }
  ok = close(fd) == 0 && ok;
  if (!ok) {
    fprintf(stderr, "[E] Cannot write bP table file\n");
    return KH_E_IO;
  }
  ptable_cache(rows, info.m3);
  return KH_OK;
}

// The reference's table-setup lines, which the first context's worker prints in the reference's order
// (keyhunt.cpp:1631-1845, 2225-2503); every number follows from M, M2, M3 and the shard geometry.
// The other workers wait for them (setup_done / setup_wait) before they print a base line.
//
// The three layers as initBloomFilter reports them (1687-1781 with 7605-7626): per layer the element
// count, then per shard its item count and bloom_init2 size, then the layer's total.  The --mapped
// path prints the same lines as it opens the shard files (kh_mapped.h bsgs_layers).
void print_layer_lines(const kh_bsgs_info &I) {
  const uint64_t ms[3] = {I.m, I.m2, I.m3}, floor_[3] = {10000, 1000, 1000};
  for (int l = 0; l < 3; l++) {
    const uint64_t items = ms[l] / 256 > floor_[l] ? ms[l] / 256 + (ms[l] % 256 ? 1 : 0) : 1000;
    const uint64_t bytes = mapped::init2_bytes(items <= 10000 ? 10000 : (uint64_t)opt.bloom_mult * items);
    printf("[+] Bloom filter for %llu elements ", (unsigned long long)ms[l]);
    for (int i = 0; i < 256; i++) {
      printf("[+] Bloom filter for %llu elements.\n", (unsigned long long)items);
      printf("[+] Loading data to the bloomfilter total: %.2f MB\n", (double)bytes / 1048576.0);
    }
    printf(": %.2f MB\n", mapped::layer_mb(256 * bytes));
  }
}

// 1845: the bP table's size, in whole MB (the integer division is the reference's)
void print_allocating(const kh_bsgs_info &I) {
  printf("[+] Allocating %.2f MB for %llu bP Points\n", (double)(I.m3 * 16 / 1048576), (unsigned long long)I.m3);
}

// The baby-step build (2362-2503): its progress lines as one reference thread (-t 1) prints them -- the
// count before the work units start, again at the loop's first pass, after each finished unit of
// THREADBPWORKLOAD = 1048576 babies (93, clamped to M) but the last, then the 100 % line (2457) -- the
// checksums of the three layers, and the sort of the bP rows (not with --load-ptable, 2495).  With more
// threads the reference's count lines depend on its threads' timing; these are the single-thread ones.
void print_build_lines(const kh_bsgs_info &I) {
  const uint64_t m = I.m, w = std::min<uint64_t>(1048576, m), units = m / w + (m % w ? 1 : 0);
  auto count = [&](uint64_t f) {
    printf("\r[+] processing %llu/%llu bP points : %i%%\r", (unsigned long long)f, (unsigned long long)m,
           (int)(((double)f / (double)m) * 100));
  };
  count(0);
  for (uint64_t u = 0; u < units; u++) count(u * w);
  printf("\r[+] processing %llu/%llu bP points : 100%%     \n", (unsigned long long)m, (unsigned long long)m);
  printf("[+] Making checkums .. ... done\n");
  if (!opt.load_ptable) printf("[+] Sorting %llu elements... Done!\n", (unsigned long long)I.m3);
}

std::mutex g_setup_mtx;
std::condition_variable g_setup_cv;
bool g_setup_done = false;
void setup_done() {
  fflush(stdout);
  {
    std::lock_guard<std::mutex> lk(g_setup_mtx);
    g_setup_done = true;
  }
  g_setup_cv.notify_all();
}
void setup_wait() {
  std::unique_lock<std::mutex> lk(g_setup_mtx);
  g_setup_cv.wait(lk, [] { return g_setup_done; });
}

// -S (keyhunt.cpp:1983-2230, 2504-2652): the files of this N/k in the working directory are read
// when they are all there, else the tables are built and (by the first GPU's worker) written.
// -S with --mapped (keyhunt.cpp:1983 skips the reads, 2504-2652 still writes): the table files hold the
// mapped shard filters -- each shard's struct bloom as the mapping left it, its bits and their sha256
// twice -- and the sorted bP rows with their sha256, in the reference's order 4, 6, 2, 7
int write_mapped_tables(kh_ctx *ctx, const kh_bsgs_info &info, const std::vector<std::vector<mapped::filter>> &F) {
  const uint64_t ms[3] = {info.m, info.m2, info.m3};
  const int kinds[3] = {4, 6, 7};
  auto layer = [&](int l) {
    char fn[96];
    snprintf(fn, sizeof fn, "keyhunt_bsgs_%d_%llu.blm", kinds[l], (unsigned long long)ms[l]);
    FILE *f = fopen(fn, "wb");
    if (!f) {
      fprintf(stderr, "[E] Error can't create the file %s\n", fn);
      return false;
    }
    bool ok = true;
    for (int i = 0; i < 256 && ok; i++) {
      uint8_t h[112], ck[32];
      mapped::struct_bloom(F[l][i], h);
      sha256(F[l][i].bf.data(), F[l][i].bytes, ck);
      ok = fwrite(h, 1, 112, f) == 112 && (F[l][i].bytes == 0 || fwrite(F[l][i].bf.data(), 1, F[l][i].bytes, f) == F[l][i].bytes) &&
           fwrite(ck, 1, 32, f) == 32 && fwrite(ck, 1, 32, f) == 32;
    }
    ok = fclose(f) == 0 && ok;
    if (!ok) fprintf(stderr, "[E] Error writing the file %s\n", fn);
    else printf("[+] Writing bloom filter to file %s .... Done!\n", fn);
    return ok;
  };
  if (!layer(0) || !layer(1)) return KH_E_IO;
  if (opt.load_ptable) return layer(2) ? KH_OK : KH_E_IO;  // no .tbl with --load-ptable (2588)
  const uint8_t *rows = nullptr;
  uint64_t n = 0;
  int r = kh_bsgs_table_rows(ctx, &rows, &n);
  if (r) return r;
  char fn[96];
  snprintf(fn, sizeof fn, "keyhunt_bsgs_2_%llu.tbl", (unsigned long long)info.m3);
  FILE *f = fopen(fn, "wb");
  if (!f) {
    fprintf(stderr, "[E] Error can't create the file %s\n", fn);
    return KH_E_IO;
  }
  uint8_t ck[32];
  sha256(rows, n * 16, ck);
  bool ok = (n == 0 || fwrite(rows, 1, n * 16, f) == n * 16) && fwrite(ck, 1, 32, f) == 32;
  ok = fclose(f) == 0 && ok;
  if (!ok) {
    fprintf(stderr, "[E] Error writing the file %s\n", fn);
    return KH_E_IO;
  }
  printf("[+] Writing bP Table to file %s .. Done!\n", fn);
  return layer(2) ? KH_OK : KH_E_IO;
}

int bsgs_tables(kh_ctx *ctx, const kh_bsgs_info &info, bool first) {
  if (opt.mapped) {  // -S is skipped with --mapped (keyhunt.cpp:1983); the shards live in files
    int r = kh_bsgs_build(ctx);
    std::vector<std::vector<mapped::filter>> F;
    if (!r && first && !mapped::bsgs_layers(ctx, info, opt.save_read ? &F : nullptr)) r = KH_E_IO;
    if (!r && first) {
      print_allocating(info);
      ptable_md5_loaded();
      print_build_lines(info);
      if (opt.save_read) r = write_mapped_tables(ctx, info, F);
    }
    return r;
  }
  if (first) {
    print_layer_lines(info);
    print_allocating(info);
    ptable_md5_loaded();
  }
  if (!opt.save_read) {
    int r = kh_bsgs_build(ctx);
    if (!r && first) print_build_lines(info);
    return r;
  }
  char f4[96], f6[96], f7[96], f2[96];
  if (opt.load_ptable) {
    // -S with --load-ptable (keyhunt.cpp:2153-2186): the reference reads the .tbl into its
    // read-only mapping of the --ptable file, which fails, or reports the .tbl missing; it never
    // writes the .tbl (2588)
    snprintf(f2, sizeof f2, "keyhunt_bsgs_2_%llu.tbl", (unsigned long long)info.m3);
    if (access(f2, F_OK) == 0) {
      fprintf(stderr, "[E] Error reading the file %s\n", f2);
    } else {
      fprintf(stderr, "[E] Missing bP table file %s\n", f2);
      fprintf(stderr, "    Remove --loadptable or generate the table first.\n");
    }
    return KH_E_IO;
  }
  snprintf(f4, sizeof f4, "keyhunt_bsgs_4_%llu.blm", (unsigned long long)info.m);
  snprintf(f6, sizeof f6, "keyhunt_bsgs_6_%llu.blm", (unsigned long long)info.m2);
  snprintf(f7, sizeof f7, "keyhunt_bsgs_7_%llu.blm", (unsigned long long)info.m3);
  snprintf(f2, sizeof f2, "keyhunt_bsgs_2_%llu.tbl", (unsigned long long)info.m3);
  static std::mutex mtx;
  static int decided = 0;  // 1: every worker reads the files, 2: every worker builds, the first writes
  {
    std::lock_guard<std::mutex> lk(mtx);
    if (!decided) {
      bool all = true;
      for (const char *f : {f4, f6, f7, f2}) all = all && access(f, R_OK) == 0;
      decided = all ? 1 : 2;
    }
  }
  if (decided == 1) {
    int r = kh_bsgs_load(ctx, ".", opt.skip_checksum ? KH_LOAD_SKIP_CHECKSUM : 0);
    if (r) {
      fprintf(stderr, "[E] %s\n", kh_last_error(ctx));
      return r;
    }
    if (first) {  // 1994-2225: a dot per 64 shards; nothing is built, checked or sorted after it
      printf("[+] Reading bloom filter from file %s .... Done!\n", f4);
      printf("[+] Reading bloom filter from file %s .... Done!\n", f6);
      printf("[+] Reading bP Table from file %s .... Done!\n", f2);
      printf("[+] Reading bloom filter from file %s .... Done!\n", f7);
    }
    return KH_OK;
  }
  int r = kh_bsgs_build(ctx);
  if (r || !first) return r;
  print_build_lines(info);
  r = kh_bsgs_save(ctx, ".");
  if (r) {
    fprintf(stderr, "[E] %s\n", kh_last_error(ctx));
    return r;
  }
  printf("[+] Writing bloom filter to file %s .... Done!\n", f4);
  printf("[+] Writing bloom filter to file %s .... Done!\n", f6);
  printf("[+] Writing bP Table to file %s .. Done!\n", f2);
  printf("[+] Writing bloom filter to file %s .... Done!\n", f7);
  return KH_OK;
}

// One found target, printed and recorded as the reference's worker does (keyhunt.cpp:4790-4830);
// returns true when every target is now found (the run then ends, 4811-4814)
bool print_found(kh_ctx *ctx, const bsgs_job *j, const kh_bsgs_found &fd) {
  uint32_t t = fd.target;
  {
    std::lock_guard<std::mutex> lk(g_found_mtx);
    if (g_found[t]) return false;
    g_found[t] = 1;
  }
  std::string k = u_hex(u_from_be32(fd.key));
  uint8_t pxy[64];
  kh_pubkeys(ctx, fd.key, 1, pxy);
  std::string pub;
  if ((*j->comp)[t]) {
    uint8_t p = (pxy[63] & 1) ? 3 : 2;
    pub = hex(&p, 1) + hex(pxy, 32);
  } else {
    uint8_t p = 4;
    pub = hex(&p, 1) + hex(pxy, 64);
  }
  {
    std::lock_guard<std::mutex> lk2(g_keys_mtx);
    // each BSGS worker of the reference has its own format: the sequential one (also -B ggsb and
    // angrygiant) continues its string over a backslash-newline, so no newline is printed
    // (keyhunt.cpp:4826-4827); random 5079, dance 5885, backward 6144, both 6429
    const int bm = opt.bsgs_mode;
    printf(bm == BM_SEQUENTIAL || bm == BM_GGSB || bm == BM_ANGRYGIANT ? "[+] Thread Key found privkey %s   "
           : bm == BM_RANDOM                                          ? "[+] Thread Key found privkey %s    \n"
                                                                      : "[+] Thread Key found privkey %s   \n",
           k.c_str());
    printf("[+] Publickey %s\n", pub.c_str());
    FILE *f = fopen("KEYFOUNDKEYFOUND.txt", "a");
    if (f) {
      fprintf(f, "Key found privkey %s\nPublickey %s\n", k.c_str(), pub.c_str());
      fclose(f);
    }
    fflush(stdout);
  }
  std::lock_guard<std::mutex> lk(g_found_mtx);
  return std::all_of(g_found.begin(), g_found.end(), [](uint8_t v) { return v != 0; });
}

// The per-base progress lines of the reference's BSGS workers, each printed as the worker takes the
// base (keyhunt.cpp:4618-4633; random 4955-4968, dance 5762-5774, backward 6023-6035, both
// 6308-6320): "[+] Thread 0x%s \n" with -M, else, unless -q, "\r[+] Thread 0x%s   \r" overwritten in
// place (the random worker pads with two spaces).  A call walks many bases: with -M every base's
// line is printed in the reference's order, each before the keys found in that base; otherwise the
// lines of a run of bases would overwrite one another, so the run's overlay is printed once -- what
// they leave on the terminal (the last line, completed by any longer earlier line).
struct base_lines {
  const bool on = opt.matrix || !opt.quiet;
  const char *sp = opt.bsgs_mode == BM_RANDOM ? "  " : opt.matrix ? " " : "   ";
  std::string overlay;  // the pending in-place lines, rendered
  void add(const U &base) {
    if (!on) return;
    const std::string ln = "[+] Thread 0x" + u_hex(base) + sp;
    if (opt.matrix) {
      printf("%s\n", ln.c_str());
      return;
    }
    if (ln.size() >= overlay.size())
      overlay = ln;
    else
      overlay.replace(0, ln.size(), ln);
  }
  void flush() {
    if (!overlay.empty()) printf("\r%s\r", overlay.c_str());
    overlay.clear();
    fflush(stdout);
  }
};

// The bases of one call, in the order the reference's worker takes them: `count` bases from `start`
// `step` apart, or an explicit list.  Each found key is reported after the progress line of the
// first base whose window (base, base + 2M * cycles * 1024] holds it -- the base a single reference
// thread finds it in.  Exits (status 1) when every target is found.
void report_call(kh_ctx *ctx, const bsgs_job *j, const kh_bsgs_info &info, const U &start, const U &step,
                 uint64_t count, const std::vector<U> *list, const std::vector<kh_bsgs_found> &found, uint32_t nf) {
  const uint64_t W = 2 * info.m * info.cycles * 1024;
  auto base_at = [&](uint64_t i) { return list ? (*list)[i] : u_add(start, u_mul_u64(step, i)); };
  std::vector<std::pair<uint64_t, uint32_t>> at;  // (base position, found index)
  for (uint32_t f = 0; f < nf && f < found.size(); f++) {
    const U key = u_from_be32(found[f].key);
    const uint64_t none = ~0ULL;
    uint64_t pos = none;
    if (list) {
      for (uint64_t i = 0; i < count; i++) {
        const U b = (*list)[i];
        if (u_cmp(key, b) > 0 && u_cmp(u_sub(key, b), u_from_u64(W)) <= 0) {
          pos = i;
          break;
        }
      }
    } else if (u_cmp(key, start) > 0 && step.v[1] == 0 && step.v[2] == 0 && step.v[3] == 0 && step.v[4] == 0 &&
               step.v[0]) {
      const U rel = u_sub(key, start);  // smallest b with rel <= b * step + W
      if (u_cmp(rel, u_from_u64(W)) > 0) {
        uint64_t rem = 0;
        const U q = u_divmod_u64(u_sub(rel, u_from_u64(W)), step.v[0], &rem);
        if (u_bitlen(q) < 63 && q.v[0] + (rem ? 1 : 0) < count) pos = q.v[0] + (rem ? 1 : 0);
      } else {
        pos = 0;
      }
    }
    if (pos == none) {
      // no base of the call holds the key in its window (base, base + W]: the engine found a key the
      // reference's per-base windows do not cover; it is printed after the call's last base line
      fprintf(stderr, "[W] key %s lies outside every base window of its call; printed after the call's last base\n",
              u_hex(key).c_str());
      pos = count ? count - 1 : 0;
    }
    at.push_back({pos, f});
  }
  std::sort(at.begin(), at.end());
  base_lines bl;
  uint64_t next = 0;
  for (auto &p : at) {
    if (bl.on) {
      for (; next <= p.first && next < count; next++) bl.add(base_at(next));
      bl.flush();
    }
    if (print_found(ctx, j, found[p.second])) {
      printf("All points were found\n");
      fflush(stdout);
      _exit(EXIT_FAILURE);  // keyhunt.cpp:4811-4814
    }
  }
  if (bl.on) {
    for (; next < count; next++) bl.add(base_at(next));
    bl.flush();
  }
}

void bsgs_worker(bsgs_job *j) {
  kh_ctx *ctx = nullptr;
  int r = kh_open(j->device, &ctx);
  if (r) {
    j->rc = r;
    if (j->first) setup_done();
    g_running--;
    return;
  }
  kh_bsgs_info info;
  r = kh_bsgs_set_layer1(ctx, opt.layer1);
  if (!r) r = kh_bsgs_set_bloom_multiplier(ctx, (uint32_t)opt.bloom_mult);
  if (!r) r = kh_bsgs_setup(ctx, j->n, j->k, &info);
  if (!r) r = bsgs_tables(ctx, info, j->first);
  if (!r) r = bsgs_ptable(ctx, info, j->first);
  // the first worker has printed the setup lines (or failed): the others' base lines follow them
  if (j->first)
    setup_done();
  else
    setup_wait();
  size_t nt = j->tx->size();
  std::vector<uint8_t> xy(64 * nt);
  for (size_t i = 0; i < nt; i++) {
    fe_to_be(&xy[64 * i], (*j->tx)[i]);
    fe_to_be(&xy[64 * i + 32], (*j->ty)[i]);
  }
  if (!r) r = kh_bsgs_set_targets(ctx, xy.data(), (uint32_t)nt);
  const U twoN = u_mul_u64(u_from_u64(info.n), 2);
  std::vector<kh_bsgs_found> found(nt + 1);
  std::vector<uint8_t> list_be;
  const bool progression = opt.bsgs_mode == BM_SEQUENTIAL || opt.bsgs_mode == BM_ANGRYGIANT || opt.bsgs_mode == BM_GGSB;
  // listed schedules (backward, both, random, dance): the next call's bases are drawn and packed on a
  // helper thread while the GPU walks the current call's (drawing, checking and packing 2^20 bases
  // took ~1/4 of a call's time on the host between calls)
  list_batch cur, nxt;
  if (!progression && !r) prepare_batch(twoN, j->list_bases_per_call, cur);
  while (!r) {
    if (!progression) {
      if (!cur.ok) break;
      std::thread pre([&]() { prepare_batch(twoN, j->list_bases_per_call, nxt); });
      const uint64_t nb = cur.drawn.size();
      uint32_t nf = 0;
      if (cur.consecutive)
        r = kh_bsgs_scan(ctx, cur.st_be, nb, found.data(), (uint32_t)found.size(), &nf);
      else
        r = kh_bsgs_scan_list(ctx, cur.be.data(), nb, found.data(), (uint32_t)found.size(), &nf);
      pre.join();
      if (r) {
        fprintf(stderr, "[E] kh_bsgs_scan: %s (%s)\n", kh_strerror(r), kh_last_error(ctx));
        break;
      }
      g_bases_done += nb;
      report_call(ctx, j, info, U{}, g_step, nb, &cur.drawn, found, nf);
      std::swap(cur, nxt);
      continue;
    }
    {
      U st;
      uint64_t nb = 0;
      if (!take_progression(g_step, u_cmp(g_step, twoN) == 0 ? j->bases_per_call : j->list_bases_per_call, st, nb))
        break;
      uint8_t st_be[32];
      u_to_be32(st, st_be);
      uint32_t nf = 0;
      if (u_cmp(g_step, twoN) == 0) {
        r = kh_bsgs_scan(ctx, st_be, nb, found.data(), (uint32_t)found.size(), &nf);
      } else {  // ggsb: bases 2 x block size apart, each walking its own 2N keys
        list_be.resize(32 * nb);
        U b = st;
        for (uint64_t i = 0; i < nb; i++, b = u_add(b, g_step)) u_to_be32(b, &list_be[32 * i]);
        r = kh_bsgs_scan_list(ctx, list_be.data(), nb, found.data(), (uint32_t)found.size(), &nf);
      }
      if (r) {
        fprintf(stderr, "[E] kh_bsgs_scan: %s (%s)\n", kh_strerror(r), kh_last_error(ctx));
        break;
      }
      g_bases_done += nb;
      report_call(ctx, j, info, st, g_step, nb, nullptr, found, nf);
    }
  }
  j->rc = r;
  kh_close(ctx);
  g_running--;
}

void usage(const char *p) {
  printf("Usage: %s -m address|rmd160|xpoint|bsgs -f FILE [-b BITS | -r START:END] [-l compress|uncompress|both]\n"
         "       [-n N] [-k K] [-I STRIDE] [-g GPUS] [-q] [-s SECONDS] [-M] [-L blocked|reference]\n"
         "       [-e] [-c btc|eth] [-R] [-B sequential|backward|both|random|dance|angrygiant] [-S] [-6]\n"
         "       [-z MULT] [-m vanity -v PREFIX ...] [--rmd-batch-size N] [-d] [-h]\n", p);
}

}  // namespace

int main(int argc, char **argv) {
  printf("[+] Version %s\n", VERSION);
  const char *mode_names[] = {"address", "rmd160", "xpoint", "bsgs", "vanity"};
  int c;
  U order;
  u_from_hex(ORDER_HEX, order);
  static const struct option long_opts[] = {{"bsgs-block-count", required_argument, 0, 1},
                                           {"bsgs-block-size", required_argument, 0, 2},
                                           {"ptable", required_argument, 0, 3},
                                           {"ptable-size", required_argument, 0, 4},
                                           {"load-ptable", no_argument, 0, 5},
                                           {"ptable-cache", no_argument, 0, 6},
                                           {"mapped", optional_argument, 0, 7},
                                           {"mapped-size", required_argument, 0, 8},
                                           {"mapped-chunks", required_argument, 0, 9},
                                           {"bloom-file", required_argument, 0, 10},
                                           {"load-bloom", no_argument, 0, 11},
                                           {"bloom-bytes", required_argument, 0, 12},
                                           {"create-mapped", optional_argument, 0, 13},
                                           {"tmpdir", required_argument, 0, 14},
                                           {"rmd-batch-size", required_argument, 0, 15},
                                           {0, 0, 0, 0}};
  // --mapped-size / --bloom-bytes / --create-mapped N: the entry count and error the byte budget
  // allows (bloom_entries_for_bytes, keyhunt.cpp:7510-7530)
  auto size_override = [](uint64_t bytes) {
    uint64_t n;
    uint32_t k;
    mapped::entries_for(bytes, &n, &k);
    opt.mapped_entries = n;
    opt.mapped_error = powl(0.5L, (long double)k);
  };
  while ((c = getopt_long(argc, argv, "m:f:l:r:b:k:n:t:g:qs:I:L:MRec:B:S6v:z:dh", long_opts, nullptr)) != -1) {
    switch (c) {
      case 1:  // keyhunt.cpp:809-811: implies GGSB
        opt.ggsb_count = strtoull(optarg, NULL, 10);
        opt.ggsb = opt.ggsb_count > 0;
        break;
      case 2:  // keyhunt.cpp:812-814
        opt.ggsb_size = strtoull(optarg, NULL, 10);
        opt.ggsb = opt.ggsb_size > 0;
        break;
      case 3: opt.ptable = optarg; break;  // keyhunt.cpp:772-773
      case 4: {                            // keyhunt.cpp:774-785
        char *end;
        uint64_t v = strtoull(optarg, &end, 10);
        if (*end) {
          switch (tolower(*end)) {
            case 'k': v *= 1024ull; break;
            case 'm': v *= 1024ull * 1024ull; break;
            case 'g': v *= 1024ull * 1024ull * 1024ull; break;
            case 't': v *= 1024ull * 1024ull * 1024ull * 1024ull; break;
          }
        }
        opt.ptable_size = v;
        break;
      }
      case 5: opt.load_ptable = true; break;  // keyhunt.cpp:786-787
      case 6: opt.ptable_cache = true; break;  // keyhunt.cpp:788-789
      case 7:                                  // keyhunt.cpp:744-748
        opt.mapped = true;
        if (optarg) opt.mapped_name = optarg;
        break;
      case 8: {  // keyhunt.cpp:749-765, with the k/m/g/t suffixes
        opt.mapped = true;
        char *end;
        uint64_t v = strtoull(optarg, &end, 10);
        if (*end) {
          switch (tolower(*end)) {
            case 'k': v *= 1024ull; break;
            case 'm': v *= 1024ull * 1024ull; break;
            case 'g': v *= 1024ull * 1024ull * 1024ull; break;
            case 't': v *= 1024ull * 1024ull * 1024ull * 1024ull; break;
          }
        }
        size_override(v);
        break;
      }
      case 9:  // keyhunt.cpp:766-768
        opt.mapped = true;
        opt.mapped_chunks = (uint32_t)strtoul(optarg, NULL, 10);
        break;
      case 10: opt.mapped_name = optarg; break;  // keyhunt.cpp:768-769 (does not set --mapped)
      case 11: opt.load_bloom = true; break;     // keyhunt.cpp:770-771
      case 12:                                   // keyhunt.cpp:790-796
        opt.mapped = true;
        size_override(strtoull(optarg, NULL, 10));
        break;
      case 13:  // keyhunt.cpp:797-806
        opt.mapped = true;
        opt.create_mapped = true;
        if (optarg) size_override(strtoull(optarg, NULL, 10));
        break;
      case 14: break;  // --tmpdir: where the reference puts an unnamed bP table mapping; unused here
      case 15: {       // keyhunt.cpp:815-829: clamped to [4, 1024], rounded down to a multiple of 4
        long v = strtol(optarg, NULL, 10);
        if (v < 4) v = 4;
        if (v > 1024) v = 1024;
        if (v % 4) {
          v -= v % 4;
          if (v < 4) v = 4;
        }
        opt.rmd_batch = (int)v;
        break;
      }
      case 'm': {
        int m = -1;
        for (int i = 0; i < 5; i++)
          if (!strcmp(optarg, mode_names[i])) m = i;
        if (m < 0) {
          fprintf(stderr, "[E] Unsupported mode %s (engine covers address, rmd160, xpoint, bsgs, vanity)\n", optarg);
          return EXIT_FAILURE;
        }
        opt.mode = m;
        if (m != MODE_BSGS) printf("[+] Mode %s\n", optarg);  // BSGS: "[+] Mode BSGS <schedule>" later
        break;
      }
      case 'f': opt.file = optarg; break;
      case 'v':  // keyhunt.cpp:1083-1100
        if (is_base58(optarg)) {
          if (addvanity(optarg, opt.vanity) > 0)
            printf("[+] Added Vanity search : %s\n", optarg);
          else
            printf("[+] Vanity search \"%s\" was NOT Added\n", optarg);
        } else {
          fprintf(stderr, "[+] The string \"%s\" is not Valid Base58\n", optarg);
        }
        break;
      case 'l':
        // keyhunt.cpp:945-960
        if (!strcmp(optarg, "compress")) { opt.search = KH_SEARCH_COMPRESS; printf("[+] Search compress only\n"); }
        else if (!strcmp(optarg, "uncompress")) { opt.search = KH_SEARCH_UNCOMPRESS; printf("[+] Search uncompress only\n"); }
        else if (!strcmp(optarg, "both")) { opt.search = KH_SEARCH_BOTH; printf("[+] Search both compress and uncompress\n"); }
        else { fprintf(stderr, "[E] Unknow search type %s\n", optarg); return EXIT_FAILURE; }
        break;
      case 'r': {  // keyhunt.cpp:1024-1055: START[:END]; START alone runs to the group order
        std::string s(optarg);
        size_t p = s.find(':');
        const std::string a = s.substr(0, p), b = p == std::string::npos ? std::string(ORDER_HEX) : s.substr(p + 1);
        if (!u_from_hex(a.c_str(), opt.start)) {
          fprintf(stderr, p == std::string::npos ? "[E] Invalid hexstring : %s.\n" : "[E] Invalid hexstring : %s\n",
                  a.c_str());
        } else if (!u_from_hex(b.c_str(), opt.end)) {
          fprintf(stderr, "[E] Invalid hexstring : %s\n", b.c_str());
        } else {
          opt.have_range = true;
          opt.range_start_str = a;
          opt.range_end_str = p == std::string::npos ? std::string() : b;  // empty: the order
        }
        break;
      }
      case 'b':
        opt.bits = atoi(optarg);
        if (opt.bits > 0 && opt.bits <= 256) {
          opt.have_bits = true;
        } else {
          fprintf(stderr, "[E] invalid bits param: %s.\n", optarg);
        }
        break;
      case 'k': opt.kfactor = strtoull(optarg, nullptr, 10); if (!opt.kfactor) opt.kfactor = 1; printf("[+] K factor %llu\n", (unsigned long long)opt.kfactor); break;
      case 'n': opt.flag_n = true; opt.str_n = optarg; break;
      case 't': {  // host threads: one per GPU context here (see -g); echoed as keyhunt.cpp:1076-1082 does
        long t = strtol(optarg, NULL, 10);
        if (t <= 0) t = 1;
        printf(t > 1 ? "[+] Threads : %u\n" : "[+] Thread : %u\n", (unsigned)t);
        break;
      }
      case 'g': opt.gpus = atoi(optarg); break;
      case 'q': opt.quiet = true; printf("[+] Quiet thread output\n"); break;
      case 's':  // keyhunt.cpp:1059-1072
        opt.seconds = atoi(optarg);
        if (opt.seconds < 0) opt.seconds = 30;
        if (opt.seconds == 0)
          printf("[+] Turn off stats output\n");
        else
          printf("[+] Stats output every %d seconds\n", opt.seconds);
        break;
      case 'I': {
        U s;
        bool ok = (optarg[0] == '0' && optarg[1] == 'x') ? u_from_hex(optarg, s) : u_from_dec(optarg, s);
        if (!ok || u_is_zero(s)) { fprintf(stderr, "[E] invalid stride %s\n", optarg); return EXIT_FAILURE; }
        opt.stride = s;
        opt.stride_set = true;
        break;
      }
      case 'M': opt.matrix = true; printf("[+] Matrix screen\n"); break;  // keyhunt.cpp:960-963
      case 'L':  // BSGS layer-1 layout on the GPU (engine option; the reference has one layout)
        if (!strcmp(optarg, "reference")) opt.layer1 = KH_LAYER1_REFERENCE;
        else if (!strcmp(optarg, "blocked")) opt.layer1 = KH_LAYER1_BLOCKED;
        else { fprintf(stderr, "[E] -L reference|blocked\n"); return EXIT_FAILURE; }
        break;
      case 'R':  // keyhunt.cpp:1019-1023
        printf("[+] Random mode\n");
        opt.random = true;
        opt.bsgs_mode = BM_RANDOM;
        break;
      case 'B': {  // keyhunt.cpp:841-853
        int idx = -1;
        for (int i = 0; i < 7; i++)
          if (!strcmp(optarg, BSGS_MODES[i])) idx = i;
        if (idx < 0) {
          fprintf(stderr, "[W] Ignoring unknow bsgs mode %s\n", optarg);
        } else {
          opt.bsgs_mode = idx;  // GGSB reuses the sequential worker (keyhunt.cpp:2764-2767)
          if (idx == BM_GGSB) opt.ggsb = true;
        }
        break;
      }
      case 'e':  // keyhunt.cpp:925-931
        opt.endo = true;
        printf("[+] Endomorphism enabled\n");
        break;
      case 'S': opt.save_read = true; break;  // keyhunt.cpp:1073-1075
      case '6':  // keyhunt.cpp:837-840
        opt.skip_checksum = true;
        fprintf(stderr, "[W] Skipping checksums on files\n");
        break;
      case 'c':  // keyhunt.cpp:874-891
        opt.crypto_given = true;
        if (!strcmp(optarg, "btc")) {
          opt.eth = false;
        } else if (!strcmp(optarg, "eth")) {
          opt.eth = true;
          printf("[+] Setting search for ETH adddress.\n");
        } else {
          fprintf(stderr, "[E] Unknow crypto value %s\n", optarg);
          return EXIT_FAILURE;
        }
        break;
      case 'z':  // keyhunt.cpp:1112-1118: bloom entries = multiplier x items above 10000 (7608)
        opt.bloom_mult = (int)strtol(optarg, NULL, 10);
        if (opt.bloom_mult <= 0) opt.bloom_mult = 1;
        printf("[+] Bloom Size Multiplier %i\n", opt.bloom_mult);
        break;
      case 'd':  // keyhunt.cpp:1019-1022
        printf("[+] Flag DEBUG enabled\n");
        break;
      case 'h':
        usage(argv[0]);
        return EXIT_SUCCESS;
      default: usage(argv[0]); return EXIT_FAILURE;
    }
  }
  if (opt.load_ptable && !opt.ptable) {  // keyhunt.cpp:1126-1129
    fprintf(stderr, "--load-ptable requires --ptable <file>\n");
    return EXIT_FAILURE;
  }
  mapped::cfg.name = opt.mapped_name;
  mapped::cfg.chunks = opt.mapped_chunks;
  mapped::cfg.load_bloom = opt.load_bloom;
  mapped::cfg.entries = opt.mapped_entries;
  mapped::cfg.error = opt.mapped_error;
  mapped::cfg.bloom_mult = opt.bloom_mult;
  if (opt.create_mapped) return mapped::create();  // keyhunt.cpp:1131-1172: make the file(s) and exit
  if (!opt.file && !(opt.mode == MODE_VANITY && opt.vanity.targets)) {
    fprintf(stderr, "[E] -f FILE is required\n");
    return EXIT_FAILURE;
  }
  // validate_nk (keyhunt.cpp:1173-1183): applied to every mode
  uint64_t nk_n = 0x100000000000ULL;
  if (opt.flag_n) nk_n = (opt.str_n[0] == '0' && (opt.str_n[1] == 'x' || opt.str_n[1] == 'X')) ? strtoull(opt.str_n + 2, nullptr, 16) : strtoull(opt.str_n, nullptr, 10);
  if (!validate_nk(nk_n, opt.kfactor)) return EXIT_FAILURE;
  // keyhunt.cpp:1185-1193 compares the -B index with MODE_BSGS (2), i.e. these two guards fire
  // for -B both whatever -m is (SURVEY 8a parity note 7); BSGS itself ignores -e and -I
  if (opt.bsgs_mode == BM_BOTH && opt.endo) {
    fprintf(stderr, "[E] Endomorphism doesn't work with BSGS\n");
    return EXIT_FAILURE;
  }
  if (opt.bsgs_mode == BM_BOTH && opt.stride_set) {
    fprintf(stderr, "[E] Stride doesn't work with BSGS\n");
    return EXIT_FAILURE;
  }
  if (opt.stride_set) printf("[+] Stride : %s\n", u_dec(opt.stride).c_str());  // keyhunt.cpp:1195-1203
  if (opt.mode == MODE_BSGS) printf("[+] Mode BSGS %s\n", BSGS_MODES[opt.bsgs_mode]);  // keyhunt.cpp:1209-1211
  if (opt.mode == MODE_ADDRESS && !opt.crypto_given) printf("[+] Setting search for btc adddress\n");  // 1217-1220
  // ranges (keyhunt.cpp:854-873, 1221-1269)
  if (opt.have_bits) {
    opt.start = u_shl1(opt.bits - 1);
    opt.end = u_shl1(opt.bits);
    if (u_cmp(opt.end, order) > 0) opt.end = order;
  } else if (opt.have_range) {
    if (u_is_zero(opt.start)) opt.start = u_from_u64(1);
    if (u_cmp(opt.start, opt.end) == 0) {
      fprintf(stderr, "[E] Start and End range can't be the same\nFallback to random mode!\n");
      opt.have_range = false;
    } else if (u_cmp(opt.start, order) >= 0 || u_cmp(opt.end, order) > 0) {
      fprintf(stderr, "[E] Start and End range can't be great than N\nFallback to random mode!\n");
      opt.have_range = false;
    } else {
      if (u_cmp(opt.start, opt.end) > 0) {
        fprintf(stderr, "[W] Opps, start range can't be great than end range. Swapping them\n");
        std::swap(opt.start, opt.end);
      }
    }
  }
  if (!opt.have_bits && !opt.have_range) {
    // no usable range (keyhunt.cpp:1250-1255, 1534-1540): the address family walks sequentially
    // from 1 to the group order; BSGS starts at a random key below the order and walks up
    opt.start = opt.mode == MODE_BSGS ? u_rand_range(u_from_u64(1), order) : u_from_u64(1);
    opt.end = order;
  }
  // the range lines: the address family prints them after "[+] N =" with the range as used
  // (keyhunt.cpp:1325-1339); BSGS after reading its targets, with -r's strings as typed and nothing
  // for a random start (1517-1540)
  auto print_range = [&]() {
    if (opt.mode == MODE_BSGS && !opt.have_bits && !opt.have_range) return;
    printf(opt.have_bits ? "[+] Bit Range %d\n" : "[+] Range \n", opt.bits);
    if (opt.mode == MODE_BSGS && !opt.have_bits)
      printf("[+] -- from : 0x%s\n[+] -- to   : 0x%s\n", opt.range_start_str.c_str(),
             opt.range_end_str.empty() ? u_hex(order).c_str() : opt.range_end_str.c_str());
    else
      printf("[+] -- from : 0x%s\n[+] -- to   : 0x%s\n", u_hex(opt.start).c_str(), u_hex(opt.end).c_str());
  };
  // -g contexts: one host thread + kh_ctx each, on device d % ndev.  More contexts than devices
  // share a device (as the reference's -t threads share the host's cores); each keeps its own
  // tables and lanes, and they all take work from the one cursor (keyhunt.cpp:3321-3324, 4600-4617).
  // The devices are counted once the targets are read, so the reference's lines come first.
  int ndev = 0, gpus = 0;
  std::vector<addr_job> aj;
  std::vector<bsgs_job> bj;
  auto open_devices = [&]() {
    kh_device_count(&ndev);
    if (ndev < 1) {
      fprintf(stderr, "[E] no GPU found\n");
      return false;
    }
    gpus = opt.gpus > 0 ? opt.gpus : ndev;
    printf("[+] GPUs : %d (%d context%s)\n", std::min(gpus, ndev), gpus, gpus == 1 ? "" : "s");
    aj.resize(gpus);
    bj.resize(gpus);
    return true;
  };
  g_cursor = opt.start;
  g_end = opt.end;
  g_top = opt.end;
  U twoN;
  std::vector<std::thread> th;
  std::vector<uint8_t> rows;
  std::string data_file;  // -S target cache (outlives the GPU threads)
  std::vector<fe> tx, ty;
  std::vector<bool> comp;

  if (opt.mode != MODE_BSGS) {
    uint64_t nseq = 0x100000000ULL;  // N_SEQUENTIAL_MAX (keyhunt.cpp:464, 1272-1292)
    if (opt.flag_n) {
      nseq = nk_n;
      if (nseq < 1024 || nseq % 1024) nseq = 0x100000000ULL;
    }
    printf("[+] N = %p\n", (void *)nseq);
    print_range();
    uint64_t items = 0;
    // -S: read the target cache if it exists (FLAGREADEDFILE1), else read the file and write it
    bool have_data = false;
    if (opt.save_read && opt.mode != MODE_VANITY) {
      if (!data_file_name(opt.file, data_file)) {
        fprintf(stderr, "[E] sha256_file error\n");
        return EXIT_FAILURE;
      }
      FILE *df = fopen(data_file.c_str(), "rb");
      if (df) {
        fseeko(df, 0, SEEK_END);
        const off_t size = ftello(df);
        fclose(df);
        have_data = true;
        printf("[+] Reading file %s\n", data_file.c_str());
        // a file too short for the bloom checksum or its struct bloom fails the reference's first two
        // reads (readFileAddress, keyhunt.cpp:7068, 7076; the caller's message at 1347): e.g. the empty
        // data file an -S --mapped-chunks N>1 run leaves behind (below)
        if (size < 32 + 112) {  // checksum + struct bloom (112 B, kh_mapped.h struct_bloom)
          fprintf(stderr, "[E] %s reading file, code line %d\n", size < 32 ? "Errore" : "Error", size < 32 ? 7068 : 7076);
          fprintf(stderr, "[E] Unenexpected error\n");
          return EXIT_FAILURE;
        }
      }
    }
    // -S with --mapped and no cache yet: the target filter is the mapped file's (bloom.dat, or the
    // --mapped / --bloom-file name), and that filter -- its struct bloom and bits -- goes into the
    // data file (keyhunt.cpp:7033-7049, 7630-7706, 7756-7855).  With --mapped-chunks above 1 the
    // reference writes bloom.bytes from its FIRST chunk's mapping (bloom.bf = bf_chunks[0],
    // bloom.cpp:395), past that mapping's end (handled below)
    const bool mapped_data = opt.mapped && opt.save_read && opt.mode != MODE_VANITY && !have_data;
    const bool mapped_data_chunked = mapped_data && opt.mapped_chunks > 1;
    mapped::filter tf;
    std::vector<uint8_t> adds;  // the items the reference adds to its (mapped) target bloom
    std::vector<uint8_t> *addp = opt.mapped ? &adds : nullptr;
    if (have_data) {
      // rows and bloom come from the file, in each GPU's kh_targets_load
    } else if (opt.mode == MODE_VANITY) {
      if (!read_vanity(opt.file)) return EXIT_FAILURE;
    } else if (opt.eth && opt.mode == MODE_ADDRESS) {
      if (!read_targets_eth(opt.file, rows, items, addp)) return EXIT_FAILURE;
    } else if (!read_targets(opt.file, opt.mode, rows, items, addp)) {
      return EXIT_FAILURE;
    }
    if (opt.mapped) {
      bool ok;
      if (opt.mode == MODE_VANITY) {  // the vanity bloom: the first min_bytes bytes of every A
        const uint32_t L = (uint32_t)opt.vanity.min_bytes;
        for (size_t j = 0; j < opt.vanity.ranges.size(); j += 40)
          adds.insert(adds.end(), opt.vanity.ranges.begin() + j, opt.vanity.ranges.begin() + j + L);
        ok = mapped::targets(opt.vanity.total, adds, L);
      } else {
        ok = mapped::targets(items, adds, 20, mapped_data && !mapped_data_chunked ? &tf : nullptr);
      }
      if (!ok) return EXIT_FAILURE;
    }
    if (mapped_data_chunked) {
      // The reference maps and fills the chunk files, opens data_<hex>.dat for writing, then hashes
      // bloom.bytes from the first chunk's mapping and dies of SIGBUS past its end (writeFileIfNeeded,
      // keyhunt.cpp:7770-7809): the chunk files hold the filter, the data file is left empty, and the next
      // -S run fails reading it (tests/golden/ref_mapped.json "rmd160_S_mapped_chunks").  This CLI leaves
      // the same files and exits with an error status instead of the signal.
      FILE *f = fopen(data_file.c_str(), "wb");
      if (f) fclose(f);
      fflush(stdout);
      fprintf(stderr, "[E] -S with --mapped-chunks %u: the data file would be written from the first chunk's mapping "
                      "past its end (the reference dies of SIGBUS there); %s left empty\n",
              (unsigned)opt.mapped_chunks, data_file.c_str());
      return EXIT_FAILURE;
    }
    if (!have_data)
      printf("[+] Sorting data ... done! %llu values were loaded and sorted\n", (unsigned long long)(rows.size() / 20));
    if (mapped_data) {
      printf("[D] size data %llu\n", (unsigned long long)rows.size());
      if (!write_mapped_data_file(data_file, tf, rows)) {
        fprintf(stderr, "[E] Error writing file %s\n", data_file.c_str());
        return EXIT_FAILURE;
      }
      printf("[+] Writing file %s ........\n", data_file.c_str());
      data_file.clear();  // the contexts take their targets from the rows
    }
    if (!open_devices()) return EXIT_FAILURE;
    {
      // contexts stacked on one device must fit its free memory (each holds its own inversion pad,
      // kh_scan_memory): checked before any is opened, as bsgsd-amd checks its BSGS tables
      const uint32_t smode = opt.mode == MODE_XPOINT ? KH_MODE_XPOINT
                             : (opt.eth && (opt.mode == MODE_ADDRESS || opt.mode == MODE_RMD160)) ? KH_MODE_ETH
                                                                                                   : KH_MODE_ADDRESS;
      uint64_t need = 0;
      if (kh_scan_memory(nseq, smode | (opt.endo ? KH_MODE_ENDO : 0), (uint32_t)opt.search, &need) == KH_OK) {
        for (int dev = 0; dev < ndev && dev < gpus; dev++) {
          const uint64_t per = (uint64_t)(gpus / ndev + (dev < gpus % ndev ? 1 : 0));
          uint64_t fr = 0, tot = 0;
          if (kh_device_memory(dev, &fr, &tot) == KH_OK && fr && per * need > fr) {
            fprintf(stderr, "[E] -g %d: %llu context(s) on GPU %d need %.1f GB of device memory (%.1f GB each), "
                            "%.1f GB are free; use fewer contexts (-g) or a smaller -n\n",
                    gpus, (unsigned long long)per, dev, per * need / 1e9, need / 1e9, fr / 1e9);
            return EXIT_FAILURE;
          }
        }
      }
    }
    g_running = gpus;
    for (int d = 0; d < gpus; d++) {
      aj[d].device = d % ndev;
      aj[d].index = d;
      aj[d].rows = &rows;
      // initBloomFilter (keyhunt.cpp:7608): max(10000, items), times -z above the floor
      const uint64_t nitems = items ? items : rows.size() / 20;
      aj[d].bloom_items = nitems <= 10000 ? nitems : nitems * (uint64_t)opt.bloom_mult;
      aj[d].nseq = nseq;
      if (!data_file.empty()) {
        aj[d].data_file = data_file.c_str();
        aj[d].save_data = !have_data && d == 0;  // one GPU writes the cache
      }
      th.emplace_back(addr_worker, &aj[d]);
    }
  } else {
    FILE *f = fopen(opt.file, "r");
    if (!f) {
      fprintf(stderr, "[E] Can't open file %s\n", opt.file);
      return EXIT_FAILURE;
    }
    printf("[+] Opening file %s\n", opt.file);
    // keyhunt.cpp:1369-1446: N = lines of 66+ characters; each such line's first token (separators
    // " \t:") is a public key of 66 or 130 characters (ParsePublicKeyHex), else "Invalid length"
    std::vector<std::string> lines = fgets_pieces(f, 1022);
    fclose(f);
    size_t counted = 0;
    for (auto &ln : lines) counted += ln.size() >= 66;
    if (!counted) {
      fprintf(stderr, "[E] There is no valid data in the file\n");
      return EXIT_FAILURE;
    }
    for (auto &ln : lines) {
      if (ln.size() < 66) continue;
      std::vector<char> buf(ln.begin(), ln.end());
      buf.push_back(0);
      char *tok = strtok(buf.data(), " \t:");
      const size_t tl = tok ? strlen(tok) : 0;
      fe x, y;
      bool cp = false;
      if (tl == 66 || tl == 130) {
        const int r = parse_pubkey_hex_ref(tok, x, y, cp);
        if (r < 0) return 255;  // the reference's exit(-1)
        if (r > 0) {
          tx.push_back(x);
          ty.push_back(y);
          comp.push_back(cp);
        }
      } else {
        printf("Invalid length: %s\n", tok ? tok : "");
      }
    }
    if (tx.empty()) {
      fprintf(stderr, "[E] The file don't have any valid publickeys\n");
      return EXIT_FAILURE;
    }
    printf("[+] Added %zu points from file\n", tx.size());
    print_range();
    g_found.assign(tx.size(), 0);
    // BSGS N: -n or 2^44 (keyhunt.cpp:1454-1471); the library validates sqrt / 1024 and derives M
    uint64_t n = nk_n;
    U diff = u_sub(opt.end, opt.start);
    if (u_cmp(diff, u_from_u64(n)) < 0) {
      fprintf(stderr, "[E] the given range is small\n");
      return EXIT_FAILURE;
    }
    uint64_t m = 1;
    while ((m + 1) * (m + 1) <= n) m++;
    uint64_t M = m * opt.kfactor;
    uint64_t Nr = (n / M) * M;
    twoN = u_mul_u64(u_from_u64(Nr), 2);
    printf("[+] N = 0x%llx\n", (unsigned long long)Nr);
    // GGSB block geometry from sqrt(N) (keyhunt.cpp:1477-1499) and the base step (1617-1627)
    g_step = twoN;
    uint64_t ggsb_blocks = 1, ggsb_babies = M;
    if (opt.ggsb) {
      uint64_t bc = opt.ggsb_count, bs = opt.ggsb_size;
      if (bc == 0 && bs == 0) bc = 1;
      if (bc > 0 && bs == 0)
        bs = (m + bc - 1) / bc;
      else if (bs > 0 && bc == 0)
        bc = (m + bs - 1) / bs;
      if (bc == 0) bc = 1;
      if (bs == 0) bs = m;
      if (bc > 1 && bs) g_step = u_mul_u64(u_from_u64(bs), 2);
      ggsb_blocks = bc > 1 ? bc : 1;
      if (bs) ggsb_babies = bs;
    }
    {
      // keyhunt.cpp:1663-1685 (stderr): the build's layout and the expected layer / table sizes
      const uint64_t items = M / 256 > 10000 ? M / 256 + (M % 256 ? 1 : 0) : 1000;
      const long double err = opt.mapped && opt.mapped_error ? opt.mapped_error : 0.000001L;
      const double shard_mb = (double)mapped::bytes_for(items, err) / 1048576.0;
      fprintf(stderr, "[i] BSGS table build: %s layout, creating %llu block(s) of %llu babies each.\n",
              ggsb_blocks > 1 ? "GGSB" : "classic", (unsigned long long)ggsb_blocks, (unsigned long long)ggsb_babies);
      fprintf(stderr, "[i] Expected sizes: each bloom layer ~%.2f MB (256 shards), bPtable ~%.2f MB per block (%.2f MB total).\n",
              shard_mb * 256.0, (double)(ggsb_babies * 16) / 1048576.0, (double)(M * 16) / 1048576.0);
    }
    if (opt.mapped && opt.save_read && opt.mapped_chunks > 1) {
      // the reference writes each shard's bits from its first chunk's mapping, past that mapping's end
      fprintf(stderr, "[E] -S with --mapped-chunks above 1: the reference writes the table files from each shard's "
                      "first chunk mapping past its end; not provided\n");
      return EXIT_FAILURE;
    }
    if (!open_devices()) return EXIT_FAILURE;
    g_running = gpus;
    for (int d = 0; d < gpus; d++) {
      bj[d].device = d % ndev;
      bj[d].first = d == 0;
      bj[d].tx = &tx;
      bj[d].ty = &ty;
      bj[d].comp = &comp;
      bj[d].n = n;
      bj[d].k = opt.kfactor;
      // ~2^35 giant points per engine call (16 pipelined rounds, ~1 s): the end of a call drains
      // the pipeline (the last round's second check, the hit copies), which at 2^31 points per call
      // cost 7 % of the rate (profiles/r03f_cli_rate_bsgs.json); a call returns as soon as every
      // target is found.  Listed schedules take calls of the same size (at 2^31 points per call,
      // -B random ran 17 % and -B both 9 % below sequential: profiles/r05k_cli_rate_bsgs_*.json).
      // A range of fewer bases than that is dealt out evenly over the contexts (the reference's
      // threads take one base each, keyhunt.cpp:4600-4617)
      {
        uint64_t aux = Nr / M, pts = ((aux + 1023) / 1024) * 1024;
        bj[d].bases_per_call = std::max<uint64_t>(1, (1ULL << 35) / pts);
        bj[d].list_bases_per_call = bj[d].bases_per_call;
        const U span = u_sub(opt.end, opt.start);
        if (g_step.v[1] == 0 && g_step.v[2] == 0 && g_step.v[3] == 0 && g_step.v[4] == 0) {
          uint64_t rem = 0;
          U nb = u_divmod_u64(span, g_step.v[0], &rem);
          if (u_bitlen(nb) <= 40) {
            const uint64_t bases = nb.v[0] + (rem ? 1 : 0), share = (bases + gpus - 1) / gpus;
            bj[d].bases_per_call = std::max<uint64_t>(1, std::min(bj[d].bases_per_call, share));
            bj[d].list_bases_per_call = std::max<uint64_t>(1, std::min(bj[d].list_bases_per_call, share));
          }
        }
      }
      th.emplace_back(bsgs_worker, &bj[d]);
    }
  }
  // stats loop (keyhunt.cpp:2850-2962)
  uint64_t secs = 0;
  while (g_running > 0) {
    sleep(1);
    secs++;
    if (opt.seconds > 0 && secs % opt.seconds == 0) print_stats(secs, keys_done(twoN));
  }
  for (auto &t : th) t.join();
  int rc = 0;
  for (int d = 0; d < gpus; d++) rc |= (opt.mode == MODE_BSGS ? bj[d].rc : aj[d].rc);
  printf("\nEnd\n");
  return rc ? EXIT_FAILURE : EXIT_SUCCESS;
}
