// kh_mapped.h -- the reference's memory-mapped bloom files (--mapped, --mapped-size,
// --mapped-chunks, --bloom-file, --load-bloom, --bloom-bytes, --create-mapped; keyhunt.cpp:724-806,
// 1131-1172, 1631-1785, 7495-7530, 7630-7706; bsgsd.cpp:517-535, 584-660, 955-995, 1180-1255;
// bloom/bloom.cpp:491-747), shared by bin/keyhunt-amd and bin/bsgsd-amd.
//
// The engine keeps its own filters in HBM; these files are what the reference leaves on disk for
// the same options, written with the reference's geometry and bit layout (the bits set by the GPU
// through kh_bloom_add / kh_bsgs_layer_bits), and read back the way bloom_load_mmap reads them.
#ifndef KH_MAPPED_H
#define KH_MAPPED_H

#include <fcntl.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <string>
#include <vector>

#include "kh_gpu.h"

namespace mapped {

// the options of the host that uses the files (keyhunt-amd or bsgsd-amd)
struct config {
  const char *name = nullptr;  // --mapped NAME / --bloom-file NAME (mapped_filename)
  uint32_t chunks = 1;         // --mapped-chunks
  bool load_bloom = false;     // --load-bloom
  uint64_t entries = 0;        // mapped_entries_override
  long double error = 0;       // mapped_error_override
  int bloom_mult = 1;          // -z (FLAGBLOOMMULTIPLIER)
  bool bsgsd = false;          // bsgsd's initBloomFilterMapped (bsgsd.cpp:584-660): its messages,
                               // every shard reported, the non-mapped branch
};
inline config cfg;

// (uint64_t) of a long double as the reference's x86-64 build converts it: a value past 2^64 (or an
// infinite one) gives 0 -- bloom_init_mmap's bit count for an entry count that large, and the
// "0 bytes" bsgsd prints for it
inline uint64_t u64_of(long double v) {
  if (!(v >= 0) || v >= 18446744073709551616.0L) return 0;
  return (uint64_t)v;
}

// bloom_bytes_for_entries_error (keyhunt.cpp:7495-7507) == bytes_for_entries_error (bloom.cpp:454-464)
inline uint64_t bytes_for(uint64_t entries, long double error) {
  long double num = -logl(error);
  long double denom = 0.480453013918201L;
  long double bpe = num / denom;
  long double allbits = (long double)entries * bpe;
  uint64_t bits = u64_of(allbits);
  return bits / 8 + ((bits % 8) ? 1 : 0);
}
// bloom_init2's byte count (bloom/bloom.cpp:154-187): bpe kept as a double (struct bloom's field),
// bits = entries x bpe in long double; the size initBloomFilter's "Loading data" line reports
inline uint64_t init2_bytes(uint64_t entries) {
  long double num = -logl(0.000001L);
  long double denom = 0.480453013918201;
  const double bpe = (double)(num / denom);
  const uint64_t bits = u64_of((long double)entries * bpe);
  return bits / 8 + ((bits % 8) ? 1 : 0);
}
// the layer totals keyhunt prints after the 256 shards of a layer, computed in float
// (keyhunt.cpp:1719, 1750, 1781; bsgsd.cpp:1200, 1222, 1244)
inline double layer_mb(uint64_t total) { return (double)(float)((float)total / (float)1048576); }
// bloom_entries_for_bytes (keyhunt.cpp:7510-7530) == entries_hashes_for_bytes (bloom.cpp:465-489)
inline void entries_for(uint64_t bytes, uint64_t *entries, uint32_t *hashes) {
  uint64_t best_n = 0;
  uint32_t best_k = 0;
  for (uint32_t b = 20; b <= 64; b += 2) {
    const uint64_t n = 1ULL << (b == 64 ? 63 : b);
    const uint32_t k = 1U << ((b - 20) / 2);
    if (b == 64 || bytes_for(n, powl(0.5L, (long double)k)) > bytes) break;
    best_n = n;
    best_k = k;
  }
  if (best_n == 0) {
    best_n = 1ULL << 20;
    best_k = 1;
  }
  *entries = best_n;
  *hashes = (uint32_t)(uint8_t)best_k;
}
// bsgsd's bloom_entries_for_bytes (bsgsd.cpp:517-535) has no early exit: from bits = 50 on,
// 0.5^k underflows to 0, the need is -log(0) bits per entry, 0 bytes after the conversion, and so
// every size picks n = 2^62 (bits = 64 shifts 1 by 64: n = 1 on x86-64, no larger) with
// k = 2^21, i.e. an error override of 0.5^(2^21) = 0 -- which initBloomFilterMapped then reads
// as "no override" (1e-6).  The 2^62-entry filter cannot be mapped: every --mapped-size,
// --bloom-bytes or --create-mapped=N start of the reference daemon fails
inline void entries_for_bsgsd(uint64_t bytes, uint64_t *entries, long double *error) {
  uint64_t best_n = 0;
  uint32_t best_k = 0;
  for (uint32_t b = 20; b <= 64; b += 2) {
    const uint64_t n = b == 64 ? 1 : 1ULL << b;
    const uint32_t k = 1U << ((b - 20) / 2);
    if (bytes_for(n, powl(0.5L, (long double)k)) <= bytes && n > best_n) {
      best_n = n;
      best_k = k;
    }
  }
  if (best_n == 0) {
    best_n = 1000;
    best_k = 1;
  }
  *entries = best_n;
  *error = powl(0.5L, (long double)best_k);
}

struct filter {
  std::string name;                 // NAME, or the base of NAME.i
  uint32_t chunks = 1;
  uint64_t bits = 0, bytes = 0;
  uint32_t hashes = 0;
  uint64_t entries = 0;             // struct bloom's entries, error and bpe as the mapping left them
  long double error = 0;
  double bpe = 0;
  std::vector<uint64_t> chunk_bytes;  // size of each file
  std::vector<uint8_t> bf;          // flat bit array
  std::string file(uint32_t i) const { return chunks > 1 ? name + "." + std::to_string(i) : name; }
};
inline bool applied = false;  // initBloomFilterMapped's static mapped_override_applied
inline bool open_failed = false;  // bsgs_layers stopped at a shard it could not open (the reference exits 0)

inline bool exists(const std::string &f) {
  struct stat st;
  return stat(f.c_str(), &st) == 0;
}

// bloom_load_mmap (bloom.cpp:491-578): geometry from the files' total size
inline bool load(filter &F) {
  F.chunk_bytes.assign(F.chunks, 0);
  F.bf.clear();
  for (uint32_t i = 0; i < F.chunks; i++) {
    FILE *f = fopen(F.file(i).c_str(), "rb");
    if (!f) return false;
    std::vector<uint8_t> b;
    uint8_t buf[1 << 16];
    size_t n;
    while ((n = fread(buf, 1, sizeof buf, f)) > 0) b.insert(b.end(), buf, buf + n);
    fclose(f);
    F.chunk_bytes[i] = b.size();
    F.bf.insert(F.bf.end(), b.begin(), b.end());
  }
  F.bytes = F.bf.size();
  F.bits = F.bytes * 8;
  entries_for(F.bytes, &F.entries, &F.hashes);
  F.bpe = (double)F.bits / (double)F.entries;
  F.error = powl(0.5L, (long double)F.hashes);
  return true;
}

// bloom_init_mmap (bloom.cpp:589-700): geometry from entries and error (bpe kept as a double, the
// ln(2)^2 denominator a double literal); existing files are kept, resized only when `resize`
inline bool init(filter &F, uint64_t entries, long double error, bool resize) {
  if (entries < 1000 || error <= 0 || error >= 1) return false;
  long double num = -logl(error);
  long double denom = 0.480453013918201;
  const double bpe = (double)(num / denom);
  F.entries = entries;
  F.error = error;
  F.bpe = bpe;
  F.bits = u64_of((long double)entries * bpe);
  F.bytes = F.bits / 8 + ((F.bits % 8) ? 1 : 0);
  F.hashes = (uint32_t)(uint8_t)ceil(0.693147180559945 * bpe);
  const uint64_t cb = F.chunks > 1 ? F.bytes / F.chunks : F.bytes;
  F.chunk_bytes.assign(F.chunks, cb);
  F.chunk_bytes[F.chunks - 1] = F.bytes - cb * (F.chunks - 1);
  if (cb == 0) {
    // more chunks than bytes, or no bytes at all: the reference creates (or truncates) the first
    // chunk's file and fails to map its 0 bytes (bloom.cpp:647-711)
    const std::string fn = F.file(0);
    struct stat st;
    if (stat(fn.c_str(), &st) == 0 && st.st_size != 0 && !resize) {
      fprintf(stderr, "bloom_init_mmap: file '%s' size %lld does not match expected 0\n", fn.c_str(), (long long)st.st_size);
      return false;
    }
    int fd = open(fn.c_str(), O_RDWR | O_CREAT, 0644);
    if (fd >= 0) {
      if (ftruncate(fd, 0) != 0) fprintf(stderr, "bloom_init_mmap: ftruncate('%s', 0) failed\n", fn.c_str());
      close(fd);
    }
    fprintf(stderr, "bloom_init_mmap: mmap('%s', 0) failed: Invalid argument\n", fn.c_str());
    return false;
  }
  F.bf.assign(F.bytes, 0);
  uint64_t off = 0;
  for (uint32_t i = 0; i < F.chunks; i++) {
    const std::string fn = F.file(i);
    struct stat st;
    if (stat(fn.c_str(), &st) == 0) {
      if ((uint64_t)st.st_size != F.chunk_bytes[i] && !resize) {
        fprintf(stderr, "bloom_init_mmap: file '%s' size %lld does not match expected %llu\n", fn.c_str(),
                (long long)st.st_size, (unsigned long long)F.chunk_bytes[i]);
        return false;
      }
      FILE *f = fopen(fn.c_str(), "rb");  // the bytes it keeps (ftruncate never moves them)
      if (f) {
        size_t got = fread(F.bf.data() + off, 1, (size_t)std::min<uint64_t>(st.st_size, F.chunk_bytes[i]), f);
        (void)got;
        fclose(f);
      }
    }
    off += F.chunk_bytes[i];
  }
  return true;
}

inline bool save(const filter &F) {
  uint64_t off = 0;
  for (uint32_t i = 0; i < F.chunks; i++) {
    FILE *f = fopen(F.file(i).c_str(), "wb");
    bool ok = f && (F.chunk_bytes[i] == 0 || fwrite(F.bf.data() + off, F.chunk_bytes[i], 1, f) == 1);
    if (f) ok = fclose(f) == 0 && ok;
    if (!ok) {
      fprintf(stderr, "[E] Error writing the mapped bloom file %s\n", F.file(i).c_str());
      return false;
    }
    off += F.chunk_bytes[i];
  }
  return true;
}

// initBloomFilterMapped (keyhunt.cpp:7630-7706; bsgsd.cpp:584-656), FLAGMAPPED set: load or create
// the filter of `items` elements; fname names a BSGS shard file, else --mapped/--bloom-file or
// bloom.dat
inline bool open_filter(filter &F, uint64_t items, const char *fname) {
  F.name = fname ? fname : (cfg.name ? cfg.name : "bloom.dat");
  F.chunks = cfg.chunks ? cfg.chunks : 1;
  printf("[+] Bloom filter for %llu elements.\n", (unsigned long long)items);
  if (cfg.load_bloom) {
    struct stat st;
    if (cfg.bsgsd ? (stat(F.file(0).c_str(), &st) != 0 || st.st_size == 0) : !exists(F.file(0))) {
      fprintf(stderr, cfg.bsgsd ? "[E] --load-bloom specified but mapped bloom file '%s' does not exist or is empty\n"
                                : "[E] --load-bloom specified but mapped bloom file '%s' does not exist\n",
              F.file(0).c_str());
      return false;
    }
    if (!load(F)) {
      fprintf(stderr, "[E] bloom_load_mmap failed for '%s'\n", F.name.c_str());
      return false;
    }
    if (!F.bytes) {
      fprintf(stderr, "[E] Mapped bloom file '%s' has zero length; regenerate it or remove --load-bloom\n", F.name.c_str());
      return false;
    }
    return true;
  }
  if (!cfg.entries && exists(F.file(0))) {
    if (!load(F)) {
      fprintf(stderr, "[E] bloom_load_mmap failed for '%s'\n", F.name.c_str());
      return false;
    }
    if (!F.bytes) {
      fprintf(stderr, "[E] Existing mapped bloom file '%s' is empty; delete it or rerun without --load-bloom\n",
              F.name.c_str());
      return false;
    }
    return true;
  }
  uint64_t total;
  if (cfg.entries && (!applied || items >= cfg.entries)) {
    total = cfg.entries;
    applied = true;  // the override is applied once (to the first filter) by default
  } else {
    total = items <= 10000 ? 10000 : (uint64_t)cfg.bloom_mult * items;
  }
  const long double error = cfg.error ? cfg.error : 0.000001L;
  if (!init(F, total, error, cfg.entries != 0)) {
    fprintf(stderr, "[E] bloom_init_mmap failed for '%s' (%llu bytes for %llu elements).\n", F.name.c_str(),
            (unsigned long long)bytes_for(total, error), (unsigned long long)total);
    return false;
  }
  return true;
}

// --create-mapped (keyhunt.cpp:1131-1172): the zeroed file(s) of the override's size, then exit 0
inline int create() {
  if (!cfg.entries) {
    fprintf(stderr, "[E] --create-mapped requires size via argument or --bloom-bytes\n");
    return EXIT_FAILURE;
  }
  filter F;
  F.name = cfg.name ? cfg.name : "bloom.dat";
  F.chunks = cfg.chunks ? cfg.chunks : 1;
  const long double error = cfg.error ? cfg.error : 0.000001L;
  if (!init(F, cfg.entries, error, true)) {
    fprintf(stderr, "[E] bloom_init_mmap failed for '%s' (%llu bytes for %llu elements).\n", F.name.c_str(),
            (unsigned long long)bytes_for(cfg.entries, error), (unsigned long long)cfg.entries);
    return EXIT_FAILURE;
  }
  std::fill(F.bf.begin(), F.bf.end(), 0);
  return save(F) ? EXIT_SUCCESS : EXIT_FAILURE;
}

// struct bloom (bloom/bloom.h, 112 bytes on x86-64) of a mapped filter of ONE file as bloom_init_mmap /
// bloom_load_mmap leave it (bloom.cpp:491-578, 589-724): what writeFileIfNeeded stores in data_<hex>.dat
// when -S meets --mapped (keyhunt.cpp:7756-7855).  The mapping's address (bf) is written as 0; bf_chunks
// is NULL for one file.
inline void struct_bloom(const filter &F, uint8_t h[112]) {
  memset(h, 0, 112);
  memcpy(h + 0, &F.entries, 8);
  memcpy(h + 8, &F.bits, 8);
  memcpy(h + 16, &F.bytes, 8);
  h[24] = (uint8_t)F.hashes;
  const long double e = F.error;
  memcpy(h + 32, &e, 10);  // the x87 value; its 6 padding bytes stay 0, as the memset left them
  h[48] = 1;               // ready, BLOOM_VERSION_MAJOR 2, _MINOR 201
  h[49] = 2;
  h[50] = 201;
  memcpy(h + 56, &F.bpe, 8);
  const uint32_t mc = 1;
  memcpy(h + 80, &mc, 4);
  memcpy(h + 88, &F.bytes, 8);  // chunk_bytes, last_chunk_bytes
  memcpy(h + 96, &F.bytes, 8);
}

// a target filter (address / rmd160 / xpoint / eth / vanity): open it, add the items, write it back;
// out: the filter as the reference's run holds it afterwards (for -S's data file)
inline bool targets(uint64_t items, const std::vector<uint8_t> &adds, uint32_t len, filter *out = nullptr) {
  filter F;
  if (!open_filter(F, items, nullptr)) return false;
  if (kh_bloom_add(F.bf.data(), F.bits, F.hashes, adds.data(), adds.size() / len, len) != KH_OK) return false;
  printf("[+] Loading data to the bloomfilter total: %.2f MB\n", (double)F.bytes / 1048576.0);
  if (!save(F)) return false;
  if (out) *out = std::move(F);
  return true;
}

// the BSGS layers (keyhunt.cpp:1631-1785; bsgsd.cpp:1180-1255): 3 x 256 shard files bloom-%u.dat,
// bloom2-%u.dat, bloom3-%u.dat of itemsbloom / itemsbloom2 / itemsbloom3 elements each, all opened
// in that order first (the size override is applied to the first), then filled by the baby steps
// of their layer on the GPU.  A shard that cannot be opened stops the start: the files opened
// before it are left as the reference's mmap left them (created, or loaded and unchanged)
inline bool bsgs_layers(kh_ctx *ctx, const kh_bsgs_info &I, std::vector<std::vector<filter>> *keep = nullptr) {
  const uint64_t ms[3] = {I.m, I.m2, I.m3};
  const uint64_t floor_[3] = {10000, 1000, 1000};
  const char *pfx[3] = {"bloom-", "bloom2-", "bloom3-"};
  std::vector<std::vector<filter>> F(3, std::vector<filter>(256));
  for (int l = 0; l < 3; l++) {
    const uint64_t items = ms[l] / 256 > floor_[l] ? ms[l] / 256 + (ms[l] % 256 ? 1 : 0) : 1000;
    printf("[+] Bloom filter for %llu elements ", (unsigned long long)ms[l]);
    uint64_t total = 0;
    for (int i = 0; i < 256; i++) {
      const std::string fn = pfx[l] + std::to_string(i) + ".dat";
      if (!open_filter(F[l][i], items, fn.c_str())) {
        if (cfg.bsgsd)
          fprintf(stderr, l < 2 ? "[E] error bloom_init _ %i\n" : "[E] error bloom_init %i\n", i);
        else
          fprintf(stderr, l < 2 ? "[E] error bloom_init _ [%d]\n" : "[E] error bloom_init [%d]\n", i);
        for (int q = 0; q <= l; q++)
          for (int j = 0; j < (q < l ? 256 : i); j++) save(F[q][j]);
        open_failed = true;
        return false;
      }
      printf("[+] Loading data to the bloomfilter total: %.2f MB\n", (double)F[l][i].bytes / 1048576.0);
      total += F[l][i].bytes;
    }
    printf(": %.2f MB\n", layer_mb(total));
  }
  for (int l = 0; l < 3; l++) {
    // one GPU pass per distinct shard geometry
    std::vector<bool> done(256, false);
    for (int i = 0; i < 256; i++) {
      if (done[i]) continue;
      const uint64_t bits = F[l][i].bits, bytes = F[l][i].bytes;
      const uint32_t hashes = F[l][i].hashes;
      std::vector<uint8_t> all(256 * bytes, 0);
      std::vector<int> group;
      for (int j = i; j < 256; j++)
        if (!done[j] && F[l][j].bits == bits && F[l][j].bytes == bytes && F[l][j].hashes == hashes) {
          group.push_back(j);
          memcpy(&all[(size_t)j * bytes], F[l][j].bf.data(), bytes);
        }
      int r = kh_bsgs_layer_bits(ctx, (uint32_t)l + 1, bits, hashes, bytes, all.data());
      if (r) {
        fprintf(stderr, "[E] %s (%s)\n", kh_strerror(r), kh_last_error(ctx));
        return false;
      }
      for (int j : group) {
        memcpy(F[l][j].bf.data(), &all[(size_t)j * bytes], bytes);
        done[j] = true;
      }
    }
    for (int i = 0; i < 256; i++)
      if (!save(F[l][i])) return false;
  }
  if (keep) *keep = std::move(F);  // -S writes the layers' filters as the run left them
  return true;
}

}  // namespace mapped

#endif  // KH_MAPPED_H
