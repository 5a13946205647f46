// bsgsd_amd.cpp -- the reference's BSGS daemon (bsgsd.cpp, BSGSD.md) on the MI355X engine
// (bin/bsgsd-amd).
//
// The three bloom layers and the bP table stay resident in every GPU's HBM.  A client sends one
// request and reads one reply, as in bsgsd.cpp:3307-3579:
//   line mode:  "<publickey> <from>:<to>\n" (or "<publickey> <from> <to>\n")
//               -> "<privkey hex>\n" | "404 Not Found\n" | "400 Bad Request"
//   HTTP mode:  POST with a JSON body {"pubkey": "...", "from": "...", "to": "..."}
//               -> HTTP/1.1 200 OK (body "<privkey hex>\n") | 404 Not Found | 400 Bad Request,
//                  Content-Type text/plain, Content-Length, Connection: close, X-Elapsed-Seconds
// The range is walked in whole bases of 2N from <from> while base < <to> (bsgsd.cpp:2510-2525),
// split across the GPUs; found keys are appended to KEYFOUNDKEYFOUND.txt like the reference's.
// Tables come from the -S files in the working directory when all four exist, else they are
// built and written (bsgsd sets FLAGSAVEREADFILE = 1, bsgsd.cpp:238).  Requests are served one
// at a time ("One client at the time", BSGSD.md).
//
// Like the reference daemon, the .tbl file is followed by its MD5 in keyhunt_bsgs_2_<M3>.tbl.md5
// whenever it is written or read (bsgsd.cpp:1625-1670, 2073-2095).
//
// Options: -k K, -n N, -i IP (127.0.0.1), -p PORT (8080), -6 (skip file checksums), -g contexts
// (default: one per GPU; more than the GPUs share them), -L reference|blocked (layer-1 layout),
// -t (accepted; one host thread per context), --ptable FILE, --ptable-size SIZE, --load-ptable,
// --ptable-cache (the bP table file, its FILE.md5 and FILE.cache, bsgsd.cpp:1314-1470, 1719-1755),
// and the bloom-file options (bsgsd.cpp:776-889): --mapped[=NAME], --mapped-size SIZE,
// --mapped-chunks N, --bloom-file NAME, --load-bloom, --bloom-bytes SIZE, --create-mapped[=SIZE]
// (kh_mapped.h: with --mapped the 3 x 256 shard files bloom-%u.dat, bloom2-%u.dat, bloom3-%u.dat
// are written as the reference's mmap leaves them, and no -S files are read or written), --tmpdir
// (where the reference maps an unnamed bP table; the table lives in HBM here),
// --bsgs-block-count / --bsgs-block-size (parsed and sized by the reference, then unused,
// bsgsd.cpp:1047-1066) and --rmd-batch-size (unused by the daemon, bsgsd.cpp:887-888).
#include <arpa/inet.h>
#include <ctype.h>
#include <errno.h>
#include <fcntl.h>
#include <getopt.h>
#include <netinet/in.h>
#include <signal.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/socket.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "kh_gpu.h"
#include "kh_host_util.h"
#include "kh_mapped.h"

using namespace kh;
using namespace khh;

namespace {

struct gpu {
  kh_ctx *ctx = nullptr;
  kh_bsgs_info info{};
};

struct options {
  uint64_t k = 1, n = 0x100000000000ULL;
  const char *ip = "127.0.0.1";
  int port = 8080;
  bool skip_checksum = false;
  int gpus = 0;
  uint32_t layer1 = KH_LAYER1_BLOCKED;
  const char *ptable = nullptr;
  uint64_t ptable_size = 0;
  bool load_ptable = false, ptable_cache = false;
  bool mapped = false, create_mapped = false;  // FLAGMAPPED, FLAGCREATEMAPPED (mapped::cfg holds the rest)
} opt;

std::vector<gpu> g_gpus;

bool send_all(int fd, const char *buf, size_t len) {
  size_t sent = 0;
  while (sent < len) {
    ssize_t n = send(fd, buf + sent, len - sent, MSG_NOSIGNAL);
    if (n < 0 && errno == EINTR) continue;
    if (n <= 0) return false;
    sent += (size_t)n;
  }
  return true;
}

std::string tbl_name(const kh_bsgs_info &I) {
  char f[96];
  snprintf(f, sizeof f, "keyhunt_bsgs_2_%llu.tbl", (unsigned long long)I.m3);
  return f;
}

bool files_present(const kh_bsgs_info &I) {
  if (opt.mapped) return false;  // -S files are skipped with --mapped (bsgsd.cpp:1465, 1991)
  char f[3][96];
  snprintf(f[0], 96, "keyhunt_bsgs_4_%llu.blm", (unsigned long long)I.m);
  snprintf(f[1], 96, "keyhunt_bsgs_6_%llu.blm", (unsigned long long)I.m2);
  snprintf(f[2], 96, "keyhunt_bsgs_7_%llu.blm", (unsigned long long)I.m3);
  for (auto &x : f)
    if (access(x, R_OK) != 0) return false;
  return access(tbl_name(I).c_str(), R_OK) == 0;
}

// MD5 of `path` into path.md5, reporting an earlier one (bsgsd.cpp:1444-1462, 1648-1665)
bool md5_refresh(const std::string &path, uint8_t md5[16], bool report) {
  const std::string md5_path = path + ".md5";
  if (!md5_of_file(path.c_str(), md5)) {
    fprintf(stderr, "[W] Unable to compute MD5 for bP table %s\n", path.c_str());
    return false;
  }
  uint8_t disk[16];
  if (report && read_md5_file(md5_path.c_str(), disk))
    printf(memcmp(disk, md5, 16) == 0 ? "[+] bP table MD5 verified (%s)\n" : "[W] bP table MD5 mismatch (%s); refreshing\n",
           md5_path.c_str());
  if (!write_md5_file(md5_path.c_str(), md5)) fprintf(stderr, "[W] Unable to write bP table MD5 file %s\n", md5_path.c_str());
  return true;
}

// The table files of the first context, in the reference daemon's order (bsgsd.cpp:1314-1470,
// 1473-1755, 2073-2095): the --ptable file is opened (read-only with --load-ptable: its rows are the
// table), the -S files are read when all four exist (the .tbl only without --ptable), --ptable-cache
// then writes CACHE_TARGET.md5 / .cache from the rows the target holds AT THAT POINT (a fresh --ptable
// file still holds zeros), and only then are the tables built and the files written.  `rows` returns
// the --load-ptable rows for every context.
int first_tables(gpu &g, std::vector<uint8_t> &rows, bool &present) {
  const kh_bsgs_info &I = g.info;
  const uint64_t bytes = I.m3 * 16;
  const std::string tbl = tbl_name(I);
  std::string target;  // bptable_cache_target
  std::vector<uint8_t> target_rows(bytes, 0);
  uint8_t md5[16];
  bool md5_ready = false;
  if (opt.ptable) {
    target = opt.ptable;
    if (opt.load_ptable) {
      FILE *f = fopen(opt.ptable, "rb");
      if (!f) {
        fprintf(stderr, "[E] Cannot open bP table file\n");
        return KH_E_IO;
      }
      struct stat st;
      if (fstat(fileno(f), &st) != 0 || (uint64_t)st.st_size < bytes) {
        fclose(f);
        fprintf(stderr, "[E] Existing bP table file too small\n");
        return KH_E_IO;
      }
      rows.resize(bytes);
      const bool ok = bytes == 0 || fread(rows.data(), bytes, 1, f) == 1;
      fclose(f);
      if (!ok) {
        fprintf(stderr, "[E] Cannot read bP table file\n");
        return KH_E_IO;
      }
      target_rows = rows;
      md5_ready = md5_refresh(opt.ptable, md5, true);
    } else {
      const uint64_t map_bytes = std::max(bytes, opt.ptable_size);
      int fd = open(opt.ptable, O_RDWR | O_CREAT, 0600);
      if (fd < 0) {
        fprintf(stderr, "[E] Cannot create bP table file\n");
        return KH_E_IO;
      }
      struct stat st;
      bool ok = fstat(fd, &st) == 0;
      if (ok && (uint64_t)st.st_size < map_bytes) ok = ftruncate(fd, (off_t)map_bytes) == 0;
      if (ok && map_bytes < (1ull << 20)) {  // small mappings are zeroed (bsgsd.cpp:1424-1431)
        std::vector<uint8_t> zero(map_bytes, 0);
        ok = pwrite(fd, zero.data(), map_bytes, 0) == (ssize_t)map_bytes;
      }
      if (ok && bytes) ok = pread(fd, target_rows.data(), bytes, 0) == (ssize_t)bytes;
      close(fd);
      if (!ok) {
        fprintf(stderr, "[E] Cannot resize bP table file\n");
        return KH_E_IO;
      }
    }
  }
  present = files_present(I);
  if (present) {
    int r = kh_bsgs_load(g.ctx, ".", opt.skip_checksum ? KH_LOAD_SKIP_CHECKSUM : 0);
    if (r) return r;
    if (!opt.ptable) {  // the .tbl was read: it is now the cache target, with its MD5 refreshed
      target = tbl;
      uint64_t got = 0;
      r = kh_get_bsgs_table(g.ctx, target_rows.data(), I.m3, &got);
      if (r) return r;
      md5_ready = md5_refresh(tbl, md5, true);
    }
  }
  if (opt.ptable_cache && !target.empty()) {
    if (!md5_ready) md5_ready = md5_refresh(target, md5, false);
    if (md5_ready) {
      const std::string cache = target + ".cache";
      const int st = bptable_cache_status(cache.c_str(), md5, I.m3);
      if (st == 1) {
        printf("[+] bP table cache hit (%s)\n", cache.c_str());
      } else {
        printf(st < 0 ? "[W] bP table cache mismatch (%s); rebuilding\n" : "[I] bP table cache not found (%s); creating\n",
               cache.c_str());
        if (bptable_cache_write(cache.c_str(), md5, target_rows.data(), I.m3))
          printf("[+] bP table cache refreshed (%s)\n", cache.c_str());
        else
          printf("[W] Unable to write bP table cache to %s\n", cache.c_str());
      }
    }
  }
  if (!present) {
    const bool had_tbl = access(tbl.c_str(), F_OK) == 0;
    int r = kh_bsgs_build(g.ctx);
    if (!r && !opt.mapped) r = kh_bsgs_save(g.ctx, ".");
    if (r) return r;
    if (opt.mapped) {
      // the shard files instead, filled from the tables just built (bsgsd.cpp:1180-1255, 1850-1980)
      if (!mapped::bsgs_layers(g.ctx, I)) return KH_E_IO;
    } else if (opt.load_ptable && !had_tbl) {
      unlink(tbl.c_str());  // the table came from the --ptable file: no .tbl is written
    } else {
      md5_refresh(tbl, md5, false);
    }
  }
  if (present && opt.ptable && !opt.load_ptable) {
    // the reference never reads the .tbl with --ptable: it rebuilds and rewrites it (the same
    // bytes) and its MD5 (bsgsd.cpp:2073-2095)
    uint8_t m[16];
    md5_refresh(tbl, m, false);
  }
  if (opt.ptable && !opt.load_ptable) {  // the built rows land in the --ptable file
    std::vector<uint8_t> built(bytes);
    uint64_t got = 0;
    int r = kh_get_bsgs_table(g.ctx, built.data(), I.m3, &got);
    if (r) return r;
    int fd = open(opt.ptable, O_RDWR);
    bool ok = fd >= 0 && (bytes == 0 || pwrite(fd, built.data(), bytes, 0) == (ssize_t)bytes);
    if (fd >= 0) ok = close(fd) == 0 && ok;
    if (!ok) {
      fprintf(stderr, "[E] Cannot write bP table file\n");
      return KH_E_IO;
    }
  }
  if (opt.load_ptable) return kh_bsgs_set_table(g.ctx, rows.data(), I.m3);
  return KH_OK;
}

// bsgsd's initBloomFilterMapped without --mapped (bsgsd.cpp:657-680), per shard in the order of
// bsgsd.cpp:1180-1255: --load-bloom, or a shard file already in the directory, makes it bloom_load
// that file (bloom/bloom.cpp:323-372), which needs the BLOOM_MAGIC header bloom_save writes -- the
// daemon never writes one, and a mapped shard file (raw bits) fails it -- so the start stops there
// (exit 0) before any table is built
bool plain_shards_ok() {
  const char *pfx[3] = {"bloom-", "bloom2-", "bloom3-"};
  for (int l = 0; l < 3; l++)
    for (int i = 0; i < 256; i++) {
      const std::string fn = pfx[l] + std::to_string(i) + ".dat";
      struct stat st;
      const bool have = stat(fn.c_str(), &st) == 0;
      bool fail = false;
      if (mapped::cfg.load_bloom) {
        if (!have || st.st_size == 0)
          fprintf(stderr, "[E] --load-bloom specified but bloom file '%s' does not exist or is empty\n", fn.c_str());
        else
          fprintf(stderr, "[E] bloom_load failed for '%s'\n", fn.c_str());
        fail = true;
      } else if (!mapped::cfg.entries && have) {
        fprintf(stderr, "[E] bloom_load failed for '%s'\n", fn.c_str());
        fail = true;
      }
      if (fail) {
        fprintf(stderr, l < 2 ? "[E] error bloom_init _ %i\n" : "[E] error bloom_init %i\n", i);
        return false;
      }
    }
  return true;
}

// the walk of one request: bases from, from + 2N, ... while base < to, over every GPU
bool search(const fe &qx, const fe &qy, const U &from, const U &to, U &key) {
  uint8_t xy[64];
  fe_to_be(xy, qx);
  fe_to_be(xy + 32, qy);
  const U twoN = u_mul_u64(u_from_u64(g_gpus[0].info.n), 2);
  for (auto &g : g_gpus) {
    kh_bsgs_reset_found(g.ctx);
    kh_bsgs_set_targets(g.ctx, xy, 1);
  }
  std::mutex mtx;
  U cursor = from;
  std::atomic<bool> found{false};
  const uint64_t per_call = 65536;  // bases per engine call (2^31 giant points at k = 128)
  auto worker = [&](gpu &g) {
    for (;;) {
      U base;
      uint64_t nb = 0;
      {
        std::lock_guard<std::mutex> lk(mtx);
        if (found || u_cmp(cursor, to) >= 0) return;
        base = cursor;
        while (nb < per_call && u_cmp(cursor, to) < 0) {
          cursor = u_add(cursor, twoN);
          nb++;
        }
      }
      uint8_t st[32];
      u_to_be32(base, st);
      kh_bsgs_found f[2];
      uint32_t nf = 0;
      int r = kh_bsgs_scan(g.ctx, st, nb, f, 2, &nf);
      if (r) {
        fprintf(stderr, "[E] kh_bsgs_scan: %s (%s)\n", kh_strerror(r), kh_last_error(g.ctx));
        return;
      }
      if (nf) {
        std::lock_guard<std::mutex> lk(mtx);
        if (!found) key = u_from_be32(f[0].key);
        found = true;
        return;
      }
    }
  };
  std::vector<std::thread> th;
  for (auto &g : g_gpus) th.emplace_back(worker, std::ref(g));
  for (auto &t : th) t.join();
  return found;
}

void record_key(const U &key, bool compressed, bool at_base) {
  uint8_t kb[32], pxy[64];
  u_to_be32(key, kb);
  kh_pubkeys(g_gpus[0].ctx, kb, 1, pxy);
  std::string pub;
  if (compressed) {
    uint8_t p = (pxy[63] & 1) ? 3 : 2;
    pub = hex(&p, 1) + hex(pxy, 32);
  } else {
    uint8_t p = 4;
    pub = hex(&p, 1) + hex(pxy, 64);
  }
  const std::string k = u_hex(key);
  // a key at the very start of a base is caught by the reference's base-point check, whose line
  // ends in two spaces (bsgsd.cpp:2544-2548); the giant-step path prints none (2724)
  printf(at_base ? "[+] Thread Key found privkey %s  \n[+] Publickey %s\n" : "[+] Thread Key found privkey %s\n[+] Publickey %s\n",
         k.c_str(), pub.c_str());
  FILE *f = fopen("KEYFOUNDKEYFOUND.txt", "a");
  if (f) {
    fprintf(f, "Key found privkey %s\nPublickey %s\n", k.c_str(), pub.c_str());
    fclose(f);
  }
  fflush(stdout);
}

bool json_value(const std::string &src, const char *key, std::string &out) {  // bsgsd.cpp:3393-3405
  const std::string needle = "\"" + std::string(key) + "\"";
  size_t pos = src.find(needle);
  if (pos == std::string::npos) return false;
  pos = src.find(':', pos + needle.size());
  if (pos == std::string::npos) return false;
  pos = src.find('"', pos);
  if (pos == std::string::npos) return false;
  size_t end = src.find('"', pos + 1);
  if (end == std::string::npos) return false;
  out.assign(src.begin() + pos + 1, src.begin() + end);
  return true;
}

void handle(int fd) {
  const auto t0 = std::chrono::steady_clock::now();
  char buf[1024];
  ssize_t n = recv(fd, buf, sizeof buf - 1, MSG_PEEK);
  if (n <= 0) return;
  const bool http = memcmp(buf, "POST", n < 4 ? (size_t)n : 4) == 0;
  const char *bad = http ? "HTTP/1.1 400 Bad Request\r\nConnection: close\r\n\r\n" : "400 Bad Request";
  std::string pub, from_s, to_s;
  if (http) {
    std::string req;
    size_t hdr_end;
    do {
      n = recv(fd, buf, sizeof buf, 0);
      if (n <= 0) return;
      req.append(buf, (size_t)n);
      if (req.size() > (1u << 20)) {
        const char *m = "HTTP/1.1 413 Request Entity Too Large\r\nConnection: close\r\n\r\n";
        send_all(fd, m, strlen(m));
        return;
      }
      hdr_end = req.find("\r\n\r\n");
    } while (hdr_end == std::string::npos);
    const std::string head = req.substr(0, hdr_end);
    std::string body = req.substr(hdr_end + 4);
    size_t clen = 0, p = head.find("Content-Length:");
    if (p != std::string::npos) clen = strtoull(head.c_str() + p + 15, nullptr, 10);
    while (body.size() < clen) {
      n = recv(fd, buf, sizeof buf, 0);
      if (n <= 0) return;
      body.append(buf, (size_t)n);
      if (body.size() > (1u << 20)) {
        const char *m = "HTTP/1.1 413 Request Entity Too Large\r\nConnection: close\r\n\r\n";
        send_all(fd, m, strlen(m));
        return;
      }
    }
    if (!(json_value(body, "pubkey", pub) && json_value(body, "from", from_s) && json_value(body, "to", to_s))) {
      send_all(fd, bad, strlen(bad));
      return;
    }
  } else {
    std::string line;
    do {
      n = recv(fd, buf, sizeof buf, 0);
      if (n <= 0) return;
      line.append(buf, (size_t)n);
      if (line.size() > 4096) {
        printf("Invalid input too long from client\n");
        send_all(fd, bad, strlen(bad));
        return;
      }
    } while (line.find('\n') == std::string::npos);
    std::vector<std::string> tok;
    size_t i = 0;
    while (i < line.size()) {
      while (i < line.size() && isspace((unsigned char)line[i])) i++;
      size_t j = i;
      while (j < line.size() && !isspace((unsigned char)line[j])) j++;
      if (j > i) tok.push_back(line.substr(i, j - i));
      i = j;
    }
    if (tok.size() < 2) {
      printf("Invalid input format from client, tokens %zu : %s\n", tok.size(), line.c_str());
      send_all(fd, bad, strlen(bad));
      return;
    }
    pub = tok[0];
    if (tok.size() >= 3) {
      from_s = tok[1];
      to_s = tok[2];
    } else {
      size_t c = tok[1].find(':');
      if (c == std::string::npos || c == 0 || c + 1 == tok[1].size()) {
        printf("Invalid range format from client: %s\n", tok[1].c_str());
        send_all(fd, bad, strlen(bad));
        return;
      }
      from_s = tok[1].substr(0, c);
      to_s = tok[1].substr(c + 1);
    }
  }
  fe qx, qy;
  bool compressed = false;
  U from, to;
  // Secp256K1::ParsePublicKeyHex prints its own message first (SECP256K1.cpp:303-380); where the
  // reference exits (a 04 key of the wrong length, an unreadable digit pair) the request is refused
  // like the others instead
  if (parse_pubkey_hex_ref(pub.c_str(), qx, qy, compressed) <= 0) {
    printf("Invalid publickey format from client %s\n", pub.c_str());
    send_all(fd, bad, strlen(bad));
    return;
  }
  if (!u_from_hex(from_s.c_str(), from) || !u_from_hex(to_s.c_str(), to)) {
    printf("Invalid hexadecimal format from client %s:%s\n", from_s.c_str(), to_s.c_str());
    send_all(fd, bad, strlen(bad));
    return;
  }
  U key;
  const bool ok = search(qx, qy, from, to, key);
  if (ok) {
    uint64_t rem = 1;
    if (u_cmp(key, from) >= 0) u_divmod_u64(u_sub(key, from), 2 * g_gpus[0].info.n, &rem);
    record_key(key, compressed, rem == 0);
  }
  const double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  std::string body = ok ? u_hex(key) + "\n" : std::string("404 Not Found\n");
  std::string reply;
  if (http) {
    char h[256];
    snprintf(h, sizeof h,
             "%sContent-Type: text/plain\r\nContent-Length: %zu\r\nConnection: close\r\nX-Elapsed-Seconds: %.3f\r\n\r\n",
             ok ? "HTTP/1.1 200 OK\r\n" : "HTTP/1.1 404 Not Found\r\n", body.size(), secs);
    reply = h + body;
  } else {
    reply = body;
  }
  if (!send_all(fd, reply.data(), reply.size())) printf("Failed to send message to client\n");
}

}  // namespace

int main(int argc, char **argv) {
  signal(SIGPIPE, SIG_IGN);
  printf("[+] Version 0.2.230519 Satoshi Quest (bsgsd-amd: MI355X engine)\n");
  int c;
  bool have_n = false;
  static const struct option long_opts[] = {{"ptable", required_argument, 0, 1},
                                           {"ptable-size", required_argument, 0, 2},
                                           {"load-ptable", no_argument, 0, 3},
                                           {"ptable-cache", no_argument, 0, 4},
                                           {"mapped", optional_argument, 0, 5},
                                           {"mapped-size", required_argument, 0, 6},
                                           {"mapped-chunks", required_argument, 0, 7},
                                           {"bloom-file", required_argument, 0, 8},
                                           {"load-bloom", no_argument, 0, 9},
                                           {"bloom-bytes", required_argument, 0, 10},
                                           {"create-mapped", optional_argument, 0, 11},
                                           {"tmpdir", required_argument, 0, 12},
                                           {"bsgs-block-count", required_argument, 0, 13},
                                           {"bsgs-block-size", required_argument, 0, 13},
                                           {"rmd-batch-size", required_argument, 0, 13},
                                           {0, 0, 0, 0}};
  mapped::cfg.bsgsd = true;
  // --mapped-size / --bloom-bytes / --create-mapped SIZE, with the k/m/g/t suffixes: the entry count
  // and error bsgsd's bloom_entries_for_bytes gives any size (kh_mapped.h entries_for_bsgsd)
  auto size_override = [](const char *arg) {
    char *end;
    uint64_t v = strtoull(arg, &end, 10);
    if (*end) {
      switch (tolower(*end)) {
        case 'k': v *= 1024ull; break;
        case 'm': v *= 1024ull * 1024ull; break;
        case 'g': v *= 1024ull * 1024ull * 1024ull; break;
        case 't': v *= 1024ull * 1024ull * 1024ull * 1024ull; break;
      }
    }
    mapped::entries_for_bsgsd(v, &mapped::cfg.entries, &mapped::cfg.error);
  };
  while ((c = getopt_long(argc, argv, "6hk:n:t:p:i:g:L:B:", long_opts, nullptr)) != -1) {
    switch (c) {
      case 1: opt.ptable = optarg; break;  // bsgsd.cpp:828-829
      case 2: {                            // bsgsd.cpp:830-841
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
      case 3: opt.load_ptable = true; break;
      case 4: opt.ptable_cache = true; break;
      case 5:  // bsgsd.cpp:799-803
        opt.mapped = true;
        if (optarg) mapped::cfg.name = optarg;
        break;
      case 6:  // bsgsd.cpp:804-820
        opt.mapped = true;
        size_override(optarg);
        break;
      case 7:  // bsgsd.cpp:821-823
        opt.mapped = true;
        mapped::cfg.chunks = (uint32_t)strtoul(optarg, NULL, 10);
        break;
      case 8: mapped::cfg.name = optarg; break;        // bsgsd.cpp:824-825 (does not set --mapped)
      case 9: mapped::cfg.load_bloom = true; break;    // bsgsd.cpp:826-827
      case 10:                                         // bsgsd.cpp:844-859
        opt.mapped = true;
        size_override(optarg);
        break;
      case 11:  // bsgsd.cpp:860-878
        opt.mapped = true;
        opt.create_mapped = true;
        if (optarg) size_override(optarg);
        break;
      case 12: break;  // --tmpdir
      case 13: break;  // --bsgs-block-count/--bsgs-block-size/--rmd-batch-size: no effect on the daemon
      case '6':
        opt.skip_checksum = true;
        fprintf(stderr, "[W] Skipping checksums on files\n");
        break;
      case 'k':
        opt.k = strtoull(optarg, nullptr, 10);
        if (!opt.k) opt.k = 1;
        printf("[+] K factor %llu\n", (unsigned long long)opt.k);
        break;
      case 'n':
        opt.n = (optarg[0] == '0' && (optarg[1] == 'x' || optarg[1] == 'X')) ? strtoull(optarg + 2, nullptr, 16)
                                                                             : strtoull(optarg, nullptr, 10);
        have_n = true;
        break;
      case 't': break;  // one host thread per GPU
      case 'p': opt.port = atoi(optarg); break;
      case 'i': opt.ip = optarg; break;
      case 'g': opt.gpus = atoi(optarg); break;
      case 'L':
        if (!strcmp(optarg, "reference")) opt.layer1 = KH_LAYER1_REFERENCE;
        else if (!strcmp(optarg, "blocked")) opt.layer1 = KH_LAYER1_BLOCKED;
        else { fprintf(stderr, "[E] -L reference|blocked\n"); return EXIT_FAILURE; }
        break;
      case 'B':
        if (strcmp(optarg, "sequential")) {
          fprintf(stderr, "[E] bsgsd-amd walks the requested range sequentially (-B %s not provided)\n", optarg);
          return EXIT_FAILURE;
        }
        break;
      case 'h':
      default:
        printf("usage: %s [-k K] [-n N] [-i IP] [-p PORT] [-6] [-g CONTEXTS] [-L reference|blocked]\n"
               "       [--ptable FILE [--ptable-size SIZE] [--load-ptable] [--ptable-cache]]\n"
               "       [--mapped[=NAME]] [--mapped-size SIZE] [--mapped-chunks N] [--bloom-file NAME]\n"
               "       [--load-bloom] [--bloom-bytes SIZE] [--create-mapped[=SIZE]] [--tmpdir DIR]\n", argv[0]);
        return c == 'h' ? EXIT_SUCCESS : EXIT_FAILURE;
    }
  }
  (void)have_n;
  if (opt.load_ptable && !opt.ptable) {  // bsgsd.cpp:951-954
    fprintf(stderr, "--load-ptable requires --ptable <file>\n");
    return EXIT_FAILURE;
  }
  if (opt.create_mapped) return mapped::create();  // bsgsd.cpp:955-995: the zeroed file(s), then exit
  if (!validate_nk(opt.n, opt.k)) return EXIT_FAILURE;
  printf("[+] Mode BSGS secuential\n[+] N = 0x%llx\n", (unsigned long long)opt.n);
  if (!opt.mapped && !plain_shards_ok()) return 0;
  int ndev = 0;
  if (kh_device_count(&ndev) || ndev <= 0) {
    fprintf(stderr, "[E] no GPU\n");
    return EXIT_FAILURE;
  }
  // -g contexts on devices d % ndev: more contexts than devices share a device, each with its own
  // tables and lanes, all taking bases from the request's one cursor
  if (opt.gpus <= 0) opt.gpus = ndev;
  g_gpus.resize(opt.gpus);
  bool present = false;
  std::vector<uint8_t> ptable_rows;
  // every context holds its own tables and walk pad: before any table is built, the contexts each
  // device will carry must fit its free memory (measured before the first context allocates)
  std::vector<uint64_t> dev_free(ndev, 0);
  for (int d = 0; d < ndev && d < opt.gpus; d++) kh_device_memory(d, &dev_free[d], nullptr);
  for (int d = 0; d < opt.gpus; d++) {
    gpu &g = g_gpus[d];
    int r = kh_open(d % ndev, &g.ctx);
    if (!r) r = kh_bsgs_set_layer1(g.ctx, opt.layer1);
    if (!r) r = kh_bsgs_set_base_check(g.ctx, 1);  // bsgsd.cpp:2544-2561
    if (!r) r = kh_bsgs_setup(g.ctx, opt.n, opt.k, &g.info);
    if (!r && d == 0) {
      uint64_t need = 0;
      kh_bsgs_memory(g.ctx, &need, nullptr);
      for (int dev = 0; dev < ndev && dev < opt.gpus; dev++) {
        const uint64_t per = (uint64_t)(opt.gpus / ndev + (dev < opt.gpus % ndev ? 1 : 0));
        if (dev_free[dev] && per * need > dev_free[dev]) {
          fprintf(stderr, "[E] -g %d: %llu context(s) on GPU %d need %.1f GB of device memory (%.1f GB each), "
                          "%.1f GB are free; use fewer contexts (-g) or a smaller -n / -k\n",
                  opt.gpus, (unsigned long long)per, dev, per * need / 1e9, need / 1e9, dev_free[dev] / 1e9);
          return EXIT_FAILURE;
        }
      }
    }
    if (!r && d == 0) {
      r = first_tables(g, ptable_rows, present);
    } else if (!r && opt.mapped) {
      // --mapped skips the -S files (bsgsd.cpp:1465, 1991): the first context built its tables and
      // the shard files; the others build theirs too rather than read any -S file left in the
      // directory by an earlier run
      r = kh_bsgs_build(g.ctx);
      if (!r && opt.load_ptable) r = kh_bsgs_set_table(g.ctx, ptable_rows.data(), g.info.m3);
    } else if (!r) {  // the first context left the four files (or the --ptable rows) for the others
      r = kh_bsgs_load(g.ctx, ".", opt.skip_checksum ? KH_LOAD_SKIP_CHECKSUM : 0);
      if (r == KH_E_IO) r = kh_bsgs_build(g.ctx);  // --load-ptable without a .tbl
      if (!r && opt.load_ptable) r = kh_bsgs_set_table(g.ctx, ptable_rows.data(), g.info.m3);
    }
    if (r && mapped::open_failed) return 0;  // a shard file the reference cannot map either: exit(0)
    if (r) {
      fprintf(stderr, "[E] GPU %d: %s (%s)\n", d, kh_strerror(r), g.ctx ? kh_last_error(g.ctx) : "");
      return EXIT_FAILURE;
    }
  }
  printf("[+] %s %d GPU table set(s): M %llu, M2 %llu, M3 %llu\n", present ? "Read" : "Built", opt.gpus,
         (unsigned long long)g_gpus[0].info.m, (unsigned long long)g_gpus[0].info.m2,
         (unsigned long long)g_gpus[0].info.m3);
  int srv = socket(AF_INET, SOCK_STREAM, 0);
  if (srv < 0) {
    perror("socket failed");
    return EXIT_FAILURE;
  }
  int one = 1;
  setsockopt(srv, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
  sockaddr_in addr;
  memset(&addr, 0, sizeof addr);
  addr.sin_family = AF_INET;
  addr.sin_port = htons((uint16_t)opt.port);
  if (inet_pton(AF_INET, opt.ip, &addr.sin_addr) != 1) {
    fprintf(stderr, "[W] Invalid IP address: %s, defaulting to 127.0.0.1\n", opt.ip);
    opt.ip = "127.0.0.1";
    inet_pton(AF_INET, opt.ip, &addr.sin_addr);
  }
  if (bind(srv, (sockaddr *)&addr, sizeof addr) < 0) {
    perror("bind failed");
    return EXIT_FAILURE;
  }
  if (listen(srv, 3) < 0) {
    perror("listen failed");
    return EXIT_FAILURE;
  }
  printf("[+] Listening in %s:%i\n", opt.ip, opt.port);
  fflush(stdout);
  for (;;) {
    sockaddr_in cli;
    socklen_t len = sizeof cli;
    int fd = accept(srv, (sockaddr *)&cli, &len);
    if (fd < 0) {
      if (errno == EINTR) continue;
      perror("accept failed");
      return EXIT_FAILURE;
    }
    char ip[INET_ADDRSTRLEN];
    inet_ntop(AF_INET, &cli.sin_addr, ip, sizeof ip);
    printf("[+] Accepting incoming conection from %s:%i\n", ip, ntohs(cli.sin_port));
    fflush(stdout);
    handle(fd);
    close(fd);
    printf("[+] Closing conection from %s:%i\n", ip, ntohs(cli.sin_port));
    fflush(stdout);
  }
}
