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
// Options: -k K, -n N, -i IP (127.0.0.1), -p PORT (8080), -6 (skip file checksums), -g GPUs
// (default all), -L reference|blocked (layer-1 layout), -t (accepted; one host thread per GPU).
#include <arpa/inet.h>
#include <ctype.h>
#include <errno.h>
#include <getopt.h>
#include <netinet/in.h>
#include <signal.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/socket.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "kh_gpu.h"
#include "kh_host_util.h"

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

// -S files of this N/k: read when all four exist, else build (+ write from the first GPU)
int load_or_build(gpu &g, bool first, bool files_present) {
  if (files_present) return kh_bsgs_load(g.ctx, ".", opt.skip_checksum ? KH_LOAD_SKIP_CHECKSUM : 0);
  int r = kh_bsgs_build(g.ctx);
  if (!r && first) r = kh_bsgs_save(g.ctx, ".");
  return r;
}

bool files_present(const kh_bsgs_info &I) {
  char f[4][96];
  snprintf(f[0], 96, "keyhunt_bsgs_4_%llu.blm", (unsigned long long)I.m);
  snprintf(f[1], 96, "keyhunt_bsgs_6_%llu.blm", (unsigned long long)I.m2);
  snprintf(f[2], 96, "keyhunt_bsgs_7_%llu.blm", (unsigned long long)I.m3);
  snprintf(f[3], 96, "keyhunt_bsgs_2_%llu.tbl", (unsigned long long)I.m3);
  for (auto &x : f)
    if (access(x, R_OK) != 0) return false;
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

void record_key(const U &key, bool compressed) {
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
  printf("[+] Thread Key found privkey %s\n[+] Publickey %s\n", k.c_str(), pub.c_str());
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
  if (!parse_pubkey(pub.c_str(), qx, qy, compressed)) {
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
  if (ok) record_key(key, compressed);
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
  while ((c = getopt(argc, argv, "6hk:n:t:p:i:g:L:B:")) != -1) {
    switch (c) {
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
        printf("usage: %s [-k K] [-n N] [-i IP] [-p PORT] [-6] [-g GPUS] [-L reference|blocked]\n", argv[0]);
        return c == 'h' ? EXIT_SUCCESS : EXIT_FAILURE;
    }
  }
  (void)have_n;
  if (!validate_nk(opt.n, opt.k)) return EXIT_FAILURE;
  printf("[+] Mode BSGS secuential\n[+] N = 0x%llx\n", (unsigned long long)opt.n);
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
  for (int d = 0; d < opt.gpus; d++) {
    gpu &g = g_gpus[d];
    int r = kh_open(d % ndev, &g.ctx);
    if (!r) r = kh_bsgs_set_layer1(g.ctx, opt.layer1);
    if (!r) r = kh_bsgs_setup(g.ctx, opt.n, opt.k, &g.info);
    if (!r && d == 0) present = files_present(g.info);
    if (!r) r = load_or_build(g, d == 0, present);
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
