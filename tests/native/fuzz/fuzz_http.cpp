// libFuzzer target: the native HTTP/1.1 ops server (httpd.cpp: request-line/header
// parsing, pipelining, Content-Length bodies, limits, CORS, routing).
//
// One HttpServer on 127.0.0.1 (ephemeral port, 2 workers, an Exporter with a fixture
// inventory so /metrics renders real text).  Each input is written on a fresh TCP
// connection, followed by a write half-close; the harness drains until the server
// closes.  Every response must start with a status line; every 256 inputs a plain
// GET /health on a new connection must answer 200.
#include <arpa/inet.h>
#include <netinet/in.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <dirent.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "fuzz_common.h"
#include "httpd.h"
#include "telemetry.h"

using namespace amdgpu_dp;

namespace {

// Every connection the harness opened has been closed by then; a growing count means
// the server leaks descriptors (or connections it never closes).
int open_fds() {
  int n = 0;
  if (DIR* d = opendir("/proc/self/fd")) {
    while (readdir(d)) ++n;
    closedir(d);
  }
  return n;
}
int g_fd_baseline = -1;

void check_fds() {
  const int n = open_fds();
  if (g_fd_baseline < 0) g_fd_baseline = n;
  if (n > g_fd_baseline + 64) {
    std::fprintf(stderr, "descriptor leak: %d open fds (baseline %d)\n", n, g_fd_baseline);
    std::abort();
  }
}

std::shared_ptr<Exporter> g_ex;
std::unique_ptr<HttpServer> g_http;
int g_port = 0;
uint64_t g_iter = 0;

std::string roundtrip(const char* data, size_t size) {
  const int fd = socket(AF_INET, SOCK_STREAM | SOCK_CLOEXEC, 0);
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_port = htons(static_cast<uint16_t>(g_port));
  a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
  if (!fuzzutil::connect_retry(fd, reinterpret_cast<sockaddr*>(&a), sizeof(a))) {
    std::fprintf(stderr, "connect failed: %s\n", std::strerror(errno));
    std::abort();
  }
  size_t off = 0;
  while (off < size) {
    const ssize_t w = send(fd, data + off, size - off, MSG_NOSIGNAL);
    if (w < 0 && errno == EINTR) continue;
    if (w <= 0) break;  // server answered 4xx and closed early: fine
    off += static_cast<size_t>(w);
  }
  shutdown(fd, SHUT_WR);
  std::string resp;
  if (!fuzzutil::drain_until_close(fd, &resp)) {
    std::fprintf(stderr, "server did not close a half-closed connection within 5 s\n");
    std::abort();
  }
  // Linger-free close: the fuzzer opens tens of thousands of connections.
  struct linger lg {1, 0};
  setsockopt(fd, SOL_SOCKET, SO_LINGER, &lg, sizeof(lg));
  close(fd);
  return resp;
}

}  // namespace

extern "C" int LLVMFuzzerInitialize(int*, char***) {
  if (const char* dir = fuzzutil::seed_dir()) {
    fuzzutil::write_seed(dir, "get_health", "GET /health HTTP/1.1\r\nHost: x\r\n\r\n");
    fuzzutil::write_seed(dir, "pipelined",
                         "GET / HTTP/1.1\r\nOrigin: http://a\r\n\r\nGET /metrics?x=1 HTTP/1.1\r\n\r\n"
                         "OPTIONS /health HTTP/1.1\r\n\r\n");
    fuzzutil::write_seed(dir, "post_body", "POST /health HTTP/1.1\r\nContent-Length: 5\r\n\r\nhelloGET /nope HTTP/1.0\r\n\r\n");
    fuzzutil::write_seed(dir, "keepalive_10", "GET /health HTTP/1.0\r\nConnection: keep-alive\r\n\r\n"
                                              "DELETE /metrics HTTP/1.1\r\nConnection: close\r\n\r\n");
    fuzzutil::write_seed(dir, "metrics_gzip", "GET /metrics HTTP/1.1\r\nAccept-Encoding: deflate, gzip;q=1\r\n\r\n"
                                              "GET /metrics HTTP/1.1\r\naccept-encoding: br\r\n\r\n");
    fuzzutil::write_seed(dir, "chunked", "PUT / HTTP/1.1\r\nTransfer-Encoding: chunked\r\n\r\n5\r\nhello\r\n0\r\n\r\n");
    std::exit(0);
  }
  g_ex = std::make_shared<Exporter>();
  std::vector<GpuInfo> gpus(2);
  for (int i = 0; i < 2; ++i) {
    gpus[i].index = i;
    gpus[i].uuid = "gpu-" + std::to_string(i);
    gpus[i].market_name = "AMD Instinct MI355X";
    gpus[i].gfx_target = "gfx950";
  }
  g_ex->set_inventory(gpus);
  g_ex->set_tables({fuzzutil::make_table(2, 1)});
  HttpConfig hc;
  hc.host = "127.0.0.1";
  hc.port = 0;
  hc.threads = 2;
  hc.access_log = false;
  g_http = std::make_unique<HttpServer>(hc, g_ex);
  g_http->set_restart_hook([] {});
  g_port = g_http->start();
  return 0;
}

extern "C" int LLVMFuzzerTestOneInput(const uint8_t* data, size_t size) {
  const std::string resp = roundtrip(reinterpret_cast<const char*>(data), size);
  // HTTP/1.0 requests are answered "HTTP/1.0 ..." like Go's net/http writeStatusLine
  if (!resp.empty() && resp.compare(0, 9, "HTTP/1.1 ") != 0 && resp.compare(0, 9, "HTTP/1.0 ") != 0) {
    std::fprintf(stderr, "response does not start with a status line: %.40s\n", resp.c_str());
    std::abort();
  }
  if ((++g_iter & 255) == 0) {
    check_fds();
    static const char kHealth[] = "GET /health HTTP/1.1\r\nConnection: close\r\n\r\n";
    const std::string r = roundtrip(kHealth, sizeof(kHealth) - 1);
    if (r.compare(0, 15, "HTTP/1.1 200 OK") != 0) {
      std::fprintf(stderr, "liveness GET /health failed: %.60s\n", r.c_str());
      std::abort();
    }
  }
  return 0;
}
