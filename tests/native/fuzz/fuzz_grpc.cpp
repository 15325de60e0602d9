// libFuzzer target: the native HTTP/2 gRPC server (grpc_h2.cpp) on its unix socket.
//
// One GrpcServer (2 worker threads, a 8x8 CPX device table) lives for the whole run.
// Each input becomes one connection: client preface + SETTINGS, then the input bytes
// as raw frames, then a write half-close; the harness drains the socket until the
// server closes it.  Every 256 inputs a well-formed Allocate on a fresh connection
// must still succeed, so a wedged worker, a leaked stream state or a server that stops
// closing connections is a finding, not just a crash.
//
// The table has pre_start_required set and a verifier thread completes PreStartContainer
// jobs (pass, fail, or after a short delay, in turn), so the asynchronous completion
// path - answers arriving after the client reset the stream, closed the connection, or
// after the fd number was reused - is fuzzed too.
#include <poll.h>
#include <sys/socket.h>
#include <sys/un.h>
#include <unistd.h>

#include <dirent.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>

#include "fuzz_common.h"
#include "grpc_h2.h"

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

std::unique_ptr<GrpcServer> g_srv;
std::shared_ptr<DeviceTable> g_table;

void verifier() {  // runs for the whole fuzzing session
  uint64_t n = 0;
  for (;;) {
    for (auto& job : g_table->pop_prestart(50)) {
      ++n;
      if (n % 3 == 2) std::this_thread::sleep_for(std::chrono::milliseconds(2));
      g_table->complete_prestart(job.id, n % 3 != 1, n % 3 == 1 ? "injected canary failure" : "");
    }
  }
}
std::string g_path;
uint64_t g_iter = 0;

const char kPreface[] = "PRI * HTTP/2.0\r\n\r\nSM\r\n\r\n";

std::string client_prefix() {
  std::string o(kPreface, 24);
  fuzzutil::h2_frame(&o, 0x4, 0, 0, "");  // empty SETTINGS
  return o;
}

bool write_all(int fd, const char* p, size_t n) {
  while (n > 0) {
    const ssize_t w = send(fd, p, n, MSG_NOSIGNAL);
    if (w < 0 && errno == EINTR) continue;
    if (w <= 0) return false;  // the server closed early (GOAWAY): fine
    p += w;
    n -= static_cast<size_t>(w);
  }
  return true;
}

void one_connection(const uint8_t* data, size_t size) {
  const int fd = socket(AF_UNIX, SOCK_STREAM | SOCK_CLOEXEC, 0);
  struct sockaddr_un addr {};
  addr.sun_family = AF_UNIX;
  std::memcpy(addr.sun_path, g_path.c_str(), g_path.size() + 1);
  if (!fuzzutil::connect_retry(fd, reinterpret_cast<sockaddr*>(&addr), sizeof(addr))) {
    std::fprintf(stderr, "connect failed: %s\n", std::strerror(errno));
    std::abort();
  }
  const std::string pre = client_prefix();
  if (write_all(fd, pre.data(), pre.size())) write_all(fd, reinterpret_cast<const char*>(data), size);
  shutdown(fd, SHUT_WR);
  if (!fuzzutil::drain_until_close(fd, nullptr)) {
    std::fprintf(stderr, "server did not close a half-closed connection within 5 s\n");
    std::abort();
  }
  close(fd);
}

void liveness_check() {
  H2Client c(g_path, 5.0);
  std::string resp, msg;
  const int st = c.unary("/v1beta1.DevicePlugin/Allocate", fuzzutil::alloc_req({{"gpu2-xcp3"}}), &resp, &msg);
  if (st != 0 || resp.empty()) {
    std::fprintf(stderr, "liveness Allocate failed: status %d %s\n", st, msg.c_str());
    std::abort();
  }
}

}  // namespace

extern "C" int LLVMFuzzerInitialize(int*, char***) {
  if (const char* dir = fuzzutil::seed_dir()) {
    using fuzzutil::h2_call;
    fuzzutil::write_seed(dir, "allocate", h2_call(1, "/v1beta1.DevicePlugin/Allocate",
                                                  fuzzutil::alloc_req({{"gpu0-xcp0", "gpu0-xcp1"}})));
    fuzzutil::write_seed(dir, "preferred_huffman",
                         h2_call(1, "/v1beta1.DevicePlugin/GetPreferredAllocation",
                                 fuzzutil::preferred_req({"gpu1-xcp0", "gpu1-xcp1", "gpu3-xcp2"}, {}, 2), true));
    std::string two = h2_call(1, "/v1beta1.DevicePlugin/GetDevicePluginOptions", "") +
                      h2_call(3, "/v1beta1.DevicePlugin/ListAndWatch", "");
    fuzzutil::h2_frame(&two, 0x8, 0, 3, std::string("\x00\x01\x00\x00", 4));  // stream WINDOW_UPDATE
    fuzzutil::h2_frame(&two, 0x6, 0, 0, "12345678");                          // PING
    fuzzutil::write_seed(dir, "options_law_ping", two);
    // HEADERS split across CONTINUATION, padded DATA, then RST_STREAM
    std::string cont;
    const std::string hb = fuzzutil::grpc_headers("/v1beta1.DevicePlugin/PreStartContainer", false);
    fuzzutil::h2_frame(&cont, 0x1, 0x0, 5, hb.substr(0, 7));
    fuzzutil::h2_frame(&cont, 0x9, 0x4, 5, hb.substr(7));
    fuzzutil::h2_frame(&cont, 0x0, 0x9, 5, std::string("\x02", 1) + fuzzutil::grpc_body("") + "pp");
    fuzzutil::h2_frame(&cont, 0x3, 0, 5, std::string(4, '\0'));
    fuzzutil::write_seed(dir, "continuation_padded", cont);
    // PreStartContainer answered asynchronously, interleaved with an Allocate and a reset
    std::string pre = h2_call(1, "/v1beta1.DevicePlugin/PreStartContainer",
                              fuzzutil::alloc_req({{"gpu4-xcp1", "gpu4-xcp2"}}).substr(2)) +
                      h2_call(3, "/v1beta1.DevicePlugin/Allocate", fuzzutil::alloc_req({{"gpu0-xcp0"}})) +
                      h2_call(5, "/v1beta1.DevicePlugin/PreStartContainer", "");
    fuzzutil::h2_frame(&pre, 0x3, 0, 5, std::string(4, '\0'));
    fuzzutil::write_seed(dir, "prestart_async", pre);
    std::exit(0);
  }
  char tmpl[] = "/tmp/fuzz-grpc-XXXXXX";
  const char* dir = mkdtemp(tmpl);
  if (!dir) std::abort();
  g_path = std::string(dir) + "/plugin.sock";
  g_srv = std::make_unique<GrpcServer>(g_path, 2);
  g_table = fuzzutil::make_table(8, 8, 0, true);
  g_srv->set_table(g_table);
  g_srv->start();
  std::thread(verifier).detach();
  liveness_check();
  return 0;
}

extern "C" int LLVMFuzzerTestOneInput(const uint8_t* data, size_t size) {
  one_connection(data, size);
  if ((++g_iter & 255) == 0) {
    liveness_check();
    check_fds();
  }
  return 0;
}
