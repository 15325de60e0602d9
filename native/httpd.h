// Native HTTP/1.1 ops server: GET / /metrics /health /restart /ready /health/clear.
//
// Reference: echo v4 server (server/server.go:35-69) with middleware chain
// Recover -> Cros -> Logger -> MetricsMiddleware (server/server.go:39-43,
// middleware/echo_metric.go:78-124) and routes from router/api.go:27-54.
// Wire behaviour kept byte-compatible: JSON envelope {"code":0,"data":..,"msg":"success"},
// echo's error bodies {"message":"Not Found"}, CORS headers, OPTIONS -> 200, and the
// echo_http_requests_total / echo_http_request_duration_seconds families with the same
// labels and buckets.  Implementation: epoll workers sharing one listening socket
// (EPOLLEXCLUSIVE), keep-alive + pipelining, lock-free metric atomics, buffered access
// log, and /metrics served from the exporter's pre-rendered bytes without the GIL.
#pragma once

#include <atomic>
#include <condition_variable>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "metrics.h"
#include "telemetry.h"

namespace amdgpu_dp {

struct HttpConfig {
  std::string host = "0.0.0.0";
  int port = 9100;
  int threads = 2;
  bool access_log = true;
  int idle_timeout_s = 60;
  int read_timeout_s = 30;
  int busy_poll_us = 0;  // keep polling this long after a request before sleeping (0 = off)
  // GET /restart only from a loopback peer (others get 403); off = the reference's
  // behaviour, where anyone who reaches the port can reload the plugins
  bool restart_local_only = false;
  // GET /health/clear only from a loopback peer (others get 403)
  bool clear_local_only = true;
  std::string version = "0.1.0";
};

class HttpServer {
 public:
  // echo_http_* label dimensions: methods, handlers (routes), status classes
  static constexpr int kMethods = 8;
  static constexpr int kHandlers = 7;
  static constexpr int kStatus = 5;
  HttpServer(HttpConfig cfg, std::shared_ptr<Exporter> exporter);
  ~HttpServer();
  // Returns the bound port (cfg.port may be 0 = ephemeral).  Throws on bind failure.
  int start();
  void stop();
  bool running() const { return running_.load(); }
  int port() const { return bound_port_; }
  void set_restart_hook(std::function<void()> hook);
  // GET /health/clear?<query>: an operator drops a GPU's health latches.  The hook gets
  // the raw query string and returns (HTTP status, JSON body).
  using ClearHook = std::function<std::pair<int, std::string>(const std::string& query)>;
  void set_clear_hook(ClearHook hook);
  // GET /ready answers 200 while ready, else 503 with the reason (the plugin manager
  // pushes its registration state here)
  void set_ready(bool ready, const std::string& reason);
  uint64_t requests_total() const { return requests_.load(); }
  uint64_t shed_connections() const { return shed_.load(); }  // closed at accept: out of fds
  std::vector<int> worker_connections() const;  // connections owned per worker thread
  // Renders the echo_http_* families (exposed for tests).
  void render_http_metrics(std::string* out) const;

  // Internal, public for the worker implementation
  struct Worker;

 private:
  friend struct Worker;
  // direct_fd >= 0: nothing is queued on that connection, so a /metrics answer may go
  // to the socket straight from the exposition's cached segments (one sendmsg, no copy
  // into *out); what the socket does not take is appended to *out as usual.
  void handle(const std::string& method, const std::string& path, const std::string& origin, bool keep_alive,
              bool http10, std::string* out, int* status_out, size_t* body_bytes_out, bool gzip_ok = false,
              bool peer_local = true, int direct_fd = -1, const std::string& query = std::string());
  void record(int method_idx, int handler_idx, int status, double seconds);
  void log_access(const std::string& remote, const std::string& host, const std::string& method,
                  const std::string& uri, const std::string& ua, int status, double seconds, size_t bytes_in,
                  size_t bytes_out);
  void flush_log();

  HttpConfig cfg_;
  std::shared_ptr<Exporter> exporter_;
  std::function<void()> restart_hook_;
  ClearHook clear_hook_;
  std::mutex hook_mu_;
  bool ready_ = true;  // GET /ready (guarded by hook_mu_)
  std::string not_ready_reason_;
  int listen_fd_ = -1;
  int bound_port_ = 0;
  std::atomic<bool> running_{false};
  std::atomic<bool> stop_{false};
  std::vector<std::thread> threads_;
  std::vector<std::unique_ptr<Worker>> workers_;
  std::thread log_thread_;
  ShardedCounter requests_;
  ShardedCounter shed_;

  // echo_http_requests_total per (status class, method, handler), one copy per thread
  // shard (metrics.h) so that concurrent workers never write the same line
  struct alignas(64) CountShard {
    std::atomic<uint64_t> c[kStatus][kMethods][kHandlers];
  };
  std::unique_ptr<CountShard[]> counts_;
  // bit m * kHandlers + h: (method, handler) seen at least once; a scrape walks only these
  // instead of every (status, method, handler) counter and every histogram
  std::atomic<uint64_t> used_mh_{0};
  std::unique_ptr<Histogram> hist_[kMethods][kHandlers];

  std::mutex log_mu_;
  std::condition_variable log_cv_;  // log_buf_ became non-empty, or stop
  std::string log_buf_;
  int stop_efd_ = -1;
};

}  // namespace amdgpu_dp
