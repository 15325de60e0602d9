// Load generators for the BASELINE.md measurement protocol.
//
//   http_load : N keep-alive HTTP/1.1 connections issuing GET <path>; closed-loop (max
//               rate) or open-loop at a fixed target rate, where latency is measured from
//               each request's *scheduled* send time (no coordinated omission).
//   grpc_load : N native HTTP/2 clients issuing unary calls, closed-loop.
#pragma once

#include <string>
#include <thread>
#include <vector>

#include <cstdint>
#include <string>
#include <memory>
#include <vector>

namespace amdgpu_dp {

struct LoadResult {
  uint64_t ok = 0;
  uint64_t errors = 0;
  uint64_t bytes = 0;
  double elapsed_s = 0;
  std::vector<double> latencies_s;  // one per completed request
};

LoadResult http_load(const std::string& host, int port, const std::string& path, int conns, double duration_s,
                     double target_rps, bool accept_gzip = false);

LoadResult grpc_load(const std::string& socket_path, const std::string& method, const std::string& req, int conns,
                     double duration_s);

// Speed-of-light reference for one unary RPC on a unix socket: a client thread and an
// epoll server thread exchange `req_bytes` / `resp_bytes` with exactly the syscalls the
// plugin's Allocate path makes (client send + blocking recv; server epoll_wait + recv +
// send) and no protocol work at all.  Per-round-trip latency in seconds, n samples after
// `warmup` untimed ones.  Allocate p50 minus this p50 is what HTTP/2 + HPACK + protobuf +
// the device table cost.  tcp=true: the same over a loopback TCP connection, the floor
// of one /metrics scrape of resp_bytes (what the kernel's copies and wake-ups cost).
// client_cpu / server_cpu >= 0 pin the two threads (the calling thread's own affinity is
// restored afterwards): the same exchange between two chosen CPUs - SMT siblings, two
// cores of one L3, two L3 domains - is what says what a placement costs on this host.
// peek: the server reads each request with MSG_PEEK and consumes it after its send (the
// plugin's grpc.peekReads): the bare exchange without the write-space wake-up of the client
// that consuming its data causes.
std::vector<double> uds_pingpong(int n, int warmup, int req_bytes, int resp_bytes, bool server_spin = false,
                                 bool tcp = false, int gap_us = 0, int client_cpu = -1, int server_cpu = -1,
                                 bool peek = false);

// Effective core clock of the calling thread, GHz: a chain of `iters` dependent integer
// adds (one per cycle on x86-64) timed with CLOCK_MONOTONIC; the best of `reps`.  Tells a
// box whose cores run at 2 GHz from one whose cores boost to 4+.
double core_ghz(int64_t iters = 20000000, int reps = 5);

// The same bare exchange, one at a time on demand: a persistent socket pair whose server
// thread sleeps in epoll_wait(timeout_ms) between exchanges the way the plugin's worker
// does (its loop wakes every 100 ms).  once() is one round trip, in seconds; interleaved
// with real RPCs after the same idle gap it gives each a paired floor
// (scripts/idle_probe.py).
class UdsPinger {
 public:
  UdsPinger(int req_bytes, int resp_bytes, int server_timeout_ms);
  ~UdsPinger();
  double once();

 private:
  int cfd_ = -1, sfd_ = -1, ep_ = -1;
  std::string req_;
  std::vector<char> buf_;
  std::thread server_;
};

class Exporter;
class HttpServer;

// What one /metrics response costs in user space, without sockets: `threads` threads
// each assemble `iters` expositions (Exporter::render + the HTTP server's echo_http_*
// families, appended to a reused buffer) concurrently.  Mean ns per exposition, per
// thread: if 4 threads take longer each than 1 does, the scrape path shares something.
std::vector<double> render_bench(std::shared_ptr<Exporter> ex, std::shared_ptr<HttpServer> http, int threads,
                                 int iters);

class FixtureBackend;

// Health propagation as a kubelet sees it: inject alternating PRE_RESET / POST_RESET
// events for `gpu` into a fixture backend and time each until a ListAndWatch message
// with the matching health arrives on a compiled watcher.  Runs without the GIL, so the
// Python side of the plugin is measured, not the measuring client.  Returns
// (1 = Unhealthy transition / 0 = Healthy, seconds) per event.
std::vector<std::pair<int, double>> health_propagation(FixtureBackend& be, const std::string& socket_path, int gpu,
                                                       int events);

// The bare exchange in the benchmark's rhythm: `batches` batches of `batch` back-to-back
// exchanges, `batch_gap_us` apart, to a server thread that polls for `server_poll_us`
// after each request and sleeps in epoll_wait otherwise (the plugin worker's policy):
// the host's own tail for the pattern bench.py times Allocate in.
std::vector<double> uds_pingpong_batched(int batches, int batch, int batch_gap_us, int req_bytes, int resp_bytes,
                                         int server_poll_us);

// n sequential unary calls on one connection; per-call latency in seconds.
std::vector<double> h2_bench_unary(const std::string& socket_path, const std::string& path, const std::string& req,
                                   int n);

}  // namespace amdgpu_dp
