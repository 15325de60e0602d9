#include "loadgen.h"

#include <arpa/inet.h>
#include <errno.h>
#include <netdb.h>
#include <netinet/in.h>
#include <fcntl.h>
#include <sched.h>
#include <netinet/tcp.h>
#include <sys/epoll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cstring>
#include <mutex>
#include <stdexcept>
#include <thread>

#include "backend.h"
#include "fixture_backend.h"
#include "grpc_h2.h"
#include "httpd.h"
#include "telemetry.h"

namespace amdgpu_dp {

namespace {

int tcp_connect(const std::string& host, int port) {
  struct addrinfo hints {};
  hints.ai_family = AF_UNSPEC;
  hints.ai_socktype = SOCK_STREAM;
  struct addrinfo* res = nullptr;
  if (getaddrinfo(host.c_str(), std::to_string(port).c_str(), &hints, &res) != 0) return -1;
  int fd = -1;
  for (auto* ai = res; ai; ai = ai->ai_next) {
    fd = socket(ai->ai_family, ai->ai_socktype | SOCK_CLOEXEC, ai->ai_protocol);
    if (fd < 0) continue;
    if (connect(fd, ai->ai_addr, ai->ai_addrlen) == 0) break;
    close(fd);
    fd = -1;
  }
  freeaddrinfo(res);
  if (fd >= 0) {
    int one = 1;
    setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
  }
  return fd;
}

// Reads one HTTP/1.1 response (Content-Length framed) from fd; `buf` keeps leftovers.
bool read_response(int fd, std::string* buf, size_t* body_len, int* status) {
  char tmp[65536];
  for (;;) {
    const size_t he = buf->find("\r\n\r\n");
    if (he != std::string::npos) {
      *status = std::atoi(buf->c_str() + 9);
      size_t cl = 0;
      const size_t p = buf->find("Content-Length:");
      if (p != std::string::npos && p < he) cl = std::strtoull(buf->c_str() + p + 15, nullptr, 10);
      if (buf->size() >= he + 4 + cl) {
        *body_len = cl;
        buf->erase(0, he + 4 + cl);
        return true;
      }
    }
    const ssize_t r = recv(fd, tmp, sizeof(tmp), 0);
    if (r <= 0) {
      if (r < 0 && errno == EINTR) continue;
      return false;
    }
    buf->append(tmp, static_cast<size_t>(r));
  }
}

}  // namespace

LoadResult http_load(const std::string& host, int port, const std::string& path, int conns, double duration_s,
                     double target_rps, bool accept_gzip) {
  LoadResult total;
  std::mutex mu;
  std::vector<std::thread> ts;
  const int64_t t0 = mono_ns() + 2000000;  // common start 2 ms out
  const int64_t t_end = t0 + static_cast<int64_t>(duration_s * 1e9);
  const std::string req = "GET " + path + " HTTP/1.1\r\nHost: " + host + "\r\nUser-Agent: amdgpu-dp-loadgen\r\n" +
                          (accept_gzip ? "Accept-Encoding: gzip\r\n" : "") + "\r\n";
  for (int c = 0; c < conns; ++c) {
    ts.emplace_back([&, c] {
      LoadResult r;
      int fd = tcp_connect(host, port);
      std::string buf;
      // open loop: this connection's requests are scheduled every conns/target_rps seconds
      const double interval_ns = target_rps > 0 ? 1e9 * conns / target_rps : 0;
      int64_t next = t0 + static_cast<int64_t>(interval_ns * c / std::max(1, conns));
      while (mono_ns() < t0) {
      }
      for (;;) {
        int64_t sched = mono_ns();
        if (interval_ns > 0) {
          // sleep until ~150 us before the slot, then spin: a sleep alone wakes up to one
          // timer slack (50 us) late, and the latency is counted from the slot (open loop)
          for (int64_t now = mono_ns(); now < next; now = mono_ns()) {
            if (next - now > 200000) std::this_thread::sleep_for(std::chrono::nanoseconds(next - now - 150000));
            else cpu_relax();
          }
          sched = next;
          next += static_cast<int64_t>(interval_ns);
        }
        if (sched >= t_end) break;
        if (fd < 0) fd = tcp_connect(host, port);
        size_t body = 0;
        int status = 0;
        bool ok = fd >= 0 && send(fd, req.data(), req.size(), MSG_NOSIGNAL) == static_cast<ssize_t>(req.size()) &&
                  read_response(fd, &buf, &body, &status) && status == 200;
        const int64_t done = mono_ns();
        if (ok) {
          ++r.ok;
          r.bytes += body;
          r.latencies_s.push_back((done - sched) * 1e-9);
        } else {
          ++r.errors;
          if (fd >= 0) close(fd);
          fd = -1;
          buf.clear();
        }
      }
      if (fd >= 0) close(fd);
      std::lock_guard<std::mutex> lk(mu);
      total.ok += r.ok;
      total.errors += r.errors;
      total.bytes += r.bytes;
      total.latencies_s.insert(total.latencies_s.end(), r.latencies_s.begin(), r.latencies_s.end());
    });
  }
  for (auto& t : ts) t.join();
  total.elapsed_s = duration_s;  // every connection issues requests over [t0, t_end)
  return total;
}

std::vector<double> render_bench(std::shared_ptr<Exporter> ex, std::shared_ptr<HttpServer> http, int threads,
                                 int iters) {
  if (!ex || threads < 1 || threads > 64 || iters < 1) throw std::invalid_argument("render_bench: bad arguments");
  std::vector<double> out(static_cast<size_t>(threads), 0.0);
  std::atomic<int> ready{0};
  std::vector<std::thread> ts;
  for (int t = 0; t < threads; ++t)
    ts.emplace_back([&, t] {
      std::string buf;
      ready.fetch_add(1);
      while (ready.load() < threads) {
      }
      const int64_t t0 = mono_ns();
      Exposition e;  // reused like the HTTP worker's
      for (int i = 0; i < iters; ++i) {
        buf.clear();
        e.clear();
        ex->render(&e);
        buf.append(256, ' ');  // the response header's share
        e.append_to(&buf);
        if (http) http->render_http_metrics(&buf);
      }
      out[static_cast<size_t>(t)] = static_cast<double>(mono_ns() - t0) / iters;
    });
  for (auto& t : ts) t.join();
  return out;
}

LoadResult grpc_load(const std::string& socket_path, const std::string& method, const std::string& req, int conns,
                     double duration_s) {
  LoadResult total;
  std::mutex mu;
  std::vector<std::thread> ts;
  const int64_t t0 = mono_ns() + 2000000;
  const int64_t t_end = t0 + static_cast<int64_t>(duration_s * 1e9);
  for (int c = 0; c < conns; ++c) {
    ts.emplace_back([&] {
      LoadResult r;
      try {
        H2Client cl(socket_path);
        std::string resp, msg;
        while (mono_ns() < t0) {
        }
        for (;;) {
          const int64_t s = mono_ns();
          if (s >= t_end) break;
          const int st = cl.unary(method, req, &resp, &msg);
          const int64_t e = mono_ns();
          if (st == 0) {
            ++r.ok;
            r.bytes += resp.size();
            r.latencies_s.push_back((e - s) * 1e-9);
          } else {
            ++r.errors;
          }
        }
      } catch (const std::exception&) {
        ++r.errors;
      }
      std::lock_guard<std::mutex> lk(mu);
      total.ok += r.ok;
      total.errors += r.errors;
      total.bytes += r.bytes;
      total.latencies_s.insert(total.latencies_s.end(), r.latencies_s.begin(), r.latencies_s.end());
    });
  }
  for (auto& t : ts) t.join();
  total.elapsed_s = duration_s;
  return total;
}

namespace {

// A connected loopback TCP pair (client, server), both with TCP_NODELAY like the
// loadgen's and the HTTP server's sockets.
bool tcp_pair(int sv[2]) {
  const int lfd = socket(AF_INET, SOCK_STREAM | SOCK_CLOEXEC, 0);
  if (lfd < 0) return false;
  struct sockaddr_in a {};
  a.sin_family = AF_INET;
  a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
  socklen_t al = sizeof(a);
  bool ok = bind(lfd, reinterpret_cast<sockaddr*>(&a), sizeof(a)) == 0 && listen(lfd, 1) == 0 &&
            getsockname(lfd, reinterpret_cast<sockaddr*>(&a), &al) == 0;
  sv[0] = ok ? socket(AF_INET, SOCK_STREAM | SOCK_CLOEXEC, 0) : -1;
  ok = ok && sv[0] >= 0 && connect(sv[0], reinterpret_cast<sockaddr*>(&a), sizeof(a)) == 0;
  sv[1] = ok ? accept4(lfd, nullptr, nullptr, SOCK_CLOEXEC) : -1;
  close(lfd);
  if (!ok || sv[1] < 0) {
    if (sv[0] >= 0) close(sv[0]);
    return false;
  }
  int one = 1;
  setsockopt(sv[0], IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
  setsockopt(sv[1], IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
  return true;
}

}  // namespace

namespace {

// Pins the calling thread to `cpu` (no-op for cpu < 0); the mask it had goes to *saved.
bool pin_self(int cpu, cpu_set_t* saved) {
  if (cpu < 0) return true;
  if (saved && sched_getaffinity(0, sizeof(*saved), saved) != 0) return false;
  cpu_set_t one;
  CPU_ZERO(&one);
  CPU_SET(cpu, &one);
  return sched_setaffinity(0, sizeof(one), &one) == 0;
}

}  // namespace

double core_ghz(int64_t iters, int reps) {
  if (iters < 1000 || reps < 1) throw std::invalid_argument("core_ghz: bad arguments");
  double best = 0;
  for (int r = 0; r < reps; ++r) {
    uint64_t x = static_cast<uint64_t>(r) + 1;
    const int64_t t0 = mono_ns();
    for (int64_t i = 0; i < iters; ++i) asm volatile("add $1, %0" : "+r"(x));  // 1 cycle, dependent
    const int64_t dt = mono_ns() - t0;
    if (dt > 0) best = std::max(best, static_cast<double>(iters) / static_cast<double>(dt));
  }
  return best;
}

std::vector<double> uds_pingpong(int n, int warmup, int req_bytes, int resp_bytes, bool server_spin, bool tcp,
                                 int gap_us, int client_cpu, int server_cpu, bool peek) {
  if (n < 0 || warmup < 0 || gap_us < 0 || req_bytes <= 0 || resp_bytes <= 0 || req_bytes > (1 << 20) || resp_bytes > (4 << 20))
    throw std::invalid_argument("uds_pingpong: bad sizes");
  if (client_cpu >= CPU_SETSIZE || server_cpu >= CPU_SETSIZE) throw std::invalid_argument("uds_pingpong: bad cpu");
  int sv[2];
  if (tcp ? !tcp_pair(sv) : socketpair(AF_UNIX, SOCK_STREAM | SOCK_CLOEXEC, 0, sv) != 0)
    throw std::runtime_error(std::string(tcp ? "tcp loopback pair: " : "socketpair: ") + strerror(errno));
  const int cfd = sv[0], sfd = sv[1];
  fcntl(sfd, F_SETFL, fcntl(sfd, F_GETFL) | O_NONBLOCK);
  struct timeval tv {5, 0};  // a dead server thread ends the client's recv, not the process
  setsockopt(cfd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof(tv));
  if (peek) {
    int zero = 0;
    if (tcp || setsockopt(sfd, SOL_SOCKET, SO_PEEK_OFF, &zero, sizeof(zero)) != 0) peek = false;
  }
  const int ep = epoll_create1(EPOLL_CLOEXEC);
  struct epoll_event ev {};
  ev.events = EPOLLIN | EPOLLRDHUP;
  ev.data.fd = sfd;
  epoll_ctl(ep, EPOLL_CTL_ADD, sfd, &ev);
  std::atomic<int> server_pinned{-1};
  std::thread server([&] {  // the plugin server's syscall pattern: epoll_wait, recv, send
    server_pinned.store(pin_self(server_cpu, nullptr) ? 1 : 0);
    std::vector<char> in(static_cast<size_t>(req_bytes) + 65536), out(static_cast<size_t>(resp_bytes), 'r');
    std::vector<char> sink(65536);
    size_t have = 0;
    epoll_event evs[4];
    for (;;) {
      // server_spin: the busy-poll worker (grpc.busyPollUs) never sleeps between requests
      const int k = epoll_wait(ep, evs, 4, server_spin ? 0 : 1000);
      if (k == 0 && server_spin) cpu_relax();
      if (k < 0 && errno != EINTR) return;
      if (k <= 0) continue;
      bool closed = false;
      size_t peeked = 0;
      for (;;) {
        const ssize_t r = recv(sfd, in.data() + have, in.size() - have, peek ? MSG_PEEK : 0);
        if (r > 0) {
          have += static_cast<size_t>(r);
          peeked += peek ? static_cast<size_t>(r) : 0;
          if (have >= in.size()) break;
        } else if (r < 0 && errno == EINTR) {
          continue;
        } else {
          if (r == 0 || errno != EAGAIN) closed = true;
          break;
        }
      }
      while (have >= static_cast<size_t>(req_bytes)) {
        have -= static_cast<size_t>(req_bytes);
        size_t off = 0;
        while (off < out.size()) {
          const ssize_t w = send(sfd, out.data() + off, out.size() - off, MSG_NOSIGNAL);
          if (w > 0)
            off += static_cast<size_t>(w);
          else if (w < 0 && (errno == EAGAIN || errno == EINTR))
            continue;
          else
            return;
        }
      }
      while (peeked > 0) {  // consume what was peeked, after the answer went out
        const ssize_t r = recv(sfd, sink.data(), std::min(peeked, sink.size()), MSG_DONTWAIT);
        if (r > 0) peeked -= static_cast<size_t>(r);
        else if (r < 0 && errno == EINTR) continue;
        else break;
      }
      if (closed) return;
    }
  });
  cpu_set_t saved;
  CPU_ZERO(&saved);
  const bool client_pinned = pin_self(client_cpu, &saved);
  while (server_pinned.load() < 0) std::this_thread::yield();
  std::vector<double> lat;
  lat.reserve(static_cast<size_t>(n));
  const std::string req(static_cast<size_t>(req_bytes), 'q');
  std::vector<char> buf(static_cast<size_t>(resp_bytes));
  bool failed = !client_pinned || server_pinned.load() == 0;
  for (int i = 0; i < n + warmup && !failed; ++i) {
    // gap_us > 0: both threads idle between exchanges, as the cold Allocate's do
    if (gap_us > 0) std::this_thread::sleep_for(std::chrono::microseconds(gap_us));
    const int64_t t0 = mono_ns();
    if (send(cfd, req.data(), req.size(), MSG_NOSIGNAL) != static_cast<ssize_t>(req.size())) {
      failed = true;
      break;
    }
    size_t got = 0;
    while (got < buf.size()) {
      const ssize_t r = recv(cfd, buf.data() + got, buf.size() - got, 0);
      if (r > 0) {
        got += static_cast<size_t>(r);
      } else if (r < 0 && errno == EINTR) {
        continue;
      } else {
        failed = true;
        break;
      }
    }
    if (i >= warmup && !failed) lat.push_back((mono_ns() - t0) * 1e-9);
  }
  shutdown(cfd, SHUT_RDWR);  // the server sees EOF and leaves its loop
  server.join();
  if (client_cpu >= 0 && client_pinned) sched_setaffinity(0, sizeof(saved), &saved);
  close(cfd);
  close(sfd);
  close(ep);
  if (failed) throw std::runtime_error(!client_pinned || server_pinned.load() == 0 ? "uds_pingpong: cannot pin to the CPU"
                                                                                    : "uds_pingpong: socket error");
  return lat;
}

std::vector<double> uds_pingpong_batched(int batches, int batch, int batch_gap_us, int req_bytes, int resp_bytes,
                                         int server_poll_us) {
  if (batches <= 0 || batch <= 0 || batch_gap_us < 0 || server_poll_us < 0 || req_bytes <= 0 || resp_bytes <= 0 ||
      req_bytes > (1 << 20) || resp_bytes > (4 << 20))
    throw std::invalid_argument("uds_pingpong_batched: bad arguments");
  int sv[2];
  if (socketpair(AF_UNIX, SOCK_STREAM | SOCK_CLOEXEC, 0, sv) != 0)
    throw std::runtime_error(std::string("socketpair: ") + strerror(errno));
  const int cfd = sv[0], sfd = sv[1];
  fcntl(sfd, F_SETFL, fcntl(sfd, F_GETFL) | O_NONBLOCK);
  struct timeval tv {5, 0};
  setsockopt(cfd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof(tv));
  const int ep = epoll_create1(EPOLL_CLOEXEC);
  struct epoll_event ev {};
  ev.events = EPOLLIN | EPOLLRDHUP;
  ev.data.fd = sfd;
  epoll_ctl(ep, EPOLL_CTL_ADD, sfd, &ev);
  // the plugin worker's policy: after a request, poll for server_poll_us, then sleep in
  // epoll_wait (100 ms timeouts) until the next one
  std::thread server([&] {
    std::vector<char> in(static_cast<size_t>(req_bytes) + 65536), out(static_cast<size_t>(resp_bytes), 'r');
    size_t have = 0;
    epoll_event evs[4];
    int64_t poll_until = 0;
    for (;;) {
      const bool polling = poll_until != 0;
      const int k = epoll_wait(ep, evs, 4, polling ? 0 : 100);
      if (k == 0 && polling) {
        if (mono_ns() >= poll_until) poll_until = 0;
        else cpu_relax();
        continue;
      }
      if (k < 0 && errno != EINTR) return;
      if (k <= 0) continue;
      bool closed = false;
      for (;;) {
        const ssize_t r = recv(sfd, in.data() + have, in.size() - have, 0);
        if (r > 0) {
          have += static_cast<size_t>(r);
          if (have >= in.size()) break;
        } else if (r < 0 && errno == EINTR) {
          continue;
        } else {
          if (r == 0 || errno != EAGAIN) closed = true;
          break;
        }
      }
      while (have >= static_cast<size_t>(req_bytes)) {
        have -= static_cast<size_t>(req_bytes);
        size_t off = 0;
        while (off < out.size()) {
          const ssize_t w = send(sfd, out.data() + off, out.size() - off, MSG_NOSIGNAL);
          if (w > 0)
            off += static_cast<size_t>(w);
          else if (w < 0 && (errno == EAGAIN || errno == EINTR))
            continue;
          else
            return;
        }
      }
      if (server_poll_us > 0) poll_until = mono_ns() + static_cast<int64_t>(server_poll_us) * 1000;
      if (closed) return;
    }
  });
  std::vector<double> lat;
  lat.reserve(static_cast<size_t>(batches) * batch);
  const std::string req(static_cast<size_t>(req_bytes), 'q');
  std::vector<char> buf(static_cast<size_t>(resp_bytes));
  bool failed = false;
  for (int b = 0; b < batches && !failed; ++b) {
    std::this_thread::sleep_for(std::chrono::microseconds(batch_gap_us));
    for (int i = 0; i < batch && !failed; ++i) {
      const int64_t t0 = mono_ns();
      if (send(cfd, req.data(), req.size(), MSG_NOSIGNAL) != static_cast<ssize_t>(req.size())) {
        failed = true;
        break;
      }
      size_t got = 0;
      while (got < buf.size()) {
        const ssize_t r = recv(cfd, buf.data() + got, buf.size() - got, 0);
        if (r > 0) {
          got += static_cast<size_t>(r);
        } else if (r < 0 && errno == EINTR) {
          continue;
        } else {
          failed = true;
          break;
        }
      }
      if (!failed) lat.push_back((mono_ns() - t0) * 1e-9);
    }
  }
  shutdown(cfd, SHUT_RDWR);
  server.join();
  close(cfd);
  close(sfd);
  close(ep);
  if (failed) throw std::runtime_error("uds_pingpong_batched: socket error");
  return lat;
}

UdsPinger::UdsPinger(int req_bytes, int resp_bytes, int server_timeout_ms)
    : req_(static_cast<size_t>(req_bytes), 'q'), buf_(static_cast<size_t>(resp_bytes)) {
  if (req_bytes <= 0 || resp_bytes <= 0 || req_bytes > (1 << 20) || resp_bytes > (4 << 20) || server_timeout_ms < 0)
    throw std::invalid_argument("UdsPinger: bad sizes");
  int sv[2];
  if (socketpair(AF_UNIX, SOCK_STREAM | SOCK_CLOEXEC, 0, sv) != 0)
    throw std::runtime_error(std::string("socketpair: ") + strerror(errno));
  cfd_ = sv[0];
  sfd_ = sv[1];
  fcntl(sfd_, F_SETFL, fcntl(sfd_, F_GETFL) | O_NONBLOCK);
  struct timeval tv {5, 0};
  setsockopt(cfd_, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof(tv));
  ep_ = epoll_create1(EPOLL_CLOEXEC);
  struct epoll_event ev {};
  ev.events = EPOLLIN | EPOLLRDHUP;
  ev.data.fd = sfd_;
  epoll_ctl(ep_, EPOLL_CTL_ADD, sfd_, &ev);
  server_ = std::thread([this, req_bytes, resp_bytes, server_timeout_ms] {
    std::vector<char> in(static_cast<size_t>(req_bytes) + 65536), out(static_cast<size_t>(resp_bytes), 'r');
    size_t have = 0;
    epoll_event evs[4];
    for (;;) {
      const int k = epoll_wait(ep_, evs, 4, server_timeout_ms);
      if (k < 0 && errno != EINTR) return;
      if (k <= 0) continue;
      bool closed = false;
      for (;;) {
        const ssize_t r = recv(sfd_, in.data() + have, in.size() - have, 0);
        if (r > 0) {
          have += static_cast<size_t>(r);
          if (have >= in.size()) break;
        } else if (r < 0 && errno == EINTR) {
          continue;
        } else {
          if (r == 0 || errno != EAGAIN) closed = true;
          break;
        }
      }
      while (have >= static_cast<size_t>(req_bytes)) {
        have -= static_cast<size_t>(req_bytes);
        size_t off = 0;
        while (off < out.size()) {
          const ssize_t w = send(sfd_, out.data() + off, out.size() - off, MSG_NOSIGNAL);
          if (w > 0)
            off += static_cast<size_t>(w);
          else if (w < 0 && (errno == EAGAIN || errno == EINTR))
            continue;
          else
            return;
        }
      }
      if (closed) return;
    }
  });
}

UdsPinger::~UdsPinger() {
  shutdown(cfd_, SHUT_RDWR);
  if (server_.joinable()) server_.join();
  close(cfd_);
  close(sfd_);
  close(ep_);
}

double UdsPinger::once() {
  const int64_t t0 = mono_ns();
  if (send(cfd_, req_.data(), req_.size(), MSG_NOSIGNAL) != static_cast<ssize_t>(req_.size()))
    throw std::runtime_error("UdsPinger: send failed");
  size_t got = 0;
  while (got < buf_.size()) {
    const ssize_t r = recv(cfd_, buf_.data() + got, buf_.size() - got, 0);
    if (r > 0) got += static_cast<size_t>(r);
    else if (r < 0 && errno == EINTR) continue;
    else throw std::runtime_error("UdsPinger: recv failed");
  }
  return (mono_ns() - t0) * 1e-9;
}

namespace {

int count_unhealthy(const std::string& law) {
  int n = 0;
  for (size_t p = law.find("Unhealthy"); p != std::string::npos; p = law.find("Unhealthy", p + 9)) ++n;
  return n;
}

}  // namespace

std::vector<std::pair<int, double>> health_propagation(FixtureBackend& be, const std::string& socket_path, int gpu,
                                                       int events) {
  H2Client c(socket_path);
  c.open_stream("/v1beta1.DevicePlugin/ListAndWatch", "");
  std::string msg;
  if (c.next_stream_message(&msg, 10000) != 0) throw std::runtime_error("ListAndWatch ended");
  const int base = count_unhealthy(msg);
  std::vector<std::pair<int, double>> out;
  for (int i = 0; i < events; ++i) {
    const bool down = i % 2 == 0;
    HwEvent e;
    e.kind = down ? kEvtPreReset : kEvtPostReset;
    e.gpu = gpu;
    e.message = "propagation bench";
    const int64_t t0 = mono_ns();
    be.inject_event(e);
    for (;;) {
      if (c.next_stream_message(&msg, 10000) != 0) throw std::runtime_error("ListAndWatch ended");
      if ((count_unhealthy(msg) > base) == down) break;
    }
    out.emplace_back(down ? 1 : 0, (mono_ns() - t0) * 1e-9);
  }
  return out;
}

std::vector<double> h2_bench_unary(const std::string& socket_path, const std::string& path, const std::string& req,
                                   int n) {
  H2Client c(socket_path);
  std::vector<double> out;
  out.reserve(static_cast<size_t>(n));
  std::string resp, msg;
  for (int i = 0; i < n; ++i) {
    const int64_t t0 = mono_ns();
    const int st = c.unary(path, req, &resp, &msg);
    out.push_back((mono_ns() - t0) * 1e-9);
    if (st != 0) throw std::runtime_error("h2_bench_unary: grpc-status " + std::to_string(st) + ": " + msg);
  }
  return out;
}

}  // namespace amdgpu_dp
