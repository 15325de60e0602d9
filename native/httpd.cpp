#include "httpd.h"

#include <charconv>
#include <limits>

#include <pthread.h>

#include <arpa/inet.h>
#include <errno.h>
#include <fcntl.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/epoll.h>
#include <sys/eventfd.h>
#include <sys/socket.h>
#include <sys/uio.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <ctime>
#include <stdexcept>
#include <unordered_map>

namespace amdgpu_dp {

namespace {

const char* kMethodNames[] = {"GET", "POST", "PUT", "DELETE", "PATCH", "HEAD", "OPTIONS", "OTHER"};
const char* kHandlerNames[] = {"/", "/metrics", "/health", "/restart", "/ready", "/not-found", "/health/clear"};
const char* kStatusNames[] = {"1xx", "2xx", "3xx", "4xx", "5xx"};

int method_index(const std::string& m) {
  for (int i = 0; i < 7; ++i)
    if (m == kMethodNames[i]) return i;
  return 7;
}

int status_class(int status) {  // middleware/echo_metric.go:50-61
  if (status < 200) return 0;
  if (status < 300) return 1;
  if (status < 400) return 2;
  if (status < 500) return 3;
  return 4;
}

// a JSON string body (quotes, backslashes and control characters escaped)
void append_json_string_body(std::string* out, const std::string& s) {
  for (unsigned char c : s) {
    if (c == '"' || c == '\\') {
      out->push_back('\\');
      out->push_back(static_cast<char>(c));
    } else if (c < 0x20) {
      char buf[8];
      std::snprintf(buf, sizeof(buf), "\\u%04x", c);
      out->append(buf);
    } else {
      out->push_back(static_cast<char>(c));
    }
  }
}

const char* reason(int status) {
  switch (status) {
    case 200: return "OK";
    case 400: return "Bad Request";
    case 403: return "Forbidden";
    case 404: return "Not Found";
    case 405: return "Method Not Allowed";
    case 413: return "Request Entity Too Large";
    case 431: return "Request Header Fields Too Large";
    case 500: return "Internal Server Error";
    case 501: return "Not Implemented";
    case 503: return "Service Unavailable";
    default: return "Unknown";
  }
}

// echo_http_request_duration_seconds buckets (middleware/echo_metric.go:25-48)
std::vector<double> echo_buckets() {
  return {0.0005, 0.001, 0.002, 0.005, 0.01, 0.02, 0.05, 0.1, 0.2, 0.5, 1.0, 2.0, 5.0, 10.0, 15.0, 20.0, 30.0};
}

inline char lower_ascii(char c) { return c >= 'A' && c <= 'Z' ? static_cast<char>(c + ('a' - 'A')) : c; }

// header-name match against a lower-case literal (field names are ASCII, RFC 9110 5.1)
template <size_t N>
bool ieq(const char* a, size_t n, const char (&lower)[N]) {
  if (n != N - 1) return false;
  for (size_t i = 0; i < n; ++i)
    if (lower_ascii(a[i]) != lower[i]) return false;
  return true;
}

bool icontains(std::string_view h, std::string_view lower) {
  if (lower.size() > h.size()) return false;
  for (size_t i = 0; i + lower.size() <= h.size(); ++i) {
    size_t k = 0;
    while (k < lower.size() && lower_ascii(h[i + k]) == lower[k]) ++k;
    if (k == lower.size()) return true;
  }
  return false;
}

// promhttp's gzipAccepted: any comma-separated part equal to "gzip" or starting with
// "gzip;" (q-values are not weighed, as in the reference's client_golang v1.19).
bool accepts_gzip(std::string_view v) {
  size_t i = 0;
  while (i <= v.size()) {
    size_t j = v.find(',', i);
    if (j == std::string_view::npos) j = v.size();
    size_t a = i, b = j;
    while (a < b && (v[a] == ' ' || v[a] == '\t')) ++a;
    while (b > a && (v[b - 1] == ' ' || v[b - 1] == '\t')) --b;
    const std::string_view part = v.substr(a, b - a);
    if (part == "gzip" || part.substr(0, 5) == "gzip;") return true;
    i = j + 1;
  }
  return false;
}

std::string http_date() {
  char buf[64];
  time_t t = time(nullptr);
  struct tm tmv;
  gmtime_r(&t, &tmv);
  const size_t n = strftime(buf, sizeof(buf), "%a, %d %b %Y %H:%M:%S GMT", &tmv);
  return std::string(buf, n);
}

struct Conn {
  int fd = -1;
  std::string in;
  std::string out;
  size_t out_off = 0;
  int64_t last_ns = 0;
  std::string remote;
  bool local = false;  // the peer is on a loopback address
  bool close_after = false;
  bool want_out = false;
  bool want_in = true;
};

// Unsent response bytes above which a connection's further requests wait (a /metrics
// answer is up to ~100 KB; 4 MiB is dozens of pipelined scrapes).
constexpr size_t kMaxPendingOut = 4u << 20;
inline size_t backlog(const Conn* c) { return c->out.size() - c->out_off; }

}  // namespace

struct HttpServer::Worker {
  int ep = -1;
  std::unordered_map<int, std::unique_ptr<Conn>> conns;
  // the accepting worker hands each connection to the least-loaded worker (see
  // GrpcServer::Worker): concurrent scrapers are served in parallel, not queued on one
  std::mutex in_mu;
  std::vector<std::unique_ptr<Conn>> incoming;
  std::atomic<int> load{0};
};

HttpServer::HttpServer(HttpConfig cfg, std::shared_ptr<Exporter> exporter)
    : cfg_(std::move(cfg)), exporter_(std::move(exporter)) {
  counts_.reset(new CountShard[kMetricShards]);
  for (int k = 0; k < kMetricShards; ++k)
    for (auto& a : counts_[k].c)
      for (auto& b : a)
        for (auto& c : b) c.store(0, std::memory_order_relaxed);
  for (auto& row : hist_)
    for (auto& h : row) h = std::make_unique<Histogram>(echo_buckets());
}

HttpServer::~HttpServer() { stop(); }

void HttpServer::set_clear_hook(ClearHook hook) {
  std::lock_guard<std::mutex> lk(hook_mu_);
  clear_hook_ = std::move(hook);
}

void HttpServer::set_restart_hook(std::function<void()> hook) {
  std::lock_guard<std::mutex> lk(hook_mu_);
  restart_hook_ = std::move(hook);
}

void HttpServer::set_ready(bool ready, const std::string& reason) {
  std::lock_guard<std::mutex> lk(hook_mu_);
  ready_ = ready;
  not_ready_reason_ = ready ? std::string() : reason;
}

int HttpServer::start() {
  if (running_) return bound_port_;
  struct addrinfo hints {};
  hints.ai_family = AF_UNSPEC;
  hints.ai_socktype = SOCK_STREAM;
  hints.ai_flags = AI_PASSIVE | AI_NUMERICSERV;
  struct addrinfo* res = nullptr;
  const std::string port = std::to_string(cfg_.port);
  const char* host = cfg_.host.empty() ? nullptr : cfg_.host.c_str();
  if (getaddrinfo(host, port.c_str(), &hints, &res) != 0 || !res)
    throw std::runtime_error("httpd: cannot resolve listen address " + cfg_.host + ":" + port);
  int fd = -1;
  for (auto* ai = res; ai; ai = ai->ai_next) {
    fd = socket(ai->ai_family, ai->ai_socktype | SOCK_NONBLOCK | SOCK_CLOEXEC, ai->ai_protocol);
    if (fd < 0) continue;
    int one = 1;
    setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
    if (bind(fd, ai->ai_addr, ai->ai_addrlen) == 0 && listen(fd, 1024) == 0) break;
    close(fd);
    fd = -1;
  }
  freeaddrinfo(res);
  if (fd < 0) throw std::runtime_error("httpd: bind/listen failed on " + cfg_.host + ":" + port + ": " + strerror(errno));
  struct sockaddr_storage ss {};
  socklen_t sl = sizeof(ss);
  getsockname(fd, reinterpret_cast<sockaddr*>(&ss), &sl);
  bound_port_ = ntohs(ss.ss_family == AF_INET6 ? reinterpret_cast<sockaddr_in6*>(&ss)->sin6_port
                                               : reinterpret_cast<sockaddr_in*>(&ss)->sin_port);
  listen_fd_ = fd;
  stop_ = false;
  running_ = true;
  const int nthreads = std::max(1, cfg_.threads);
  // stop() writes this (never read: level-triggered, it wakes every worker at once), so the
  // workers can sleep 5 s at a time when no scraper is around
  stop_efd_ = eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);
  for (int t = 0; t < nthreads; ++t) {
    auto w = std::make_unique<Worker>();
    w->ep = epoll_create1(EPOLL_CLOEXEC);
    struct epoll_event ev {};
    ev.events = EPOLLIN | EPOLLEXCLUSIVE;
    ev.data.fd = listen_fd_;
    epoll_ctl(w->ep, EPOLL_CTL_ADD, listen_fd_, &ev);
    if (stop_efd_ >= 0) {
      struct epoll_event sev {};
      sev.events = EPOLLIN;
      sev.data.fd = stop_efd_;
      epoll_ctl(w->ep, EPOLL_CTL_ADD, stop_efd_, &sev);
    }
    workers_.push_back(std::move(w));
  }
  for (int t = 0; t < nthreads; ++t) {
    Worker* w = workers_[t].get();
    threads_.emplace_back([this, w, t] {
      pthread_setname_np(pthread_self(), ("dphttp-" + std::to_string(t)).c_str());
      foreground_thread();
      set_thread_shard(kMetricShards - 1 - static_cast<int>(t));
      std::vector<epoll_event> evs(128);
      char rbuf[16384];
      int spare = -1;  // reserve descriptor for accept_or_shed
      int64_t last_sweep = mono_ns();
      auto close_conn = [&](int cfd) {
        epoll_ctl(w->ep, EPOLL_CTL_DEL, cfd, nullptr);
        close(cfd);
        w->conns.erase(cfd);
        w->load.fetch_sub(1, std::memory_order_relaxed);
      };
      auto adopt = [&] {
        std::lock_guard<std::mutex> lk(w->in_mu);
        for (auto& c : w->incoming) {
          const int cfd = c->fd;
          w->conns.emplace(cfd, std::move(c));
        }
        w->incoming.clear();
      };
      auto flush = [&](Conn* c) -> bool {  // false => connection closed
        while (c->out_off < c->out.size()) {
          const ssize_t n = send(c->fd, c->out.data() + c->out_off, c->out.size() - c->out_off, MSG_NOSIGNAL);
          if (n > 0) {
            c->out_off += static_cast<size_t>(n);
          } else if (n < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) {
            break;
          } else if (n < 0 && errno == EINTR) {
            continue;
          } else {
            close_conn(c->fd);
            return false;
          }
        }
        if (c->out_off >= c->out.size()) {
          c->out.clear();
          c->out_off = 0;
          if (c->close_after) {
            close_conn(c->fd);
            return false;
          }
        }
        const bool want = c->out_off < c->out.size() || !c->out.empty();
        const bool want_in = backlog(c) <= kMaxPendingOut;
        if (want != c->want_out || want_in != c->want_in) {
          struct epoll_event ev {};
          // throttled: no read interest, and no EPOLLRDHUP either (level-triggered, it
          // would fire on every wait once the peer half-closes)
          ev.events = (want_in ? EPOLLIN | EPOLLRDHUP : 0u) | (want ? EPOLLOUT : 0u);
          ev.data.fd = c->fd;
          epoll_ctl(w->ep, EPOLL_CTL_MOD, c->fd, &ev);
          c->want_out = want;
          c->want_in = want_in;
        }
        return true;
      };
      // Parses and answers every complete request in the buffer (pipelining) while the
      // connection's unsent output stays under kMaxPendingOut: a client that pipelines
      // requests without reading the answers is throttled (its socket leaves the epoll
      // read set, TCP flow control holds the rest) instead of growing our buffer.
      auto serve = [&](Conn* c) {
        // parse and answer every complete request in the buffer (pipelining)
        size_t pos = 0;
        while (!c->close_after && backlog(c) <= kMaxPendingOut) {
          const size_t hdr_end = c->in.find("\r\n\r\n", pos);
          if (hdr_end == std::string::npos) {
            if (c->in.size() - pos > 65536) {  // header block too large
              std::string o;
              int st = 431;
              size_t bytes = 0;
              handle("", "", "", false, false, &o, &st, &bytes);
              c->out.append(o);
              c->close_after = true;
            }
            break;
          }
          const char* p = c->in.data() + pos;
          const size_t hlen = hdr_end - pos;
          const char* le = static_cast<const char*>(memchr(p, '\n', hlen + 2));
          std::string_view reqline(p, le ? static_cast<size_t>(le - p) : hlen);
          if (!reqline.empty() && reqline.back() == '\r') reqline.remove_suffix(1);
          const size_t sp1 = reqline.find(' ');
          const size_t sp2 = sp1 == std::string_view::npos ? std::string_view::npos : reqline.find(' ', sp1 + 1);
          std::string method, uri;
          std::string_view proto;
          if (sp1 != std::string_view::npos && sp2 != std::string_view::npos) {
            method.assign(reqline.substr(0, sp1));
            uri.assign(reqline.substr(sp1 + 1, sp2 - sp1 - 1));
            proto = reqline.substr(sp2 + 1);
          }
          std::string origin, hosth, ua;
          size_t content_len = 0;
          bool conn_close = false, conn_keep = false, chunked = false, gzip_ok = false;
          const char* q = le ? le + 1 : p + hlen;
          const char* hend = p + hlen;
          while (q < hend) {
            const char* e = static_cast<const char*>(memchr(q, '\n', static_cast<size_t>(hend - q)));
            if (!e) e = hend;
            const char* colon = static_cast<const char*>(memchr(q, ':', static_cast<size_t>(e - q)));
            if (colon) {
              const size_t nlen = static_cast<size_t>(colon - q);
              const char* v = colon + 1;
              while (v < e && (*v == ' ' || *v == '\t')) ++v;
              const char* ve = e;
              while (ve > v && (ve[-1] == '\r' || ve[-1] == ' ')) --ve;
              const std::string_view val(v, static_cast<size_t>(ve - v));
              if (ieq(q, nlen, "origin")) origin.assign(val);
              else if (ieq(q, nlen, "host")) hosth.assign(val);
              else if (ieq(q, nlen, "user-agent")) ua.assign(val);
              else if (ieq(q, nlen, "content-length")) {
                // leading digits, as strtoull reads them: a malformed value is 0; a
                // negative or overflowing one is huge, and refused below as too large
                std::string_view d = val;
                if (!d.empty() && d[0] == '+') d.remove_prefix(1);
                unsigned long long cl = 0;
                const auto r = std::from_chars(d.data(), d.data() + d.size(), cl);
                content_len = (!d.empty() && d[0] == '-') || r.ec == std::errc::result_out_of_range
                                  ? std::numeric_limits<size_t>::max()
                                  : static_cast<size_t>(cl);
              } else if (ieq(q, nlen, "transfer-encoding")) chunked = true;
              else if (ieq(q, nlen, "accept-encoding")) gzip_ok = gzip_ok || accepts_gzip(val);
              else if (ieq(q, nlen, "connection")) {
                if (icontains(val, "close")) conn_close = true;
                if (icontains(val, "keep-alive")) conn_keep = true;
              }
            }
            q = e + 1;
          }
          const size_t body_start = hdr_end + 4;
          if (content_len > (1u << 20)) {
            std::string o;
            int st = 413;
            size_t bytes = 0;
            handle("", "", origin, false, false, &o, &st, &bytes);
            c->out.append(o);
            c->close_after = true;
            break;
          }
          if (c->in.size() < body_start + content_len) break;  // wait for the body
          const bool http10 = proto == "HTTP/1.0";
          const bool keep = !chunked && !method.empty() && (http10 ? conn_keep : !conn_close);
          const int64_t t0 = mono_ns();
          int status = 0;
          size_t body_bytes = 0;
          // responses are appended straight to the connection's output buffer (its
          // capacity is reused across requests): no per-request copy of the body
          if (method.empty() || chunked) {
            status = method.empty() ? 400 : 501;
            handle("", "", origin, false, http10, &c->out, &status, &body_bytes);
          } else {
            const size_t qm = uri.find('?');
            handle(method, qm == std::string::npos ? uri : uri.substr(0, qm), origin, keep, http10, &c->out,
                   &status, &body_bytes, gzip_ok, c->local, c->out.empty() ? c->fd : -1,
                   qm == std::string::npos ? std::string() : uri.substr(qm + 1));
          }
          const double dt = (mono_ns() - t0) * 1e-9;
          requests_.add();
          if (cfg_.access_log && method != "OPTIONS" && !method.empty())
            log_access(c->remote, hosth, method, uri, ua, status, dt, content_len, body_bytes);
          pos = body_start + content_len;
          if (!keep) c->close_after = true;
        }
        c->in.erase(0, pos);
      };
      // busy-poll window (see GrpcServer): a scraper's next request on a keep-alive
      // connection usually lands while the worker is still polling
      const int64_t spin_ns = static_cast<int64_t>(std::max(0, std::min(cfg_.busy_poll_us, 100000))) * 1000;
      int64_t spin_until = 0;
      while (!stop_.load(std::memory_order_relaxed)) {
        // 5 s: the idle-connection sweep below needs no finer grain (timeouts are 30-60 s)
        const int n = epoll_wait(w->ep, evs.data(), static_cast<int>(evs.size()), spin_until ? 0 : 5000);
        const int64_t now = mono_ns();
        if (spin_until) {
          if (n == 0 && now < spin_until) {
            cpu_relax();
            continue;
          }
          if (n == 0) spin_until = 0;
        }
        for (int i = 0; i < n; ++i) {
          const int fd = evs[i].data.fd;
          if (fd == stop_efd_) continue;  // stop(): the loop condition ends it
          if (fd == listen_fd_) {
            for (;;) {
              struct sockaddr_storage peer {};
              socklen_t pl = sizeof(peer);
              bool shed = false;
              const int cfd = accept_or_shed(listen_fd_, reinterpret_cast<sockaddr*>(&peer), &pl, &spare, &shed);
              if (cfd < 0) {
                if (!shed) break;
                shed_.add();
                continue;
              }
              int one = 1;
              setsockopt(cfd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
              auto c = std::make_unique<Conn>();
              c->fd = cfd;
              c->last_ns = now;
              char ip[INET6_ADDRSTRLEN] = {0};
              if (peer.ss_family == AF_INET)
                inet_ntop(AF_INET, &reinterpret_cast<sockaddr_in*>(&peer)->sin_addr, ip, sizeof(ip));
              else if (peer.ss_family == AF_INET6)
                inet_ntop(AF_INET6, &reinterpret_cast<sockaddr_in6*>(&peer)->sin6_addr, ip, sizeof(ip));
              c->remote = ip;
              if (peer.ss_family == AF_INET)
                c->local = (ntohl(reinterpret_cast<sockaddr_in*>(&peer)->sin_addr.s_addr) >> 24) == 127;
              else if (peer.ss_family == AF_INET6) {
                const in6_addr& a6 = reinterpret_cast<sockaddr_in6*>(&peer)->sin6_addr;
                c->local = IN6_IS_ADDR_LOOPBACK(&a6) || (IN6_IS_ADDR_V4MAPPED(&a6) && a6.s6_addr[12] == 127);
              }
              Worker* t = pick_least_loaded(workers_, w);  // this one on a tie
              struct epoll_event ev {};
              ev.events = EPOLLIN | EPOLLRDHUP;
              ev.data.fd = cfd;
              if (t != w) {  // EPOLLOUT: the owner wakes at once and adopts it (idle sweep included)
                c->want_out = true;
                ev.events |= EPOLLOUT;
                {
                  std::lock_guard<std::mutex> lk(t->in_mu);
                  t->incoming.push_back(std::move(c));
                }
                epoll_ctl(t->ep, EPOLL_CTL_ADD, cfd, &ev);
                continue;
              }
              epoll_ctl(w->ep, EPOLL_CTL_ADD, cfd, &ev);
              w->conns.emplace(cfd, std::move(c));
            }
            continue;
          }
          auto it = w->conns.find(fd);
          if (it == w->conns.end()) {
            adopt();
            it = w->conns.find(fd);
            if (it == w->conns.end()) continue;
          }
          Conn* c = it->second.get();
          c->last_ns = now;
          if (evs[i].events & EPOLLERR) {
            close_conn(fd);
            continue;
          }
          bool peer_closed = false;
          if ((evs[i].events & (EPOLLIN | EPOLLRDHUP | EPOLLHUP)) && backlog(c) <= kMaxPendingOut) {
            for (;;) {
              const ssize_t r = recv(fd, rbuf, sizeof(rbuf), 0);
              if (r > 0) {
                c->in.append(rbuf, static_cast<size_t>(r));
                if (c->in.size() > (1u << 20)) break;
                if (static_cast<size_t>(r) < sizeof(rbuf)) break;
              } else if (r == 0) {
                peer_closed = true;
                break;
              } else if (errno == EINTR) {
                continue;
              } else {
                if (errno != EAGAIN && errno != EWOULDBLOCK) peer_closed = true;
                break;
              }
            }
            if (spin_ns > 0) spin_until = now + spin_ns;
          }
          serve(c);
          if (!c->out.empty() || (evs[i].events & EPOLLOUT)) {
            if (!flush(c)) continue;
            // Drained below the limit with requests still waiting (a throttled pipelining
            // client): answer them now, no further EPOLLIN may come for them.  A few rounds
            // per event, so one such client does not hold the worker; if requests remain
            // and nothing is queued to send, EPOLLOUT (writable at once) brings us back.
            bool closed = false;
            for (int round = 0; round < 8 && !c->in.empty() && !c->close_after &&
                                backlog(c) <= kMaxPendingOut;
                 ++round) {
              const size_t before = c->in.size();
              serve(c);
              if (!c->out.empty() && !flush(c)) {
                closed = true;
                break;
              }
              if (c->in.size() == before) break;  // only an incomplete request is left
              if (round == 7 && !c->want_out) {
                struct epoll_event ev {};
                ev.events = EPOLLIN | EPOLLRDHUP | EPOLLOUT;
                ev.data.fd = c->fd;
                epoll_ctl(w->ep, EPOLL_CTL_MOD, c->fd, &ev);
                c->want_out = true;
                c->want_in = true;
              }
            }
            if (closed) continue;
          }
          if (peer_closed && c->out.empty()) close_conn(fd);
        }
        if (now - last_sweep > 1000000000LL) {  // idle / slow-client sweep
          last_sweep = now;
          std::vector<int> dead;
          for (auto& kv : w->conns) {
            const int64_t idle = now - kv.second->last_ns;
            const int64_t limit = kv.second->in.empty() ? cfg_.idle_timeout_s : cfg_.read_timeout_s;
            if (idle > limit * 1000000000LL) dead.push_back(kv.first);
          }
          for (int fd : dead) close_conn(fd);
        }
      }
      adopt();
      for (auto& kv : w->conns) close(kv.first);
      w->conns.clear();
      if (spare >= 0) close(spare);
    });
  }
  if (cfg_.access_log) {
    log_thread_ = std::thread([this] {
      background_thread("dpaccesslog");
      for (;;) {
        {  // asleep until there is something to write (no periodic wake-ups on an idle node)
          std::unique_lock<std::mutex> lk(log_mu_);
          log_cv_.wait(lk, [&] { return stop_.load() || !log_buf_.empty(); });
        }
        if (stop_.load()) break;
        // batch what the next 100 ms bring into one write
        std::unique_lock<std::mutex> lk(log_mu_);
        log_cv_.wait_for(lk, std::chrono::milliseconds(100), [&] { return stop_.load(); });
        lk.unlock();
        flush_log();
      }
      flush_log();
    });
  }
  return bound_port_;
}

std::vector<int> HttpServer::worker_connections() const {
  std::vector<int> out;
  for (const auto& w : workers_) out.push_back(w->load.load(std::memory_order_relaxed));
  return out;
}

void HttpServer::stop() {
  if (!running_.exchange(false)) return;
  stop_ = true;
  if (stop_efd_ >= 0) {
    const uint64_t one = 1;
    (void)!write(stop_efd_, &one, sizeof(one));
  }
  {
    std::lock_guard<std::mutex> lk(log_mu_);
  }
  log_cv_.notify_all();
  for (auto& t : threads_)
    if (t.joinable()) t.join();
  threads_.clear();
  if (log_thread_.joinable()) log_thread_.join();
  if (stop_efd_ >= 0) close(stop_efd_);
  stop_efd_ = -1;
  for (auto& w : workers_) {
    for (auto& c : w->incoming) close(c->fd);  // handed over after its owner had left its loop
    w->incoming.clear();
    if (w->ep >= 0) close(w->ep);
  }
  workers_.clear();
  if (listen_fd_ >= 0) close(listen_fd_);
  listen_fd_ = -1;
}

void HttpServer::record(int mi, int hi, int status, double seconds) {
  hist_[mi][hi]->observe(seconds);
  counts_[thread_shard()].c[status_class(status)][mi][hi].fetch_add(1, std::memory_order_relaxed);
  const uint64_t bit = uint64_t{1} << (mi * kHandlers + hi);
  if (!(used_mh_.load(std::memory_order_relaxed) & bit)) used_mh_.fetch_or(bit, std::memory_order_relaxed);
}

void HttpServer::handle(const std::string& method, const std::string& path, const std::string& origin,
                        bool keep_alive, bool http10, std::string* out, int* status_out, size_t* body_bytes_out,
                        bool gzip_ok, bool peer_local, int direct_fd, const std::string& query) {
  const int64_t t0 = mono_ns();
  int status = 200;
  static thread_local std::string body_buf;  // per worker thread, capacity reused
  std::string& body = body_buf;
  body.clear();
  const char* ctype = "application/json";
  int handler = -1;
  const bool cors = true;
  bool gz = false;
  // plain /metrics: the exposition's segments are appended after the header, each once
  // (per worker thread, its per-scrape strings keep their capacity across scrapes)
  static thread_local Exposition expo;
  expo.clear();
  bool have_expo = false;
  if (method.empty()) {
    status = *status_out ? *status_out : 400;
    body = std::string("{\"message\":\"") + reason(status) + "\"}\n";
  } else if (method == "OPTIONS") {
    // server/server.go:92-94: Cros answers every OPTIONS with HTTPError(200); echo's
    // error handler renders {"message":"OK"}.  Logger/Metrics are not reached.
    body = "{\"message\":\"OK\"}\n";
  } else try {
    if (path == "/") handler = 0;
    else if (path == "/metrics") handler = 1;
    else if (path == "/health") handler = 2;
    else if (path == "/restart") handler = 3;
    else if (path == "/ready") handler = 4;
    else if (path == "/health/clear") handler = 6;
    if (handler < 0) {
      status = 404;
      body = "{\"message\":\"Not Found\"}\n";
      handler = 5;
    } else if (method != "GET") {
      status = 405;
      body = "{\"message\":\"Method Not Allowed\"}\n";
    } else if (handler == 0) {  // router/api.go:40-42
      body = "{\"code\":0,\"data\":\"version : " + cfg_.version + "\",\"msg\":\"success\"}\n";
    } else if (handler == 2) {  // router/api.go:45-47
      body = "{\"code\":0,\"data\":\"ok\",\"msg\":\"success\"}\n";
    } else if (handler == 4) {  // readiness: every resource registered with kubelet
      std::lock_guard<std::mutex> lk(hook_mu_);
      if (ready_) {
        body = "{\"code\":0,\"data\":\"ready\",\"msg\":\"success\"}\n";
      } else {
        status = 503;  // util.Failed's envelope (modules/util/http.go:13-15)
        body = "{\"code\":-1,\"data\":null,\"msg\":\"";
        append_json_string_body(&body, not_ready_reason_);
        body += "\"}\n";
      }
    } else if (handler == 6 && cfg_.clear_local_only && !peer_local) {
      status = 403;  // http.healthClearLocalOnly: dropping a health latch is an operator's act
      body = "{\"message\":\"Forbidden\"}\n";
    } else if (handler == 6) {
      ClearHook hook;
      {
        std::lock_guard<std::mutex> lk(hook_mu_);
        hook = clear_hook_;
      }
      if (hook) {
        auto r = hook(query);
        status = r.first;
        body = std::move(r.second);
      } else {
        status = 503;
        body = "{\"code\":-1,\"data\":null,\"msg\":\"no health monitor\"}\n";
      }
    } else if (handler == 3 && cfg_.restart_local_only && !peer_local) {
      status = 403;  // http.restartLocalOnly: a reload is not for remote callers
      body = "{\"message\":\"Forbidden\"}\n";
    } else if (handler == 3) {  // router/api.go:50-54
      std::function<void()> hook;
      {
        std::lock_guard<std::mutex> lk(hook_mu_);
        hook = restart_hook_;
      }
      if (hook) hook();
      body = "{\"code\":0,\"data\":\"ok\",\"msg\":\"success\"}\n";
    } else {  // /metrics
      ctype = "text/plain; version=0.0.4; charset=utf-8";
      if (gzip_ok) {  // promhttp compresses when the scraper accepts gzip (Prometheus does)
        std::string httpm;
        render_http_metrics(&httpm);
        if (exporter_) exporter_->render_gzip(&body, httpm);
        else gzip_member(httpm.data(), httpm.size(), &body);
        gz = true;
      } else if (exporter_) {
        exporter_->render(&expo);
        have_expo = true;
        render_http_metrics(&body);  // small; follows the exposition
      } else {
        render_http_metrics(&body);
      }
    }
    const double dt = (mono_ns() - t0) * 1e-9;
    record(method_index(method), handler, status, dt);
  } catch (const std::exception& e) {  // echo's Recover middleware: a failing handler is a 500, not a crash
    status = 500;
    body = "{\"message\":\"Internal Server Error\"}\n";
    ctype = "application/json";
    gz = false;
    have_expo = false;
    std::fprintf(stderr, "httpd: handler for %s %s failed: %s\n", method.c_str(), path.c_str(), e.what());
    if (handler >= 0) record(method_index(method), handler, status, (mono_ns() - t0) * 1e-9);
  }
  static thread_local std::string date;
  static thread_local int64_t date_ns = 0;
  const int64_t now = mono_ns();
  if (now - date_ns > 500000000LL) {
    date = http_date();
    date_ns = now;
  }
  const size_t body_len = body.size() + (have_expo ? expo.size() : 0);
  std::string& o = *out;
  o.reserve(o.size() + body_len + 512);
  o.append(http10 ? "HTTP/1.0 " : "HTTP/1.1 ").append(std::to_string(status)).append(" ").append(reason(status)).append("\r\n");
  if (cors) {  // server/server.go:77-96
    o.append("Access-Control-Allow-Credentials: true\r\n");
    o.append("Access-Control-Allow-Headers: Content-Type, Content-Length, Accept-Encoding, Authorization, Origin\r\n");
    o.append("Access-Control-Allow-Methods: POST, GET, OPTIONS, PATCH, PUT, DELETE\r\n");
    o.append("Access-Control-Allow-Origin: ").append(origin.empty() ? std::string("*") : origin).append("\r\n");
  }
  if (!keep_alive) o.append("Connection: close\r\n");
  else if (http10) o.append("Connection: keep-alive\r\n");
  if (gz) o.append("Content-Encoding: gzip\r\n");
  o.append("Content-Length: ").append(std::to_string(body_len)).append("\r\n");
  o.append("Content-Type: ").append(ctype).append("\r\n");
  o.append("Date: ").append(date).append("\r\n");
  if (handler == 1) o.append("Vary: Accept-Encoding\r\n");
  o.append("\r\n");
  *status_out = status;
  *body_bytes_out = body_len;
  if (have_expo && direct_fd >= 0 && keep_alive) {
    // Nothing queued before this answer (direct_fd): hand the header and the exposition's
    // segments to the kernel in one sendmsg instead of copying ~20-80 KB into the
    // connection buffer first.  The segments are this thread's cached views, valid until
    // its next render; what the socket does not take now is copied into *out.
    struct iovec iov[6];
    int k = 0;
    auto add = [&](const char* p, size_t n) {
      if (n) iov[k++] = {const_cast<char*>(p), n};
    };
    add(o.data(), o.size());
    add(expo.head.data(), expo.head.size());
    add(expo.counters.data(), expo.counters.size());
    add(expo.health.data(), expo.health.size());
    add(expo.tail.data(), expo.tail.size());
    add(body.data(), body.size());
    struct msghdr mh {};
    mh.msg_iov = iov;
    mh.msg_iovlen = static_cast<size_t>(k);
    ssize_t sent;
    do {
      sent = sendmsg(direct_fd, &mh, MSG_NOSIGNAL | MSG_DONTWAIT);
    } while (sent < 0 && errno == EINTR);
    size_t skip = sent > 0 ? static_cast<size_t>(sent) : 0;  // errors: queue it all, flush reports them
    o.clear();
    for (int i = 0; i < k; ++i) {
      if (skip >= iov[i].iov_len) {
        skip -= iov[i].iov_len;
        continue;
      }
      o.append(static_cast<const char*>(iov[i].iov_base) + skip, iov[i].iov_len - skip);
      skip = 0;
    }
    return;
  }
  if (have_expo) expo.append_to(&o);
  o.append(body);
}

namespace {
// the fixed text of every echo_http_* line, built once: a scrape re-renders these
// families each time (its own request moves them), so only the numbers are formatted
struct EchoText {
  std::string requests[HttpServer::kStatus][HttpServer::kMethods][HttpServer::kHandlers];
  std::string labels[HttpServer::kMethods][HttpServer::kHandlers];
  EchoText() {
    for (int m = 0; m < HttpServer::kMethods; ++m)
      for (int h = 0; h < HttpServer::kHandlers; ++h) {
        labels[m][h].append("handler=\"").append(kHandlerNames[h]).append("\",method=\"").append(kMethodNames[m])
            .append("\",");
        for (int s = 0; s < HttpServer::kStatus; ++s)
          requests[s][m][h].append("echo_http_requests_total{handler=\"").append(kHandlerNames[h])
              .append("\",method=\"").append(kMethodNames[m]).append("\",status=\"").append(kStatusNames[s])
              .append("\"} ");
      }
  }
};
const EchoText& echo_text() {
  static const EchoText t;
  return t;
}
}  // namespace

void HttpServer::render_http_metrics(std::string* out) const {
  // middleware/echo_metric.go:80-93 family names / help strings
  static_assert(kMethods * kHandlers <= 64, "used_mh_ is one 64-bit mask");
  const EchoText& et = echo_text();
  const uint64_t used = used_mh_.load(std::memory_order_relaxed);
  bool any = false;
  for (int s = 0; s < kStatus; ++s) {
    for (uint64_t bits = used; bits; bits &= bits - 1) {
      const int mh = __builtin_ctzll(bits);
      const int m = mh / kHandlers, h = mh % kHandlers;
      uint64_t v = 0;
      for (int k = 0; k < kMetricShards; ++k) v += counts_[k].c[s][m][h].load(std::memory_order_relaxed);
      if (!v) continue;
      if (!any) {
        append_header(out, "echo_http_requests_total", "Number of HTTP operations", "counter");
        any = true;
      }
      out->append(et.requests[s][m][h]);
      append_u64(out, v);
      out->push_back('\n');
    }
  }
  any = false;
  for (uint64_t bits = used; bits; bits &= bits - 1) {
    const int mh = __builtin_ctzll(bits);
    const int m = mh / kHandlers, h = mh % kHandlers;
    if (!hist_[m][h]->count()) continue;
    if (!any) {
      append_header(out, "echo_http_request_duration_seconds", "Spend time by processing a route", "histogram");
      any = true;
    }
    hist_[m][h]->render(out, "echo_http_request_duration_seconds", et.labels[m][h]);
  }
}

void HttpServer::log_access(const std::string& remote, const std::string& host, const std::string& method,
                            const std::string& uri, const std::string& ua, int status, double seconds, size_t bytes_in,
                            size_t bytes_out) {
  // echo middleware.Logger() default JSON format (server/server.go:42)
  char ts[64];
  struct timespec tsv;
  clock_gettime(CLOCK_REALTIME, &tsv);
  struct tm tmv;
  gmtime_r(&tsv.tv_sec, &tmv);
  const size_t n = strftime(ts, sizeof(ts), "%Y-%m-%dT%H:%M:%S", &tmv);
  std::snprintf(ts + n, sizeof(ts) - n, ".%09ldZ", tsv.tv_nsec);
  std::string line;
  line.reserve(256);
  line.append("{\"time\":\"").append(ts).append("\",\"id\":\"\",\"remote_ip\":\"");
  append_label_value(&line, remote);
  line.append("\",\"host\":\"");
  append_label_value(&line, host);
  line.append("\",\"method\":\"").append(method).append("\",\"uri\":\"");
  append_label_value(&line, uri);
  line.append("\",\"user_agent\":\"");
  append_label_value(&line, ua);
  line.append("\",\"status\":").append(std::to_string(status)).append(",\"error\":\"\",\"latency\":");
  line.append(std::to_string(static_cast<long long>(seconds * 1e9)));
  char human[32];
  std::snprintf(human, sizeof(human), "%.3fµs", seconds * 1e6);
  line.append(",\"latency_human\":\"").append(human).append("\",\"bytes_in\":").append(std::to_string(bytes_in));
  line.append(",\"bytes_out\":").append(std::to_string(bytes_out)).append("}\n");
  bool was_empty;
  {
    std::lock_guard<std::mutex> lk(log_mu_);
    was_empty = log_buf_.empty();
    log_buf_.append(line);
    if (log_buf_.size() > (256u << 10)) {
      fwrite(log_buf_.data(), 1, log_buf_.size(), stdout);
      fflush(stdout);
      log_buf_.clear();
    }
  }
  if (was_empty) log_cv_.notify_one();  // the writer thread sleeps until there is a first line
}

void HttpServer::flush_log() {
  std::string buf;
  {
    std::lock_guard<std::mutex> lk(log_mu_);
    buf.swap(log_buf_);
  }
  if (!buf.empty()) {
    fwrite(buf.data(), 1, buf.size(), stdout);
    fflush(stdout);
  }
}

}  // namespace amdgpu_dp
