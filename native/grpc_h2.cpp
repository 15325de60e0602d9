#include "grpc_h2.h"

#include "core_escape.h"
#include "hpack.h"
#include "pbwire.h"

#include <errno.h>
#include <fcntl.h>
#include <poll.h>
#include <pthread.h>
#include <sched.h>
#include <sys/mman.h>
#include <sys/epoll.h>
#include <sys/eventfd.h>
#include <sys/socket.h>
#include <sys/time.h>
#include <sys/stat.h>
#include <sys/un.h>
#include <unistd.h>

#include <algorithm>
#include <cstring>
#include <new>
#include <stdexcept>
#include <unordered_map>

namespace amdgpu_dp {

namespace {

constexpr char kPreface[] = "PRI * HTTP/2.0\r\n\r\nSM\r\n\r\n";
constexpr size_t kPrefaceLen = 24;

enum FrameType : uint8_t {
  kData = 0,
  kHeaders = 1,
  kPriority = 2,
  kRstStream = 3,
  kSettings = 4,
  kPushPromise = 5,
  kPing = 6,
  kGoaway = 7,
  kWindowUpdate = 8,
  kContinuation = 9,
};
enum Flags : uint8_t { kEndStream = 0x1, kAck = 0x1, kEndHeaders = 0x4, kPadded = 0x8, kPriorityFlag = 0x20 };
enum H2Error : uint32_t { kNoError = 0, kProtocolError = 1, kFlowControlError = 3, kStreamClosed = 5,
                          kFrameSizeError = 6, kRefusedStream = 7, kCompressionError = 9 };

constexpr uint32_t kMaxFrame = 16384;           // our SETTINGS_MAX_FRAME_SIZE (default)
constexpr int64_t kLocalWindow = 1 << 20;        // stream + connection receive windows we grant
constexpr size_t kMaxMessage = 4u << 20;         // grpc default max receive message size
constexpr size_t kMaxStreams = 1024;
constexpr int64_t kMaxWindow = 0x7FFFFFFF;       // RFC 9113 §6.9.1
constexpr size_t kMaxPendingOut = 16u << 20;     // a peer that never reads is dropped
constexpr size_t kMaxBuffered = 16u << 20;       // request bytes buffered per connection

void put_u32(std::string* o, uint32_t v) {
  o->push_back(static_cast<char>(v >> 24));
  o->push_back(static_cast<char>(v >> 16));
  o->push_back(static_cast<char>(v >> 8));
  o->push_back(static_cast<char>(v));
}

uint32_t get_u32(const uint8_t* p) {
  return (static_cast<uint32_t>(p[0]) << 24) | (static_cast<uint32_t>(p[1]) << 16) |
         (static_cast<uint32_t>(p[2]) << 8) | p[3];
}

void frame(std::string* o, uint32_t len, uint8_t type, uint8_t flags, uint32_t sid) {
  o->push_back(static_cast<char>(len >> 16));
  o->push_back(static_cast<char>(len >> 8));
  o->push_back(static_cast<char>(len));
  o->push_back(static_cast<char>(type));
  o->push_back(static_cast<char>(flags));
  put_u32(o, sid & 0x7FFFFFFFu);
}

void window_update(std::string* o, uint32_t sid, uint32_t inc) {
  frame(o, 4, kWindowUpdate, 0, sid);
  put_u32(o, inc & 0x7FFFFFFFu);
}

void grpc_prefix(std::string* o, size_t len) {
  o->push_back(0);
  put_u32(o, static_cast<uint32_t>(len));
}

std::string pct_encode(std::string_view s) {
  static const char* hex = "0123456789ABCDEF";
  std::string o;
  for (unsigned char c : s) {
    if (c >= 0x20 && c <= 0x7E && c != '%') {
      o.push_back(static_cast<char>(c));
    } else {
      o.push_back('%');
      o.push_back(hex[c >> 4]);
      o.push_back(hex[c & 15]);
    }
  }
  return o;
}

const std::string& response_headers() {
  static const std::string h = [] {
    std::string s;
    hpack::encode_indexed(&s, 8);                              // :status 200
    hpack::encode_literal_name_index(&s, 31, "application/grpc");  // content-type
    return s;
  }();
  return h;
}

const std::string& ok_trailers() {
  static const std::string t = [] {
    std::string s;
    hpack::encode_literal(&s, "grpc-status", "0");
    return s;
  }();
  return t;
}

enum Method { kMUnknown = -1, kMOptions = 0, kMLaw, kMPreferred, kMAllocate, kMPreStart };

Method method_of(std::string_view path) {
  static const std::string_view base = "/v1beta1.DevicePlugin/";
  if (path.size() <= base.size() || path.substr(0, base.size()) != base) return kMUnknown;
  const std::string_view m = path.substr(base.size());
  if (m == "Allocate") return kMAllocate;
  if (m == "GetPreferredAllocation") return kMPreferred;
  if (m == "ListAndWatch") return kMLaw;
  if (m == "GetDevicePluginOptions") return kMOptions;
  if (m == "PreStartContainer") return kMPreStart;
  return kMUnknown;
}

struct Stream {
  int method = -1;          // Method, resolved from :path while decoding the header block
  std::string path;         // kept only for an unknown method's error message
  std::string data;
  bool headers_done = false;
  int64_t send_window = 65535;
  int64_t recv_unacked = 0;
  std::string pend;         // queued DATA payload (flow-controlled)
  bool trailers_after = false;
  std::string trailers;     // header block sent (END_STREAM) once pend drains
  bool law = false;
  uint64_t law_version = 0;
  bool dispatched = false;  // request half-closed; later DATA/HEADERS are stream errors
  bool done = false;
};

std::string request_headers(std::string_view path) {
  std::string h;
  hpack::encode_indexed(&h, 3);  // :method POST
  hpack::encode_indexed(&h, 6);  // :scheme http
  hpack::encode_literal_name_index(&h, 4, path);          // :path
  hpack::encode_literal_name_index(&h, 1, "localhost");   // :authority
  hpack::encode_literal_name_index(&h, 31, "application/grpc");
  hpack::encode_literal(&h, "te", "trailers");
  return h;
}

}  // namespace

// Completions of asynchronous RPCs (PreStartContainer checks) for one worker.  Shared
// with the pending jobs, so a verifier finishing after the worker is gone still has a
// valid queue and eventfd to post to.
struct AsyncDone {
  struct Item {
    int fd;
    uint64_t serial;  // connection incarnation: the fd number may have been reused
    uint32_t sid;
    bool ok;
    std::string error;
    int64_t t0;
  };
  std::mutex mu;
  std::vector<Item> items;
  int efd = -1;
  AsyncDone() : efd(eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC)) {}
  ~AsyncDone() {
    if (efd >= 0) ::close(efd);
  }
  void post(Item it) {
    {
      std::lock_guard<std::mutex> lk(mu);
      items.push_back(std::move(it));
    }
    const uint64_t one = 1;
    (void)!write(efd, &one, sizeof(one));
  }
};

struct GrpcServer::Worker {
  int index = 0;
  int ep = -1;
  int efd = -1;
  std::shared_ptr<AsyncDone> done = std::make_shared<AsyncDone>();
  uint64_t next_serial = 1;
  struct Conn {
    int fd = -1;
    uint64_t serial = 0;
    std::string in;
    std::string out;
    size_t out_off = 0;
    bool preface = false;
    hpack::Decoder dec{4096};
    std::unordered_map<uint32_t, Stream> streams;
    int64_t send_window = 65535;
    int64_t peer_init_window = 65535;
    uint32_t peer_max_frame = 16384;
    uint32_t cont_sid = 0;
    uint8_t cont_flags = 0;
    std::string hblock;
    int64_t recv_unacked = 0;
    uint32_t last_sid = 0;
    size_t buffered = 0;  // request bytes held across all streams
    bool closing = false;
    bool want_out = false;
    bool internal = false;  // the keep-warm tick's private connection: no fd, no accounting
    // grpc.peekReads: requests are read with MSG_PEEK (SO_PEEK_OFF advances over what was
    // read) and consumed only after the answers went out.  Consuming the client's data runs
    // its socket's write-space callback, which wakes a client blocked in recv() on that
    // socket (one wait queue for both directions) for nothing.  Measured on the MI355X box
    // the early wake-up pays for itself: it keeps the client's CPU out of deeper idle states
    // for the real one, so this is off by default (docs/ROUND6.md).
    bool peek = false;
    size_t peeked = 0;      // bytes read by peeking, still in the socket
  };
  std::unordered_map<int, std::unique_ptr<Conn>> conns;
  // Connections are spread over the workers: the one that accepts hands a new
  // connection to the least-loaded worker, which adopts it on its first event.
  std::mutex in_mu;
  std::vector<std::unique_ptr<Conn>> incoming;
  std::atomic<int> load{0};  // owned + incoming connections
  // set once this worker has served a ListAndWatch stream: only such workers are woken
  // for a table change (kubelet holds one stream per plugin, so usually one worker;
  // waking all of them one eventfd write after another delayed the stream's push)
  std::atomic<bool> law_seen{false};
  std::atomic<int> law_open{0};  // ListAndWatch streams open on this worker's connections
};

using Conn = GrpcServer::Worker::Conn;

namespace {

void goaway(Conn& c, uint32_t code) {
  frame(&c.out, 8, kGoaway, 0, 0);
  put_u32(&c.out, c.last_sid);
  put_u32(&c.out, code);
  c.closing = true;
}

void rst_stream(Conn& c, uint32_t sid, uint32_t code) {
  frame(&c.out, 4, kRstStream, 0, sid);
  put_u32(&c.out, code);
}

void drop_data(Conn& c, Stream& s) {
  c.buffered -= s.data.size();
  std::string().swap(s.data);
}

// Drain a stream's pending DATA within the flow-control windows, then its trailers.
void flush_stream(Conn& c, uint32_t sid, Stream& s) {
  while (!s.pend.empty()) {
    const int64_t n = std::min<int64_t>({static_cast<int64_t>(s.pend.size()), c.send_window, s.send_window,
                                         static_cast<int64_t>(c.peer_max_frame)});
    if (n <= 0) return;
    frame(&c.out, static_cast<uint32_t>(n), kData, 0, sid);
    c.out.append(s.pend.data(), static_cast<size_t>(n));
    s.pend.erase(0, static_cast<size_t>(n));
    c.send_window -= n;
    s.send_window -= n;
  }
  if (s.trailers_after) {
    frame(&c.out, static_cast<uint32_t>(s.trailers.size()), kHeaders, kEndHeaders | kEndStream, sid);
    c.out.append(s.trailers);
    s.trailers_after = false;
    s.done = true;
  }
}

void send_message(Conn& c, uint32_t sid, Stream& s, std::string_view payload, bool with_ok_trailers) {
  const int64_t len = static_cast<int64_t>(payload.size()) + 5;
  if (s.pend.empty() && len <= c.send_window && len <= s.send_window && len <= c.peer_max_frame) {
    // common case (every unary response): one DATA frame straight into the output,
    // trailers right behind it - no per-stream queue
    frame(&c.out, static_cast<uint32_t>(len), kData, 0, sid);
    grpc_prefix(&c.out, payload.size());
    c.out.append(payload.data(), payload.size());
    c.send_window -= len;
    s.send_window -= len;
    if (with_ok_trailers) {
      const std::string& t = ok_trailers();
      frame(&c.out, static_cast<uint32_t>(t.size()), kHeaders, kEndHeaders | kEndStream, sid);
      c.out.append(t);
      s.done = true;
    }
    return;
  }
  grpc_prefix(&s.pend, payload.size());
  s.pend.append(payload.data(), payload.size());
  if (with_ok_trailers) {
    s.trailers = ok_trailers();
    s.trailers_after = true;
  }
  flush_stream(c, sid, s);
}

void send_error(Conn& c, uint32_t sid, Stream& s, int code, std::string_view msg) {
  std::string h = response_headers();
  hpack::encode_literal(&h, "grpc-status", std::to_string(code));
  if (!msg.empty()) hpack::encode_literal(&h, "grpc-message", pct_encode(msg));
  frame(&c.out, static_cast<uint32_t>(h.size()), kHeaders, kEndHeaders | kEndStream, sid);
  c.out.append(h);
  s.done = true;
}

void send_headers(Conn& c, uint32_t sid) {
  const std::string& h = response_headers();
  frame(&c.out, static_cast<uint32_t>(h.size()), kHeaders, kEndHeaders, sid);
  c.out.append(h);
}

}  // namespace

GrpcServer::GrpcServer(std::string socket_path, int threads, int busy_poll_us, int admission_poll_us)
    : path_(std::move(socket_path)),
      nthreads_(threads),
      busy_poll_us_(std::max(0, std::min(busy_poll_us, 100000))),
      admission_poll_us_(std::max(0, std::min(admission_poll_us, 100000))) {}

GrpcServer::~GrpcServer() {
  stop();
  if (trace_hdr_) munmap(trace_hdr_, trace_bytes_);
}

void GrpcServer::set_call_trace(const std::string& path, int capacity) {
  std::lock_guard<std::mutex> lk(mu_);
  if (running_) throw std::runtime_error("set_call_trace: server already running");
  if (capacity <= 0) throw std::invalid_argument("set_call_trace: capacity must be > 0");
  const size_t bytes = sizeof(CallTraceHeader) + static_cast<size_t>(capacity) * sizeof(CallTraceEntry);
  const int fd = ::open(path.c_str(), O_RDWR | O_CREAT | O_TRUNC | O_CLOEXEC, 0644);
  if (fd < 0) throw std::runtime_error("set_call_trace: open " + path + ": " + strerror(errno));
  if (ftruncate(fd, static_cast<off_t>(bytes)) != 0) {
    const int e = errno;
    ::close(fd);
    throw std::runtime_error("set_call_trace: ftruncate: " + std::string(strerror(e)));
  }
  void* p = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  ::close(fd);
  if (p == MAP_FAILED) throw std::runtime_error("set_call_trace: mmap: " + std::string(strerror(errno)));
  // write every page now: a page's first write faults (page-cache allocation, the file
  // system's page_mkwrite), and in the ring that happened inside every 73rd request
  // (0.017 minor faults per call in the idle probe's daemon counters)
  std::memset(p, 0, bytes);
  if (trace_hdr_) munmap(trace_hdr_, trace_bytes_);
  trace_hdr_ = new (p) CallTraceHeader();
  trace_hdr_->capacity = static_cast<uint32_t>(capacity);
  trace_ = reinterpret_cast<CallTraceEntry*>(static_cast<char*>(p) + sizeof(CallTraceHeader));
  trace_bytes_ = bytes;
  trace_hdr_->magic = kCallTraceMagic;
}

void GrpcServer::law_closed(Worker* w) {
  w->law_open.fetch_sub(1, std::memory_order_relaxed);
  stamp_law_closed();
}

void GrpcServer::stamp_law_closed() {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  law_closed_ns_.store(static_cast<int64_t>(ts.tv_sec) * 1000000000LL + ts.tv_nsec, std::memory_order_relaxed);
}

int GrpcServer::list_and_watch_streams() const {
  std::lock_guard<std::mutex> lk(mu_);  // workers_ changes only under it (start / stop)
  int n = 0;
  for (const auto& w : workers_) n += w->law_open.load(std::memory_order_relaxed);
  return n;
}

void GrpcServer::set_table(std::shared_ptr<DeviceTable> t) {
  if (!t) throw std::invalid_argument("GrpcServer: null device table");
  std::lock_guard<std::mutex> lk(mu_);
  t->add_listener(notifier_);
  {
    std::lock_guard<std::mutex> sk(swap_mu_);
    table_ = std::move(t);
    table_gen_.fetch_add(1, std::memory_order_release);
  }
  // running: wake every worker (not only those with a stream) so none serves a request
  // from the old table after an idle wait
  for (auto& w : workers_) {
    const uint64_t one = 1;
    if (w->efd >= 0) (void)!write(w->efd, &one, sizeof(one));
  }
}

void GrpcServer::start() {
  std::lock_guard<std::mutex> lk(mu_);
  if (running_) return;
  std::shared_ptr<DeviceTable> table;
  uint64_t gen;
  {
    std::lock_guard<std::mutex> sk(swap_mu_);
    table = table_;
    gen = table_gen_.load();
  }
  if (!table) throw std::runtime_error("GrpcServer: no device table");
  struct sockaddr_un addr {};
  addr.sun_family = AF_UNIX;
  if (path_.size() >= sizeof(addr.sun_path)) throw std::runtime_error("GrpcServer: socket path too long: " + path_);
  std::memcpy(addr.sun_path, path_.c_str(), path_.size() + 1);
  ::unlink(path_.c_str());
  const int fd = socket(AF_UNIX, SOCK_STREAM | SOCK_NONBLOCK | SOCK_CLOEXEC, 0);
  if (fd < 0) throw std::runtime_error(std::string("GrpcServer: socket: ") + strerror(errno));
  if (bind(fd, reinterpret_cast<sockaddr*>(&addr), sizeof(addr)) != 0 || listen(fd, 256) != 0) {
    const int e = errno;
    ::close(fd);
    throw std::runtime_error("GrpcServer: bind/listen " + path_ + ": " + strerror(e));
  }
  listen_fd_ = fd;
  struct stat st {};
  if (::stat(path_.c_str(), &st) == 0) {
    sock_dev_ = st.st_dev;
    sock_ino_ = st.st_ino;
  }
  stop_ = false;
  running_ = true;
  const int n = std::max(1, nthreads_);
  for (int i = 0; i < n; ++i) {
    auto w = std::make_unique<Worker>();
    w->index = i;
    w->ep = epoll_create1(EPOLL_CLOEXEC);
    w->efd = eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);
    struct epoll_event ev {};
    ev.events = EPOLLIN | EPOLLEXCLUSIVE;
    ev.data.fd = listen_fd_;
    epoll_ctl(w->ep, EPOLL_CTL_ADD, listen_fd_, &ev);
    struct epoll_event ev2 {};
    ev2.events = EPOLLIN;
    ev2.data.fd = w->efd;
    epoll_ctl(w->ep, EPOLL_CTL_ADD, w->efd, &ev2);
    struct epoll_event ev3 {};
    ev3.events = EPOLLIN;
    ev3.data.fd = w->done->efd;
    epoll_ctl(w->ep, EPOLL_CTL_ADD, w->done->efd, &ev3);
    workers_.push_back(std::move(w));
  }
  failed_ = false;
  {
    std::lock_guard<std::mutex> fk(fail_mu_);
    fail_reason_.clear();
  }
  for (size_t i = 0; i < workers_.size(); ++i)
    threads_.emplace_back([this, wp = workers_[i].get(), t = table, gen, i] {
      // named, so /proc/<pid>/task/*/comm tells the workers apart (scripts/idle_probe.py)
      pthread_setname_np(pthread_self(), ("dpgrpc-" + std::to_string(i)).c_str());
      foreground_thread();
      set_thread_shard(static_cast<int>(i));
      run_guarded(wp, t, gen);
    });
  std::lock_guard<std::mutex> nk(notifier_->mu);
  notifier_->srv = this;
}

std::vector<int> GrpcServer::worker_connections() const {
  std::lock_guard<std::mutex> lk(mu_);
  std::vector<int> out;
  for (const auto& w : workers_) out.push_back(w->load.load(std::memory_order_relaxed));
  return out;
}

void GrpcServer::notify() {
  for (auto& w : workers_) {
    const uint64_t one = 1;
    // workers that never served a stream have nothing to push (their 100 ms version
    // poll covers a stream that starts while this runs)
    if (w->efd >= 0 && w->law_seen.load(std::memory_order_acquire)) (void)!write(w->efd, &one, sizeof(one));
  }
}

void GrpcServer::stop() {
  std::lock_guard<std::mutex> lk(mu_);
  if (!running_.exchange(false)) return;
  {
    std::lock_guard<std::mutex> nk(notifier_->mu);  // no table change may notify from here on
    notifier_->srv = nullptr;
  }
  stop_ = true;
  for (auto& w : workers_) {  // every worker, streams or not: they all have to leave their loop
    const uint64_t one = 1;
    if (w->efd >= 0) (void)!write(w->efd, &one, sizeof(one));
  }
  for (auto& t : threads_)
    if (t.joinable()) t.join();
  threads_.clear();
  for (auto& w : workers_) {
    for (auto& c : w->incoming) {  // handed over after its owner had already left its loop
      ::close(c->fd);
      conns_.fetch_sub(1);
    }
    w->incoming.clear();
    if (w->ep >= 0) ::close(w->ep);
    if (w->efd >= 0) ::close(w->efd);
  }
  workers_.clear();
  if (listen_fd_ >= 0) ::close(listen_fd_);
  listen_fd_ = -1;
  struct stat st {};
  if (::stat(path_.c_str(), &st) == 0 && st.st_dev == sock_dev_ && st.st_ino == sock_ino_) ::unlink(path_.c_str());
}

void GrpcServer::fail(const std::string& why) {
  std::shared_ptr<const std::function<void()>> hook;
  {
    std::lock_guard<std::mutex> lk(fail_mu_);
    if (failed_.exchange(true)) return;  // the first fault is the one reported
    fail_reason_ = why;
    hook = fail_hook_;
  }
  if (hook && *hook) {
    try {
      (*hook)();  // (a Python callable takes the GIL itself; no lock of ours is held)
    } catch (...) {  // the manager's poll still finds failure()
    }
  }
}

std::string GrpcServer::failure() const {
  std::lock_guard<std::mutex> lk(fail_mu_);
  return fail_reason_;
}

void GrpcServer::inject_fault(const std::string& kind) {
  if (kind == "worker") {
    std::lock_guard<std::mutex> lk(mu_);
    inject_worker_fault_.store(1);
    for (auto& w : workers_) {  // wake one at once rather than at its 100 ms poll
      const uint64_t one = 1;
      if (w->efd >= 0) (void)!write(w->efd, &one, sizeof(one));
      break;
    }
  } else if (kind == "listener") {
    std::lock_guard<std::mutex> lk(mu_);
    if (listen_fd_ >= 0) ::shutdown(listen_fd_, SHUT_RDWR);
  } else {
    throw std::invalid_argument("inject_fault: unknown kind " + kind);
  }
}

void GrpcServer::run_guarded(Worker* w, std::shared_ptr<DeviceTable> table, uint64_t gen) {
  try {
    run(w, std::move(table), gen);
    return;
  } catch (const std::exception& e) {
    fail(std::string("gRPC worker died: ") + e.what());
  } catch (...) {
    fail("gRPC worker died: unknown exception");
  }
  // the dead worker's connections can no longer be served: close them, so their
  // clients (kubelet) see the failure at once instead of a silent stall
  for (auto& kv : w->conns) {
    epoll_ctl(w->ep, EPOLL_CTL_DEL, kv.first, nullptr);
    ::close(kv.first);
    conns_.fetch_sub(1);
  }
  w->conns.clear();
  if (w->law_open.exchange(0, std::memory_order_relaxed) > 0) stamp_law_closed();  // kubelet's stream went too
  w->load.store(1 << 20, std::memory_order_relaxed);  // never picked for a new connection
  if (listen_fd_ >= 0) epoll_ctl(w->ep, EPOLL_CTL_DEL, listen_fd_, nullptr);
}

void GrpcServer::run(Worker* w, std::shared_ptr<DeviceTable> table, uint64_t table_gen) {
  std::vector<epoll_event> evs(128);
  char rbuf[32768];
  int spare = -1;  // reserve descriptor for accept_or_shed
  struct SpareCloser {
    int* fd;
    ~SpareCloser() {
      if (*fd >= 0) ::close(*fd);
    }
  } spare_closer{&spare};
  auto close_conn = [&](int fd) {
    epoll_ctl(w->ep, EPOLL_CTL_DEL, fd, nullptr);
    ::close(fd);
    auto ci = w->conns.find(fd);
    if (ci != w->conns.end())
      for (const auto& st : ci->second->streams)
        if (st.second.law) law_closed(w);
    w->conns.erase(fd);
    conns_.fetch_sub(1);
    w->load.fetch_sub(1, std::memory_order_relaxed);
  };
  auto adopt = [&] {
    std::lock_guard<std::mutex> lk(w->in_mu);
    for (auto& c : w->incoming) {
      c->serial = w->next_serial++;
      const int fd = c->fd;
      w->conns.emplace(fd, std::move(c));
    }
    w->incoming.clear();
  };
  // Drops from the socket what was read by peeking (see Conn::peek), now that the answers
  // are out; what cannot be dropped yet stays counted and goes with the next batch.
  auto consume_peeked = [&](Conn* c) {
    char sink[16384];
    while (c->peeked > 0) {
      const ssize_t n = recv(c->fd, sink, std::min(c->peeked, sizeof(sink)), MSG_DONTWAIT);
      if (n > 0) {
        c->peeked -= static_cast<size_t>(n);
      } else if (n < 0 && errno == EINTR) {
        continue;
      } else {
        break;
      }
    }
  };
  // returns false if the connection was closed
  auto flush = [&](Conn* c) -> bool {
    while (c->out_off < c->out.size()) {
      const ssize_t n = send(c->fd, c->out.data() + c->out_off, c->out.size() - c->out_off, MSG_NOSIGNAL);
      if (n > 0) {
        c->out_off += static_cast<size_t>(n);
      } else if (n < 0 && errno == EINTR) {
        continue;
      } else if (n < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) {
        break;
      } else {
        close_conn(c->fd);
        return false;
      }
    }
    if (c->out_off >= c->out.size()) {
      c->out.clear();
      c->out_off = 0;
      if (c->closing) {
        close_conn(c->fd);
        return false;
      }
    }
    const bool want = !c->out.empty();
    if (want != c->want_out) {
      struct epoll_event ev {};
      ev.events = EPOLLIN | EPOLLRDHUP | (want ? EPOLLOUT : 0);
      ev.data.fd = c->fd;
      epoll_ctl(w->ep, EPOLL_CTL_MOD, c->fd, &ev);
      c->want_out = want;
    }
    return true;
  };
  std::string scratch;
  bool admitting = false;  // a GetPreferredAllocation was answered in this batch
  int64_t last_rpc = 0;    // mono ns of this worker's last kubelet RPC (admission window)
  // call trace (set_call_trace): when the events being handled were delivered, whether the
  // worker was polling then, and the records of this batch still waiting for their send
  int64_t wake_ts = 0;
  int64_t recv_done = 0;  // (call trace) when the request's recv() returned
  bool wake_spin = false;
  int64_t wake_idle = 0;      // the worker's time without work before this wake-up
  uint16_t last_cpu = 0xFFFF;  // CPU of the worker's previous work
  // Each worker writes its own slice of the ring with its own counter: one shared counter
  // was a cache line every traced call of every worker wrote (N ranks -> N cores)
  // Records are filled at dispatch and written to the ring after the response's send(),
  // like the histogram observations below: nothing the bench's attribution needs sits on
  // the request's critical path (a ring slot is a cache line missed once per lap)
  std::vector<std::pair<uint64_t, CallTraceEntry>> trace_pending;  // (slot, record) awaiting the send
  const uint64_t trace_slice = trace_ ? std::max<uint64_t>(1, trace_hdr_->capacity / std::max(1, nthreads_)) : 1;
  const uint64_t trace_base = trace_ ? (static_cast<uint64_t>(w->index) * trace_slice) % trace_hdr_->capacity : 0;
  uint64_t trace_next = 0;
  int64_t send_begin = 0;  // (call trace) when the flush that carries the responses began
  auto stamp_sent = [&] {
    const int64_t t = mono_ns();
    for (auto& ps : trace_pending) {
      ps.second.t_sent = t;
      if (send_begin > ps.second.t_dispatch)
        ps.second.handle_ns = static_cast<uint16_t>(std::min<int64_t>(send_begin - ps.second.t_dispatch, 0xFFFF));
      trace_[ps.first] = ps.second;
    }
    trace_pending.clear();
  };
  struct PendingObs {
    int rpc;
    double dt;
    bool err;
  };
  std::vector<PendingObs> pending_obs;  // RPC histogram observations, applied after the send
  auto apply_observes = [&] {
    for (const auto& o : pending_obs) table->observe(o.rpc, o.dt, o.err);
    pending_obs.clear();
  };
  auto push_law = [&](Conn* c) {
    const uint64_t v = table->version();
    std::string payload;
    for (auto& kv : c->streams) {
      Stream& s = kv.second;
      if (!s.law || s.done || s.law_version == v) continue;
      const int64_t t0 = mono_ns();
      if (payload.empty()) payload = table->list_and_watch();
      s.law_version = v;
      send_message(*c, kv.first, s, payload, false);
      table->observe(kRpcListAndWatch, (mono_ns() - t0) * 1e-9, false);
    }
  };
  // the keep-warm connection's requests are not kubelet's: no counter or histogram sees them
  auto observe = [&](const Conn& c, int rpc, double dt, bool err) {
    if (!c.internal) pending_obs.push_back({rpc, dt, err});
  };
  auto dispatch = [&](Conn& c, uint32_t sid, Stream& s, std::string_view body) {
    if (s.dispatched) {  // END_STREAM seen twice (trailers or DATA after the request)
      rst_stream(c, sid, kStreamClosed);
      s.done = true;
      return;
    }
    s.dispatched = true;
    const int64_t t0 = mono_ns();
    if (!c.internal) {
      requests_.add();
      last_rpc = t0;  // opens (extends) this worker's admission window
    }
    const Method m = static_cast<Method>(s.method);
    if (trace_ && !c.internal && m != kMLaw && m != kMPreStart) {
      const uint64_t idx = trace_next++;
      const uint64_t slot = trace_base + idx % trace_slice;
      trace_pending.emplace_back(slot, CallTraceEntry{});
      CallTraceEntry& e = trace_pending.back().second;
      e.t_ready = wake_ts;
      e.t_dispatch = t0;
      e.t_sent = 0;
      e.conn = (static_cast<uint64_t>(w->index) << 48) | (c.serial & 0xFFFFFFFFFFFFull);
      e.method = static_cast<uint8_t>(m == kMAllocate ? kRpcAllocate : m == kMPreferred ? kRpcPreferred
                                      : m == kMOptions ? kRpcOptions : 255);
      e.spinning = wake_spin ? 1 : 0;
      e.idle_ns = wake_idle;
      e.recv_ns = recv_done > wake_ts ? static_cast<uint32_t>(std::min<int64_t>(recv_done - wake_ts, 0xFFFFFFFF)) : 0;
      const int cpu = sched_getcpu();
      e.cpu = static_cast<uint16_t>(cpu < 0 ? 0xFFFF : cpu);
      e.prev_cpu = last_cpu;
      last_cpu = e.cpu;
      e.seq = static_cast<uint32_t>(idx + 1);
    }
    if (m == kMUnknown) {
      send_error(c, sid, s, 12, "unknown method " + s.path);  // UNIMPLEMENTED
      return;
    }
    if (body.size() < 5) {
      send_error(c, sid, s, 13, "missing gRPC message");  // INTERNAL
      return;
    }
    const uint8_t* d = reinterpret_cast<const uint8_t*>(body.data());
    if (d[0] != 0) {
      send_error(c, sid, s, 12, "compressed gRPC messages are not supported");
      return;
    }
    const uint32_t len = get_u32(d + 1);
    if (len != body.size() - 5) {
      send_error(c, sid, s, 13, "unary request must carry exactly one message");
      return;
    }
    const std::string_view msg(body.data() + 5, len);
    std::string& out = scratch;  // per-worker response buffer, capacity reused
    out.clear();
    bool ok = true;
    int rpc = kRpcAllocate;
    try {
      switch (m) {
        case kMAllocate:
          ok = table->allocate(msg, &out);
          break;
        case kMPreferred:
          rpc = kRpcPreferred;
          ok = table->preferred(msg, &out);
          if (!c.internal) admitting = true;  // this container's Allocate is next
          break;
        case kMOptions:
          rpc = kRpcOptions;
          out = table->options_bytes();
          break;
        case kMPreStart: {
          rpc = kRpcPreStart;
          if (!table->config().pre_start_required) break;  // reference behaviour: empty OK
          // answered when the verifier completes the job (see the done-queue below)
          auto q = w->done;
          const int fd = c.fd;
          const uint64_t serial = c.serial;
          std::string err;
          if (!table->submit_prestart(
                  msg,
                  [q, fd, serial, sid, t0](bool pass, const std::string& e) {
                    q->post({fd, serial, sid, pass, e, t0});
                  },
                  &err)) {
            send_error(c, sid, s, 2, err);
            observe(c, rpc, (mono_ns() - t0) * 1e-9, true);
          }
          return;
        }
        case kMLaw: {
          rpc = kRpcListAndWatch;
          w->law_seen.store(true, std::memory_order_release);
          if (!s.law) w->law_open.fetch_add(1, std::memory_order_relaxed);
          s.law = true;
          s.law_version = table->version();
          send_headers(c, sid);
          send_message(c, sid, s, table->list_and_watch(), false);
          observe(c, rpc, (mono_ns() - t0) * 1e-9, false);
          return;
        }
        default:
          break;
      }
    } catch (const std::exception& e) {  // e.g. bad_alloc on a hostile request: INTERNAL, keep serving
      send_error(c, sid, s, 13, std::string("internal error: ") + e.what());
      observe(c, rpc, (mono_ns() - t0) * 1e-9, true);
      return;
    }
    if (ok) {
      send_headers(c, sid);
      send_message(c, sid, s, out, true);
    } else {
      send_error(c, sid, s, 2, out);  // UNKNOWN, like a plain Go error from a handler
    }
    observe(c, rpc, (mono_ns() - t0) * 1e-9, !ok);
  };
  struct PathSink {
    bool seen = false;
    int method = kMUnknown;
    std::string unknown;
  };
  auto on_header = [](void* ctx, std::string_view name, std::string_view value) {
    if (name != ":path") return;
    auto* ps = static_cast<PathSink*>(ctx);
    ps->seen = true;
    ps->method = method_of(value);
    if (ps->method == kMUnknown) ps->unknown.assign(value.data(), value.size());
  };
  auto on_headers_block = [&](Conn& c, uint32_t sid, uint8_t flags) -> bool {
    PathSink ps;
    if (!c.dec.decode(reinterpret_cast<const uint8_t*>(c.hblock.data()), c.hblock.size(), on_header, &ps)) {
      goaway(c, kCompressionError);
      return false;
    }
    c.hblock.clear();
    auto it = c.streams.find(sid);
    if (it == c.streams.end()) {
      if ((sid & 1) == 0 || sid <= c.last_sid) {  // must be a new, odd, increasing stream id
        goaway(c, kProtocolError);
        return false;
      }
      c.last_sid = sid;
      if (c.streams.size() >= kMaxStreams) {
        rst_stream(c, sid, kRefusedStream);
        return true;
      }
      Stream s;
      s.send_window = c.peer_init_window;
      s.method = ps.method;
      s.path = std::move(ps.unknown);
      s.headers_done = true;
      it = c.streams.emplace(sid, std::move(s)).first;
    }
    if (flags & kEndStream) {
      dispatch(c, sid, it->second, it->second.data);
      drop_data(c, it->second);
    }
    return true;
  };
  auto process = [&](Conn& c) -> bool {  // false = fatal, close after flushing
    size_t pos = 0;
    if (!c.preface) {
      if (c.in.size() < kPrefaceLen) return true;
      if (std::memcmp(c.in.data(), kPreface, kPrefaceLen) != 0) {
        goaway(c, kProtocolError);
        return false;
      }
      pos = kPrefaceLen;
      c.preface = true;
    }
    while (c.in.size() - pos >= 9) {
      const uint8_t* h = reinterpret_cast<const uint8_t*>(c.in.data() + pos);
      const uint32_t len = (static_cast<uint32_t>(h[0]) << 16) | (static_cast<uint32_t>(h[1]) << 8) | h[2];
      const uint8_t type = h[3], flags = h[4];
      const uint32_t sid = get_u32(h + 5) & 0x7FFFFFFFu;
      if (len > kMaxFrame) {
        goaway(c, kFrameSizeError);
        return false;
      }
      if (c.in.size() - pos < 9 + len) break;
      const uint8_t* p = h + 9;
      pos += 9 + len;
      if (c.cont_sid && type != kContinuation) {
        goaway(c, kProtocolError);
        return false;
      }
      switch (type) {
        case kSettings: {
          if (sid != 0 || (!(flags & kAck) && len % 6)) {
            goaway(c, kProtocolError);
            return false;
          }
          if (flags & kAck) break;
          for (uint32_t i = 0; i + 6 <= len; i += 6) {
            const uint16_t id = static_cast<uint16_t>((p[i] << 8) | p[i + 1]);
            const uint32_t v = get_u32(p + i + 2);
            if (id == 4) {  // INITIAL_WINDOW_SIZE: adjust every open stream by the delta
              if (v > 0x7FFFFFFFu) {
                goaway(c, kFlowControlError);
                return false;
              }
              const int64_t delta = static_cast<int64_t>(v) - c.peer_init_window;
              c.peer_init_window = v;
              for (auto& kv : c.streams) {
                kv.second.send_window += delta;
                if (kv.second.send_window > kMaxWindow) {
                  goaway(c, kFlowControlError);
                  return false;
                }
              }
            } else if (id == 5) {
              if (v < 16384 || v > 16777215) {
                goaway(c, kProtocolError);
                return false;
              }
              c.peer_max_frame = v;
            }
          }
          frame(&c.out, 0, kSettings, kAck, 0);
          for (auto& kv : c.streams) flush_stream(c, kv.first, kv.second);
          break;
        }
        case kPing:
          if (len != 8) {
            goaway(c, kFrameSizeError);
            return false;
          }
          if (!(flags & kAck)) {
            frame(&c.out, 8, kPing, kAck, 0);
            c.out.append(reinterpret_cast<const char*>(p), 8);
          }
          break;
        case kWindowUpdate: {
          if (len != 4) {
            goaway(c, kFrameSizeError);
            return false;
          }
          const uint32_t inc = get_u32(p) & 0x7FFFFFFFu;
          if (sid == 0) {
            c.send_window += inc;
            if (inc == 0 || c.send_window > kMaxWindow) {
              goaway(c, inc == 0 ? kProtocolError : kFlowControlError);
              return false;
            }
            for (auto& kv : c.streams) flush_stream(c, kv.first, kv.second);
          } else {
            auto it = c.streams.find(sid);
            if (it != c.streams.end()) {
              it->second.send_window += inc;
              if (inc == 0 || it->second.send_window > kMaxWindow) {
                rst_stream(c, sid, inc == 0 ? kProtocolError : kFlowControlError);
                it->second.done = true;
                it->second.pend.clear();
                it->second.trailers_after = false;
              } else {
                flush_stream(c, sid, it->second);
              }
            }
          }
          break;
        }
        case kHeaders: {
          if (sid == 0) {
            goaway(c, kProtocolError);
            return false;
          }
          size_t off = 0, pad = 0;
          if (flags & kPadded) {
            if (len < 1) return goaway(c, kProtocolError), false;
            pad = p[0];
            off = 1;
          }
          if (flags & kPriorityFlag) off += 5;
          if (off + pad > len) {
            goaway(c, kProtocolError);
            return false;
          }
          // Fast unary path (every kubelet unary call): a complete header block for a new
          // stream, followed in the buffer by the stream's one DATA frame with END_STREAM.
          // Decoded and dispatched in place from the frames, on a stack Stream that enters
          // the stream map only if it outlives the call (flow-controlled response,
          // ListAndWatch, an asynchronous PreStartContainer).
          if ((flags & (kEndHeaders | kEndStream)) == kEndHeaders && !c.cont_sid && (sid & 1) && sid > c.last_sid &&
              c.streams.size() < kMaxStreams && c.in.size() - pos >= 9) {
            const uint8_t* dh = reinterpret_cast<const uint8_t*>(c.in.data() + pos);
            const uint32_t dlen = (static_cast<uint32_t>(dh[0]) << 16) | (static_cast<uint32_t>(dh[1]) << 8) | dh[2];
            if (dh[3] == kData && (dh[4] & (kEndStream | kPadded)) == kEndStream && (get_u32(dh + 5) & 0x7FFFFFFFu) == sid &&
                dlen <= kMaxFrame && c.in.size() - pos >= 9 + dlen) {
              PathSink ps;
              if (!c.dec.decode(p + off, len - off - pad, on_header, &ps)) {
                goaway(c, kCompressionError);
                return false;
              }
              c.last_sid = sid;
              Stream s;
              s.send_window = c.peer_init_window;
              s.method = ps.method;
              s.path = std::move(ps.unknown);
              s.headers_done = true;
              const char* body = reinterpret_cast<const char*>(dh + 9);
              pos += 9 + dlen;
              c.recv_unacked += dlen;
              dispatch(c, sid, s, std::string_view(body, dlen));
              if (!s.done || !s.pend.empty()) c.streams.emplace(sid, std::move(s));
              if (c.recv_unacked > kLocalWindow / 2) {
                window_update(&c.out, 0, static_cast<uint32_t>(c.recv_unacked));
                c.recv_unacked = 0;
              }
              break;
            }
          }
          c.hblock.assign(reinterpret_cast<const char*>(p + off), len - off - pad);
          if (flags & kEndHeaders) {
            if (!on_headers_block(c, sid, flags)) return false;
          } else {
            c.cont_sid = sid;
            c.cont_flags = flags;
          }
          break;
        }
        case kContinuation:
          if (sid != c.cont_sid || c.hblock.size() + len > (1u << 20)) {
            goaway(c, kProtocolError);
            return false;
          }
          c.hblock.append(reinterpret_cast<const char*>(p), len);
          if (flags & kEndHeaders) {
            const uint32_t s = c.cont_sid;
            c.cont_sid = 0;
            if (!on_headers_block(c, s, c.cont_flags)) return false;
          }
          break;
        case kData: {
          if (sid == 0) {
            goaway(c, kProtocolError);
            return false;
          }
          size_t off = 0, pad = 0;
          if (flags & kPadded) {
            if (len < 1) return goaway(c, kProtocolError), false;
            pad = p[0];
            off = 1;
          }
          if (off + pad > len) {
            goaway(c, kProtocolError);
            return false;
          }
          c.recv_unacked += len;
          auto it = c.streams.find(sid);
          if (it != c.streams.end() && it->second.dispatched && !it->second.done) {
            rst_stream(c, sid, kStreamClosed);  // DATA after the request half-closed
            it->second.done = true;
          } else if (it != c.streams.end() && !it->second.done && it->second.data.empty() &&
                     (flags & kEndStream)) {
            // the whole request in one DATA frame (every kubelet unary call): dispatch
            // from the frame in place, no per-stream copy
            dispatch(c, sid, it->second,
                     std::string_view(reinterpret_cast<const char*>(p + off), len - off - pad));
          } else if (it != c.streams.end() && !it->second.done) {
            Stream& s = it->second;
            s.data.append(reinterpret_cast<const char*>(p + off), len - off - pad);
            c.buffered += len - off - pad;
            s.recv_unacked += len;
            if (s.data.size() > kMaxMessage + 5 || c.buffered > kMaxBuffered) {
              send_error(c, sid, s, 8, "request exceeds the receive limit");  // RESOURCE_EXHAUSTED
              drop_data(c, s);
            } else if (flags & kEndStream) {
              dispatch(c, sid, s, s.data);
              drop_data(c, s);
            } else if (s.recv_unacked > kLocalWindow / 2) {
              window_update(&c.out, sid, static_cast<uint32_t>(s.recv_unacked));
              s.recv_unacked = 0;
            }
          }
          if (c.recv_unacked > kLocalWindow / 2) {
            window_update(&c.out, 0, static_cast<uint32_t>(c.recv_unacked));
            c.recv_unacked = 0;
          }
          break;
        }
        case kRstStream: {
          auto it = c.streams.find(sid);
          if (it != c.streams.end()) {
            drop_data(c, it->second);
            if (it->second.law) law_closed(w);
            c.streams.erase(it);
          }
          break;
        }
        case kGoaway:
          c.closing = true;
          break;
        default:  // PRIORITY, PUSH_PROMISE (invalid from clients; ignored), unknown
          break;
      }
    }
    c.in.erase(0, pos);
    for (auto it = c.streams.begin(); it != c.streams.end();)
      if (it->second.done && it->second.pend.empty()) {
        drop_data(c, it->second);
        if (it->second.law) law_closed(w);
        it = c.streams.erase(it);
      } else {
        ++it;
      }
    return true;
  };

  uint64_t seen_version = table->version();
  // canned requests for the keep-warm tick: typical request header blocks and an
  // Allocate / GetPreferredAllocation of the table's first device
  std::string warm_hdrs, warm_hdrs_pref, warm_alloc, warm_pref, warm_out;
  {
    auto headers = [](std::string* h, std::string_view path) {
      hpack::encode_indexed(h, 3);                                    // :method POST
      hpack::encode_indexed(h, 6);                                    // :scheme http
      hpack::encode_literal_name_index(h, 4, path);                   // :path
      hpack::encode_literal_name_index(h, 1, "localhost");            // :authority
      hpack::encode_literal(h, "content-type", "application/grpc");
      hpack::encode_literal(h, "te", "trailers");
    };
    headers(&warm_hdrs, "/v1beta1.DevicePlugin/Allocate");
    headers(&warm_hdrs_pref, "/v1beta1.DevicePlugin/GetPreferredAllocation");
  }
  auto warm_requests = [&] {  // for the table's first device (again after a table swap)
    warm_alloc.clear();
    warm_pref.clear();
    const std::vector<std::string> ids = table->ids();
    if (!ids.empty()) {
      std::string ctr;
      pb::put_bytes(&ctr, 1, ids[0]);
      pb::put_bytes(&warm_alloc, 1, ctr);
      std::string pctr;
      pb::put_bytes(&pctr, 1, ids[0]);
      pb::put_bytes(&pctr, 2, ids[0]);
      pb::put_int_nz(&pctr, 3, 1);
      pb::put_bytes(&warm_pref, 1, pctr);
    }
  };
  warm_requests();
  // The full tick: a private in-memory connection (no socket) gets an Allocate and a
  // GetPreferredAllocation as kubelet's client would frame them, and the worker runs them
  // through the same path as a real request - frame parsing, HPACK, dispatch, the table,
  // response framing - then drops the answer.  Marked internal: nothing is counted.
  std::unique_ptr<Conn> warm_conn;
  uint32_t warm_sid = 1;
  auto warm_full = [&] {
    if (warm_alloc.empty()) return;
    if (!warm_conn || warm_sid > (1u << 30)) {  // (re)start: preface + empty SETTINGS
      warm_conn = std::make_unique<Conn>();
      warm_conn->internal = true;
      warm_sid = 1;
      warm_conn->in.assign(kPreface, kPrefaceLen);
      frame(&warm_conn->in, 0, kSettings, 0, 0);
    }
    Conn& c = *warm_conn;
    for (int k = 0; k < 2; ++k) {
      const std::string& h = k == 0 ? warm_hdrs : warm_hdrs_pref;
      const std::string& m = k == 0 ? warm_alloc : warm_pref;
      frame(&c.in, static_cast<uint32_t>(h.size()), kHeaders, kEndHeaders, warm_sid);
      c.in.append(h);
      frame(&c.in, static_cast<uint32_t>(5 + m.size()), kData, kEndStream, warm_sid);
      grpc_prefix(&c.in, m.size());
      c.in.append(m);
      warm_sid += 2;
    }
    if (!process(c)) warm_conn.reset();  // cannot happen with these frames; start over if it does
    if (warm_conn) {
      c.out.clear();
      c.out_off = 0;
      c.send_window = 65535;  // no peer sends WINDOW_UPDATEs here
    }
  };
  int64_t last_activity = mono_ns();
  const int64_t spin_ns = static_cast<int64_t>(busy_poll_us_) * 1000;
  const int64_t admission_ns = static_cast<int64_t>(admission_poll_us_) * 1000;
  int64_t spin_until = 0;  // busy-poll window end (mono ns); 0 = closed
  SpinGuard guard;
  bool polite = false;  // the open window gives way to other threads (see SpinGuard)
  ContentionDetector contention;  // grpc.coreEscape
  unsigned escape_rotate = static_cast<unsigned>(w->index);
  while (!stop_.load(std::memory_order_relaxed)) {
    if (table_gen_.load(std::memory_order_acquire) != table_gen) {
      // hot table swap (set_table): serve from the new table from here on and send every
      // ListAndWatch stream its device list (versions of two tables do not compare)
      {
        std::lock_guard<std::mutex> sk(swap_mu_);
        table = table_;
        table_gen = table_gen_.load(std::memory_order_relaxed);
      }
      for (auto& kv : w->conns)
        for (auto& st : kv.second->streams)
          if (st.second.law) st.second.law_version = 0;
      warm_requests();
      seen_version = 0;  // table versions start at 1: the push below runs
    }
    if (inject_worker_fault_.load(std::memory_order_relaxed)) {
      int armed = 1;
      if (inject_worker_fault_.compare_exchange_strong(armed, 0)) throw std::runtime_error("injected worker fault");
    }
    int n;
    const bool polling = spin_until != 0;
    if (polling) {
      // (polling the last request's connection with a direct recv instead, one syscall less
      // on the request's path, measured slower: 2.87 vs 2.67 us p50, profiles/r5/ab_hot_recv.jsonl)
      n = epoll_wait(w->ep, evs.data(), static_cast<int>(evs.size()), 0);
      if (n == 0) {
        const int64_t now = mono_ns();
        if (now >= spin_until) {
          spin_until = 0;
        } else if (!polite) {
          const int gap = poll_gap_ns_.load(std::memory_order_relaxed);
          if (gap > 0) {
            const int64_t until = now + gap;
            do {
              cpu_relax();
            } while (mono_ns() < until);
          } else {
            cpu_relax();
          }
        } else if (!guard.keep_polling(now)) {  // preempted: the CPU is wanted (maybe by the client)
          spin_until = 0;
          poll_windows_yielded_.add();
        } else {
          guard.pause(now);
        }
        continue;
      }
    } else {
      // Within the admission window (a kubelet RPC less than active_window_ms ago): keep-warm
      // ticks, and a worker that holds a connection wakes at least every idle_wake_ms (keeps
      // its core out of deep idle states: what the first request after a long idle pays most
      // of).  Outside it: nothing runs; the worker sleeps until a request, a notify, a table
      // swap or stop (all of which write its eventfd), with a 5 s safety tick.
      const int window = active_window_ms_.load(std::memory_order_relaxed);
      const bool active = window == 0 || (last_rpc != 0 && mono_ns() - last_rpc < static_cast<int64_t>(window) * 1000000);
      const int warm = active ? keep_warm_ms_.load(std::memory_order_relaxed) : 0;
      const int wake = (!active || w->conns.empty()) ? 0 : idle_wake_ms_.load(std::memory_order_relaxed);
      int timeout = warm > 0 ? std::min(warm, 100) : (active ? 100 : 5000);
      if (wake > 0) timeout = std::min(timeout, wake);
      n = epoll_wait(w->ep, evs.data(), static_cast<int>(evs.size()), timeout);
      if (n == 0) idle_wakeups_.fetch_add(1, std::memory_order_relaxed);
      if (n == 0 && warm > 0 && !w->conns.empty() && !warm_alloc.empty()) {
        const int64_t now = mono_ns();
        if (now - last_activity >= static_cast<int64_t>(warm) * 1000000) {
          if (keep_warm_full_.load(std::memory_order_relaxed)) {
            warm_full();
          } else {
            hpack::Decoder d(4096);
            d.decode(reinterpret_cast<const uint8_t*>(warm_hdrs.data()), warm_hdrs.size(),
                     [](void*, std::string_view, std::string_view) {}, nullptr);
            warm_out.clear();
            table->allocate(warm_alloc, &warm_out);
            warm_out.clear();
            table->preferred(warm_pref, &warm_out);
          }
          warm_ticks_.fetch_add(1, std::memory_order_relaxed);
          last_activity = now;
          if (trace_) {
            const int cpu = sched_getcpu();
            last_cpu = static_cast<uint16_t>(cpu < 0 ? 0xFFFF : cpu);
          }
        }
      }
    }
    if (n > 0) {
      const int64_t now = mono_ns();
      wake_idle = now - last_activity;
      last_activity = now;
      wake_ts = now;
      wake_spin = polling;
    }
    bool law_tick = false;
    bool got_input = false;  // this event carried input: (re)open the busy-poll window after the send
    for (int i = 0; i < n; ++i) {
      const int fd = evs[i].data.fd;
      if (fd == w->efd) {
        uint64_t x;
        while (read(w->efd, &x, sizeof(x)) > 0) {
        }
        law_tick = true;
        continue;
      }
      if (fd == w->done->efd) {  // asynchronous RPCs completed: answer their streams
        uint64_t x;
        while (read(w->done->efd, &x, sizeof(x)) > 0) {
        }
        std::vector<AsyncDone::Item> items;
        {
          std::lock_guard<std::mutex> lk(w->done->mu);
          items.swap(w->done->items);
        }
        for (auto& it : items) {
          auto ci = w->conns.find(it.fd);
          if (ci == w->conns.end() || ci->second->serial != it.serial) continue;  // client went away
          Conn* c = ci->second.get();
          auto si = c->streams.find(it.sid);
          if (si == c->streams.end() || si->second.done) continue;
          if (it.ok) {
            send_headers(*c, it.sid);
            send_message(*c, it.sid, si->second, std::string_view(), true);  // PreStartContainerResponse{}
          } else {
            send_error(*c, it.sid, si->second, 2, it.error);  // UNKNOWN, like a Go handler error
          }
          table->observe(kRpcPreStart, (mono_ns() - it.t0) * 1e-9, !it.ok);
          flush(c);
        }
        continue;
      }
      if (fd == listen_fd_) {
        if (evs[i].events & (EPOLLERR | EPOLLHUP)) {  // the listening socket itself broke
          epoll_ctl(w->ep, EPOLL_CTL_DEL, listen_fd_, nullptr);
          fail("listening socket " + path_ + " reported an error");
          continue;
        }
        for (;;) {
          bool shed = false;
          const int cfd = accept_or_shed(listen_fd_, nullptr, nullptr, &spare, &shed);
          if (cfd < 0) {
            if (shed) {
              shed_.add();
              continue;
            }
            // only a listener that is gone or no longer listening is a server fault;
            // the rest (ECONNABORTED, EPROTO, ENOBUFS, pending network errors) concern
            // one connection and the next accept may succeed
            if (errno == EBADF || errno == EINVAL || errno == ENOTSOCK) {
              const int e = errno;
              epoll_ctl(w->ep, EPOLL_CTL_DEL, listen_fd_, nullptr);
              fail("accept on " + path_ + ": " + strerror(e));
            }
            break;
          }
          Worker* t = pick_least_loaded(workers_, w);  // this one on a tie
          auto c = std::make_unique<Conn>();
          c->fd = cfd;
          {
            int zero = 0;  // peek offset 0: MSG_PEEK reads advance it, consuming reads take it back
            c->peek = peek_reads_.load(std::memory_order_relaxed) &&
                      setsockopt(cfd, SOL_SOCKET, SO_PEEK_OFF, &zero, sizeof(zero)) == 0;
          }
          // server preface: SETTINGS(MAX_CONCURRENT_STREAMS, INITIAL_WINDOW_SIZE) + conn window
          frame(&c->out, 12, kSettings, 0, 0);
          c->out.push_back(0);
          c->out.push_back(3);
          put_u32(&c->out, kMaxStreams);
          c->out.push_back(0);
          c->out.push_back(4);
          put_u32(&c->out, static_cast<uint32_t>(kLocalWindow));
          window_update(&c->out, 0, static_cast<uint32_t>(kLocalWindow - 65535));
          conns_.fetch_add(1);
          struct epoll_event ev {};
          ev.events = EPOLLIN | EPOLLRDHUP;
          ev.data.fd = cfd;
          if (t != w) {  // EPOLLOUT: the owner wakes at once, adopts it and sends the preface
            c->want_out = true;
            {
              std::lock_guard<std::mutex> lk(t->in_mu);
              t->incoming.push_back(std::move(c));
            }
            ev.events |= EPOLLOUT;
            epoll_ctl(t->ep, EPOLL_CTL_ADD, cfd, &ev);
            continue;
          }
          c->serial = w->next_serial++;
          epoll_ctl(w->ep, EPOLL_CTL_ADD, cfd, &ev);
          Conn* cp = c.get();
          w->conns.emplace(cfd, std::move(c));
          flush(cp);
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
      if (evs[i].events & EPOLLERR) {
        close_conn(fd);
        continue;
      }
      bool peer_closed = false;
      if (evs[i].events & (EPOLLIN | EPOLLRDHUP | EPOLLHUP)) {
        for (;;) {
          const ssize_t r = recv(fd, rbuf, sizeof(rbuf), c->peek ? MSG_PEEK : 0);
          if (r > 0) {
            c->in.append(rbuf, static_cast<size_t>(r));
            if (c->peek) c->peeked += static_cast<size_t>(r);
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
        if (trace_) recv_done = mono_ns();
        if (!process(*c)) c->closing = true;
        got_input = true;
      }
      if (c->out.size() - c->out_off > kMaxPendingOut) {  // e.g. a PING flood that is never read
        close_conn(fd);
        continue;
      }
      if (!trace_pending.empty()) send_begin = mono_ns();
      const bool alive = flush(c);  // the response goes out first; the bookkeeping follows
      // (a call answered inside a busy-poll window: its service time feeds the core
      // contention check, grpc.coreEscape)
      const int64_t sent_at = got_input && wake_spin && core_escape_.load(std::memory_order_relaxed) ? mono_ns() : 0;
      if (alive && c->peeked) consume_peeked(c);
      if (!trace_pending.empty()) stamp_sent();
      if (!pending_obs.empty()) apply_observes();
      if (sent_at && alive && contention.note(sent_at - wake_ts, sent_at) && peer_on_sibling(c->fd, sched_getcpu(), sent_at) &&
          escape_core(escape_rotate++) >= 0)
        core_escapes_.fetch_add(1, std::memory_order_relaxed);
      if (got_input) {
        got_input = false;
        const int64_t window = admitting ? std::max(spin_ns, admission_ns) : spin_ns;
        if (window > 0) {
          const int64_t now = mono_ns();
          spin_until = std::max(spin_until, now + window);
          if (admitting && admission_ns > spin_ns) admission_windows_.add();
          // only a window that reaches past a busy-poll window (an admission window, or
          // what is left of one) is long enough to keep a client on this CPU waiting for
          // long; a busy-poll window (tens of us) polls throughout, so a call that comes
          // after a short client hiccup still finds the worker awake
          polite = spin_until - now > spin_ns;
          if (polite) guard.reset(now);
        }
        admitting = false;
      }
      if (!alive) continue;
      if (peer_closed) close_conn(fd);
    }
    if (!pending_obs.empty()) apply_observes();  // (a connection closed before its flush)
    // ListAndWatch: push on notify() and on any version change seen by the poll tick
    const uint64_t v = table->version();
    if (law_tick || v != seen_version) {
      seen_version = v;
      std::vector<int> fds;
      for (auto& kv : w->conns) fds.push_back(kv.first);
      for (int fd : fds) {
        auto it = w->conns.find(fd);
        if (it == w->conns.end()) continue;
        push_law(it->second.get());
        flush(it->second.get());
      }
    }
  }
  adopt();
  // shutdown: finish open streams with OK trailers (like the reference's ListAndWatch
  // returning nil on stop), GOAWAY, best-effort flush, close.
  for (auto& kv : w->conns) {
    Conn* c = kv.second.get();
    for (auto& s : c->streams) {
      if (s.second.done) continue;
      frame(&c->out, static_cast<uint32_t>(ok_trailers().size()), kHeaders, kEndHeaders | kEndStream, s.first);
      c->out.append(ok_trailers());
    }
    goaway(*c, kNoError);
    (void)!send(c->fd, c->out.data() + c->out_off, c->out.size() - c->out_off, MSG_NOSIGNAL | MSG_DONTWAIT);
    ::close(c->fd);
    conns_.fetch_sub(1);
  }
  w->conns.clear();
  w->law_open.store(0, std::memory_order_relaxed);
}

// ------------------------------------------------------------------- client

H2Client::H2Client(const std::string& socket_path, double timeout_s)
    : timeout_ms_(static_cast<int>(timeout_s * 1000)) {
  struct sockaddr_un addr {};
  addr.sun_family = AF_UNIX;
  if (socket_path.size() >= sizeof(addr.sun_path)) throw std::runtime_error("socket path too long");
  std::memcpy(addr.sun_path, socket_path.c_str(), socket_path.size() + 1);
  fd_ = socket(AF_UNIX, SOCK_STREAM | SOCK_CLOEXEC, 0);
  if (fd_ < 0 || connect(fd_, reinterpret_cast<sockaddr*>(&addr), sizeof(addr)) != 0) {
    const int e = errno;
    close();
    throw std::runtime_error("H2Client: connect " + socket_path + ": " + strerror(e));
  }
  set_recv_timeout(timeout_ms_);
  std::string o(kPreface, kPrefaceLen);
  frame(&o, 6, kSettings, 0, 0);
  o.push_back(0);
  o.push_back(4);
  put_u32(&o, static_cast<uint32_t>(kLocalWindow));
  window_update(&o, 0, static_cast<uint32_t>(kLocalWindow - 65535));
  send_all(o);
}

H2Client::~H2Client() { close(); }

void H2Client::close() {
  if (fd_ >= 0) ::close(fd_);
  fd_ = -1;
}

void H2Client::set_recv_timeout(int ms) {
  struct timeval tv;
  tv.tv_sec = ms / 1000;
  tv.tv_usec = (ms % 1000) * 1000;
  setsockopt(fd_, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof(tv));
}

void H2Client::send_all(const std::string& s) {
  size_t off = 0;
  while (off < s.size()) {
    const ssize_t n = send(fd_, s.data() + off, s.size() - off, MSG_NOSIGNAL);
    if (n < 0) {
      if (errno == EINTR) continue;
      throw std::runtime_error(std::string("H2Client: send: ") + strerror(errno));
    }
    off += static_cast<size_t>(n);
  }
}

bool H2Client::read_frame(uint8_t* type, uint8_t* flags, uint32_t* sid, std::string_view* payload) {
  // Frames are parsed in place: *payload views in_, valid until the next read_frame (every
  // caller uses it before reading on), and the consumed prefix goes only when more bytes
  // are needed - no per-frame copy or memmove on the response path.
  char buf[32768];
  for (;;) {
    const size_t avail = in_.size() - in_off_;
    if (avail >= 9) {
      const uint8_t* h = reinterpret_cast<const uint8_t*>(in_.data() + in_off_);
      const uint32_t len = (static_cast<uint32_t>(h[0]) << 16) | (static_cast<uint32_t>(h[1]) << 8) | h[2];
      if (avail >= 9 + static_cast<size_t>(len)) {
        *type = h[3];
        *flags = h[4];
        *sid = get_u32(h + 5) & 0x7FFFFFFFu;
        *payload = std::string_view(in_.data() + in_off_ + 9, len);
        in_off_ += 9 + len;
        return true;
      }
    }
    if (in_off_ == in_.size()) in_.clear();
    else if (in_off_ > 0) in_.erase(0, in_off_);
    in_off_ = 0;
    // blocking recv bounded by SO_RCVTIMEO: one syscall per response instead of poll + recv
    const ssize_t r = recv(fd_, buf, sizeof(buf), 0);
    if (stamp_recv_) recv_ret_ns_ = mono_ns();
    if (r <= 0) {
      if (r < 0 && errno == EINTR) continue;
      if (r < 0 && (errno == EAGAIN || errno == EWOULDBLOCK))
        throw std::runtime_error("H2Client: timed out waiting for response");
      return false;
    }
    in_.append(buf, static_cast<size_t>(r));
  }
}


bool H2Client::handle_control(uint8_t type, uint8_t flags, uint32_t sid, std::string_view payload) {
  std::string ctl;
  if (type == kSettings) {
    if (!(flags & kAck)) {
      for (size_t i = 0; i + 6 <= payload.size(); i += 6) {
        const uint8_t* p = reinterpret_cast<const uint8_t*>(payload.data()) + i;
        const uint16_t id = static_cast<uint16_t>((p[0] << 8) | p[1]);
        const uint32_t v = get_u32(p + 2);
        if (id == 4) {
          stream_window_ += static_cast<int64_t>(v) - stream_window_init_;
          stream_window_init_ = v;
        } else if (id == 5) {
          peer_max_frame_ = v;
        }
      }
      frame(&ctl, 0, kSettings, kAck, 0);
    }
  } else if (type == kPing) {
    if (!(flags & kAck)) {
      frame(&ctl, 8, kPing, kAck, 0);
      ctl.append(payload);
    }
  } else if (type == kWindowUpdate && payload.size() == 4) {
    const uint32_t inc = get_u32(reinterpret_cast<const uint8_t*>(payload.data())) & 0x7FFFFFFFu;
    if (sid == 0) send_window_ += inc;
    else if (sid == cur_sid_) stream_window_ += inc;
  } else if (type == kGoaway) {
    // RFC 7540 6.8: streams up to last_stream_id may still be answered (a gRPC server
    // shutting down gracefully sends last = 2^31-1 first); only a stream above it was
    // not processed.  No new stream goes out on this connection afterwards.
    const auto* g = reinterpret_cast<const uint8_t*>(payload.data());
    const uint32_t last = payload.size() >= 8 ? get_u32(g) & 0x7FFFFFFFu : 0;
    const uint32_t code = payload.size() >= 8 ? get_u32(g + 4) : 0;
    goaway_ = true;
    if (cur_sid_ > last || watch_sid_ > last)
      throw std::runtime_error("H2Client: GOAWAY (error code " + std::to_string(code) + ", last stream " +
                               std::to_string(last) + "): the request was not processed");
  } else {
    return false;
  }
  if (!ctl.empty()) send_all(ctl);
  return true;
}

void H2Client::send_request(uint32_t sid, std::string_view path, std::string_view req) {
  if (goaway_) throw std::runtime_error("H2Client: the server sent GOAWAY: open a new connection");
  cur_sid_ = sid;
  stream_window_ = stream_window_init_;
  std::string& o = out_buf_;  // capacity reused across calls
  o.clear();
  if (path != hpath_) {  // a client calls one or two methods: keep the encoded block
    hpath_.assign(path.data(), path.size());
    hblock_ = request_headers(path);
  }
  frame(&o, static_cast<uint32_t>(hblock_.size()), kHeaders, kEndHeaders, sid);
  o.append(hblock_);
  std::string& body = body_buf_;
  body.clear();
  grpc_prefix(&body, req.size());
  body.append(req.data(), req.size());
  size_t off = 0;
  while (off < body.size()) {
    int64_t n = std::min<int64_t>({static_cast<int64_t>(body.size() - off), send_window_, stream_window_,
                                   static_cast<int64_t>(peer_max_frame_)});
    if (n <= 0) {  // blocked on flow control: flush what we have, wait for WINDOW_UPDATE
      send_all(o);
      o.clear();
      uint8_t type, flags;
      uint32_t fsid;
      std::string_view payload;
      if (!read_frame(&type, &flags, &fsid, &payload)) throw std::runtime_error("H2Client: connection closed");
      if (!handle_control(type, flags, fsid, payload) && fsid == sid && (type == kRstStream))
        throw std::runtime_error("H2Client: stream reset while sending");
      continue;
    }
    const bool last = off + static_cast<size_t>(n) == body.size();
    frame(&o, static_cast<uint32_t>(n), kData, last ? kEndStream : 0, sid);
    o.append(body.data() + off, static_cast<size_t>(n));
    off += static_cast<size_t>(n);
    send_window_ -= n;
    stream_window_ -= n;
  }
  send_all(o);
}

int H2Client::unary(std::string_view path, std::string_view req, std::string* resp, std::string* message) {
  const uint32_t sid = next_sid_;
  next_sid_ += 2;
  send_request(sid, path, req);
  std::string& data = data_buf_;
  data.clear();
  int status = -1;
  uint8_t type, flags;
  uint32_t fsid;
  std::string_view payload;
  for (;;) {
    if (!read_frame(&type, &flags, &fsid, &payload)) throw std::runtime_error("H2Client: connection closed");
    if (handle_control(type, flags, fsid, payload)) continue;
    if (fsid == sid && type == kData) {
      data.append(payload);
      conn_consumed_ += static_cast<int64_t>(payload.size());
    } else if (fsid == sid && type == kHeaders) {
      struct Sink {
        int* status;
        std::string* message;
      } sink{&status, message};
      auto fn = [](void* ctx, std::string_view name, std::string_view value) {
        auto* k = static_cast<Sink*>(ctx);
        if (name == "grpc-status") {
          int v = 0;
          for (char ch : value) {
            if (ch < '0' || ch > '9') break;
            v = v * 10 + (ch - '0');
          }
          *k->status = v;
        } else if (name == "grpc-message" && k->message) {
          k->message->assign(value.data(), value.size());
        }
      };
      if (!dec_.decode(reinterpret_cast<const uint8_t*>(payload.data()), payload.size(), fn, &sink))
        throw std::runtime_error("H2Client: bad HPACK from server");
    } else if (fsid == sid && type == kRstStream) {
      throw std::runtime_error("H2Client: stream reset");
    }
    if (conn_consumed_ > kLocalWindow / 2) {
      std::string ctl;
      window_update(&ctl, 0, static_cast<uint32_t>(conn_consumed_));
      conn_consumed_ = 0;
      send_all(ctl);
    }
    if (fsid == sid && (flags & kEndStream) && (type == kHeaders || type == kData)) break;
  }
  if (resp) {
    resp->clear();
    if (data.size() >= 5) resp->assign(data.data() + 5, data.size() - 5);
  }
  return status;
}

void H2Client::send_unary_nowait(std::string_view path, std::string_view req) {
  const uint32_t sid = next_sid_;
  next_sid_ += 2;
  send_request(sid, path, req);
}

int H2Client::first_stream_message(std::string_view path, std::string_view req, std::string* resp) {
  const uint32_t sid = next_sid_;
  next_sid_ += 2;
  send_request(sid, path, req);
  std::string data;
  uint8_t type, flags;
  uint32_t fsid;
  std::string_view payload;
  for (;;) {
    if (!read_frame(&type, &flags, &fsid, &payload)) throw std::runtime_error("H2Client: connection closed");
    if (handle_control(type, flags, fsid, payload)) continue;
    if (fsid == sid && type == kData) {
      data.append(payload);
      conn_consumed_ += static_cast<int64_t>(payload.size());
      if (data.size() >= 5 && data.size() >= 5 + get_u32(reinterpret_cast<const uint8_t*>(data.data()) + 1)) break;
    }
    if (fsid == sid && (flags & kEndStream)) break;
  }
  std::string rst;
  frame(&rst, 4, kRstStream, 0, sid);
  put_u32(&rst, 8);  // CANCEL
  send_all(rst);
  if (resp && data.size() >= 5) resp->assign(data.data() + 5, data.size() - 5);
  return 0;
}

void H2Client::open_stream(std::string_view path, std::string_view req) {
  watch_sid_ = next_sid_;
  next_sid_ += 2;
  watch_buf_.clear();
  watch_consumed_ = 0;
  send_request(watch_sid_, path, req);
}

int H2Client::next_stream_message(std::string* resp, int timeout_ms) {
  if (watch_sid_ == 0) throw std::runtime_error("H2Client: no open stream");
  set_recv_timeout(timeout_ms);
  struct Restore {
    H2Client* c;
    ~Restore() { c->set_recv_timeout(c->timeout_ms_); }
  } restore{this};
  uint8_t type, flags;
  uint32_t fsid;
  std::string_view payload;
  for (;;) {
    if (watch_buf_.size() >= 5) {
      const uint32_t len = get_u32(reinterpret_cast<const uint8_t*>(watch_buf_.data()) + 1);
      if (watch_buf_.size() >= 5 + static_cast<size_t>(len)) {
        if (resp) resp->assign(watch_buf_.data() + 5, len);
        watch_buf_.erase(0, 5 + static_cast<size_t>(len));
        return 0;
      }
    }
    if (!read_frame(&type, &flags, &fsid, &payload)) throw std::runtime_error("H2Client: connection closed");
    if (handle_control(type, flags, fsid, payload)) continue;
    if (fsid != watch_sid_) continue;
    if (type == kData) {
      watch_buf_.append(payload);
      conn_consumed_ += static_cast<int64_t>(payload.size());
      watch_consumed_ += static_cast<int64_t>(payload.size());
      std::string ctl;  // a long watch must keep both receive windows open
      if (conn_consumed_ > kLocalWindow / 2) {
        window_update(&ctl, 0, static_cast<uint32_t>(conn_consumed_));
        conn_consumed_ = 0;
      }
      if (watch_consumed_ > kLocalWindow / 2) {
        window_update(&ctl, watch_sid_, static_cast<uint32_t>(watch_consumed_));
        watch_consumed_ = 0;
      }
      if (!ctl.empty()) send_all(ctl);
    }
    if (type == kRstStream || (flags & kEndStream)) {
      watch_sid_ = 0;
      return -1;  // the server ended the stream (plugin stopped)
    }
  }
}

}  // namespace amdgpu_dp
