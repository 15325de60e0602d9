// Native gRPC-over-HTTP/2 (h2c, unix socket) server for the kubelet DevicePlugin API.
//
// Reference: each NvidiaDevicePlugin owns a grpc-go server on its unix socket
// (plugin/plugin.go:52,100-137).  The kubelet-facing RPCs are tiny, so their latency
// is framework overhead (SURVEY.md §3.4, §7.5 hard part 2); this server removes Python
// and the GIL from that path entirely: epoll workers parse HTTP/2 frames, decode HPACK,
// hand the protobuf bytes to the native DeviceTable and write one response burst
// (HEADERS + DATA + trailers) per call.  ListAndWatch streams stay open and are
// re-sent whenever the table's health version changes (eventfd wake-up).
//
// Also: H2Client, a minimal blocking client: the plugin registers with kubelet and
// probes its own socket through it (it speaks full HPACK, so it can talk to grpcio /
// grpc-go servers too).  The load generators built on it live in tests/native/loadgen.cpp
// (the bench extension), not in the plugin.
#pragma once

#include <atomic>
#include <functional>
#include <memory>
#include <mutex>
#include <sys/types.h>

#include <string>
#include <string_view>
#include <thread>
#include <vector>

#include "device_table.h"
#include "hpack.h"

namespace amdgpu_dp {

// Per-call trace of unary RPCs (grpc.callTraceFile): a ring of fixed-size records in a
// shared file mapping, so a benchmark in another process can attribute each slow call
// it measured to a segment of the server's handling.  All times CLOCK_MONOTONIC ns.
struct CallTraceEntry {
  int64_t t_ready = 0;     // the epoll_wait return that delivered the request
  int64_t t_dispatch = 0;  // request decoded, handler entered
  int64_t t_sent = 0;      // response handed to send() (the worker's flush of the batch)
  uint64_t conn = 0;       // worker index << 48 | connection serial
  int64_t idle_ns = 0;     // how long the worker had been without work (requests or keep-warm ticks)
  uint32_t seq = 0;        // write order + 1 (0: slot never written)
  uint8_t method = 0;      // Rpc
  uint8_t spinning = 0;    // 1: the worker was polling (busy-poll window), 0: it slept in epoll_wait
  uint16_t cpu = 0;        // CPU the worker ran on at dispatch
  uint16_t prev_cpu = 0;   // CPU of the worker's previous work (0xFFFF: none yet)
  uint16_t handle_ns = 0;  // t_dispatch -> the response's send() began (capped at 65535)
  uint32_t recv_ns = 0;    // t_ready -> the connection's recv() returned (the rest to t_dispatch is parsing)
};
static_assert(sizeof(CallTraceEntry) == 56, "trace record layout is read by bench.py");
struct CallTraceHeader {
  uint64_t magic = 0;      // kCallTraceMagic
  uint32_t version = 2;    // 2: worker i writes records [i * slice, (i + 1) * slice)
  uint32_t capacity = 0;   // records after the header
  std::atomic<uint64_t> next{0};  // unused since version 2 (kept for the layout)
  uint64_t pad[5] = {};
};
static_assert(sizeof(CallTraceHeader) == 64, "trace header layout is read by bench.py");
constexpr uint64_t kCallTraceMagic = 0x5452434c4c414344ull;  // "DCALLCRT"

class GrpcServer {
 public:
  // busy_poll_us: after a worker handles a request it keeps polling its epoll set
  // without sleeping for this long (0 = always block).  A kubelet admits a pod as a
  // burst of RPCs (GetPreferredAllocation, Allocate, PreStartContainer); a worker that
  // is still polling when the next one lands skips the idle-CPU wake-up, which is most
  // of a unix-socket round trip.  An idle plugin never spins: the window only opens on
  // request activity and closes after busy_poll_us without any.
  // admission_poll_us: the window after a GetPreferredAllocation.  Kubelet asks for the
  // preferred devices and then, after some bookkeeping of its own, Allocates them for
  // the same container: a longer window there (once per pod admission) keeps that
  // Allocate off the cold path.
  GrpcServer(std::string socket_path, int threads, int busy_poll_us = 0, int admission_poll_us = 0);
  ~GrpcServer();
  // Before start(): the table to serve.  While running: a hot swap (a plugin reload that
  // keeps the resource): every worker switches to the new table before its next request,
  // and every ListAndWatch stream is sent the new device list - kubelet's connection, its
  // registration and the socket stay as they are.
  void set_table(std::shared_ptr<DeviceTable> t);
  uint64_t table_swaps() const { return table_gen_.load(); }
  // Before start(): record every unary call in a ring of `capacity` CallTraceEntry records
  // mapped from `path` (created / truncated).  Costs one clock read per response batch.
  void set_call_trace(const std::string& path, int capacity);
  void start();  // throws std::runtime_error on bind/listen failure
  void stop();   // idempotent: trailers for open streams, GOAWAY, close, unlink socket
  void notify(); // wake ListAndWatch streams now (health changed)
  bool running() const { return running_.load(); }
  // Supervision (reference: the Serve crash-restart loop, plugin/plugin.go:107-129): a
  // worker thread that died on an exception, or a listener that broke (accept errors,
  // EPOLLERR/HUP on the socket), leaves the server unable to serve.  failure() names
  // the first such fault ("" while healthy); the plugin manager polls it and restarts
  // the server on a fresh socket.  The hook (set before start) runs once, on the thread
  // that hit the fault, right after failure() names it: the manager checks at once
  // instead of at its next poll.
  std::string failure() const;
  // (held by shared_ptr: copying it under fail_mu_ must not copy a Python callable,
  // whose copy takes the GIL - a thread polling failure() holds the GIL)
  void set_failure_hook(std::function<void()> hook) {
    auto h = hook ? std::make_shared<const std::function<void()>>(std::move(hook)) : nullptr;
    std::lock_guard<std::mutex> lk(fail_mu_);
    fail_hook_.swap(h);
  }  // (the previous hook is released here, after the lock)
  // Test-only fault injection: "worker" (the next worker to wake throws) or "listener"
  // (the listening socket is shut down underneath the workers).
  void inject_fault(const std::string& kind);
  uint64_t requests() const { return requests_.load(); }
  uint64_t shed_connections() const { return shed_.load(); }  // closed at accept: out of fds
  // polling windows opened by a GetPreferredAllocation (grpc.admissionPollUs), and
  // windows ended early because the worker was preempted (nothing counted per request)
  uint64_t admission_windows() const { return admission_windows_.load(); }
  uint64_t poll_windows_yielded() const { return poll_windows_yielded_.load(); }
  int connections() const { return conns_.load(); }
  // ListAndWatch streams open now (kubelet holds one per registered plugin; none while
  // registered means kubelet dropped the endpoint and waits for a new Register)
  int list_and_watch_streams() const;
  // CLOCK_MONOTONIC seconds (Python's time.monotonic) when a ListAndWatch stream last
  // ended, 0 if none has: the manager's stream watch times its grace from this, so it
  // can look only every few seconds while the node is quiet
  double list_and_watch_closed_at() const { return law_closed_ns_.load(std::memory_order_relaxed) * 1e-9; }
  // Keep-warm (grpc.keepWarmMs, 0 = off): a worker that holds a connection and has been
  // idle this long runs the request path on canned requests (HPACK decode of a typical
  // request header block, Allocate and GetPreferredAllocation through the table), so
  // kubelet's sparse calls do not find that code and data evicted.  Experimental: see
  // scripts/idle_probe.py --keep-warm-ms and BASELINE.md.
  void set_keep_warm_ms(int ms) { keep_warm_ms_.store(ms > 0 ? ms : 0); }
  // full: the tick runs canned requests through the whole request path of a private
  // in-memory connection (frame parsing, HPACK, dispatch, table, response framing);
  // otherwise only the HPACK decode and the table calls
  void set_keep_warm_full(bool on) { keep_warm_full_.store(on); }
  uint64_t warm_ticks() const { return warm_ticks_.load(); }
  // A worker that holds a connection sleeps at most this long at a time (0 = only the
  // keep-warm period / 100 ms): the wake-ups alone, no work, keep its core from settling
  // into a deep idle state whose exit the next request would pay (grpc.idleWakeMs).
  void set_idle_wake_ms(int ms) { idle_wake_ms_.store(ms > 0 ? ms : 0); }
  // Admission window (grpc.activeWindowMs, 0 = always): idle wake-ups and keep-warm ticks
  // run only for this long after a worker's last kubelet RPC.  Outside it the worker sleeps
  // in epoll_wait for up to 5 s at a time: an idle node pays next to nothing for the plugin,
  // and a pod admission's first call (GetPreferredAllocation) opens the window for the
  // Allocate that follows it.  (Sleeping workers wake every 5 s.)
  void set_active_window_ms(int ms) { active_window_ms_.store(ms > 0 ? ms : 0); }
  // Requests read with MSG_PEEK and consumed after the answer is sent (applies to
  // connections accepted from now on; off by default, grpc.peekReads).  See Worker::Conn::peek.
  void set_peek_reads(bool on) { peek_reads_.store(on); }
  // Busy-poll spacing (grpc.pollGapNs): between two empty polls of an open busy-poll
  // window the worker pauses this long (PAUSE instructions) instead of one PAUSE, so a
  // client on the worker's SMT sibling gets most of the core.  0 = one PAUSE.
  void set_poll_gap_ns(int ns) { poll_gap_ns_.store(std::max(0, std::min(ns, 100000))); }
  // grpc.coreEscape: a worker whose calls inside a busy-poll window run 35 % slower than
  // its own best moves to another core of its L3 (core_escape.h).  core_escapes(): moves.
  void set_core_escape(bool on) { core_escape_.store(on); }
  uint64_t core_escapes() const { return core_escapes_.load(); }
  // Epoll wake-ups of the workers that found nothing to do (timeouts), all workers.
  uint64_t idle_wakeups() const { return idle_wakeups_.load(); }
  std::vector<int> worker_connections() const;  // connections owned per worker thread
  const std::string& socket_path() const { return path_; }

  struct Worker;

 private:
  // Table listener: pushes ListAndWatch as soon as the table changes, from whichever
  // thread changed it.  Live only between start() and stop().
  struct Notifier : TableListener {
    std::mutex mu;
    GrpcServer* srv = nullptr;
    void on_table_change() override {
      std::lock_guard<std::mutex> lk(mu);
      if (srv) srv->notify();
    }
  };
  // `table` is handed over at thread creation: a worker never takes mu_, which stop()
  // holds while it joins the workers (one not yet scheduled when stop() ran deadlocked)
  void run(Worker* w, std::shared_ptr<DeviceTable> table, uint64_t gen);
  void law_closed(Worker* w);  // a ListAndWatch stream of w's ended
  void stamp_law_closed();
  void run_guarded(Worker* w, std::shared_ptr<DeviceTable> table, uint64_t gen);  // run() + fault capture
  void fail(const std::string& why);
  std::atomic<bool> failed_{false};
  std::atomic<int> inject_worker_fault_{0};
  mutable std::mutex fail_mu_;
  std::string fail_reason_;
  std::shared_ptr<const std::function<void()>> fail_hook_;
  std::shared_ptr<Notifier> notifier_ = std::make_shared<Notifier>();
  std::string path_;
  int nthreads_;
  int busy_poll_us_;
  int admission_poll_us_;
  std::atomic<int> keep_warm_ms_{0};
  std::atomic<bool> keep_warm_full_{true};
  std::atomic<int> idle_wake_ms_{0};
  std::atomic<int> active_window_ms_{0};
  std::atomic<bool> peek_reads_{false};
  std::atomic<int> poll_gap_ns_{0};
  std::atomic<bool> core_escape_{false};
  std::atomic<uint64_t> core_escapes_{0};
  std::atomic<uint64_t> idle_wakeups_{0};
  std::atomic<uint64_t> warm_ticks_{0};
  // table_ and table_gen_ change together under swap_mu_ (never held across anything else);
  // workers poll table_gen_ (one relaxed load per loop) and take table_ when it moved
  std::mutex swap_mu_;
  std::shared_ptr<DeviceTable> table_;
  std::atomic<uint64_t> table_gen_{0};
  int listen_fd_ = -1;
  // the socket file this server bound (device, inode): stop() removes only that file, not
  // one a newer plugin instance (a rolling update's next pod) has bound at the same path
  dev_t sock_dev_ = 0;
  ino_t sock_ino_ = 0;
  std::atomic<bool> running_{false};
  std::atomic<bool> stop_{false};
  ShardedCounter requests_;  // every worker counts its calls: no shared line per RPC
  ShardedCounter shed_;
  ShardedCounter admission_windows_, poll_windows_yielded_;
  std::atomic<int> conns_{0};
  std::atomic<int64_t> law_closed_ns_{0};
  CallTraceHeader* trace_hdr_ = nullptr;  // mapped by set_call_trace (nullptr: off)
  CallTraceEntry* trace_ = nullptr;
  size_t trace_bytes_ = 0;
  std::vector<std::unique_ptr<Worker>> workers_;
  std::vector<std::thread> threads_;
  mutable std::mutex mu_;
};

class H2Client {
 public:
  explicit H2Client(const std::string& socket_path, double timeout_s = 5.0);
  ~H2Client();
  // Unary call. Returns the grpc-status (0 = OK), response message in *resp.
  int unary(std::string_view path, std::string_view req, std::string* resp, std::string* message);
  // Sends a unary request without waiting for the answer (tests: calls in flight).
  void send_unary_nowait(std::string_view path, std::string_view req);
  // Opens a server stream and returns its first message (ListAndWatch probe).
  int first_stream_message(std::string_view path, std::string_view req, std::string* resp);
  // A long-lived server stream (a kubelet-like ListAndWatch watcher): open it, then
  // read one message at a time.  next_stream_message returns 0 with a message, -1 when
  // the server ended the stream; throws on timeout.
  void open_stream(std::string_view path, std::string_view req);
  int next_stream_message(std::string* resp, int timeout_ms);
  void close();
  // Benchmarks: stamp when each recv() returns (one clock read per recv), so a call's
  // time after the response arrived (the client's own parsing) can be told from the wait.
  void set_stamp_recv(bool on) { stamp_recv_ = on; }
  int64_t last_recv_ns() const { return recv_ret_ns_; }

 private:
  void send_all(const std::string& s);
  void set_recv_timeout(int ms);
  bool read_frame(uint8_t* type, uint8_t* flags, uint32_t* sid, std::string_view* payload);
  // Sends HEADERS + gRPC-framed request DATA (split into frames, within flow control).
  void send_request(uint32_t sid, std::string_view path, std::string_view req);
  // Handles connection-level frames (SETTINGS/PING/WINDOW_UPDATE); true if consumed.
  bool handle_control(uint8_t type, uint8_t flags, uint32_t sid, std::string_view payload);
  int64_t send_window_ = 65535;          // connection send window
  int64_t stream_window_init_ = 65535;   // server's SETTINGS_INITIAL_WINDOW_SIZE
  int64_t stream_window_ = 0;            // current request stream's send window
  uint32_t cur_sid_ = 0;
  bool goaway_ = false;  // the server sent GOAWAY: no new streams on this connection
  uint32_t peer_max_frame_ = 16384;
  int fd_ = -1;
  uint32_t next_sid_ = 1;
  hpack::Decoder dec_;
  std::string in_;
  size_t in_off_ = 0;  // bytes of in_ already parsed (read_frame)
  bool stamp_recv_ = false;
  int64_t recv_ret_ns_ = 0;
  int64_t conn_consumed_ = 0;
  uint32_t watch_sid_ = 0;
  std::string watch_buf_;
  int64_t watch_consumed_ = 0;
  int timeout_ms_;
  std::string hpath_, hblock_;  // last request path and its encoded header block
  std::string out_buf_, body_buf_, data_buf_;  // per-call scratch, capacity reused
};


}  // namespace amdgpu_dp
