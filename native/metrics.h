// Lock-free Prometheus primitives + text-format (0.0.4) helpers.
//
// Reference: client_golang counters/histograms registered by promauto
// (middleware/echo_metric.go:80-93) and rendered by promhttp (router/api.go:32).
// Here every hot-path observation is a couple of relaxed atomic adds; rendering
// happens only on scrape.
#pragma once

#include <sched.h>
#include <sys/resource.h>

#include <atomic>
#include <charconv>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <iterator>
#include <memory>
#include <mutex>
#include <string>
#include <string_view>
#include <unordered_map>
#include <vector>

namespace amdgpu_dp {

inline void append_u64(std::string* out, uint64_t v) {
  char buf[24];
  char* p = buf + sizeof(buf);
  do {
    *--p = static_cast<char>('0' + v % 10);
    v /= 10;
  } while (v);
  out->append(p, static_cast<size_t>(buf + sizeof(buf) - p));
}

// Shortest round-trip decimal in %g style, like Go's strconv.FormatFloat(v, 'g', -1,
// 64) that promhttp uses ("0.0005", "30", "1e-05", "+Inf"); integral values below 1e15
// print as plain integers.  std::to_chars (Ryu) keeps this off the snprintf path: a
// scrape formats hundreds of numbers.
inline void append_float(std::string* out, double v) {
  if (std::isnan(v)) {
    out->append("NaN");
    return;
  }
  if (std::isinf(v)) {
    out->append(v > 0 ? "+Inf" : "-Inf");
    return;
  }
  if (v == std::floor(v) && std::fabs(v) < 1e15) {
    if (v < 0) {
      out->push_back('-');
      append_u64(out, static_cast<uint64_t>(-v));
    } else {
      append_u64(out, static_cast<uint64_t>(v));
    }
    return;
  }
  char buf[40];
  const auto r = std::to_chars(buf, buf + sizeof(buf), v, std::chars_format::general);
  out->append(buf, static_cast<size_t>(r.ptr - buf));
}

inline void append_label_value(std::string* out, std::string_view s) {
  for (char c : s) {
    if (c == '\\') out->append("\\\\");
    else if (c == '"') out->append("\\\"");
    else if (c == '\n') out->append("\\n");
    else out->push_back(c);
  }
}

inline void append_header(std::string* out, const char* name, const char* help, const char* type) {
  out->append("# HELP ").append(name).append(" ").append(help).append("\n# TYPE ").append(name).append(" ")
      .append(type).append("\n");
}

// Spin-wait hint for busy-poll loops and spin locks (x86 PAUSE; a yield hint or a
// compiler barrier elsewhere, so the native core still builds on non-x86 hosts).
inline void cpu_relax() {
#if defined(__x86_64__) || defined(__i386__)
  __builtin_ia32_pause();
#elif defined(__aarch64__) || defined(__arm__)
  __asm__ __volatile__("yield" ::: "memory");
#else
  __asm__ __volatile__("" ::: "memory");
#endif
}

// A long polling window (the gRPC admission window after a GetPreferredAllocation) must
// never keep a CPU from the thread the worker is waiting for.  When the client runs on the same CPU (the scheduler places a
// woken thread next to its waker), a polling worker and a client that is busy before
// its next call share that CPU, and the call waits for the window's end or a scheduler
// slice: on a shared host a 1 ms admission window turned a kubelet-like admission
// (GetPreferredAllocation, client work, Allocate) into ~0.8 ms.  Once a window has been
// idle for kQuietNs (back-to-back calls arrive well within it, so they never pay for
// any of this), the poller offers the CPU every 16 polls (sched_yield: a no-op when
// nothing else is runnable there) and ends the window as soon as it has been preempted
// (an involuntary context switch, getrusage every 16 polls): someone else wants this
// CPU, so sleep.  Short busy-poll windows (tens of us) do not use it: ending them early
// turned a client's brief hiccup into a cold wake-up of the worker and raised the warm
// Allocate tail on MI355X (profiles/r3/spin_guard_ab.txt).
class SpinGuard {
 public:
  static constexpr int64_t kQuietNs = 20000;
  // true while the window may keep polling; `now`: mono ns of this idle poll
  bool keep_polling(int64_t now) {
    if (now - idle_since_ < kQuietNs || (++polls_ & 15) != 0) return true;
    const long cs = nivcsw();
    if (base_ < 0) {
      base_ = cs;
      return true;
    }
    return cs == base_;
  }
  void pause(int64_t now) {
    if (now - idle_since_ >= kQuietNs && (polls_ & 15) == 8) sched_yield();
    else cpu_relax();
  }
  void reset(int64_t now) {  // a request was answered: the window's idle time starts now
    idle_since_ = now;
    polls_ = 0;
    base_ = -1;
  }
  static long nivcsw() {
    struct rusage ru;
    return getrusage(RUSAGE_THREAD, &ru) == 0 ? ru.ru_nivcsw : 0;
  }

 private:
  int64_t idle_since_ = 0;
  unsigned polls_ = 0;
  long base_ = -1;
};

// The worker of `workers` (each with an atomic `load`) with the fewest connections,
// `self` on a tie, with its load already incremented.  Claims the slot with a CAS, so
// two workers that accept at the same moment never both hand their connection to the
// same worker at the same load.
template <class Workers, class W>
W* pick_least_loaded(Workers& workers, W* self) {
  for (;;) {
    W* t = self;
    int tl = t->load.load(std::memory_order_relaxed);
    for (auto& o : workers) {
      const int ol = o->load.load(std::memory_order_relaxed);
      if (ol < tl) {
        t = o.get();
        tl = ol;
      }
    }
    if (t->load.compare_exchange_weak(tl, tl + 1, std::memory_order_relaxed)) return t;
  }
}

// Guards pointer-sized critical sections on the scrape path (copying or swapping a
// shared_ptr to a cached text).  A contended std::mutex parks the thread in futex_wait,
// and the wake-up costs more than the whole critical section: with 4 concurrent
// scrapers that alone tripled /metrics latency.  Only ever held for a few instructions.
class SpinLock {
 public:
  void lock() {
    while (f_.exchange(true, std::memory_order_acquire))
      while (f_.load(std::memory_order_relaxed)) cpu_relax();
  }
  void unlock() { f_.store(false, std::memory_order_release); }

 private:
  std::atomic<bool> f_{false};
};

// Observation shard of the calling thread.  Threads are spread round-robin over
// kMetricShards cache-line-separated copies of every counter, so concurrent kubelet RPC
// and HTTP workers never write the same line: with one shared set, 4 concurrent clients
// bounced the bucket, sum and count lines between cores on every call.
constexpr int kMetricShards = 16;
inline int& thread_shard_slot() {
  static thread_local int s = -1;
  return s;
}
inline int thread_shard() {
  static std::atomic<int> next{0};
  int& s = thread_shard_slot();
  if (s < 0) s = next.fetch_add(1, std::memory_order_relaxed) % kMetricShards;
  return s;
}
// Server workers claim their shard by index (gRPC worker i: shard i, HTTP worker j: shard
// 15 - j), so the workers of one server never share a line, whatever order they first
// count in (round-robin at first use let 8 busy workers collide with high probability).
inline void set_thread_shard(int s) { thread_shard_slot() = ((s % kMetricShards) + kMetricShards) % kMetricShards; }

// A counter incremented by many threads: one cache line per shard, summed on read.
class ShardedCounter {
 public:
  ShardedCounter() {
    for (auto& s : shards_) s.v.store(0, std::memory_order_relaxed);
  }
  void add(uint64_t n = 1) { shards_[thread_shard()].v.fetch_add(n, std::memory_order_relaxed); }
  uint64_t load() const {
    uint64_t t = 0;
    for (const auto& s : shards_) t += s.v.load(std::memory_order_relaxed);
    return t;
  }

 private:
  struct alignas(64) Slot {
    std::atomic<uint64_t> v;
  };
  Slot shards_[kMetricShards];
};

// Adds `d` to the double stored as bits in `a` (CAS loop; uncontended per shard).
inline void atomic_add_double(std::atomic<uint64_t>* a, double d) {
  uint64_t old = a->load(std::memory_order_relaxed);
  for (;;) {
    double cur;
    std::memcpy(&cur, &old, sizeof(cur));
    const double nv = cur + d;
    uint64_t nb;
    std::memcpy(&nb, &nv, sizeof(nb));
    if (a->compare_exchange_weak(old, nb, std::memory_order_relaxed)) return;
  }
}

class Histogram {
 public:
  static constexpr size_t kMaxBuckets = 23;  // finite bounds (+Inf is one more slot)

  explicit Histogram(std::vector<double> bounds)
      : bounds_(std::move(bounds)), shards_(new Shard[kMetricShards]), id_(next_id().fetch_add(1) + 1) {
    if (bounds_.size() > kMaxBuckets) bounds_.resize(kMaxBuckets);
    for (double b : bounds_) {  // the le="..." strings never change: format them once
      std::string s;
      append_float(&s, b);
      le_.push_back(std::move(s));
    }
    le_.push_back("+Inf");
    for (int k = 0; k < kMetricShards; ++k) {
      Shard& sh = shards_[k];
      sh.n.store(0, std::memory_order_relaxed);
      sh.sum.store(0, std::memory_order_relaxed);  // bits of 0.0
      for (auto& c : sh.counts) c.store(0, std::memory_order_relaxed);
    }
  }
  Histogram(const Histogram&) = delete;
  void observe(double v) {
    size_t i = 0;
    while (i < bounds_.size() && v > bounds_[i]) ++i;
    const int k = thread_shard();
    // readers sum only the shards some thread has observed into (one or two for most
    // histograms); the bit is written once per shard, the check is a shared read
    const uint32_t bit = 1u << k;
    if (!(used_.load(std::memory_order_relaxed) & bit)) used_.fetch_or(bit, std::memory_order_release);
    Shard& sh = shards_[k];
    sh.counts[i].fetch_add(1, std::memory_order_relaxed);
    atomic_add_double(&sh.sum, v);
    sh.n.fetch_add(1, std::memory_order_release);  // last: a reader that sees n sees the bucket
  }
  // Observations completed so far, never ahead of the buckets.
  uint64_t count() const { return count(used()); }
  double sum() const { return sum(used()); }

 private:
  uint32_t used() const { return used_.load(std::memory_order_acquire); }
  uint64_t count(uint32_t used) const {
    uint64_t c = 0;
    for (uint32_t b = used; b; b &= b - 1) c += shards_[__builtin_ctz(b)].n.load(std::memory_order_acquire);
    return c;
  }
  double sum(uint32_t used) const {
    double s = 0;
    for (uint32_t b = used; b; b &= b - 1) {
      const uint64_t bits = shards_[__builtin_ctz(b)].sum.load(std::memory_order_relaxed);
      double d;
      std::memcpy(&d, &bits, sizeof(d));
      s += d;
    }
    return s;
  }

 public:
  // labels: already-formatted `k="v",` prefix (may be empty).  A scrape renders every
  // histogram, but most of them (kubelet RPCs, sampling passes) have not moved since the
  // previous scrape: their text is cached under the observation count and re-used.  The
  // count only grows and is read before the buckets (each shard counts an observation
  // after its bucket), so a cached text is never older than its key: an observation that
  // lands mid-render changes the next key and forces a re-render.  The cache is per
  // thread (each HTTP worker keeps its own copy): a shared one, even behind a spin lock,
  // made concurrent scrapers bounce its lock and reference count between cores, and 4
  // scrapers each took 3.5x as long as one.
  void render(std::string* out, const char* name, std::string_view labels) const {
    const uint32_t shards = used();  // one snapshot for the key and the numbers
    const uint64_t key_count = count(shards);
    TlCache& tl = tl_cache();
    // entries of histograms that are gone (a plugin reload replaces every table's) are
    // never hit again: drop what was not rendered in the last kSweepEvery renders
    if (++tl.renders % kSweepEvery == 0) {
      for (auto e = tl.map.begin(); e != tl.map.end();)
        e = tl.renders - e->second.last_render > kSweepEvery ? tl.map.erase(e) : std::next(e);
    }
    auto& cache = tl.map;
    auto it = cache.find(id_);
    if (it != cache.end() && it->second.count == key_count && it->second.name == name &&
        it->second.labels == labels) {
      it->second.last_render = tl.renders;
      out->append(it->second.text);
      return;
    }
    Cached& c = cache[id_];
    c.last_render = tl.renders;
    c.count = key_count;
    if (c.pre.empty() || c.name != name || c.labels != labels) {
      c.name = name;
      c.labels.assign(labels.data(), labels.size());
      build_prefixes(&c);
    }
    // only the numbers move: the line texts were built once for this (name, labels)
    c.text.clear();
    c.text.reserve(c.pre.size() + 24 * c.ends.size());
    uint64_t cum = 0;
    size_t at = 0;
    for (size_t i = 0; i <= bounds_.size(); ++i) {
      for (uint32_t b = shards; b; b &= b - 1) cum += shards_[__builtin_ctz(b)].counts[i].load(std::memory_order_relaxed);
      c.text.append(c.pre, at, c.ends[i] - at);
      at = c.ends[i];
      append_u64(&c.text, cum);
      c.text.push_back('\n');
    }
    c.text.append(c.pre, at, c.ends[bounds_.size() + 1] - at);
    at = c.ends[bounds_.size() + 1];
    append_float(&c.text, sum(shards));
    c.text.push_back('\n');
    c.text.append(c.pre, at, c.ends[bounds_.size() + 2] - at);
    append_u64(&c.text, cum);
    c.text.push_back('\n');
    out->append(c.text);
  }

  void render_uncached(std::string* out, const char* name, std::string_view labels) const {
    std::string prefix(name);
    prefix.append("_bucket{").append(labels.data(), labels.size()).append("le=\"");
    out->reserve(out->size() + (prefix.size() + 24) * (bounds_.size() + 3));
    const uint32_t shards = used();
    uint64_t cum = 0;
    for (size_t i = 0; i <= bounds_.size(); ++i) {
      for (uint32_t b = shards; b; b &= b - 1) cum += shards_[__builtin_ctz(b)].counts[i].load(std::memory_order_relaxed);
      out->append(prefix).append(le_[i]).append("\"} ");
      append_u64(out, cum);
      out->push_back('\n');
    }
    std::string_view lab = labels;
    if (!lab.empty() && lab.back() == ',') lab.remove_suffix(1);
    out->append(name).append("_sum");
    if (!lab.empty()) out->append("{").append(lab.data(), lab.size()).append("}");
    out->push_back(' ');
    append_float(out, sum(shards));
    out->push_back('\n');
    out->append(name).append("_count");
    if (!lab.empty()) out->append("{").append(lab.data(), lab.size()).append("}");
    out->push_back(' ');
    append_u64(out, cum);
    out->push_back('\n');
  }

 private:
  struct alignas(64) Shard {
    std::atomic<uint64_t> n;
    std::atomic<uint64_t> sum;  // bits of a double
    std::atomic<uint64_t> counts[kMaxBuckets + 1];
  };
  std::vector<double> bounds_;
  std::vector<std::string> le_;
  std::unique_ptr<Shard[]> shards_;
  std::atomic<uint32_t> used_{0};  // bit k: shard k has seen an observation
  static_assert(kMetricShards <= 32, "used_ is a 32-bit mask");
  struct Cached {
    uint64_t count = 0;
    uint64_t last_render = 0;  // TlCache::renders when last used
    std::string name, labels, text;
    // the text before each number, concatenated: bucket lines `name_bucket{labels le="x"} `,
    // then `name_sum{labels} ` and `name_count{labels} `; ends[i] = end of prefix i
    std::string pre;
    std::vector<size_t> ends;
  };
  void build_prefixes(Cached* c) const {
    c->pre.clear();
    c->ends.clear();
    for (size_t i = 0; i <= bounds_.size(); ++i) {
      c->pre.append(c->name).append("_bucket{").append(c->labels).append("le=\"").append(le_[i]).append("\"} ");
      c->ends.push_back(c->pre.size());
    }
    std::string_view lab = c->labels;
    if (!lab.empty() && lab.back() == ',') lab.remove_suffix(1);
    for (const char* suffix : {"_sum", "_count"}) {
      c->pre.append(c->name).append(suffix);
      if (!lab.empty()) c->pre.append("{").append(lab.data(), lab.size()).append("}");
      c->pre.push_back(' ');
      c->ends.push_back(c->pre.size());
    }
  }
  // per-thread render cache, keyed by histogram id (ids are never reused, addresses are);
  // a scrape renders every live histogram, so a live entry is touched every ~100 renders
  struct TlCache {
    std::unordered_map<uint64_t, Cached> map;
    uint64_t renders = 0;
  };
  static constexpr uint64_t kSweepEvery = 4096;
  static TlCache& tl_cache() {
    static thread_local TlCache c;
    return c;
  }
  static std::atomic<uint64_t>& next_id() {
    static std::atomic<uint64_t> n{0};
    return n;
  }
  const uint64_t id_;
};

// RPC latency buckets: 5 us .. 1 s (the echo buckets start at 500 us, too coarse
// for a microsecond-scale Allocate).
inline std::vector<double> rpc_buckets() {
  return {5e-6, 1e-5, 2e-5, 5e-5, 1e-4, 2e-4, 5e-4, 1e-3, 2e-3, 5e-3, 1e-2, 5e-2, 0.1, 0.5, 1.0};
}

}  // namespace amdgpu_dp
