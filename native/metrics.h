// Lock-free Prometheus primitives + text-format (0.0.4) helpers.
//
// Reference: client_golang counters/histograms registered by promauto
// (middleware/echo_metric.go:80-93) and rendered by promhttp (router/api.go:32).
// Here every hot-path observation is a couple of relaxed atomic adds; rendering
// happens only on scrape.
#pragma once

#include <atomic>
#include <charconv>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
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

// Guards pointer-sized critical sections on the scrape path (copying or swapping a
// shared_ptr to a cached text).  A contended std::mutex parks the thread in futex_wait,
// and the wake-up costs more than the whole critical section: with 4 concurrent
// scrapers that alone tripled /metrics latency.  Only ever held for a few instructions.
class SpinLock {
 public:
  void lock() {
    while (f_.exchange(true, std::memory_order_acquire))
      while (f_.load(std::memory_order_relaxed)) __builtin_ia32_pause();
  }
  void unlock() { f_.store(false, std::memory_order_release); }

 private:
  std::atomic<bool> f_{false};
};

class AtomicDouble {
 public:
  void add(double d) {
    uint64_t old = bits_.load(std::memory_order_relaxed);
    for (;;) {
      double cur;
      std::memcpy(&cur, &old, sizeof(cur));
      const double nv = cur + d;
      uint64_t nb;
      std::memcpy(&nb, &nv, sizeof(nb));
      if (bits_.compare_exchange_weak(old, nb, std::memory_order_relaxed)) return;
    }
  }
  uint64_t bits() const { return bits_.load(std::memory_order_relaxed); }
  double load() const {
    const uint64_t b = bits_.load(std::memory_order_relaxed);
    double d;
    std::memcpy(&d, &b, sizeof(d));
    return d;
  }

 private:
  std::atomic<uint64_t> bits_{0};
};

class Histogram {
 public:
  explicit Histogram(std::vector<double> bounds)
      : bounds_(std::move(bounds)), counts_(bounds_.size() + 1), id_(next_id().fetch_add(1) + 1) {
    for (double b : bounds_) {  // the le="..." strings never change: format them once
      std::string s;
      append_float(&s, b);
      le_.push_back(std::move(s));
    }
    le_.push_back("+Inf");
  }
  Histogram(const Histogram&) = delete;
  void observe(double v) {
    size_t i = 0;
    while (i < bounds_.size() && v > bounds_[i]) ++i;
    counts_[i].fetch_add(1, std::memory_order_relaxed);
    sum_.add(v);
    n_.fetch_add(1, std::memory_order_release);  // last: a reader that sees n sees the bucket
  }
  // Observations completed so far: one load (a scrape asks every histogram, most of
  // which have not moved), never ahead of the buckets.
  uint64_t count() const { return n_.load(std::memory_order_acquire); }
  // labels: already-formatted `k="v",` prefix (may be empty).  A scrape renders every
  // histogram, but most of them (kubelet RPCs, sampling passes) have not moved since the
  // previous scrape: their text is cached under (count, sum) and re-used.  The key is
  // read before the buckets, and both only grow, so a cached text is never older than
  // its key: an observation that lands mid-render changes the next key and forces a
  // re-render.  The cache is per thread (each HTTP worker keeps its own copy): a shared
  // one, even behind a spin lock, made concurrent scrapers bounce its lock and reference
  // count between cores, and 4 scrapers each took 3.5x as long as one.
  void render(std::string* out, const char* name, std::string_view labels) const {
    const uint64_t key_count = count();
    const uint64_t key_sum = sum_.bits();
    auto& cache = tl_cache();
    auto it = cache.find(id_);
    if (it != cache.end() && it->second.count == key_count && it->second.sum == key_sum &&
        it->second.name == name && it->second.labels == labels) {
      out->append(it->second.text);
      return;
    }
    if (it == cache.end() && cache.size() >= 1024) cache.clear();  // histograms of old reloads
    Cached& c = cache[id_];
    c.count = key_count;
    c.sum = key_sum;
    c.name = name;
    c.labels.assign(labels.data(), labels.size());
    c.text.clear();
    render_uncached(&c.text, name, labels);
    out->append(c.text);
  }

  void render_uncached(std::string* out, const char* name, std::string_view labels) const {
    std::string prefix(name);
    prefix.append("_bucket{").append(labels.data(), labels.size()).append("le=\"");
    out->reserve(out->size() + (prefix.size() + 24) * (bounds_.size() + 3));
    uint64_t cum = 0;
    for (size_t i = 0; i <= bounds_.size(); ++i) {
      cum += counts_[i].load(std::memory_order_relaxed);
      out->append(prefix).append(le_[i]).append("\"} ");
      append_u64(out, cum);
      out->push_back('\n');
    }
    std::string_view lab = labels;
    if (!lab.empty() && lab.back() == ',') lab.remove_suffix(1);
    out->append(name).append("_sum");
    if (!lab.empty()) out->append("{").append(lab.data(), lab.size()).append("}");
    out->push_back(' ');
    append_float(out, sum_.load());
    out->push_back('\n');
    out->append(name).append("_count");
    if (!lab.empty()) out->append("{").append(lab.data(), lab.size()).append("}");
    out->push_back(' ');
    append_u64(out, cum);
    out->push_back('\n');
  }

 private:
  std::vector<double> bounds_;
  std::vector<std::string> le_;
  std::vector<std::atomic<uint64_t>> counts_;
  AtomicDouble sum_;
  std::atomic<uint64_t> n_{0};
  struct Cached {
    uint64_t count = 0, sum = 0;
    std::string name, labels, text;
  };
  // per-thread render cache, keyed by histogram id (ids are never reused, addresses are)
  static std::unordered_map<uint64_t, Cached>& tl_cache() {
    static thread_local std::unordered_map<uint64_t, Cached> c;
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
