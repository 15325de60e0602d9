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
#include <mutex>
#include <string>
#include <string_view>
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
  explicit Histogram(std::vector<double> bounds) : bounds_(std::move(bounds)), counts_(bounds_.size() + 1) {
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
  }
  uint64_t count() const {
    uint64_t c = 0;
    for (auto& x : counts_) c += x.load(std::memory_order_relaxed);
    return c;
  }
  // labels: already-formatted `k="v",` prefix (may be empty).  A scrape renders every
  // histogram, but most of them (kubelet RPCs, sampling passes) have not moved since the
  // previous scrape: their text is cached under (count, sum) and re-used.  The key is
  // read before the buckets, and both only grow, so a cached text is never older than
  // its key: an observation that lands mid-render changes the next key and forces a
  // re-render.
  void render(std::string* out, const char* name, std::string_view labels) const {
    const uint64_t key_count = count();
    const uint64_t key_sum = sum_.bits();
    {
      std::lock_guard<std::mutex> lk(cache_mu_);
      if (cache_valid_ && key_count == cache_count_ && key_sum == cache_sum_ && cache_name_ == name &&
          cache_labels_ == labels) {
        out->append(cache_);
        return;
      }
    }
    std::string text;
    render_uncached(&text, name, labels);
    out->append(text);
    std::lock_guard<std::mutex> lk(cache_mu_);
    cache_.swap(text);
    cache_count_ = key_count;
    cache_sum_ = key_sum;
    cache_name_ = name;
    cache_labels_.assign(labels.data(), labels.size());
    cache_valid_ = true;
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
  mutable std::mutex cache_mu_;
  mutable bool cache_valid_ = false;
  mutable uint64_t cache_count_ = 0, cache_sum_ = 0;
  mutable std::string cache_, cache_name_, cache_labels_;
};

// RPC latency buckets: 5 us .. 1 s (the echo buckets start at 500 us, too coarse
// for a microsecond-scale Allocate).
inline std::vector<double> rpc_buckets() {
  return {5e-6, 1e-5, 2e-5, 5e-5, 1e-4, 2e-4, 5e-4, 1e-3, 2e-3, 5e-3, 1e-2, 5e-2, 0.1, 0.5, 1.0};
}

}  // namespace amdgpu_dp
