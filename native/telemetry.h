// GPU telemetry sampler + Prometheus exposition.
//
// The reference's `metrics` package is empty (metrics/metrics.go:1): /metrics only
// carries Go runtime, build info and echo HTTP metrics.  This adds per-GPU and
// per-partition amdsmi telemetry (power, energy, temperatures incl. HBM stacks,
// activity, clocks, VRAM, ECC, xGMI link state and traffic) with the sampling
// decoupled from scraping: one sampler thread reads one gpu_metrics blob per physical
// GPU per tick and renders the text once; a scrape copies bytes.
#pragma once

#include <atomic>
#include <memory>
#include <mutex>
#include <string>
#include <string_view>
#include <thread>
#include <vector>

#include "backend.h"
#include "device_table.h"
#include "health.h"
#include "metrics.h"

namespace amdgpu_dp {

// Appends one complete gzip member (RFC 1952) of data[0, n).  Concatenated members
// form a valid multi-member gzip stream (Go's gzip.Reader, Python's gzip, curl).
void gzip_member(const char* data, size_t n, std::string* out, int level = 1);

// One /metrics exposition as its segments: the per-tick inventory/GPU text and the
// per-version device-health block are shared snapshots, the rest is rendered per
// scrape.  Its size is known before any byte is copied, so a server can write the
// response header and then append each segment once.
struct Exposition {
  std::shared_ptr<const std::string> head, health;
  std::string counters, tail;
  size_t size() const { return head->size() + counters.size() + (health ? health->size() : 0) + tail.size(); }
  void append_to(std::string* out) const {
    out->append(*head).append(counters);
    if (health) out->append(*health);
    out->append(tail);
  }
};

struct PartitionLabel {
  int gpu = -1;
  int partition = -1;
  std::string device_id;
  std::string resource;
};

class Exporter {
 public:
  Exporter();
  ~Exporter();

  void set_inventory(const std::vector<GpuInfo>& gpus);
  void set_partition_labels(const std::vector<PartitionLabel>& labels);
  void set_build_info(const std::string& rendered_lines);  // "# HELP..\n# TYPE..\nname{..} 1\n"
  void set_tables(const std::vector<std::shared_ptr<DeviceTable>>& tables);
  void set_extra(const std::string& rendered);  // Python-side families (manager state)

  // Sampler thread; `monitor` (optional) receives every sample for health polling.
  void start(std::shared_ptr<Backend> backend, int interval_ms, std::shared_ptr<HealthMonitor> monitor);
  void stop();
  bool running() const { return running_.load(); }
  // One synchronous sampling pass (also used before the first scrape).
  void sample_once();

  std::shared_ptr<const std::string> gpu_text() const;
  GpuSample last_sample(int gpu) const;
  // Full exposition (everything except the HTTP server's own echo_http_* families).
  void render(std::string* out) const;
  void render(Exposition* e) const;
  // Same exposition + `trailer` (the HTTP server's families) as a multi-member gzip
  // stream.  The inventory/GPU-text member is compressed once per sampling tick and
  // the device-health member once per table version; only the small per-scrape parts
  // are compressed on the request path.
  void render_gzip(std::string* out, std::string_view trailer) const;
  uint64_t samples_total() const { return samples_.load(); }

 private:
  void loop();
  void render_gpu_text(const std::vector<GpuSample>& samples, const std::vector<char>& ok, uint64_t inventory_gen);
  void render_process(std::string* out) const;
  void render_parts(std::shared_ptr<const std::string>* head, std::string* counters,
                    std::shared_ptr<const std::string>* health, std::string* tail) const;

  mutable std::mutex mu_;
  std::vector<GpuInfo> gpus_;
  uint64_t inventory_gen_ = 0;  // bumped by set_inventory; a sampling pass is tied to one
  std::vector<PartitionLabel> labels_;
  std::vector<GpuSample> last_;
  std::vector<std::shared_ptr<DeviceTable>> tables_;
  std::string build_info_;
  uint64_t build_info_version_ = 0;
  mutable std::shared_ptr<const std::string> head_;      // build_info_ + *gpu_text_
  mutable std::shared_ptr<const std::string> head_src_;  // gpu_text_ that head_ was built from
  mutable uint64_t head_build_ = 0;
  std::shared_ptr<const std::string> extra_;
  std::shared_ptr<const std::string> gpu_text_;

  std::shared_ptr<Backend> backend_;
  std::shared_ptr<HealthMonitor> monitor_;
  int interval_ms_ = 1000;
  std::thread thread_;
  std::atomic<bool> running_{false};
  std::atomic<bool> stop_{false};
  std::mutex sample_mu_;  // serialises sampling passes
  std::atomic<uint64_t> samples_{0};
  std::atomic<uint64_t> sample_errors_{0};
  Histogram sample_hist_;
  int64_t start_time_s_ = 0;
  // device-health block, re-rendered only when a table's version changes
  mutable std::mutex health_mu_;
  mutable std::vector<uint64_t> health_key_;
  mutable std::shared_ptr<const std::string> health_cache_;
  // gzip members cached against the exact segment objects they were compressed from
  mutable std::mutex gz_mu_;
  mutable std::string gz_head_, gz_health_;
  mutable std::shared_ptr<const std::string> gz_head_src_, gz_health_src_;
  mutable std::mutex proc_mu_;
  mutable std::string proc_cache_;
  mutable int64_t proc_cache_ns_ = 0;
};

}  // namespace amdgpu_dp
