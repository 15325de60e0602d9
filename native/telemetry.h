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
#include <thread>
#include <vector>

#include "backend.h"
#include "device_table.h"
#include "health.h"
#include "metrics.h"

namespace amdgpu_dp {

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
  uint64_t samples_total() const { return samples_.load(); }

 private:
  void loop();
  void render_gpu_text(const std::vector<GpuSample>& samples, const std::vector<char>& ok, double sample_s);
  void render_process(std::string* out) const;

  mutable std::mutex mu_;
  std::vector<GpuInfo> gpus_;
  std::vector<PartitionLabel> labels_;
  std::vector<GpuSample> last_;
  std::vector<std::shared_ptr<DeviceTable>> tables_;
  std::string build_info_;
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
  mutable std::string health_cache_;
  mutable std::mutex proc_mu_;
  mutable std::string proc_cache_;
  mutable int64_t proc_cache_ns_ = 0;
};

}  // namespace amdgpu_dp
