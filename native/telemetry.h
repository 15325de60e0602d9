// GPU telemetry sampler + Prometheus exposition.
//
// The reference's `metrics` package is empty (metrics/metrics.go:1): /metrics only
// carries Go runtime, build info and echo HTTP metrics.  This adds per-GPU and
// per-partition amdsmi telemetry (power, energy, temperatures incl. HBM stacks,
// activity, clocks, VRAM, ECC, xGMI link state and traffic) with the sampling
// decoupled from scraping: one sampler thread posts one sample per physical GPU per tick
// to the GPUs' lanes (backend.h), collects what came back within the tick and renders the
// text once; a scrape copies bytes.  A GPU whose call wedged keeps
// its lane busy and nothing else: the other GPUs' samples, health checks and series stay
// fresh, and each GPU's sample age is exported.
#pragma once

#include <atomic>
#include <condition_variable>
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
// per-version device-health block are views of snapshots the rendering thread holds,
// the rest is rendered per scrape.  Its size is known before any byte is copied, so a
// server can write the response header and then append each segment once.  The views
// stay valid until the same thread renders again (Exporter::render).
struct Exposition {
  std::string_view head, health;
  std::string counters, tail;
  size_t size() const { return head.size() + counters.size() + health.size() + tail.size(); }
  void append_to(std::string* out) const {
    out->append(head.data(), head.size()).append(counters);
    out->append(health.data(), health.size());
    out->append(tail);
  }
  void clear() {
    head = health = std::string_view();
    counters.clear();
    tail.clear();
  }
};

struct PartitionLabel {
  int gpu = -1;
  int partition = -1;
  std::string device_id;
  std::string resource;
  std::string hip_ids;  // host HIP ordinals the device spans, comma-joined ("" = unknown)
};

class Exporter : public std::enable_shared_from_this<Exporter> {
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
  // Watchdog (health.sampleStallS): a hardware call (sample, describe, ...) that has been
  // in flight on a GPU's lane for longer than this marks that GPU lost in the health
  // monitor.  A wedged driver never returns an error to count, so without it such a GPU
  // would stay advertised Healthy.  0 = off.  Attribution: the GPU whose call has been
  // stuck longest is the culprit; another stuck GPU is reported too only when some call
  // completed after its own began (the library is not serialised behind the first
  // wedge), otherwise it is "blocked" behind it and stays Healthy.
  void set_stall_ms(int ms) { stall_ms_.store(ms > 0 ? ms : 0); }
  // Adaptive cadence (telemetry.idleIntervalMs / activeWindowS): the sampler runs every
  // idle_ms instead of the start() interval while nothing has read the GPU metrics for
  // window_ms, the health monitor is settled (HealthMonitor::settling) and the first
  // window_ms after start() are over.  A scrape in that state wakes the sampler at once;
  // while scraped (and settled) it samples about twice per scrape interval, never less
  // often than idle_ms nor more often than the interval.  A sample costs ~1 ms of CPU per MI355X, most of it the
  // kernel fetching the firmware's metrics table (scripts/sysfs_cost_probe.py).
  // idle_ms <= the interval: always the interval.
  void set_idle_interval(int idle_ms, int window_ms) {
    idle_interval_ms_.store(idle_ms > 0 ? idle_ms : 0);
    active_window_ms_.store(window_ms > 0 ? window_ms : 0);
  }
  int current_interval_ms() const { return current_interval_ms_.load(); }
  uint64_t idle_passes() const { return idle_passes_.load(); }  // passes slower than the interval
  int stalled_gpu() const;                 // lowest stalled GPU index, -1 = none
  std::vector<int> stalled_gpus() const;   // reported lost by the watchdog
  std::vector<int> blocked_gpus() const;   // stuck behind another GPU's call
  // One synchronous sampling pass (also used before the first scrape).
  // sampler_gen: the sampler thread's own pass (0 = a caller's synchronous pass); it
  // ends early once stop() is waiting or another sampler generation started.
  void sample_once(uint64_t sampler_gen = 0);
  // Seconds since GPU `gpu`'s last successful sample (-1: none yet).
  double sample_age_s(int gpu) const;

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
  struct ThreadExit {  // outlives the exporter: the sampler signals it after letting go
    std::mutex mu;
    std::condition_variable cv;
    bool done = false;
    bool wait(int ms);  // ms < 0: no limit; true once the thread has exited
    void mark();
  };
  struct Waker {  // the sampler's and the watchdog's sleeps, cut short by stop()
    std::mutex mu;
    std::condition_variable cv;
    bool stopping = false;
    bool poked = false;  // the sampler's sleep only (a scrape while idle)
    void sleep_ms(int64_t ms, bool pokeable = false);
    void wake();
    void poke();
  };
  static void sampler_main(std::weak_ptr<Exporter> weak, std::shared_ptr<ThreadExit> exit,
                           std::shared_ptr<Waker> waker, uint64_t gen, int interval_ms);
  int sampler_step(int64_t* next, uint64_t gen, int interval_ms);  // ms to sleep before the next step, -1 = stop
  void render_gpu_text(const std::vector<GpuSample>& samples, const std::vector<char>& ok, uint64_t inventory_gen);
  // One GPU's sampling state across passes (guarded by sample_mu_).
  struct Slot {
    int index = -1;                        // backend index
    std::string key;                       // the GPU's identity (sampled by it, see sample_async)
    std::shared_ptr<LaneJob> job;          // in flight (null: none)
    std::shared_ptr<GpuSample> out;
    int64_t posted_ns = 0;
    GpuSample last;                        // last completed sample
    bool last_ok = false;
    int64_t last_ok_ns = 0;
    bool refused = false;                  // the lane took no job this pass (busy with a stuck call)
  };
  std::vector<Slot> slots_;
  uint64_t slots_gen_ = ~0ull;             // inventory generation slots_ belongs to
  // What the per-scrape counters need, published by the sampler and the watchdog.
  struct Freshness {
    std::vector<std::pair<int, int64_t>> last_ok;  // (gpu, mono ns of its last good sample)
  };
  struct Stalls {
    std::vector<int> stalled, blocked;
  };
  mutable SpinLock fresh_lock_;
  std::shared_ptr<const Freshness> fresh_;
  std::shared_ptr<const Stalls> stalls_;
  void render_process(std::string* out) const;  // reads /proc
  void render_process_cached(std::string* out) const;  // per-thread copy, refreshed each second
  // head_sp / health_sp (optional): owning references to the segments head / health view
  void render_parts(std::string_view* head, std::string* counters, std::string_view* health, std::string* tail,
                    std::shared_ptr<const std::string>* head_sp = nullptr,
                    std::shared_ptr<const std::string>* health_sp = nullptr) const;

  // What a scrape reads, as one immutable snapshot: rebuilt under mu_ by whatever changes
  // an input (a sampling tick, set_build_info / set_tables / set_extra) and read by the
  // HTTP workers through a pointer copy under a spin lock, so concurrent scrapers never
  // queue on mu_ (or on the sampler holding it).
  struct ScrapeView {
    std::shared_ptr<const std::string> head;  // build info + per-tick GPU text
    std::shared_ptr<const std::string> extra;
    std::vector<std::shared_ptr<DeviceTable>> tables;
  };
  void publish_view_locked();  // mu_ held
  std::shared_ptr<const ScrapeView> view() const;

  // What each scraping thread keeps between scrapes, so that a scrape writes no cache
  // line another scraper reads: the view (re-fetched only when view_gen_ moves), the
  // device-health text (re-rendered only when a table version moves) and the process_*
  // text (re-read from /proc at most once a second).  Shared copies behind a lock made 4
  // concurrent scrapers each 3.5x slower than one (lock and reference-count lines
  // bouncing between cores).
  struct TlCache {
    uint64_t exporter = 0;  // id_ of the exporter the entries belong to
    uint64_t view_gen = 0;
    std::shared_ptr<const ScrapeView> view;
    std::vector<uint64_t> health_key;  // (table address, version) pairs
    std::shared_ptr<const std::string> health;
    int64_t proc_ns = 0;
    std::string proc;
    // the device tables' RPC histograms, rendered once per change of their counts
    std::vector<uint64_t> tables_key;  // (table address, metrics_version) pairs
    std::string tables_text;
  };
  TlCache& tl_cache() const;
  // The last rendered device-health text, shared so that every thread serves the same
  // object (the gzip path caches its compressed member by identity); a thread consults
  // it only when its own key goes stale.
  struct HealthShared {
    std::vector<uint64_t> key;
    std::shared_ptr<const std::string> text;
  };
  mutable SpinLock health_lock_;
  mutable std::shared_ptr<const HealthShared> health_shared_;

  const uint64_t id_;
  mutable std::mutex mu_;
  mutable SpinLock view_lock_;
  std::shared_ptr<const ScrapeView> view_;
  std::atomic<uint64_t> view_gen_{0};
  std::vector<GpuInfo> gpus_;
  uint64_t inventory_gen_ = 0;  // bumped by set_inventory; a sampling pass is tied to one
  std::vector<PartitionLabel> labels_;
  std::vector<GpuSample> last_;
  std::vector<std::shared_ptr<DeviceTable>> tables_;
  std::string build_info_;
  std::shared_ptr<const std::string> extra_;
  std::shared_ptr<const std::string> gpu_text_;

  mutable std::mutex run_mu_;  // backend_, monitor_, interval_ms_, waker_: set by start(), copied by each pass
  std::shared_ptr<Backend> backend_;
  std::shared_ptr<HealthMonitor> monitor_;
  int interval_ms_ = 1000;
  std::thread thread_;
  std::atomic<bool> running_{false};
  std::atomic<bool> stop_{false};
  std::shared_ptr<ThreadExit> sampler_exit_;
  std::shared_ptr<Waker> waker_;
  std::mutex first_mu_;  // first pass of a start(): start() waits for it (bounded)
  std::condition_variable first_cv_;
  bool first_done_ = false;
  std::atomic<uint64_t> sampler_gen_{0};  // bumped by every start()
  std::mutex sample_mu_;  // serialises sampling passes
  std::atomic<uint64_t> samples_{0};
  std::atomic<uint64_t> sample_errors_{0};
  Histogram sample_hist_;
  void watchdog_loop(std::shared_ptr<HealthMonitor> monitor, std::shared_ptr<Waker> waker);
  std::thread watchdog_;
  std::atomic<int> stall_ms_{0};
  std::atomic<int64_t> last_pass_ns_{0};    // end of the last complete pass (mono ns)
  int64_t start_time_s_ = 0;
  // adaptive cadence (set_idle_interval)
  int next_interval_ms(int interval_ms);
  void note_read() const;
  std::atomic<int> idle_interval_ms_{0}, active_window_ms_{120000}, current_interval_ms_{0};
  mutable std::atomic<int64_t> last_read_ns_{0};
  mutable std::atomic<int64_t> read_gap_ns_{0};  // between the last two recorded reads (0: one read)
  std::atomic<int64_t> started_ns_{0};
  std::atomic<bool> idle_mode_{false};
  mutable std::atomic<bool> poke_{false};
  std::atomic<uint64_t> idle_passes_{0};

  // gzip members cached against the exact segment objects they were compressed from
  mutable std::mutex gz_mu_;
  mutable std::string gz_head_, gz_health_;
  mutable std::shared_ptr<const std::string> gz_head_src_, gz_health_src_;

};

}  // namespace amdgpu_dp
