// Per-resource device table: the data behind one kubelet DevicePlugin endpoint.
//
// Reference equivalents: device.Devices map + set algebra (device/devices.go:32-209),
// NvidiaDevicePlugin.ListAndWatch/GetPreferredAllocation/Allocate
// (plugin/plugin.go:173-225).  Differences by design:
//   * deterministic insertion order (reference iterates Go maps: defect D14)
//   * Allocate returns DeviceSpecs (/dev/kfd + the partition's render node) instead of
//     only an env var (defect D17), refuses Unhealthy devices
//   * responses are encoded from pre-built per-device protobuf fragments
//   * ListAndWatch bytes are cached and versioned; health changes bump the version
//   * the RPC read path takes no lock: per-device health is an atomic flag and the
//     ListAndWatch bytes / topology are immutable snapshots swapped RCU-style, so a
//     burst of Allocate/GetPreferredAllocation calls can never starve a health update
//     (a reader-preferring rwlock did, under ASan: native/selftest.cpp)
#pragma once

#include <atomic>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <string_view>
#include <unordered_map>
#include <utility>
#include <vector>

#include "allocator.h"
#include "backend.h"
#include "metrics.h"

namespace amdgpu_dp {

struct TableDevice {
  std::string id;
  int gpu = -1;
  int partition = -1;  // -1 = whole physical GPU
  int numa = -1;
  int replica = -1;    // >=0 when advertised as "<base>::<replica>"
  std::vector<std::string> host_paths;  // device nodes to expose (render/card)
  bool healthy = true;
};

struct TableConfig {
  std::string resource_name = "amd.com/gpu";
  std::string visible_env = "AMD_VISIBLE_DEVICES";
  std::vector<std::pair<std::string, std::string>> extra_envs;
  bool mount_kfd = true;
  std::string kfd_path = "/dev/kfd";
  std::string permissions = "rw";
  bool cdi = false;
  std::string cdi_prefix = "amd.com/gpu=";
  bool reject_unhealthy = true;
  bool pre_start_required = false;  // DevicePluginOptions.pre_start_required
};

// A PreStartContainer check waiting for the plugin's verifier (the gfx950 canary).
struct PreStartJob {
  uint64_t id = 0;
  std::vector<std::string> ids;
};

enum Rpc : int {
  kRpcOptions = 0,
  kRpcListAndWatch,
  kRpcPreferred,
  kRpcAllocate,
  kRpcPreStart,
  kRpcCount
};

const char* rpc_name(int rpc);

// Woken after every published health change, e.g. a GrpcServer pushing ListAndWatch.
// Tables hold listeners weakly, so a destroyed server is simply skipped.
class TableListener {
 public:
  virtual ~TableListener() = default;
  virtual void on_table_change() = 0;
};

class DeviceTable {
 public:
  DeviceTable(TableConfig cfg, std::vector<TableDevice> devices, Topology topo);

  const TableConfig& config() const { return cfg_; }
  size_t size() const { return devs_.size(); }
  const TableDevice& device(size_t i) const { return devs_[i]; }  // static fields only
  std::vector<std::string> ids() const;
  int index_of(std::string_view id) const;
  bool contains(const std::vector<std::string>& ids) const;
  bool aligned_supported() const { return aligned_ok_; }

  // Health: return true if anything changed (ListAndWatch version bumps).
  bool set_health(std::string_view id, bool healthy);
  int set_gpu_health(int gpu, int partition, bool healthy);
  // Every device of `gpu` Healthy except the partitions in `held` (and a whole-GPU device
  // containing one), in one update: a recovery that must not re-advertise partitions a
  // canary failed on.
  int set_gpu_health_except(int gpu, const std::vector<int>& held);
  bool healthy(std::string_view id) const;
  int healthy_count() const;
  void set_link_up(int a, int b, bool up);
  void set_link_bandwidth(int a, int b, double gbps);
  // n*n row-major (n = topology size): multi-GPU pods spanning each GPU pair.  Replaces
  // every count; a shorter vector clears the rest.
  void set_link_pods(const std::vector<int>& counts);
  // The node's tracker of recent multi-GPU Allocates (shared by every table): Allocate
  // records into it, GetPreferredAllocation adds its live entries to the link load.
  void set_recent_allocations(std::shared_ptr<RecentAllocations> r);
  Topology topology() const;

  uint64_t version() const { return version_.load(std::memory_order_acquire); }
  void add_listener(std::weak_ptr<TableListener> l);
  // Blocks until version() != seen, wake() is called or timeout_ms passes; returns the
  // current version.  For waiters that cannot be native listeners (the grpcio server's
  // ListAndWatch generators), called with the GIL released.
  uint64_t wait_change(uint64_t seen, int timeout_ms) const;
  void wake() const;
  std::string list_and_watch() const;  // ListAndWatchResponse bytes (cached)

  // RPC bodies.  Return true and response bytes in *out, or false and an error message.
  // Observations recorded in this table's RPC histograms so far: render_metrics' output
  // changes only when this does (a scrape caches the text under it).
  uint64_t metrics_version() const;
  bool allocate(std::string_view req, std::string* out) const;
  bool preferred(std::string_view req, std::string* out) const;
  std::string options_bytes() const;  // DevicePluginOptions

  // Convenience for Python callers / tests
  AllocResult preferred_ids(const std::vector<std::string>& avail, const std::vector<std::string>& must, int size,
                            std::vector<std::string>* out_ids) const;
  // Core of both: ids as views, result as device indices in r->chosen.
  AllocResult preferred_core(const std::string_view* avail, size_t n_avail, const std::string_view* must,
                             size_t n_must, int size) const;

  // PreStartContainer.  With pre_start_required the servers hand each request to the
  // plugin's verifier through this queue and answer when it completes, so a check
  // that runs for seconds (a canary on the allocated partitions) never occupies a
  // server thread and no native thread ever calls into Python.
  using PreStartDone = std::function<void(bool ok, const std::string& error)>;
  // Decodes PreStartContainerRequest; unknown ids fail at once (done is not queued).
  // Returns false with *error on a bad request.
  bool submit_prestart(std::string_view req, PreStartDone done, std::string* error);
  // Verifier side: blocks up to timeout_ms for jobs (GIL released by the binding).
  std::vector<PreStartJob> pop_prestart(int timeout_ms);
  void complete_prestart(uint64_t id, bool ok, const std::string& error);
  // Fails every queued/running job (plugin stopping) and wakes pop_prestart.
  void cancel_prestart(const std::string& why);
  void resume_prestart();  // accept jobs again (plugin served again after a stop)
  size_t prestart_pending() const;

  void observe(int rpc, double seconds, bool error) const;
  // Continue `prev`'s RPC histograms (call before this table serves anything).
  void inherit_stats(const DeviceTable& prev) { stats_ = prev.stats_; }
  void render_metrics(std::string* out, bool with_headers) const;
  static void render_metric_headers(std::string* out);

 private:
  void publish_law_locked();  // caller holds wmu_
  template <class F>
  void patch_topology(F&& f);  // copy-on-write edit of the topology snapshot (takes wmu_)
  void notify_listeners();    // caller must NOT hold wmu_
  void encode_container_alloc(const int* idx, size_t n, std::string* out) const;  // appends
  bool is_healthy(int i) const { return health_[i].load(std::memory_order_acquire) != 0; }

  TableConfig cfg_;
  std::vector<TableDevice> devs_;
  std::vector<AllocDevice> alloc_devs_;
  // Device ids are long (UUID + "-xcpN"); hashing three 8-byte words and the length
  // is enough to spread them and several times cheaper than hashing every byte.
  struct IdHash {
    size_t operator()(std::string_view s) const noexcept {
      uint64_t h = 0x9E3779B97F4A7C15ull ^ s.size();
      auto word = [&](size_t off) {
        uint64_t w = 0;
        std::memcpy(&w, s.data() + off, 8);
        return w;
      };
      if (s.size() >= 8) {
        const uint64_t ws[3] = {word(0), word((s.size() - 8) / 2), word(s.size() - 8)};
        for (uint64_t w : ws) {
          h ^= w;
          h *= 0xBF58476D1CE4E5B9ull;
          h ^= h >> 31;
        }
      } else {
        for (unsigned char ch : s) h = (h ^ ch) * 0x100000001B3ull;
      }
      return static_cast<size_t>(h ^ (h >> 29));
    }
  };
  std::unordered_map<std::string_view, int, IdHash> index_;
  std::vector<std::string> spec_frag_;  // per device: encoded DeviceSpec fields (tag 3)
  std::string kfd_frag_;
  std::string env_extra_frag_;
  bool aligned_ok_ = true;

  std::unique_ptr<std::atomic<uint8_t>[]> health_;
  std::mutex wmu_;                                // serialises writers only
  std::mutex lmu_;                                // listeners_
  mutable std::mutex pmu_;                        // PreStart queue
  std::condition_variable pcv_;
  uint64_t next_job_ = 1;
  std::deque<PreStartJob> pjobs_;                // not yet popped by the verifier
  std::unordered_map<uint64_t, PreStartDone> pwait_;  // queued or running -> completion
  bool pcancel_ = false;
  mutable std::mutex vmu_;                        // version waiters
  mutable std::condition_variable vcv_;
  mutable uint64_t wakes_ = 0;
  std::vector<std::weak_ptr<TableListener>> listeners_;
  std::shared_ptr<const Topology> topo_;          // atomic_load / atomic_store
  // Hot-path view of the tracker: a plain atomic pointer (no shared_ptr atomics on
  // Allocate); every tracker ever set is kept alive with the table.
  std::atomic<RecentAllocations*> recent_{nullptr};
  std::vector<std::shared_ptr<RecentAllocations>> recent_owned_;  // guarded by wmu_
  std::shared_ptr<const std::string> law_;        // cached ListAndWatchResponse
  std::atomic<uint64_t> version_{1};

  // RPC latency histograms and error counts.  Shared: a table swapped into a running
  // server in place of another (a reload that keeps the resource) carries on its
  // predecessor's series instead of resetting them (inherit_stats).
  struct RpcStats {
    std::unique_ptr<Histogram> hist[kRpcCount];
    std::atomic<uint64_t> errors[kRpcCount];
    RpcStats();
  };
  std::shared_ptr<RpcStats> stats_;
};

}  // namespace amdgpu_dp
