// Device health monitor: the producer the reference never had.
//
// Reference: plugin/plugin.go:40,53,181-186 declare a `health` channel consumed by
// ListAndWatch, but nothing ever sends on it (defect D9; README "driver monitoring"
// unimplemented).  Here two native sources feed one de-duplicated state machine:
//   * hardware events (amdsmi_get_gpu_event_notification: PRE/POST_RESET, thermal,
//     VM faults; or the fixture's scripted faults)        -> event thread
//   * telemetry polling (ECC uncorrectable deltas, xGMI link up/down, device lost)
//                                                          -> sampler thread
// Transitions go both ways (Unhealthy *and* back to Healthy) and are queued for the
// plugin manager, which pushes a fresh ListAndWatch response.
#pragma once

#include <atomic>
#include <condition_variable>
#include <deque>
#include <limits>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "backend.h"
#include "device_table.h"

namespace amdgpu_dp {

// Health checks an operator can turn off (health.disabledChecks): the condition is still
// tracked and reported as an informational update, but it no longer makes the GPU
// Unhealthy (compare NVIDIA's DP_DISABLE_HEALTHCHECKS; the reference has no checks).
enum HealthCheck : int {
  kCheckReset = 1,         // PRE_RESET .. POST_RESET
  kCheckEcc = 2,           // uncorrectable ECC count increased
  kCheckLost = 4,          // telemetry failing / device gone
  kCheckRetiredPages = 8,  // retired + pending HBM pages at the threshold
  kCheckPcie = 16,         // host PCIe link below health.pcieMinWidth / pcieMinSpeedGTs (opt-in)
  kCheckAll = 31,
};

struct HealthUpdate {
  int64_t ts_ns = 0;
  int kind = kEvtNone;
  int gpu = -1;        // index in the attached tables' inventory; -1 = not advertised now
  int partition = -1;
  int healthy = -1;  // 1 healthy, 0 unhealthy, -1 = not a health change (link/info)
  int peer = -1;     // link events
  int link_up = -1;
  std::string reason;
  std::string key;       // identity of `gpu` (Backend::gpu_key): what the state belongs to
  std::string peer_key;
  double link_gbps = 0;  // kEvtLinkQuality: the link's trained bandwidth now
};

// A latch that must outlive the plugin process (a DaemonSet rolling update, an OOM kill):
// the manager writes these to its state file, keyed by the host's boot id, and hands them
// back to the next process (HealthMonitor::restore_latches).
struct HealthLatch {
  std::string key;          // GPU identity
  bool ecc_bad = false;     // uncorrectable-ECC latch (cleared only by a reset)
  int64_t last_ue = -1;     // the UE count the latch was taken at (the next baseline)
  // CLOCK_BOOTTIME second at which the GPU's firmware started (boot time - firmware
  // clock), from a clock seen advancing; NaN = unknown.  Negative when the firmware
  // started before the kernel's clock (it does on every boot).  A later process that
  // finds the firmware started later than this knows the GPU was reset meanwhile.
  double fw_boot_s = std::numeric_limits<double>::quiet_NaN();
  std::string reason;
  int64_t since_ns = 0;     // wall clock of the latch
};

// A one-shot flag another thread can wait on with a bound.
struct ThreadExitFlag {
  std::mutex mu;
  std::condition_variable cv;
  bool done = false;
  void set() {
    {
      std::lock_guard<std::mutex> lk(mu);
      done = true;
    }
    cv.notify_all();
  }
  bool wait(int ms) {
    std::unique_lock<std::mutex> lk(mu);
    return cv_wait_ms(cv, lk, ms, [&] { return done; });
  }
};

class HealthMonitor {
 public:
  explicit HealthMonitor(std::shared_ptr<Backend> backend, int lost_after_failures = 3);
  ~HealthMonitor();

  // The advertised inventory, in the tables' index order: keys[i] is the identity
  // (Backend::gpu_key) of GPU i.  Health state is kept per identity, so a re-enumeration
  // that moves a GPU to another index moves its state with it, and a GPU that vanished
  // keeps its state (e.g. mid-reset) until it returns.
  void set_gpus(std::vector<std::string> keys);
  // Legacy form for backends without identities: GPU i is "#i".
  void set_gpu_count(int n);
  void start();
  void stop();
  bool running() const { return running_.load(); }

  // Called by the telemetry sampler after every sample of `gpu`.
  void on_sample(int gpu, bool ok, const GpuSample& s);
  // Feed an event as if it came from the backend (tests, canary failures).
  void process(const HwEvent& e);

  // Blocks up to timeout_ms; returns queued updates (possibly empty).
  std::vector<HealthUpdate> pop(int timeout_ms);
  bool gpu_healthy(int gpu) const;
  // Fail-fast path: an Unhealthy transition is applied to these tables from the
  // monitor thread itself (their gRPC servers push ListAndWatch at once), before the
  // update reaches the Python manager.  Healthy transitions stay with the manager,
  // which may hold a GPU back for the recovery canary.
  void set_fast_tables(std::vector<std::shared_ptr<DeviceTable>> tables);
  // With no recovery canary configured the manager holds nothing back, so Healthy
  // transitions take the same native path (the manager then only records them).
  void set_fast_recover(bool on);
  // Plugin reload: installs the new tables as the fast tables and, under the same lock
  // that orders every transition, marks Unhealthy in them each GPU the monitor reports
  // unhealthy or the caller holds back (`held_unhealthy`, table indices, e.g. a pending
  // recovery canary).  Call after set_gpus.
  void attach_tables(std::vector<std::shared_ptr<DeviceTable>> tables, bool fast_recover,
                     const std::vector<int>& held_unhealthy);
  // Per-GPU retired-page limits (index = table index of the GPU, as in set_gpus; <= 0
  // disables the check for that GPU).
  void set_bad_page_thresholds(std::vector<int> thresholds);
  // Host PCIe link floor (0 = no floor): a GPU whose link trained narrower or slower is
  // Unhealthy until it trains back (a failing riser or retimer halves host bandwidth).
  // `debounce` consecutive samples below the floor degrade the GPU, as many at or above
  // it restore it: one low reading (a link in a power-saving state for a moment) flaps
  // nothing.
  void set_pcie_floor(int min_width, double min_gts, int debounce = 1);
  // Identities the monitor holds state for that are unhealthy (advertised or not).
  std::vector<std::string> unhealthy_keys() const;
  // Bitmask of HealthCheck values to ignore; re-evaluates every GPU (a GPU held only by a
  // check that is now off becomes Healthy).
  void set_disabled_checks(int mask);
  uint64_t events_seen() const { return events_seen_; }
  // Latches to persist: every GPU whose uncorrectable-ECC latch is set (identity order).
  std::vector<HealthLatch> latches() const;
  // Re-applies latches a previous process persisted (same host boot): each GPU is held
  // Unhealthy as before, with the UE baseline it had, until a reset is seen.  A GPU whose
  // firmware is found to have started after the recorded time was reset meanwhile: its
  // first sample clears the latch.  Call before the first attach_tables.
  void restore_latches(const std::vector<HealthLatch>& latches);
  // Resets observed by polling (a kernel reset count that moved, a confirmed firmware
  // clock restart, an outage after which the uncorrectable-ECC counter had been reset).
  uint64_t resets_observed() const;
  // GPUs that came back from a telemetry outage with a latch set and nothing confirming
  // a reset (kEvtResetCandidate): re-verified by the recovery canary, or by an operator.
  uint64_t reset_candidates() const;
  // Firmware clock readings that went backwards without looking like a restart (the clock
  // had not been seen advancing, or the new reading exceeds the time since the last one),
  // or a restart the next reading did not confirm: ignored, counted here.
  uint64_t fw_clock_glitches() const;
  // Drops the latches of GPU `key` that only a reset clears: uncorrectable ECC (its count
  // is re-baselined on the next sample) and a reset in progress (PRE_RESET without
  // POST_RESET).  For a GPU re-verified by the recovery canary after a reset candidate,
  // and for an operator's GET /health/clear.  Levels the next samples re-judge (telemetry
  // lost, retired pages, PCIe) are not touched.  Returns the names of what was cleared
  // ("uncorrectable_ecc", "reset_in_progress"); emits kEvtLatchCleared when any was.
  std::vector<std::string> clear_latches(const std::string& key, const std::string& reason);
  // What holds GPU `key` Unhealthy now ("reset_in_progress", "uncorrectable_ecc",
  // "telemetry_lost", "retired_pages", "pcie_link"), checks turned off included.
  std::vector<std::string> holds(const std::string& key) const;
  // True while any GPU's health is in flux (failing or lost, a reset being confirmed,
  // a candidate unresolved, PCIe or a resetting latch set): the sampler keeps its
  // active cadence then (telemetry.idleIntervalMs).
  bool settling() const;
  // Partitions a recovery must leave Unhealthy (identity -> partition indices; -1 = the
  // whole GPU): failed or pending canary verdicts the manager keeps.  The fast path of a
  // Healthy transition writes the other devices of the GPU only, in one table update.
  void set_held_partitions(std::map<std::string, std::vector<int>> held);

 private:
  struct GpuState {
    bool resetting = false;
    bool ecc_bad = false;
    bool lost = false;
    bool lost_failing = false;  // lost because its samples failed (not a call that hung)
    bool pages_bad = false;  // retired + pending pages at/over the threshold (not cleared by a reset)
    bool pcie_bad = false;   // host PCIe link trained below the configured floor
    int pcie_low = 0;        // consecutive samples below the floor
    int pcie_ok = 0;         // consecutive samples at or above it
    int failures = 0;
    int64_t last_ue = -1;
    bool reported_healthy = true;
    bool restored = false;        // a latch restored from a previous process is set
    std::string ecc_reason;       // what set the ECC latch (persisted with it)
    int64_t ecc_since_ns = 0;
    // firmware clock tracking (GpuSample::fw_clock_s): last reading, the boot-time second
    // it was read at, whether the clock was seen advancing at about one second per
    // second, and the boot-time second the firmware started at (-1 unknown)
    double fw_clock = -1;
    double fw_read_at = -1;
    bool fw_advancing = false;
    int fw_adv_n = 0;             // consecutive readings that advanced at about 1 s/s
    bool fw_jump_pending = false;  // a restart-like step back, confirmed by readings that tick
    int fw_jump_confirms = 0;      // ticking intervals still needed to confirm it
    std::string fw_jump_why;
    int64_t reset_count = -1;      // last kernel reset count seen (GpuSample::reset_count)
    bool candidate = false;        // reset candidate reported, not resolved yet
    bool outage_unresolved = false;  // back from an outage with a clock restart still to confirm
    double fw_boot = std::numeric_limits<double>::quiet_NaN();
    double restored_fw_boot = std::numeric_limits<double>::quiet_NaN();  // previous process; first sample checks it
    std::map<std::string, int> link_up;  // peer key -> 1/0
    std::map<std::string, double> link_bw;  // peer key -> trained bandwidth as this end last saw it
    int page_threshold = 0;
  };
  void loop();
  void emit_locked(HealthUpdate u);
  void reconcile_locked(const std::string& key, int kind, const std::string& reason, bool latch_changed = false);
  bool healthy_locked(const GpuState& st) const;
  // Identity of backend index `gpu` (the index space of samples and events): the
  // event's own key when it carries one, else the backend's, else "#<index>".
  std::string key_of(int gpu, const std::string& given) const;
  int table_index_locked(const std::string& key) const;  // -1 = not advertised

  std::shared_ptr<Backend> backend_;
  int lost_after_;
  mutable std::mutex mu_;
  std::condition_variable cv_;
  std::deque<HealthUpdate> queue_;
  std::unordered_map<std::string, GpuState> state_;
  std::map<std::pair<std::string, std::string>, double> pair_bw_;  // link -> last reported bandwidth
  // Tables built at a reload start from discovery's view of the links, which the monitor
  // may never have reported (a link that re-trained while down, or flapped between the
  // last sample and the discovery).  attach_tables() starts a new epoch; each link's
  // state and bandwidth are reported once more in it, whether or not they changed (the
  // manager applies them only where the new tables disagree).
  uint64_t links_epoch_ = 1;
  std::map<std::pair<std::string, std::string>, uint64_t> up_epoch_, bw_epoch_;  // link -> epoch last reported in
  std::vector<std::string> table_keys_;  // table index -> key
  std::vector<std::shared_ptr<DeviceTable>> fast_tables_;
  bool fast_recover_ = false;
  int disabled_ = 0;  // HealthCheck bits
  int pcie_min_width_ = 0;
  double pcie_min_gts_ = 0;
  int pcie_debounce_ = 1;
  std::thread thread_;
  std::atomic<bool> running_{false};
  bool stop_ = false;
  uint64_t events_seen_ = 0;
  uint64_t resets_observed_ = 0;
  uint64_t reset_candidates_ = 0;
  uint64_t fw_glitches_ = 0;
  std::map<std::string, std::vector<int>> held_parts_;
  // Healthy fast path for table index `idx` of GPU `key`: every device, except the held
  // partitions, in one update per table.
  void write_healthy_locked(int idx, const std::string& key);
};

// CLOCK_BOOTTIME in seconds (monotonic across the host's uptime, suspend included).
double boottime_s();

}  // namespace amdgpu_dp
