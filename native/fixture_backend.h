// Scripted hardware backend: N fake MI355X GPUs x {SPX..CPX} x {NPS1..NPS8},
// an xGMI link matrix with per-link health, deterministic telemetry generators and
// timed fault scripts.  The reference has no fake NVML at all; this is
// the seam every CPU test and the BASELINE "Mock-device backend" config run on.
//
// A wedged driver is modelled by the lock it holds.  Every call that talks to one GPU
// (describe at discovery, a telemetry sample) holds a "driver lock" for its duration:
// per device by default (rocm_smi's per-device mutex), or one lock for the whole library
// (set_serialised(true)).  A wedged GPU's call blocks while holding that lock, so in the
// serialised model every later call to any GPU waits behind it, exactly as it would in a
// library that serialises all devices.
#pragma once

#include <condition_variable>
#include <deque>
#include <mutex>

#include "backend.h"

namespace amdgpu_dp {

class FixtureBackend : public Backend {
 public:
  static constexpr int kMaxGpus = 64;
  // A scripted event kind that is not delivered: the GPU's firmware restarts (a reset as
  // polling sees it, with no event notification) when it fires.
  static constexpr int kScriptFirmwareReset = 100;
  explicit FixtureBackend(uint64_t seed = 1);
  std::string name() const override { return "fixture"; }
  // before the first discovery, index = slot (like an amdsmi session's enumeration order)
  std::string gpu_key(int gpu) const override;
  int wait_events(int timeout_ms, std::vector<HwEvent>* out) override;
  void arm_events() override;
  int armed_event_sources() const override { return armed_at_ns_.load() != 0 && events_enabled_.load() ? 1 : 0; }
  void shutdown() override;

  // --- configuration (called before / between discoveries) ---
  // Every method below names GPUs by fixture slot (the order add_gpu added them), which
  // never changes: a script's "GPU 1" stays the same physical GPU when GPU 0 vanishes.
  // Events are delivered in the latest discovery's index space, with the GPU's key.
  void add_gpu(const GpuInfo& g);
  // Swap a GPU's description (e.g. a compute/memory partition-mode change).
  void replace_gpu(int index, const GpuInfo& g);
  // The model's own description of slot `slot` (no discovery, no device call).
  GpuInfo slot_info(int slot) const;
  void clear();
  void set_link(int a, int b, const Link& l);  // symmetric
  void set_link_up(int a, int b, bool up);      // also emits LinkDown/LinkUp events
  // The a-b link re-trains at `gbps` (all lanes); samples report it from now on, the way
  // amdsmi link metrics would (0 = back to the nominal 608 Gb/s).
  void set_link_bandwidth(int a, int b, double gbps);
  // Event `kind` fires `delay_s` seconds after arm_events().
  void schedule_event(double delay_s, const HwEvent& e);
  // Event fires immediately (wakes wait_events).
  void inject_event(const HwEvent& e);
  void set_fail_discovery(bool fail) { fail_discovery_ = fail; }
  void set_ecc_uncorrectable(int gpu, int64_t count);
  void set_retired_pages(int gpu, int64_t reserved, int64_t pending);
  void set_pcie_link(int gpu, int width, double gts);  // the host link as gpu_metrics reports it
  void set_gpu_present(int gpu, bool present);
  // The GPU's firmware restarts now (what a reset does): its clock starts again at zero.
  void reset_firmware(int gpu);
  // Whether samples report the firmware clock (some firmware does not).
  void set_fw_clock_reported(int gpu, bool reported);
  // The firmware clock stops (a hung SMU) - where it is, or at `at_s` seconds when >= 0 -
  // or runs again from there.
  void set_fw_clock_frozen(int gpu, bool frozen, double at_s = -1);
  // The next sample alone reports this clock value (one stale or garbage reading).
  void glitch_fw_clock(int gpu, double value_s);
  // Whether samples report the kernel's reset count (GpuSample::reset_count): the render
  // node can be opened (CDI-injected or privileged), or not (the default DaemonSet).
  void set_gpu_reset_query(int gpu, bool available);
  // The driver resets the GPU: the kernel's reset count moves; reload_firmware = a reset
  // that reloads the power-management firmware (mode-1: its clock starts again), else one
  // that keeps it running (mode-2, engine resets).  Telemetry failing meanwhile is the
  // caller's to model (set_sample_fail).
  void reset_gpu(int gpu, bool reload_firmware);
  // Telemetry of `gpu` fails (returns at once, unlike a wedge) while the GPU stays enumerated:
  // a GPU in the middle of a reset.
  void set_sample_fail(int gpu, bool fail);
  // false: the node delivers no hardware events (an unprivileged pod cannot open /dev/kfd):
  // arm_events arms nothing and reset / thermal / VM-fault events are dropped.
  void set_events_enabled(bool on) { events_enabled_.store(on); }
  // A wedged driver: every call to `gpu` (sample, describe) blocks, holding its driver
  // lock, until the wedge is lifted (or shutdown) - the way an amdsmi call can hang on a
  // GPU that stopped responding.
  void set_sample_stall(int gpu, bool stall);
  // One driver lock for all GPUs (a library that serialises every device) instead of one
  // per GPU.  Set it while no call is in flight.
  void set_serialised(bool on) { serialised_.store(on); }
  bool serialised() const { return serialised_.load(); }
  int discover_calls() const { return discover_calls_.load(); }

 protected:
  void enumerate(std::vector<DeviceRef>* refs) override;
  void describe(const DeviceRef& ref, const std::vector<DeviceRef>& all, GpuInfo* out,
                std::vector<Link>* row) override;
  bool sample_device(const Inventory& inv, int index, GpuSample* out) override;

 private:
  // Held for the duration of one device call; blocks while the GPU is wedged.
  std::unique_lock<std::mutex> device_call(int slot);
  mutable std::mutex mu_;  // fixture state; never held while a device call waits
  std::condition_variable cv_;
  std::vector<GpuInfo> gpus_;
  Topology topo_;
  std::deque<HwEvent> pending_;
  struct Scheduled {
    double delay_s;
    HwEvent ev;
  };
  std::vector<Scheduled> scheduled_;
  std::vector<int64_t> ecc_ue_;
  std::vector<std::pair<int, double>> pcie_;  // (lanes, GT/s) per GPU
  std::vector<std::pair<int64_t, int64_t>> pages_;  // (reserved, pending) per GPU
  std::vector<bool> present_;
  std::vector<int64_t> fw_start_ns_;   // CLOCK_MONOTONIC ns the GPU's firmware started at
  std::vector<bool> fw_reported_;
  std::vector<double> fw_frozen_at_;   // >= 0: the clock reads this, frozen
  std::vector<double> fw_glitch_;      // >= 0: the next sample reads this once
  std::vector<bool> gpu_reset_query_;
  std::vector<int64_t> reset_count_;
  std::vector<bool> sample_fail_;
  std::atomic<bool> events_enabled_{true};
  std::string key_of_slot_locked(int slot) const;
  void translate(HwEvent* e) const;  // slot -> discovered index, plus keys
  std::atomic<int64_t> armed_at_ns_{0};
  uint64_t seed_;
  int64_t t0_ns_;
  std::atomic<bool> fail_discovery_{false};
  bool shutdown_ = false;  // guarded by mu_
  std::atomic<int> discover_calls_{0};
  // driver locks and wedges
  std::atomic<bool> serialised_{false};
  std::mutex driver_mu_;              // the one lock of the serialised model
  std::mutex dev_mu_[kMaxGpus];       // per-GPU locks of the default model
  std::mutex wedge_mu_;
  std::condition_variable wedge_cv_;
  std::vector<bool> wedged_;          // guarded by wedge_mu_
  bool unwedge_all_ = false;          // shutdown: guarded by wedge_mu_
};

}  // namespace amdgpu_dp
