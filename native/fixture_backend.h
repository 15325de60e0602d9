// Scripted hardware backend: N fake MI355X GPUs x {SPX..CPX} x {NPS1..NPS8},
// an xGMI link matrix with per-link health, deterministic telemetry generators and
// timed fault scripts.  The reference has no fake NVML at all; this is
// the seam every CPU test and the BASELINE "Mock-device backend" config run on.
#pragma once

#include <condition_variable>
#include <deque>
#include <mutex>

#include "backend.h"

namespace amdgpu_dp {

class FixtureBackend : public Backend {
 public:
  explicit FixtureBackend(uint64_t seed = 1);
  std::string name() const override { return "fixture"; }
  void discover(std::vector<GpuInfo>* gpus, Topology* topo) override;
  // `gpu` is an index of the latest discover(), like amdsmi's: after a GPU vanished and
  // the node was re-discovered, index k samples the GPU that moved to k.
  bool sample(int gpu, GpuSample* out) override;
  std::string gpu_key(int gpu) const override;
  int wait_events(int timeout_ms, std::vector<HwEvent>* out) override;
  void arm_events() override;
  int armed_event_sources() const override { return armed_at_ns_ != 0 ? 1 : 0; }
  void shutdown() override;

  // --- configuration (called before / between discoveries) ---
  // Every method below names GPUs by fixture slot (the order add_gpu added them), which
  // never changes: a script's "GPU 1" stays the same physical GPU when GPU 0 vanishes.
  // Events are delivered in the latest discovery's index space, with the GPU's key.
  void add_gpu(const GpuInfo& g);
  // Swap a GPU's description (e.g. a compute/memory partition-mode change).
  void replace_gpu(int index, const GpuInfo& g);
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
  // A wedged driver: sample(gpu) blocks until the stall is lifted (or shutdown), the way
  // an amdsmi call can hang on a GPU that stopped responding.
  void set_sample_stall(int gpu, bool stall);
  int discover_calls() const { return discover_calls_; }

 private:
  mutable std::mutex mu_;
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
  std::vector<bool> stalled_;
  std::vector<int> view_;  // latest discover(): index -> slot (identity until the first)
  int slot_of_locked(int index) const;
  int index_of_locked(int slot) const;
  std::string key_of_slot_locked(int slot) const;
  void translate_locked(HwEvent* e) const;  // slot -> discovered index, plus keys
  int64_t armed_at_ns_ = 0;
  uint64_t seed_;
  int64_t t0_ns_;
  bool fail_discovery_ = false;
  bool shutdown_ = false;
  int discover_calls_ = 0;
};

}  // namespace amdgpu_dp
