#include "fixture_backend.h"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <stdexcept>

namespace amdgpu_dp {

namespace {
// splitmix64: cheap deterministic noise for the telemetry generators
uint64_t mix(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}
double unit(uint64_t x) { return (mix(x) >> 11) * (1.0 / 9007199254740992.0); }
}  // namespace

FixtureBackend::FixtureBackend(uint64_t seed) : seed_(seed), t0_ns_(mono_ns()) {}

std::string FixtureBackend::key_of_slot_locked(int slot) const {
  if (slot < 0 || slot >= static_cast<int>(gpus_.size())) return "";
  return gpus_[slot].uuid.empty() ? "fixture-gpu-" + std::to_string(slot) : gpus_[slot].uuid;
}

void FixtureBackend::translate(HwEvent* e) const {  // mu_ held
  auto inv = inventory();
  auto index_of_slot = [&](int slot) {
    // identity until the first discovery, like an amdsmi session's enumeration order
    if (inv->refs.empty()) return slot;
    for (size_t i = 0; i < inv->refs.size(); ++i)
      if (inv->refs[i].slot == slot) return static_cast<int>(i);
    return -1;
  };
  if (e->gpu >= 0) {
    e->key = key_of_slot_locked(e->gpu);
    e->gpu = index_of_slot(e->gpu);
  }
  if (e->peer >= 0) {
    e->peer_key = key_of_slot_locked(e->peer);
    e->peer = index_of_slot(e->peer);
  }
}

std::string FixtureBackend::gpu_key(int gpu) const {
  if (!inventory()->refs.empty()) return Backend::gpu_key(gpu);
  std::lock_guard<std::mutex> lk(mu_);
  return gpu >= 0 && gpu < static_cast<int>(gpus_.size()) && present_[gpu] ? key_of_slot_locked(gpu) : "";
}

std::unique_lock<std::mutex> FixtureBackend::device_call(int slot) {
  std::unique_lock<std::mutex> lk(serialised_.load() ? driver_mu_ : dev_mu_[slot >= 0 ? slot % kMaxGpus : 0]);
  std::unique_lock<std::mutex> w(wedge_mu_);
  wedge_cv_.wait(w, [&] { return unwedge_all_ || slot >= static_cast<int>(wedged_.size()) || !wedged_[slot]; });
  return lk;
}

void FixtureBackend::add_gpu(const GpuInfo& g) {
  std::lock_guard<std::mutex> lk(mu_);
  if (gpus_.size() >= static_cast<size_t>(kMaxGpus)) throw std::length_error("fixture: too many GPUs");
  GpuInfo copy = g;
  copy.index = static_cast<int>(gpus_.size());
  for (auto& p : copy.partitions) p.gpu = copy.index;
  gpus_.push_back(copy);
  Topology old = topo_;
  topo_.resize(static_cast<int>(gpus_.size()));
  for (int a = 0; a < old.n; ++a)
    for (int b = 0; b < old.n; ++b) topo_.at(a, b) = old.at(a, b);
  ecc_ue_.push_back(0);
  pcie_.emplace_back(16, 32.0);
  pages_.emplace_back(0, 0);
  present_.push_back(true);
  // as on the MI355X box (profiles/r5/reset_signal_probe.json): the firmware started before
  // the kernel did, ~180 s ahead of CLOCK_MONOTONIC zero
  fw_start_ns_.push_back(-180000000000LL);
  fw_reported_.push_back(true);
  fw_frozen_at_.push_back(-1);
  fw_glitch_.push_back(-1);
  gpu_reset_query_.push_back(false);
  reset_count_.push_back(0);
  sample_fail_.push_back(false);
}

void FixtureBackend::replace_gpu(int index, const GpuInfo& g) {
  std::lock_guard<std::mutex> lk(mu_);
  if (index < 0 || index >= static_cast<int>(gpus_.size())) throw std::out_of_range("replace_gpu: bad gpu index");
  GpuInfo copy = g;
  copy.index = index;
  for (auto& p : copy.partitions) p.gpu = index;
  gpus_[index] = copy;
}

GpuInfo FixtureBackend::slot_info(int slot) const {
  std::lock_guard<std::mutex> lk(mu_);
  if (slot < 0 || slot >= static_cast<int>(gpus_.size())) throw std::out_of_range("slot_info: bad gpu index");
  return gpus_[slot];
}

void FixtureBackend::clear() {
  std::lock_guard<std::mutex> lk(mu_);
  gpus_.clear();
  topo_.resize(0);
  ecc_ue_.clear();
  pcie_.clear();
  pages_.clear();
  present_.clear();
  fw_start_ns_.clear();
  fw_reported_.clear();
  fw_frozen_at_.clear();
  fw_glitch_.clear();
  gpu_reset_query_.clear();
  reset_count_.clear();
  sample_fail_.clear();
  scheduled_.clear();
  pending_.clear();
  {
    std::lock_guard<std::mutex> w(wedge_mu_);
    wedged_.clear();  // a call parked on a wedge returns (its GPU is gone)
  }
  wedge_cv_.notify_all();
}

void FixtureBackend::set_link(int a, int b, const Link& l) {
  std::lock_guard<std::mutex> lk(mu_);
  if (a < 0 || b < 0 || a >= topo_.n || b >= topo_.n) throw std::out_of_range("set_link: bad gpu index");
  topo_.at(a, b) = l;
  topo_.at(b, a) = l;
}

void FixtureBackend::set_link_up(int a, int b, bool up) {
  {
    std::lock_guard<std::mutex> lk(mu_);
    if (a < 0 || b < 0 || a >= topo_.n || b >= topo_.n) throw std::out_of_range("set_link_up: bad gpu index");
    topo_.at(a, b).up = up;
    topo_.at(b, a).up = up;
    HwEvent e;
    e.ts_ns = now_ns();
    e.kind = up ? kEvtLinkUp : kEvtLinkDown;
    e.gpu = a;
    e.peer = b;
    e.message = std::string("fixture xgmi link ") + std::to_string(a) + "-" + std::to_string(b) + (up ? " up" : " down");
    pending_.push_back(e);
  }
  cv_.notify_all();
}

void FixtureBackend::set_link_bandwidth(int a, int b, double gbps) {
  std::lock_guard<std::mutex> lk(mu_);
  if (a < 0 || b < 0 || a >= topo_.n || b >= topo_.n) throw std::out_of_range("set_link_bandwidth: bad gpu index");
  topo_.at(a, b).bw_gbps = topo_.at(b, a).bw_gbps = std::max(0.0, gbps);
}

void FixtureBackend::set_ecc_uncorrectable(int gpu, int64_t count) {
  std::lock_guard<std::mutex> lk(mu_);
  if (gpu < 0 || gpu >= static_cast<int>(ecc_ue_.size())) throw std::out_of_range("bad gpu");
  ecc_ue_[gpu] = count;
}

void FixtureBackend::set_pcie_link(int gpu, int width, double gts) {
  std::lock_guard<std::mutex> lk(mu_);
  if (gpu < 0 || gpu >= static_cast<int>(pcie_.size())) throw std::out_of_range("bad gpu");
  pcie_[gpu] = {width, gts};
}

void FixtureBackend::set_retired_pages(int gpu, int64_t reserved, int64_t pending) {
  std::lock_guard<std::mutex> lk(mu_);
  if (gpu < 0 || gpu >= static_cast<int>(pages_.size())) throw std::out_of_range("bad gpu");
  pages_[gpu] = {reserved, pending};
}

void FixtureBackend::set_sample_stall(int gpu, bool stall) {
  {
    std::lock_guard<std::mutex> lk(mu_);
    if (gpu < 0 || gpu >= static_cast<int>(gpus_.size())) throw std::out_of_range("bad gpu");
  }
  {
    std::lock_guard<std::mutex> w(wedge_mu_);
    if (wedged_.size() <= static_cast<size_t>(gpu)) wedged_.resize(gpu + 1, false);
    wedged_[gpu] = stall;
  }
  wedge_cv_.notify_all();
}

void FixtureBackend::set_gpu_present(int gpu, bool present) {
  std::lock_guard<std::mutex> lk(mu_);
  if (gpu < 0 || gpu >= static_cast<int>(present_.size())) throw std::out_of_range("bad gpu");
  present_[gpu] = present;
}

void FixtureBackend::reset_firmware(int gpu) {
  std::lock_guard<std::mutex> lk(mu_);
  if (gpu < 0 || gpu >= static_cast<int>(fw_start_ns_.size())) throw std::out_of_range("bad gpu");
  fw_start_ns_[gpu] = mono_ns();
}

void FixtureBackend::set_fw_clock_reported(int gpu, bool reported) {
  std::lock_guard<std::mutex> lk(mu_);
  if (gpu < 0 || gpu >= static_cast<int>(fw_reported_.size())) throw std::out_of_range("bad gpu");
  fw_reported_[gpu] = reported;
}

void FixtureBackend::set_fw_clock_frozen(int gpu, bool frozen, double at_s) {
  std::lock_guard<std::mutex> lk(mu_);
  if (gpu < 0 || gpu >= static_cast<int>(fw_frozen_at_.size())) throw std::out_of_range("bad gpu");
  if (frozen && at_s >= 0) {
    fw_frozen_at_[gpu] = at_s;
    return;
  }
  if (frozen == (fw_frozen_at_[gpu] >= 0)) return;
  if (frozen) {
    fw_frozen_at_[gpu] = std::max<int64_t>(0, mono_ns() - fw_start_ns_[gpu]) * 1e-9;
  } else {  // runs on from the frozen value
    fw_start_ns_[gpu] = mono_ns() - static_cast<int64_t>(fw_frozen_at_[gpu] * 1e9);
    fw_frozen_at_[gpu] = -1;
  }
}

void FixtureBackend::glitch_fw_clock(int gpu, double value_s) {
  std::lock_guard<std::mutex> lk(mu_);
  if (gpu < 0 || gpu >= static_cast<int>(fw_glitch_.size())) throw std::out_of_range("bad gpu");
  fw_glitch_[gpu] = std::max(0.0, value_s);
}

void FixtureBackend::set_gpu_reset_query(int gpu, bool available) {
  std::lock_guard<std::mutex> lk(mu_);
  if (gpu < 0 || gpu >= static_cast<int>(gpu_reset_query_.size())) throw std::out_of_range("bad gpu");
  gpu_reset_query_[gpu] = available;
}

void FixtureBackend::reset_gpu(int gpu, bool reload_firmware) {
  std::lock_guard<std::mutex> lk(mu_);
  if (gpu < 0 || gpu >= static_cast<int>(reset_count_.size())) throw std::out_of_range("bad gpu");
  ++reset_count_[gpu];
  if (reload_firmware) {
    fw_start_ns_[gpu] = mono_ns();
    if (fw_frozen_at_[gpu] >= 0) fw_frozen_at_[gpu] = -1;  // the reloaded firmware runs
  }
}

void FixtureBackend::set_sample_fail(int gpu, bool fail) {
  std::lock_guard<std::mutex> lk(mu_);
  if (gpu < 0 || gpu >= static_cast<int>(sample_fail_.size())) throw std::out_of_range("bad gpu");
  sample_fail_[gpu] = fail;
}

void FixtureBackend::enumerate(std::vector<DeviceRef>* refs) {
  discover_calls_.fetch_add(1);
  if (fail_discovery_.load()) throw std::runtime_error("fixture: discovery failure injected");
  std::lock_guard<std::mutex> lk(mu_);
  // A GPU that "fell off the bus" is not enumerated, like a real one, and every later GPU
  // moves down one index (amdsmi enumerates in BDF order).
  for (size_t i = 0; i < gpus_.size(); ++i) {
    if (!present_[i]) continue;
    DeviceRef r;
    r.key = key_of_slot_locked(static_cast<int>(i));
    r.bdf = gpus_[i].bdf;
    r.order = i;
    r.slot = static_cast<int>(i);
    refs->push_back(std::move(r));
  }
}

void FixtureBackend::describe(const DeviceRef& ref, const std::vector<DeviceRef>& all, GpuInfo* out,
                              std::vector<Link>* row) {
  auto call = device_call(ref.slot);
  std::lock_guard<std::mutex> lk(mu_);
  if (ref.slot < 0 || ref.slot >= static_cast<int>(gpus_.size()) || !present_[ref.slot])
    throw std::runtime_error("fixture: GPU " + std::to_string(ref.slot) + " is gone");
  *out = gpus_[ref.slot];
  row->assign(all.size(), Link{});
  for (size_t p = 0; p < all.size(); ++p)
    if (all[p].slot >= 0 && all[p].slot < topo_.n && all[p].slot != ref.slot) (*row)[p] = topo_.at(ref.slot, all[p].slot);
}

bool FixtureBackend::sample_device(const Inventory& inv, int index, GpuSample* s) {
  const int gpu = inv.refs[index].slot;
  auto call = device_call(gpu);
  std::lock_guard<std::mutex> lk(mu_);
  if (gpu < 0 || gpu >= static_cast<int>(gpus_.size()) || !present_[gpu] || sample_fail_[gpu]) return false;
  auto index_of_slot = [&](int slot) {
    for (size_t i = 0; i < inv.refs.size(); ++i)
      if (inv.refs[i].slot == slot) return static_cast<int>(i);
    return -1;
  };
  const GpuInfo& g = gpus_[gpu];
  const int64_t t = now_ns();
  const double ts = (mono_ns() - t0_ns_) * 1e-9;  // seconds since the fixture was created
  const uint64_t tick = static_cast<uint64_t>(ts * 10);  // noise changes at 10 Hz
  const uint64_t key = seed_ * 1000003ull + gpu * 7919ull;
  s->ts_ns = t;
  const double load = 0.5 + 0.45 * std::sin(ts * 0.7 + gpu);
  s->power_w = 220.0 + 1100.0 * load + 10.0 * unit(key ^ tick);
  s->energy_j = 1e6 + ts * 700.0;
  s->temp_edge_c = 40 + 30 * load;
  s->temp_hotspot_c = 45 + 45 * load + 2 * unit(key + 1 + tick);
  s->temp_mem_c = 42 + 35 * load;
  s->num_hbm = 8;
  for (int h = 0; h < 8; ++h) s->temp_hbm_c[h] = 44 + 33 * load + unit(key + 10 + h + tick);
  s->gfx_activity_pct = 100.0 * load;
  s->umc_activity_pct = 70.0 * load;
  s->gfxclk_mhz = 1500 + 900 * load;
  s->uclk_mhz = 1900;
  s->vram_total_bytes = static_cast<double>(g.vram_total_bytes);
  s->vram_used_bytes = g.vram_total_bytes * 0.6 * load;
  s->ecc_correctable = static_cast<int64_t>(ts) % 3;
  s->ecc_uncorrectable = ecc_ue_[gpu];
  s->retired_pages = pages_[gpu].first;
  s->pending_pages = pages_[gpu].second;
  s->unreservable_pages = 0;
  s->throttle_status = 0;
  s->num_links = 0;
  s->xgmi_link_width = 16;
  s->xgmi_link_speed = 38;
  s->xgmi_error_status = 0;
  s->pcie_link_width = pcie_[gpu].first;
  s->pcie_link_speed_gtps = pcie_[gpu].second;
  s->pcie_replays = 0;
  s->pcie_recoveries = 0;
  s->fw_clock_s = !fw_reported_[gpu]         ? -1
                  : fw_glitch_[gpu] >= 0     ? fw_glitch_[gpu]
                  : fw_frozen_at_[gpu] >= 0  ? fw_frozen_at_[gpu]
                                             : std::max<int64_t>(0, mono_ns() - fw_start_ns_[gpu]) * 1e-9;
  fw_glitch_[gpu] = -1;
  s->reset_count = gpu_reset_query_[gpu] && reset_query() ? reset_count_[gpu] : -1;
  for (int peer = 0; peer < topo_.n && s->num_links < kMaxXgmiLinks; ++peer) {
    if (peer == gpu || topo_.at(gpu, peer).type != kLinkXgmi) continue;
    const int k = s->num_links++;
    s->link_peer[k] = index_of_slot(peer);  // -1 while the peer is not discovered
    s->link_up[k] = topo_.at(gpu, peer).up ? 1 : 0;
    s->link_read_kb[k] = 1e6 * ts * load;
    s->link_write_kb[k] = 0.9e6 * ts * load;
    // what amdsmi reports on MI355X: 38 Gb/s per lane, 16 lanes -> 608 Gb/s per link
    const double bw = topo_.at(gpu, peer).bw_gbps > 0 ? topo_.at(gpu, peer).bw_gbps : 608.0;
    s->link_bitrate_gbps[k] = bw / 16.0;  // a slow fixture link trained at a lower rate, 16 lanes wide
    s->link_max_gbps[k] = 608.0;          // capability
    s->link_trained_gbps[k] = bw;
  }
  s->num_partitions = std::min<int>(static_cast<int>(g.partitions.size()), kMaxPartitions);
  for (int p = 0; p < s->num_partitions; ++p) {
    s->partition_gfx_busy_pct[p] = 100.0 * (0.5 + 0.45 * std::sin(ts * 0.7 + gpu + 0.3 * p));
    s->partition_busy_source[p] = 1;  // as the partition metrics API reports it
    s->partition_vram_used_bytes[p] = s->vram_used_bytes / std::max(1, s->num_partitions);
  }
  s->ok = true;
  return true;
}

void FixtureBackend::arm_events() {
  std::lock_guard<std::mutex> lk(mu_);
  // scheduled scripts run either way (their ECC / link effects are what polling sees)
  armed_at_ns_.store(mono_ns());
  shutdown_ = false;
}

void FixtureBackend::schedule_event(double delay_s, const HwEvent& e) {
  {
    std::lock_guard<std::mutex> lk(mu_);
    scheduled_.push_back({delay_s, e});
    std::stable_sort(scheduled_.begin(), scheduled_.end(),
                     [](const Scheduled& a, const Scheduled& b) { return a.delay_s < b.delay_s; });
  }
  cv_.notify_all();
}

void FixtureBackend::inject_event(const HwEvent& e) {
  {
    std::lock_guard<std::mutex> lk(mu_);
    HwEvent copy = e;
    if (copy.ts_ns == 0) copy.ts_ns = now_ns();
    pending_.push_back(copy);
  }
  cv_.notify_all();
}

void FixtureBackend::shutdown() {
  {
    std::lock_guard<std::mutex> lk(mu_);
    shutdown_ = true;
  }
  cv_.notify_all();
  {
    std::lock_guard<std::mutex> w(wedge_mu_);
    unwedge_all_ = true;
  }
  wedge_cv_.notify_all();
}

int FixtureBackend::wait_events(int timeout_ms, std::vector<HwEvent>* out) {
  std::unique_lock<std::mutex> lk(mu_);
  const int64_t deadline = mono_ns() + static_cast<int64_t>(timeout_ms) * 1000000;
  for (;;) {
    // promote due scheduled events
    const int64_t armed_at = armed_at_ns_.load();
    if (armed_at != 0) {
      const double elapsed = (mono_ns() - armed_at) * 1e-9;
      while (!scheduled_.empty() && scheduled_.front().delay_s <= elapsed) {
        HwEvent e = scheduled_.front().ev;
        e.ts_ns = now_ns();
        if (e.kind == kEvtEccUncorrectable && e.gpu >= 0 && e.gpu < static_cast<int>(ecc_ue_.size()))
          ecc_ue_[e.gpu] += 1;
        if (e.kind == kScriptFirmwareReset) {
          if (e.gpu >= 0 && e.gpu < static_cast<int>(fw_start_ns_.size())) fw_start_ns_[e.gpu] = mono_ns();
          scheduled_.erase(scheduled_.begin());
          continue;  // seen only through the firmware clock
        }
        if ((e.kind == kEvtLinkDown || e.kind == kEvtLinkUp) && e.gpu >= 0 && e.peer >= 0 &&
            e.gpu < topo_.n && e.peer < topo_.n) {
          topo_.at(e.gpu, e.peer).up = topo_.at(e.peer, e.gpu).up = (e.kind == kEvtLinkUp);
        }
        pending_.push_back(e);
        scheduled_.erase(scheduled_.begin());
      }
    }
    if (!pending_.empty()) {
      int n = 0;
      const bool delivered = events_enabled_.load();
      while (!pending_.empty()) {
        HwEvent e = pending_.front();
        pending_.pop_front();
        // what only amdsmi event notification reports is lost without it; an uncorrectable
        // ECC error is then seen by polling the count (incremented when it fired)
        if (!delivered && (e.kind == kEvtPreReset || e.kind == kEvtPostReset || e.kind == kEvtThermal ||
                           e.kind == kEvtVmFault || e.kind == kEvtEccUncorrectable))
          continue;
        translate(&e);
        out->push_back(std::move(e));
        ++n;
      }
      return n;
    }
    if (shutdown_) return 0;
    const int64_t now = mono_ns();
    if (now >= deadline) return 0;
    int64_t wait_ns = deadline - now;
    if (armed_at != 0 && !scheduled_.empty()) {
      const int64_t due = armed_at + static_cast<int64_t>(scheduled_.front().delay_s * 1e9);
      wait_ns = std::min<int64_t>(wait_ns, std::max<int64_t>(0, due - now));
    }
    cv_wait_ms(cv_, lk, wait_ns / 1000000 + 1, [&] { return !pending_.empty() || shutdown_; });
  }
}

}  // namespace amdgpu_dp
