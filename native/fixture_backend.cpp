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

int FixtureBackend::slot_of_locked(int index) const {
  if (view_.empty()) return index >= 0 && index < static_cast<int>(gpus_.size()) ? index : -1;
  return index >= 0 && index < static_cast<int>(view_.size()) ? view_[index] : -1;
}

int FixtureBackend::index_of_locked(int slot) const {
  if (view_.empty()) return slot;
  for (size_t i = 0; i < view_.size(); ++i)
    if (view_[i] == slot) return static_cast<int>(i);
  return -1;
}

std::string FixtureBackend::key_of_slot_locked(int slot) const {
  if (slot < 0 || slot >= static_cast<int>(gpus_.size())) return "";
  return gpus_[slot].uuid.empty() ? "fixture-gpu-" + std::to_string(slot) : gpus_[slot].uuid;
}

void FixtureBackend::translate_locked(HwEvent* e) const {
  if (e->gpu >= 0) {
    e->key = key_of_slot_locked(e->gpu);
    e->gpu = index_of_locked(e->gpu);
  }
  if (e->peer >= 0) {
    e->peer_key = key_of_slot_locked(e->peer);
    e->peer = index_of_locked(e->peer);
  }
}

std::string FixtureBackend::gpu_key(int gpu) const {
  std::lock_guard<std::mutex> lk(mu_);
  return key_of_slot_locked(slot_of_locked(gpu));
}

void FixtureBackend::add_gpu(const GpuInfo& g) {
  std::lock_guard<std::mutex> lk(mu_);
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
  if (!view_.empty()) view_.clear();  // a changed node: identity until it is discovered again
}

void FixtureBackend::replace_gpu(int index, const GpuInfo& g) {
  std::lock_guard<std::mutex> lk(mu_);
  if (index < 0 || index >= static_cast<int>(gpus_.size())) throw std::out_of_range("replace_gpu: bad gpu index");
  GpuInfo copy = g;
  copy.index = index;
  for (auto& p : copy.partitions) p.gpu = index;
  gpus_[index] = copy;
}

void FixtureBackend::clear() {
  std::lock_guard<std::mutex> lk(mu_);
  gpus_.clear();
  topo_.resize(0);
  ecc_ue_.clear();
  pcie_.clear();
  pages_.clear();
  present_.clear();
  stalled_.clear();
  view_.clear();
  scheduled_.clear();
  pending_.clear();
  cv_.notify_all();  // a sample() parked on a stall returns (its GPU is gone)
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
    if (stalled_.size() < gpus_.size()) stalled_.resize(gpus_.size(), false);
    stalled_[gpu] = stall;
  }
  cv_.notify_all();
}

void FixtureBackend::set_gpu_present(int gpu, bool present) {
  std::lock_guard<std::mutex> lk(mu_);
  if (gpu < 0 || gpu >= static_cast<int>(present_.size())) throw std::out_of_range("bad gpu");
  present_[gpu] = present;
}

void FixtureBackend::discover(std::vector<GpuInfo>* gpus, Topology* topo) {
  std::lock_guard<std::mutex> lk(mu_);
  ++discover_calls_;
  if (fail_discovery_) throw std::runtime_error("fixture: discovery failure injected");
  gpus->clear();
  // A GPU that "fell off the bus" disappears from discovery, like a real one, and every
  // later GPU moves down one index (amdsmi enumerates in BDF order).
  std::vector<int> remap(gpus_.size(), -1);
  view_.clear();
  for (size_t i = 0; i < gpus_.size(); ++i) {
    if (!present_[i]) continue;
    remap[i] = static_cast<int>(gpus->size());
    view_.push_back(static_cast<int>(i));
    GpuInfo g = gpus_[i];
    g.index = remap[i];
    for (auto& p : g.partitions) p.gpu = g.index;
    gpus->push_back(std::move(g));
  }
  topo->resize(static_cast<int>(gpus->size()));
  for (size_t a = 0; a < gpus_.size(); ++a)
    for (size_t b = 0; b < gpus_.size(); ++b)
      if (remap[a] >= 0 && remap[b] >= 0) topo->at(remap[a], remap[b]) = topo_.at(a, b);
}

bool FixtureBackend::sample(int index, GpuSample* s) {
  std::unique_lock<std::mutex> lk(mu_);
  const int gpu = slot_of_locked(index);
  s->key = key_of_slot_locked(gpu);
  if (gpu < 0 || gpu >= static_cast<int>(gpus_.size()) || !present_[gpu]) return false;
  cv_.wait(lk, [&] { return shutdown_ || gpu >= static_cast<int>(stalled_.size()) || !stalled_[gpu]; });
  if (gpu >= static_cast<int>(gpus_.size()) || !present_[gpu]) return false;
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
  for (int peer = 0; peer < topo_.n && s->num_links < kMaxXgmiLinks; ++peer) {
    if (peer == gpu || topo_.at(gpu, peer).type != kLinkXgmi) continue;
    const int k = s->num_links++;
    s->link_peer[k] = index_of_locked(peer);  // -1 while the peer is not discovered
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
    s->partition_vram_used_bytes[p] = s->vram_used_bytes / std::max(1, s->num_partitions);
  }
  s->ok = true;
  return true;
}

void FixtureBackend::arm_events() {
  std::lock_guard<std::mutex> lk(mu_);
  armed_at_ns_ = mono_ns();
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
}

int FixtureBackend::wait_events(int timeout_ms, std::vector<HwEvent>* out) {
  std::unique_lock<std::mutex> lk(mu_);
  const int64_t deadline = mono_ns() + static_cast<int64_t>(timeout_ms) * 1000000;
  for (;;) {
    // promote due scheduled events
    if (armed_at_ns_ != 0) {
      const double elapsed = (mono_ns() - armed_at_ns_) * 1e-9;
      while (!scheduled_.empty() && scheduled_.front().delay_s <= elapsed) {
        HwEvent e = scheduled_.front().ev;
        e.ts_ns = now_ns();
        if (e.kind == kEvtEccUncorrectable && e.gpu >= 0 && e.gpu < static_cast<int>(ecc_ue_.size()))
          ecc_ue_[e.gpu] += 1;
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
      while (!pending_.empty()) {
        HwEvent e = pending_.front();
        pending_.pop_front();
        translate_locked(&e);
        out->push_back(std::move(e));
        ++n;
      }
      return n;
    }
    if (shutdown_) return 0;
    const int64_t now = mono_ns();
    if (now >= deadline) return 0;
    int64_t wait_ns = deadline - now;
    if (armed_at_ns_ != 0 && !scheduled_.empty()) {
      const int64_t due = armed_at_ns_ + static_cast<int64_t>(scheduled_.front().delay_s * 1e9);
      wait_ns = std::min<int64_t>(wait_ns, std::max<int64_t>(0, due - now));
    }
    cv_wait_ms(cv_, lk, wait_ns / 1000000 + 1, [&] { return !pending_.empty() || shutdown_; });
  }
}

}  // namespace amdgpu_dp
