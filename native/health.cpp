#include "health.h"

#include <algorithm>
#include <chrono>

namespace amdgpu_dp {

HealthMonitor::HealthMonitor(std::shared_ptr<Backend> backend, int lost_after_failures)
    : backend_(std::move(backend)), lost_after_(lost_after_failures) {}

HealthMonitor::~HealthMonitor() { stop(); }

void HealthMonitor::set_gpu_count(int n) {
  // Called on every plugin (re)load: keep the state of GPUs that are still there, or a
  // GPU that is mid-reset when kubelet restarts would be forgotten as healthy and its
  // POST_RESET would never produce the Healthy update.
  std::lock_guard<std::mutex> lk(mu_);
  state_.resize(static_cast<size_t>(std::max(0, n)));
}

void HealthMonitor::start() {
  std::lock_guard<std::mutex> lk(mu_);
  if (running_) return;
  stop_ = false;
  running_ = true;
  backend_->arm_events();
  thread_ = std::thread([this] { loop(); });
}

void HealthMonitor::stop() {
  {
    std::lock_guard<std::mutex> lk(mu_);
    if (!running_) return;
    stop_ = true;
  }
  cv_.notify_all();
  if (thread_.joinable()) thread_.join();
  std::lock_guard<std::mutex> lk(mu_);
  running_ = false;
}

void HealthMonitor::loop() {
  std::vector<HwEvent> evs;
  for (;;) {
    {
      std::lock_guard<std::mutex> lk(mu_);
      if (stop_) return;
    }
    evs.clear();
    // bounded wait so stop() is honoured within ~200 ms
    backend_->wait_events(200, &evs);
    for (const auto& e : evs) process(e);
  }
}

void HealthMonitor::emit_locked(HealthUpdate u) {
  if (u.ts_ns == 0) u.ts_ns = now_ns();
  queue_.push_back(std::move(u));
  cv_.notify_all();
}

namespace {
int check_of(int kind) {
  switch (kind) {
    case kEvtPreReset:
    case kEvtPostReset: return kCheckReset;
    case kEvtEccUncorrectable: return kCheckEcc;
    case kEvtDeviceLost:
    case kEvtDeviceRecovered: return kCheckLost;
    case kEvtRetiredPagesExceeded:
    case kEvtRetiredPagesCleared: return kCheckRetiredPages;
    default: return 0;
  }
}
}  // namespace

bool HealthMonitor::healthy_locked(const GpuState& st) const {
  return !(st.resetting && !(disabled_ & kCheckReset)) && !(st.ecc_bad && !(disabled_ & kCheckEcc)) &&
         !(st.lost && !(disabled_ & kCheckLost)) && !(st.pages_bad && !(disabled_ & kCheckRetiredPages));
}

void HealthMonitor::reconcile_locked(int gpu, int kind, const std::string& reason) {
  GpuState& st = state_[gpu];
  const bool healthy = healthy_locked(st);
  if (healthy == st.reported_healthy) {
    if (disabled_ & check_of(kind)) {  // tracked, not acted on: still worth a log line
      HealthUpdate u;
      u.kind = kind;
      u.gpu = gpu;
      u.reason = reason + " (health check disabled)";
      emit_locked(std::move(u));
    }
    return;
  }
  st.reported_healthy = healthy;
  if (!healthy || fast_recover_)
    for (const auto& t : fast_tables_) t->set_gpu_health(gpu, -1, healthy);
  HealthUpdate u;
  u.kind = kind;
  u.gpu = gpu;
  u.healthy = healthy ? 1 : 0;
  u.reason = reason;
  emit_locked(std::move(u));
}

void HealthMonitor::process(const HwEvent& e) {
  std::lock_guard<std::mutex> lk(mu_);
  ++events_seen_;
  auto valid = [&](int g) { return g >= 0 && g < static_cast<int>(state_.size()); };
  const std::string why = std::string(event_kind_name(e.kind)) + (e.message.empty() ? "" : ": " + e.message);
  switch (e.kind) {
    case kEvtPreReset:
      if (!valid(e.gpu)) return;
      state_[e.gpu].resetting = true;
      reconcile_locked(e.gpu, e.kind, why);
      return;
    case kEvtPostReset:
      if (!valid(e.gpu)) return;
      state_[e.gpu].resetting = false;
      state_[e.gpu].ecc_bad = false;  // a reset clears the uncorrectable-error latch
      state_[e.gpu].last_ue = -1;     // re-baseline on next sample
      reconcile_locked(e.gpu, e.kind, why);
      return;
    case kEvtEccUncorrectable:
      if (!valid(e.gpu)) return;
      state_[e.gpu].ecc_bad = true;
      reconcile_locked(e.gpu, e.kind, why);
      return;
    case kEvtDeviceLost:
      if (!valid(e.gpu)) return;
      state_[e.gpu].lost = true;
      reconcile_locked(e.gpu, e.kind, why);
      return;
    case kEvtDeviceRecovered:
      if (!valid(e.gpu)) return;
      state_[e.gpu].lost = false;
      state_[e.gpu].failures = 0;
      reconcile_locked(e.gpu, e.kind, why);
      return;
    case kEvtRetiredPagesExceeded:
    case kEvtRetiredPagesCleared:
      if (!valid(e.gpu)) return;
      state_[e.gpu].pages_bad = e.kind == kEvtRetiredPagesExceeded;
      reconcile_locked(e.gpu, e.kind, why);
      return;
    case kEvtLinkDown:
    case kEvtLinkUp: {
      if (!valid(e.gpu) || e.peer < 0) return;
      const int up = e.kind == kEvtLinkUp ? 1 : 0;
      auto& m = state_[e.gpu].link_up;
      auto it = m.find(e.peer);
      if (it != m.end() && it->second == up) return;  // already known (polling + event)
      m[e.peer] = up;
      if (valid(e.peer)) state_[e.peer].link_up[e.gpu] = up;
      HealthUpdate u;
      u.kind = e.kind;
      u.gpu = e.gpu;
      u.peer = e.peer;
      u.link_up = up;
      u.reason = why;
      emit_locked(std::move(u));
      return;
    }
    default: {
      HealthUpdate u;  // informational (thermal, vm fault)
      u.kind = e.kind;
      u.gpu = e.gpu;
      u.partition = e.partition;
      u.reason = why;
      emit_locked(std::move(u));
    }
  }
}

void HealthMonitor::on_sample(int gpu, bool ok, const GpuSample& s) {
  std::vector<HwEvent> derived;
  {
    std::lock_guard<std::mutex> lk(mu_);
    if (gpu < 0 || gpu >= static_cast<int>(state_.size())) return;
    GpuState& st = state_[gpu];
    if (!ok) {
      if (++st.failures >= lost_after_ && !st.lost) {
        HwEvent e;
        e.kind = kEvtDeviceLost;
        e.gpu = gpu;
        e.message = "telemetry failed " + std::to_string(st.failures) + " times in a row";
        derived.push_back(e);
      }
    } else {
      st.failures = 0;
      if (st.lost) {
        HwEvent e;
        e.kind = kEvtDeviceRecovered;
        e.gpu = gpu;
        e.message = "telemetry responding again";
        derived.push_back(e);
      }
      if (s.ecc_uncorrectable >= 0) {
        if (st.last_ue >= 0 && s.ecc_uncorrectable > st.last_ue) {
          HwEvent e;
          e.kind = kEvtEccUncorrectable;
          e.gpu = gpu;
          e.message = "uncorrectable ECC count " + std::to_string(st.last_ue) + " -> " +
                      std::to_string(s.ecc_uncorrectable);
          derived.push_back(e);
        }
        st.last_ue = s.ecc_uncorrectable;
      }
      const int thr = gpu < static_cast<int>(page_thresholds_.size()) ? page_thresholds_[gpu] : 0;
      if (s.retired_pages >= 0) {
        const int64_t bad = s.retired_pages + std::max<int64_t>(0, s.pending_pages);
        const bool over = thr > 0 && bad >= thr;
        if (over != st.pages_bad) {
          HwEvent e;
          e.kind = over ? kEvtRetiredPagesExceeded : kEvtRetiredPagesCleared;
          e.gpu = gpu;
          e.message = std::to_string(bad) + " retired/pending HBM pages, threshold " + std::to_string(thr);
          derived.push_back(e);
        }
      }
      for (int k = 0; k < s.num_links; ++k) {
        if (s.link_peer[k] < 0 || s.link_up[k] < 0) continue;
        auto it = st.link_up.find(s.link_peer[k]);
        const int prev = it == st.link_up.end() ? 1 : it->second;  // links assumed up at start
        if (prev != s.link_up[k]) {
          HwEvent e;
          e.kind = s.link_up[k] ? kEvtLinkUp : kEvtLinkDown;
          e.gpu = gpu;
          e.peer = s.link_peer[k];
          e.message = "xgmi link status poll";
          derived.push_back(e);
        }
      }
    }
  }
  for (const auto& e : derived) process(e);
}

std::vector<HealthUpdate> HealthMonitor::pop(int timeout_ms) {
  std::unique_lock<std::mutex> lk(mu_);
  if (queue_.empty())
    cv_wait_ms(cv_, lk, timeout_ms, [&] { return !queue_.empty() || stop_; });
  std::vector<HealthUpdate> out(queue_.begin(), queue_.end());
  queue_.clear();
  return out;
}

void HealthMonitor::set_fast_tables(std::vector<std::shared_ptr<DeviceTable>> tables) {
  std::lock_guard<std::mutex> lk(mu_);
  fast_tables_ = std::move(tables);
}

void HealthMonitor::set_fast_recover(bool on) {
  std::lock_guard<std::mutex> lk(mu_);
  fast_recover_ = on;
}

void HealthMonitor::attach_tables(std::vector<std::shared_ptr<DeviceTable>> tables, bool fast_recover,
                                  const std::vector<int>& held_unhealthy) {
  // One critical section: a transition processed before it is written into the new
  // tables here, one processed after it goes to them through reconcile_locked.  No
  // window exists in which an event reaches only the outgoing tables.
  std::lock_guard<std::mutex> lk(mu_);
  fast_tables_ = std::move(tables);
  fast_recover_ = fast_recover;
  std::vector<char> down(state_.size(), 0);
  for (size_t g = 0; g < state_.size(); ++g) down[g] = running_ && !state_[g].reported_healthy;
  for (int g : held_unhealthy)
    if (g >= 0 && g < static_cast<int>(down.size())) down[g] = 1;
  for (size_t g = 0; g < down.size(); ++g)
    if (down[g])
      for (const auto& t : fast_tables_) t->set_gpu_health(static_cast<int>(g), -1, false);
}

void HealthMonitor::set_bad_page_thresholds(std::vector<int> thresholds) {
  std::lock_guard<std::mutex> lk(mu_);
  page_thresholds_ = std::move(thresholds);
}

void HealthMonitor::set_disabled_checks(int mask) {
  std::lock_guard<std::mutex> lk(mu_);
  disabled_ = mask & kCheckAll;
  for (size_t g = 0; g < state_.size(); ++g) reconcile_locked(static_cast<int>(g), kEvtNone, "health checks changed");
}

bool HealthMonitor::gpu_healthy(int gpu) const {
  std::lock_guard<std::mutex> lk(mu_);
  if (gpu < 0 || gpu >= static_cast<int>(state_.size())) return false;
  return state_[gpu].reported_healthy;
}

}  // namespace amdgpu_dp
