#include "health.h"

#include <time.h>

#include <cstdio>

#include <algorithm>
#include <chrono>
#include <cmath>

namespace amdgpu_dp {

HealthMonitor::HealthMonitor(std::shared_ptr<Backend> backend, int lost_after_failures)
    : backend_(std::move(backend)), lost_after_(lost_after_failures) {}

HealthMonitor::~HealthMonitor() { stop(); }

std::string HealthMonitor::key_of(int gpu, const std::string& given) const {
  if (!given.empty()) return given;
  if (gpu < 0) return "";
  // The backend names the GPU at `gpu` in its current enumeration; "" means there is none
  // (an index from before a re-discovery that dropped a GPU), and nothing is recorded for
  // it.  Only a monitor without a backend numbers GPUs itself.
  if (!backend_) return "#" + std::to_string(gpu);
  return backend_->gpu_key(gpu);
}

int HealthMonitor::table_index_locked(const std::string& key) const {
  if (key.empty()) return -1;
  for (size_t i = 0; i < table_keys_.size(); ++i)
    if (table_keys_[i] == key) return static_cast<int>(i);
  return -1;
}

void HealthMonitor::set_gpus(std::vector<std::string> keys) {
  // Called on every plugin (re)load.  State is never dropped here: a GPU that is
  // mid-reset when kubelet restarts, or that fell off the bus and is coming back, keeps
  // its latches; its POST_RESET (or recovery) still produces the Healthy update.
  std::lock_guard<std::mutex> lk(mu_);
  table_keys_ = std::move(keys);
  for (const auto& k : table_keys_)
    if (!k.empty()) state_[k];
}

void HealthMonitor::set_gpu_count(int n) {
  std::vector<std::string> keys;
  for (int i = 0; i < n; ++i) keys.push_back(key_of(i, ""));
  set_gpus(std::move(keys));
}

void HealthMonitor::start() {
  auto armed = std::make_shared<ThreadExitFlag>();
  {
    std::lock_guard<std::mutex> lk(mu_);
    if (running_) return;
    stop_ = false;
    running_ = true;
    // arming talks to every GPU (on their lanes, bounded): the event thread does it, so
    // nothing that needs mu_ waits on a wedged GPU
    thread_ = std::thread([this, armed] {
      background_thread("dpevents");
      backend_->arm_events();
      armed->set();
      loop();
    });
  }
  // the caller reads armed_event_sources() next: give arming a short, bounded wait
  armed->wait(std::min(2000, backend_->call_timeout_ms()));
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
    if (!backend_->delivers_events()) {
      // nothing armed (an unprivileged pod): health runs on polling; sleep until stop() or
      // 5 s have passed (arming may happen later, after a re-initialisation)
      std::unique_lock<std::mutex> lk(mu_);
      cv_wait_ms(cv_, lk, 5000, [&] { return stop_; });
      continue;
    }
    // bounded wait so stop() is honoured: 200 ms, a second for
    // amdsmi (an idle node then pays one wake-up a second for event delivery)
    backend_->wait_events(backend_->event_wait_ms(), &evs);
    for (const auto& e : evs) process(e);
  }
}

void HealthMonitor::emit_locked(HealthUpdate u) {
  if (u.ts_ns == 0) u.ts_ns = now_ns();
  queue_.push_back(std::move(u));
  cv_.notify_all();
}

namespace {
std::pair<std::string, std::string> link_of(const std::string& a, const std::string& b) {
  return a < b ? std::make_pair(a, b) : std::make_pair(b, a);
}

int check_of(int kind) {
  switch (kind) {
    case kEvtPreReset:
    case kEvtPostReset:
    case kEvtResetObserved: return kCheckReset;
    case kEvtEccUncorrectable: return kCheckEcc;
    case kEvtDeviceLost:
    case kEvtDeviceRecovered: return kCheckLost;
    case kEvtRetiredPagesExceeded:
    case kEvtRetiredPagesCleared: return kCheckRetiredPages;
    case kEvtPcieDegraded:
    case kEvtPcieRestored: return kCheckPcie;
    default: return 0;
  }
}
}  // namespace

bool HealthMonitor::healthy_locked(const GpuState& st) const {
  return !(st.resetting && !(disabled_ & kCheckReset)) && !(st.ecc_bad && !(disabled_ & kCheckEcc)) &&
         !(st.lost && !(disabled_ & kCheckLost)) && !(st.pages_bad && !(disabled_ & kCheckRetiredPages)) &&
         !(st.pcie_bad && !(disabled_ & kCheckPcie));
}

void HealthMonitor::reconcile_locked(const std::string& key, int kind, const std::string& reason,
                                     bool latch_changed) {
  GpuState& st = state_[key];
  const int idx = table_index_locked(key);
  const bool healthy = healthy_locked(st);
  if (healthy == st.reported_healthy) {
    // tracked, not acted on (check disabled), or a persisted latch that moved without a
    // health transition (a UE on a GPU already Unhealthy for another reason): the manager
    // still hears of it, logs it and persists the latch
    if ((disabled_ & check_of(kind)) || latch_changed) {
      HealthUpdate u;
      u.kind = kind;
      u.gpu = idx;
      u.key = key;
      u.reason = reason + ((disabled_ & check_of(kind)) ? " (health check disabled)" : " (latched)");
      emit_locked(std::move(u));
    }
    return;
  }
  st.reported_healthy = healthy;
  if (idx >= 0 && !healthy)
    for (const auto& t : fast_tables_) t->set_gpu_health(idx, -1, false);
  else if (idx >= 0 && fast_recover_)
    write_healthy_locked(idx, key);
  HealthUpdate u;
  u.kind = kind;
  u.gpu = idx;
  u.key = key;
  u.healthy = healthy ? 1 : 0;
  u.reason = reason;
  emit_locked(std::move(u));
}

void HealthMonitor::write_healthy_locked(int idx, const std::string& key) {
  const auto it = held_parts_.find(key);
  if (it == held_parts_.end() || it->second.empty()) {
    for (const auto& t : fast_tables_) t->set_gpu_health(idx, -1, true);
    return;
  }
  if (std::find(it->second.begin(), it->second.end(), -1) != it->second.end()) return;  // the whole GPU is held
  for (const auto& t : fast_tables_) t->set_gpu_health_except(idx, it->second);
}

void HealthMonitor::process(const HwEvent& e) {
  // identities first, outside mu_ (the backend answers them from its own small lock)
  const std::string key = key_of(e.gpu, e.key);
  const std::string peer_key = key_of(e.peer, e.peer_key);
  std::lock_guard<std::mutex> lk(mu_);
  ++events_seen_;
  const std::string why = std::string(event_kind_name(e.kind)) + (e.message.empty() ? "" : ": " + e.message);
  const bool known = !key.empty();
  switch (e.kind) {
    case kEvtPreReset:
      if (!known) return;
      state_[key].resetting = true;
      reconcile_locked(key, e.kind, why);
      return;
    case kEvtPostReset:
    case kEvtResetObserved: {
      if (!known) return;
      GpuState& st = state_[key];
      const bool had_latch = st.ecc_bad;
      st.resetting = false;
      st.ecc_bad = false;  // a reset clears the uncorrectable-error latch
      st.restored = false;
      st.candidate = false;
      st.ecc_reason.clear();
      // POST_RESET arrives on its own: re-baseline on the next sample.  A reset observed
      // by polling comes from the sample that already took the new baseline.
      if (e.kind == kEvtPostReset) st.last_ue = -1;
      if (e.kind == kEvtResetObserved) ++resets_observed_;
      reconcile_locked(key, e.kind, why, had_latch);
      return;
    }
    case kEvtEccUncorrectable: {
      if (!known) return;
      GpuState& st = state_[key];
      const bool fresh = !st.ecc_bad;
      if (fresh) {
        st.ecc_reason = why;
        st.ecc_since_ns = now_ns();
      }
      st.ecc_bad = true;
      reconcile_locked(key, e.kind, why, fresh);
      return;
    }
    case kEvtDeviceLost:
      if (!known) return;
      state_[key].lost = true;
      reconcile_locked(key, e.kind, why);
      return;
    case kEvtDeviceRecovered: {
      if (!known) return;
      GpuState& st = state_[key];
      st.lost = false;
      st.lost_failing = false;
      st.failures = 0;
      reconcile_locked(key, e.kind, why);
      return;
    }
    case kEvtRetiredPagesExceeded:
    case kEvtRetiredPagesCleared:
      if (!known) return;
      state_[key].pages_bad = e.kind == kEvtRetiredPagesExceeded;
      reconcile_locked(key, e.kind, why);
      return;
    case kEvtPcieDegraded:
    case kEvtPcieRestored:
      if (!known) return;
      state_[key].pcie_bad = e.kind == kEvtPcieDegraded;
      reconcile_locked(key, e.kind, why);
      return;
    case kEvtLinkDown:
    case kEvtLinkUp: {
      if (!known || peer_key.empty()) return;
      const int up = e.kind == kEvtLinkUp ? 1 : 0;
      auto& m = state_[key].link_up;
      auto it = m.find(peer_key);
      uint64_t& ep = up_epoch_[link_of(key, peer_key)];
      if (it != m.end() && it->second == up && ep == links_epoch_) return;  // already known (polling + event)
      ep = links_epoch_;
      m[peer_key] = up;
      state_[peer_key].link_up[key] = up;
      HealthUpdate u;
      u.kind = e.kind;
      u.gpu = table_index_locked(key);
      u.key = key;
      u.peer = table_index_locked(peer_key);
      u.peer_key = peer_key;
      u.link_up = up;
      u.reason = why;
      emit_locked(std::move(u));
      return;
    }
    case kEvtLinkQuality: {
      // e.value: the link's bandwidth now (the slower end's view); one update per pair
      if (!known || peer_key.empty() || e.value <= 0) return;
      const auto pk = link_of(key, peer_key);
      auto it = pair_bw_.find(pk);
      uint64_t& ep = bw_epoch_[pk];
      if (it != pair_bw_.end() && std::fabs(it->second - e.value) <= 0.05 * std::max(it->second, e.value) &&
          ep == links_epoch_)
        return;
      ep = links_epoch_;
      pair_bw_[pk] = e.value;
      HealthUpdate u;
      u.kind = e.kind;
      u.gpu = table_index_locked(key);
      u.key = key;
      u.peer = table_index_locked(peer_key);
      u.peer_key = peer_key;
      u.link_gbps = e.value;
      u.reason = why;
      emit_locked(std::move(u));
      return;
    }
    default: {
      HealthUpdate u;  // informational (thermal, vm fault)
      u.kind = e.kind;
      u.gpu = table_index_locked(key);
      u.key = key;
      u.partition = e.partition;
      u.reason = why;
      emit_locked(std::move(u));
    }
  }
}

void HealthMonitor::on_sample(int gpu, bool ok, const GpuSample& s) {
  if (gpu < 0) return;
  // The sample names the GPU it read (backends fill s.key under the lock that also
  // guards their enumeration), so a re-discovery between the read and this call cannot
  // attribute one GPU's counters to another.
  const std::string key = key_of(gpu, s.key);
  if (key.empty()) return;  // no GPU at that index any more: its health is nobody's
  std::vector<std::string> peer_keys(static_cast<size_t>(std::max(0, s.num_links)));
  if (ok)
    for (int k = 0; k < s.num_links; ++k)
      if (s.link_peer[k] >= 0)
        peer_keys[k] = !s.link_peer_key[k].empty() ? s.link_peer_key[k] : key_of(s.link_peer[k], "");
  std::vector<HwEvent> derived;
  {
    std::lock_guard<std::mutex> lk(mu_);
    GpuState& st = state_[key];
    auto event = [&](int kind, std::string msg) {
      HwEvent e;
      e.kind = kind;
      e.gpu = gpu;
      e.key = key;
      e.message = std::move(msg);
      return e;
    };
    if (!ok) {
      if (++st.failures >= lost_after_ && !st.lost) {
        st.lost_failing = true;
        derived.push_back(event(kEvtDeviceLost, "telemetry failed " + std::to_string(st.failures) + " times in a row"));
      }
    } else {
      st.failures = 0;
      // back from an outage of failed samples (a driver refuses calls while it resets the
      // GPU); a call that merely hung and returned is not one
      const bool outage = st.lost && st.lost_failing;
      if (st.lost) derived.push_back(event(kEvtDeviceRecovered, "telemetry responding again"));
      // Resets seen without event delivery (an unprivileged pod cannot arm amdsmi events),
      // strongest evidence first.
      std::string reset_why;
      const double now_b = boottime_s();
      char msg[240];
      // 1. The kernel's own reset counter (amdgpu context query on the render node): every
      //    reset the driver performs moves it, also those that keep the firmware running.
      if (s.reset_count >= 0) {
        if (st.reset_count >= 0 && s.reset_count > st.reset_count) {
          std::snprintf(msg, sizeof(msg), "the kernel reports %lld GPU reset(s) (amdgpu context query)",
                        static_cast<long long>(s.reset_count - st.reset_count));
          reset_why = msg;
        }
        st.reset_count = s.reset_count;
      }
      // 2. The power-management firmware's clock starting again (a reset that reloads the
      //    firmware).  A step back counts only if the new reading is no larger than the
      //    time since the previous one (the firmware started after it), and only once the
      //    new clock is seen ticking at about 1 s/s - for one interval after a clock this
      //    process saw ticking for two, for two intervals otherwise: a frozen, garbage or
      //    one-off reading never clears a latch.
      bool jump_dropped = false;
      bool too_close = false;
      if (s.fw_clock_s >= 0) {
        const double fw_boot = now_b - s.fw_clock_s;
        if (st.fw_clock >= 0 && s.fw_clock_s + 1.0 < st.fw_clock) {
          const double since = now_b - st.fw_read_at;
          if (s.fw_clock_s <= since + 5.0) {
            std::snprintf(msg, sizeof(msg), "firmware clock restarted (%.1f s -> %.1f s)", st.fw_clock, s.fw_clock_s);
            st.fw_jump_pending = true;
            st.fw_jump_confirms = st.fw_adv_n >= 2 ? 1 : 2;
            st.fw_jump_why = msg;
          } else {
            ++fw_glitches_;
            jump_dropped = st.fw_jump_pending;
            st.fw_jump_pending = false;
          }
          st.fw_adv_n = 0;
          st.fw_advancing = false;
        } else if (st.fw_clock >= 0) {
          const double dt = now_b - st.fw_read_at, dc = s.fw_clock_s - st.fw_clock;
          // two readings closer than 20 ms say nothing about the rate: this one is skipped
          // and the next is compared with the previous one (never with an unjudged reading)
          too_close = dt < 0.02;
          if (!too_close) {
            if (dc > 0 && dc / dt > 0.5 && dc / dt < 2.0) {
              ++st.fw_adv_n;
              st.fw_advancing = true;
              if (st.fw_jump_pending && --st.fw_jump_confirms <= 0) {
                if (reset_why.empty()) reset_why = st.fw_jump_why;
                st.fw_jump_pending = false;
              }
            } else {
              st.fw_adv_n = 0;
              st.fw_advancing = false;
              if (st.fw_jump_pending) {
                ++fw_glitches_;
                jump_dropped = true;
                st.fw_jump_pending = false;
              }
            }
          }
        }
        if (!too_close) {
          st.fw_clock = s.fw_clock_s;
          st.fw_read_at = now_b;
        }
        if (st.fw_advancing) st.fw_boot = fw_boot;
        // a latch from a previous process: did the firmware start after it was recorded?
        // Judged once this process has seen the clock tick (a frozen clock never is).
        if (!std::isnan(st.restored_fw_boot) && st.fw_adv_n >= 2) {
          const double tol = std::max(30.0, 1e-4 * std::max(0.0, now_b - st.restored_fw_boot));
          if (fw_boot > st.restored_fw_boot + tol && reset_why.empty()) {
            std::snprintf(msg, sizeof(msg), "firmware restarted while the plugin was not running (%.0f s after the "
                          "start recorded with the latch)", fw_boot - st.restored_fw_boot);
            reset_why = msg;
          }
          st.restored_fw_boot = std::numeric_limits<double>::quiet_NaN();
        }
      } else {
        st.restored_fw_boot = std::numeric_limits<double>::quiet_NaN();  // nothing to compare it with
        st.fw_jump_pending = false;
      }
      // 3. Back from an outage with nothing above confirming a reset: a reset only if the
      //    uncorrectable-ECC counter restarted below the latched baseline; otherwise a
      //    candidate - the latches hold and the manager re-verifies the GPU (recovery
      //    canary) or an operator clears it (GET /health/clear).  An outage alone is also
      //    what an amdsmi re-init, a busy driver or a library error look like.
      const bool undecided = outage || (jump_dropped && st.outage_unresolved);
      if (!reset_why.empty() || !undecided) {
        if (!reset_why.empty()) st.outage_unresolved = false;
      } else if (st.fw_jump_pending) {
        st.outage_unresolved = true;  // the next reading decides (a confirmed restart, or a candidate)
      } else {
        st.outage_unresolved = false;
        if (s.ecc_uncorrectable >= 0 && st.last_ue > 0 && s.ecc_uncorrectable < st.last_ue) {
          std::snprintf(msg, sizeof(msg), "telemetry back after an outage with the uncorrectable ECC count reset "
                        "(%lld -> %lld)", static_cast<long long>(st.last_ue),
                        static_cast<long long>(s.ecc_uncorrectable));
          reset_why = msg;
        } else if ((st.ecc_bad || st.resetting) && !st.candidate) {
          st.candidate = true;
          ++reset_candidates_;
          derived.push_back(event(kEvtResetCandidate,
                                  "telemetry back after an outage of failed samples, no reset confirmed (no kernel "
                                  "reset count, no firmware clock restart)"));
        }
      }
      if (!reset_why.empty()) {
        derived.push_back(event(kEvtResetObserved, reset_why));
        st.last_ue = -1;  // counters after a reset start a new baseline (taken just below)
      }
      if (s.ecc_uncorrectable >= 0) {
        if (st.last_ue >= 0 && s.ecc_uncorrectable > st.last_ue)
          derived.push_back(event(kEvtEccUncorrectable, "uncorrectable ECC count " + std::to_string(st.last_ue) +
                                                            " -> " + std::to_string(s.ecc_uncorrectable)));
        st.last_ue = s.ecc_uncorrectable;
      }
      if (pcie_min_width_ > 0 || pcie_min_gts_ > 0) {
        const bool narrow = pcie_min_width_ > 0 && s.pcie_link_width > 0 && s.pcie_link_width < pcie_min_width_;
        const bool slow = pcie_min_gts_ > 0 && s.pcie_link_speed_gtps > 0 && s.pcie_link_speed_gtps < pcie_min_gts_;
        if (narrow || slow) {
          st.pcie_ok = 0;
          ++st.pcie_low;
        } else {
          st.pcie_low = 0;
          ++st.pcie_ok;
        }
        const bool settled = (narrow || slow) ? st.pcie_low >= pcie_debounce_ : st.pcie_ok >= pcie_debounce_;
        if (settled && (narrow || slow) != st.pcie_bad) {
          char msg[160];
          std::snprintf(msg, sizeof(msg), "host PCIe link x%d at %.1f GT/s (floor x%d, %.1f GT/s)",
                        static_cast<int>(s.pcie_link_width), s.pcie_link_speed_gtps, pcie_min_width_, pcie_min_gts_);
          derived.push_back(event(narrow || slow ? kEvtPcieDegraded : kEvtPcieRestored, msg));
        }
      }
      const int thr = st.page_threshold;
      if (s.retired_pages >= 0) {
        const int64_t bad = s.retired_pages + std::max<int64_t>(0, s.pending_pages);
        const bool over = thr > 0 && bad >= thr;
        if (over != st.pages_bad)
          derived.push_back(event(over ? kEvtRetiredPagesExceeded : kEvtRetiredPagesCleared,
                                  std::to_string(bad) + " retired/pending HBM pages, threshold " + std::to_string(thr)));
      }
      for (int k = 0; k < s.num_links; ++k) {
        if (s.link_peer[k] < 0 || s.link_up[k] < 0 || peer_keys[k].empty()) continue;
        const auto pk = link_of(key, peer_keys[k]);
        auto it = st.link_up.find(peer_keys[k]);
        const int prev = it == st.link_up.end() ? 1 : it->second;  // links assumed up at start
        const auto ue = up_epoch_.find(pk);
        if (prev != s.link_up[k] || ue == up_epoch_.end() || ue->second != links_epoch_) {
          HwEvent e = event(s.link_up[k] ? kEvtLinkUp : kEvtLinkDown, "xgmi link status poll");
          e.peer = s.link_peer[k];
          e.peer_key = peer_keys[k];
          derived.push_back(e);
        }
        // Trained bandwidth, as this end sees it.  A link runs at the slower of its two
        // ends' views: the pair's value is reported when it is first known (the link may
        // have re-trained between discovery and this sample; the manager applies it only
        // where the tables disagree) and whenever it moves by more than 5 %.
        const double bw = s.link_trained_gbps[k];
        if (s.link_up[k] == 1 && bw > 0) {
          st.link_bw[peer_keys[k]] = bw;
          const auto pt = state_.find(peer_keys[k]);
          double eff = bw;
          if (pt != state_.end()) {
            const auto pv = pt->second.link_bw.find(key);
            if (pv != pt->second.link_bw.end()) eff = std::min(eff, pv->second);
          }
          const auto last = pair_bw_.find(pk);
          const auto be = bw_epoch_.find(pk);
          if (last == pair_bw_.end() || std::fabs(last->second - eff) > 0.05 * std::max(last->second, eff) ||
              be == bw_epoch_.end() || be->second != links_epoch_) {
            const bool moved =
                last != pair_bw_.end() && std::fabs(last->second - eff) > 0.05 * std::max(last->second, eff);
            HwEvent e = event(kEvtLinkQuality,
                              !moved
                                  ? "xgmi link bandwidth: " + std::to_string(static_cast<int>(eff)) + " Gb/s"
                                  : "xgmi link re-trained: " + std::to_string(static_cast<int>(last->second)) + " -> " +
                                        std::to_string(static_cast<int>(eff)) + " Gb/s");
            e.peer = s.link_peer[k];
            e.peer_key = peer_keys[k];
            e.value = eff;
            derived.push_back(e);
          }
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
  ++links_epoch_;  // the new tables hold discovery's view of the links: report each link once more
  std::vector<char> down(table_keys_.size(), 0);
  for (size_t g = 0; g < table_keys_.size(); ++g) {
    if (table_keys_[g].empty()) continue;
    auto it = state_.find(table_keys_[g]);
    // (a restored latch holds before the monitor runs: it came from a previous process)
    down[g] = it != state_.end() && !it->second.reported_healthy && (running_ || it->second.restored);
  }
  for (int g : held_unhealthy)
    if (g >= 0 && g < static_cast<int>(down.size())) down[g] = 1;
  for (size_t g = 0; g < down.size(); ++g)
    if (down[g])
      for (const auto& t : fast_tables_) t->set_gpu_health(static_cast<int>(g), -1, false);
  // partitions the manager holds (canary verdicts) start Unhealthy in the new tables too
  for (size_t g = 0; g < table_keys_.size(); ++g) {
    const auto it = held_parts_.find(table_keys_[g]);
    if (table_keys_[g].empty() || it == held_parts_.end()) continue;
    for (int part : it->second)
      for (const auto& t : fast_tables_) t->set_gpu_health(static_cast<int>(g), part, false);
  }
}

void HealthMonitor::set_bad_page_thresholds(std::vector<int> thresholds) {
  std::lock_guard<std::mutex> lk(mu_);
  for (size_t g = 0; g < thresholds.size() && g < table_keys_.size(); ++g)
    if (!table_keys_[g].empty()) state_[table_keys_[g]].page_threshold = thresholds[g];
}

void HealthMonitor::set_pcie_floor(int min_width, double min_gts, int debounce) {
  std::lock_guard<std::mutex> lk(mu_);
  pcie_min_width_ = std::max(0, min_width);
  pcie_min_gts_ = std::max(0.0, min_gts);
  pcie_debounce_ = std::max(1, debounce);
  if (pcie_min_width_ > 0 || pcie_min_gts_ > 0) return;  // the next samples re-judge every GPU
  std::vector<std::string> keys;  // no floor any more: nothing is held for its link
  for (auto& kv : state_)
    if (kv.second.pcie_bad) {
      kv.second.pcie_bad = false;
      keys.push_back(kv.first);
    }
  std::sort(keys.begin(), keys.end());
  for (const auto& k : keys) reconcile_locked(k, kEvtPcieRestored, "PCIe link floor removed");
}

void HealthMonitor::set_disabled_checks(int mask) {
  std::lock_guard<std::mutex> lk(mu_);
  disabled_ = mask & kCheckAll;
  std::vector<std::string> keys;
  for (const auto& kv : state_) keys.push_back(kv.first);
  std::sort(keys.begin(), keys.end());  // deterministic update order
  for (const auto& k : keys) reconcile_locked(k, kEvtNone, "health checks changed");
}

bool HealthMonitor::gpu_healthy(int gpu) const {
  std::lock_guard<std::mutex> lk(mu_);
  if (gpu < 0 || gpu >= static_cast<int>(table_keys_.size()) || table_keys_[gpu].empty()) return false;
  auto it = state_.find(table_keys_[gpu]);
  return it == state_.end() || it->second.reported_healthy;
}

std::vector<std::string> HealthMonitor::unhealthy_keys() const {
  std::lock_guard<std::mutex> lk(mu_);
  std::vector<std::string> out;
  for (const auto& kv : state_)
    if (!kv.second.reported_healthy) out.push_back(kv.first);
  std::sort(out.begin(), out.end());
  return out;
}

std::vector<HealthLatch> HealthMonitor::latches() const {
  std::lock_guard<std::mutex> lk(mu_);
  std::vector<HealthLatch> out;
  for (const auto& kv : state_) {
    const GpuState& st = kv.second;
    if (!st.ecc_bad) continue;
    HealthLatch l;
    l.key = kv.first;
    l.ecc_bad = true;
    l.last_ue = st.last_ue;
    l.fw_boot_s = !std::isnan(st.fw_boot) ? st.fw_boot : st.restored_fw_boot;
    l.reason = st.ecc_reason;
    l.since_ns = st.ecc_since_ns;
    out.push_back(std::move(l));
  }
  std::sort(out.begin(), out.end(), [](const HealthLatch& a, const HealthLatch& b) { return a.key < b.key; });
  return out;
}

void HealthMonitor::restore_latches(const std::vector<HealthLatch>& latches) {
  std::lock_guard<std::mutex> lk(mu_);
  for (const auto& l : latches) {
    if (l.key.empty() || !l.ecc_bad) continue;
    GpuState& st = state_[l.key];
    if (st.ecc_bad) continue;  // this process has its own verdict already
    st.ecc_bad = true;
    st.restored = true;
    st.last_ue = l.last_ue;
    st.ecc_reason = l.reason;
    st.ecc_since_ns = l.since_ns;
    st.restored_fw_boot = l.fw_boot_s;
    st.fw_boot = l.fw_boot_s;
    reconcile_locked(l.key, kEvtEccUncorrectable,
                     "uncorrectable ECC latch restored from the previous plugin process" +
                         (l.reason.empty() ? std::string() : " (" + l.reason + ")"));
  }
}

uint64_t HealthMonitor::resets_observed() const {
  std::lock_guard<std::mutex> lk(mu_);
  return resets_observed_;
}

uint64_t HealthMonitor::reset_candidates() const {
  std::lock_guard<std::mutex> lk(mu_);
  return reset_candidates_;
}

uint64_t HealthMonitor::fw_clock_glitches() const {
  std::lock_guard<std::mutex> lk(mu_);
  return fw_glitches_;
}

std::vector<std::string> HealthMonitor::clear_latches(const std::string& key, const std::string& reason) {
  std::lock_guard<std::mutex> lk(mu_);
  std::vector<std::string> out;
  auto it = state_.find(key);
  if (key.empty() || it == state_.end()) return out;
  GpuState& st = it->second;
  if (st.ecc_bad) out.push_back("uncorrectable_ecc");
  if (st.resetting) out.push_back("reset_in_progress");
  st.ecc_bad = false;
  st.resetting = false;
  st.restored = false;
  st.candidate = false;
  st.ecc_reason.clear();
  st.restored_fw_boot = std::numeric_limits<double>::quiet_NaN();
  st.last_ue = -1;  // the next sample takes a new baseline
  if (!out.empty()) {
    std::string what;
    for (const auto& w : out) what += (what.empty() ? "" : ", ") + w;
    reconcile_locked(key, kEvtLatchCleared, reason + " (cleared: " + what + ")", true);
  }
  return out;
}

bool HealthMonitor::settling() const {
  std::lock_guard<std::mutex> lk(mu_);
  for (const auto& kv : state_) {
    const GpuState& st = kv.second;
    if (st.failures > 0 || st.lost || st.resetting || st.fw_jump_pending || st.candidate || st.outage_unresolved ||
        st.pcie_low > 0 || (st.pcie_bad && st.pcie_ok > 0))
      return true;
  }
  return false;
}

std::vector<std::string> HealthMonitor::holds(const std::string& key) const {
  std::lock_guard<std::mutex> lk(mu_);
  std::vector<std::string> out;
  auto it = state_.find(key);
  if (it == state_.end()) return out;
  const GpuState& st = it->second;
  if (st.resetting) out.push_back("reset_in_progress");
  if (st.ecc_bad) out.push_back("uncorrectable_ecc");
  if (st.lost) out.push_back("telemetry_lost");
  if (st.pages_bad) out.push_back("retired_pages");
  if (st.pcie_bad) out.push_back("pcie_link");
  return out;
}

void HealthMonitor::set_held_partitions(std::map<std::string, std::vector<int>> held) {
  std::lock_guard<std::mutex> lk(mu_);
  held_parts_ = std::move(held);
}

double boottime_s() {
  struct timespec ts;
  clock_gettime(CLOCK_BOOTTIME, &ts);
  return static_cast<double>(ts.tv_sec) + ts.tv_nsec * 1e-9;
}

}  // namespace amdgpu_dp
