// Backend base: discovery and sampling over per-GPU lanes (lanes.h).
//
// The reference enumerates with NVML inline on the manager goroutine
// (plugin/manager.go:156-174 loadPlugins -> device/device_map.go:48-98) and rebuilds the
// NVLink graph inside GetPreferredAllocation (plugin/plugin.go:259-264); one hung NVML
// call there hangs the manager.  Here discover() enumerates without touching any single
// device, then describes every GPU on its own lane in parallel, each waited for at most
// the call bound.  A GPU that does not answer keeps its previous description and is
// reported stale; the caller is never held longer than one bound.
#include <algorithm>
#include <cstdio>
#include <stdexcept>

#include "backend.h"

namespace amdgpu_dp {

Backend::Backend() : inv_(std::make_shared<const Inventory>()) {}

std::shared_ptr<const Inventory> Backend::inventory() const {
  std::lock_guard<std::mutex> lk(inv_mu_);
  return inv_;
}

DiscoveryReport Backend::last_discovery() const {
  std::lock_guard<std::mutex> lk(inv_mu_);
  return report_;
}

std::string Backend::gpu_key(int gpu) const { return inventory()->key_of(gpu); }

int64_t Backend::last_completion_ns() const { return last_completion_ns_.load(); }

std::shared_ptr<LaneJob> Backend::post_job(const std::string& key, const char* what, uint64_t session,
                                       std::function<void()> fn, uint64_t batch) {
  // The closure keeps the backend alive, so the gate and the completion clock it touches
  // outlive a caller that stopped waiting - and a backend destroyed while a wedged call
  // (a lane thread the destructor detached) is still inside the library.  A
  // backend not owned by a shared_ptr (a stack object in a test) has no keep-alive.
  auto job = std::make_shared<LaneJob>(what, [this, self = weak_from_this().lock(), session, fn = std::move(fn)] {
    if (!gate_.enter(session)) return;  // handles of an older session: never use them
    struct Leave {  // also when fn throws (LaneJob::run catches it): a call left inside
      SessionGate& g;  // the gate for good would defer every re-initialisation
      ~Leave() { g.leave(); }
    } leave{gate_};
    fn();
    last_completion_ns_.store(mono_ns());
  }, batch);
  const int stall = stall_ms_.load();
  if (!lanes_.get(key)->post(job, static_cast<int64_t>(stall) * 1000000)) return nullptr;
  return job;
}

bool Backend::run_on_lane(const std::string& key, const char* what, uint64_t session, std::function<void()> fn,
                          int64_t ms) {
  auto job = post_job(key, what, session, std::move(fn));
  return job && job->wait(ms) && !job->dropped();
}

std::shared_ptr<LaneJob> Backend::sample_async(int gpu, std::shared_ptr<GpuSample> out, const std::string& key) {
  auto inv = inventory();
  if (!key.empty()) gpu = inv->index_of(key);
  if (gpu < 0 || gpu >= static_cast<int>(inv->refs.size())) return nullptr;
  out->key = inv->refs[gpu].key;
  auto self = shared_from_this();
  return post_job(inv->refs[gpu].key, "sample", inv->session, [self, inv, gpu, out] {
    out->ok = self->sample_device(*inv, gpu, out.get());
    for (int k = 0; k < out->num_links && k < kMaxXgmiLinks; ++k) out->link_peer_key[k] = inv->key_of(out->link_peer[k]);
  });
}

bool Backend::sample(int gpu, GpuSample* out) {
  auto s = std::make_shared<GpuSample>();
  auto job = sample_async(gpu, s);
  out->key = gpu_key(gpu);
  if (!job || !job->wait(call_timeout_ms_.load()) || job->dropped()) return false;
  *out = *s;
  return out->ok;
}

std::vector<LaneReport> Backend::lanes() const {
  auto inv = inventory();
  std::vector<LaneState> states = lanes_.states();
  std::vector<LaneReport> out(inv->refs.size());
  for (size_t i = 0; i < inv->refs.size(); ++i) {
    out[i].index = static_cast<int>(i);
    out[i].lane.key = inv->refs[i].key;
  }
  for (auto& st : states) {
    const int i = inv->index_of(st.key);
    if (i >= 0) {
      out[i].lane = std::move(st);
    } else if (st.inflight_since_ns != 0) {  // a GPU that left the inventory mid-call
      LaneReport r;
      r.lane = std::move(st);
      out.push_back(std::move(r));
    }
  }
  return out;
}

namespace {
std::string secs(int64_t ns) {
  char b[32];
  std::snprintf(b, sizeof(b), "%.1f s", ns * 1e-9);
  return b;
}
}  // namespace

void Backend::discover(std::vector<GpuInfo>* gpus, Topology* topo) {
  {
    std::unique_lock<std::mutex> lk(discover_mu_);
    if (!cv_wait_ms(discover_cv_, lk, call_timeout_ms_.load(), [&] { return !discovering_; }))
      throw std::runtime_error("another discovery has been running for longer than the call bound");
    discovering_ = true;
  }
  struct Done {
    Backend* b;
    ~Done() {
      {
        std::lock_guard<std::mutex> lk(b->discover_mu_);
        b->discovering_ = false;
      }
      b->discover_cv_.notify_all();
    }
  } done{this};
  const int64_t t0 = mono_ns();
  DiscoveryReport rep;
  auto self = shared_from_this();
  struct Out {
    GpuInfo info;
    std::vector<Link> row;
    std::string error;
    bool ok = false;
  };
  std::vector<DeviceRef> refs;
  std::vector<std::shared_ptr<Out>> outs;
  std::vector<std::shared_ptr<LaneJob>> jobs;
  uint64_t session = 0;
  for (int attempt = 0;; ++attempt) {
    refs.clear();
    outs.clear();
    jobs.clear();
    session = gate_.session();
    enumerate(&refs);  // throws: nothing installed, the previous inventory stays
    auto all = std::make_shared<const std::vector<DeviceRef>>(refs);
    const uint64_t batch = next_batch();  // posted to every lane at once
    for (size_t i = 0; i < refs.size(); ++i) {
      auto out = std::make_shared<Out>();
      outs.push_back(out);
      jobs.push_back(post_job(refs[i].key, "describe", session, [self, all, i, out] {
        try {
          self->describe((*all)[i], *all, &out->info, &out->row);
          out->ok = !out->info.partitions.empty();
          if (!out->ok) out->error = "no partitions described";
        } catch (const std::exception& e) {
          out->error = e.what();
        }
      }, batch));
    }
    const int64_t deadline = mono_ns() + static_cast<int64_t>(call_timeout_ms_.load()) * 1000000;
    for (auto& j : jobs)
      if (j) j->wait(std::max<int64_t>(0, (deadline - mono_ns()) / 1000000));
    if (attempt > 0) break;
    std::vector<GpuInfo> fresh;
    for (size_t i = 0; i < jobs.size(); ++i)
      if (jobs[i] && jobs[i]->done() && !jobs[i]->dropped() && outs[i]->ok) fresh.push_back(outs[i]->info);
    if (!handles_stale(fresh)) break;
    // A call still inside the library (a wedged GPU) keeps it from being re-initialised:
    // describe with the handles there are and try again at the next discovery.
    if (!gate_.close(call_timeout_ms_.load())) {
      rep.reinit_deferred = true;
      break;
    }
    bool ok = false;
    try {
      ok = reopen_session();
    } catch (...) {
      gate_.reopen();
      throw;
    }
    gate_.reopen();
    if (!ok) break;
  }

  // Collect: fresh descriptions, else the last ones that reached this GPU, else leave it out.
  const int64_t now = mono_ns();
  std::vector<int> kept;                       // positions in refs
  std::vector<const Described*> desc;          // per kept GPU (map nodes do not move)
  for (size_t i = 0; i < refs.size(); ++i) {
    const std::string& key = refs[i].key;
    const bool done = jobs[i] && jobs[i]->done() && !jobs[i]->dropped();
    if (done && outs[i]->ok) {
      Described d;
      d.info = outs[i]->info;
      for (size_t p = 0; p < refs.size() && p < outs[i]->row.size(); ++p) d.links[refs[p].key] = outs[i]->row[p];
      last_described_[key] = std::move(d);
      kept.push_back(static_cast<int>(i));
      desc.push_back(&last_described_[key]);
      continue;
    }
    std::string why;
    if (!jobs[i]) {
      auto lane = lanes_.find(key);
      const LaneState st = lane ? lane->state() : LaneState{};
      why = st.inflight_since_ns ? st.inflight_what + " call in flight for " + secs(now - st.inflight_since_ns)
                                 : std::string("lane refused the call");
    } else if (!jobs[i]->done()) {
      why = "no answer within " + std::to_string(call_timeout_ms_.load()) + " ms";
    } else if (jobs[i]->dropped()) {
      why = "call dropped";
    } else {
      why = outs[i]->error.empty() ? std::string("description failed") : outs[i]->error;
    }
    DiscoveryReport::Stale s;
    s.key = key;
    s.reason = why;
    auto it = last_described_.find(key);
    if (it != last_described_.end()) {
      s.index = static_cast<int>(kept.size());
      kept.push_back(static_cast<int>(i));
      desc.push_back(&it->second);
    }
    rep.stale.push_back(std::move(s));
  }
  // forget GPUs enumeration no longer lists
  for (auto it = last_described_.begin(); it != last_described_.end();) {
    const bool listed = std::any_of(refs.begin(), refs.end(), [&](const DeviceRef& r) { return r.key == it->first; });
    it = listed ? std::next(it) : last_described_.erase(it);
  }

  auto inv = std::make_shared<Inventory>();
  inv->gen = ++gen_;
  inv->session = session;
  const int n = static_cast<int>(kept.size());
  for (int k = 0; k < n; ++k) {
    inv->refs.push_back(refs[kept[k]]);
    GpuInfo g = desc[k]->info;
    g.index = k;
    g.key = refs[kept[k]].key;
    for (auto& p : g.partitions) p.gpu = k;
    inv->gpus.push_back(std::move(g));
  }
  topo->resize(n);
  for (int a = 0; a < n; ++a) {
    for (int b = 0; b < n; ++b) {
      if (a == b) continue;
      const auto& la = desc[a]->links;
      const auto& lb = desc[b]->links;
      auto ia = la.find(inv->refs[b].key);
      auto ib = lb.find(inv->refs[a].key);
      Link l = ia != la.end() ? ia->second : (ib != lb.end() ? ib->second : Link{});
      // a link is up only if both ends see it up; it runs at the slower end's rate
      if (ia != la.end() && ib != lb.end()) {
        l.up = ia->second.up && ib->second.up;
        const double x = ia->second.bw_gbps, y = ib->second.bw_gbps;
        l.bw_gbps = x > 0 && y > 0 ? std::min(x, y) : std::max(x, y);
      }
      topo->at(a, b) = l;
    }
  }
  for (auto& s : rep.stale)
    if (s.index >= 0) s.index = inv->index_of(s.key);
  rep.gen = inv->gen;
  rep.seconds = (mono_ns() - t0) * 1e-9;
  *gpus = inv->gpus;
  std::shared_ptr<const Inventory> published = inv;
  {
    std::lock_guard<std::mutex> lk(inv_mu_);
    inv_ = published;
    report_ = rep;
  }
  std::vector<std::string> keep;
  for (const auto& r : refs) keep.push_back(r.key);
  lanes_.prune(keep);
  installed(published);
}

}  // namespace amdgpu_dp
