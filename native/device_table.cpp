#include "device_table.h"

#include <algorithm>
#include <mutex>

#include "pbwire.h"

namespace amdgpu_dp {

const char* rpc_name(int rpc) {
  switch (rpc) {
    case kRpcOptions: return "GetDevicePluginOptions";
    case kRpcListAndWatch: return "ListAndWatch";
    case kRpcPreferred: return "GetPreferredAllocation";
    case kRpcAllocate: return "Allocate";
    case kRpcPreStart: return "PreStartContainer";
    default: return "unknown";
  }
}

namespace {
std::string map_entry(std::string_view k, std::string_view v) {
  std::string e;
  pb::put_bytes(&e, 1, k);
  pb::put_bytes(&e, 2, v);
  return e;
}
std::string device_spec(std::string_view container, std::string_view host, std::string_view perms) {
  std::string s;
  pb::put_string_nz(&s, 1, container);
  pb::put_string_nz(&s, 2, host);
  pb::put_string_nz(&s, 3, perms);
  return s;
}
std::string base_of(const std::string& id) {
  const size_t p = id.find("::");
  return p == std::string::npos ? id : id.substr(0, p);
}
}  // namespace

DeviceTable::RpcStats::RpcStats() {
  for (int r = 0; r < kRpcCount; ++r) {
    hist[r] = std::make_unique<Histogram>(rpc_buckets());
    errors[r].store(0);
  }
}

DeviceTable::DeviceTable(TableConfig cfg, std::vector<TableDevice> devices, Topology topo)
    : cfg_(std::move(cfg)), devs_(std::move(devices)), topo_(std::make_shared<const Topology>(std::move(topo))) {
  health_.reset(new std::atomic<uint8_t>[devs_.size() ? devs_.size() : 1]);
  for (size_t i = 0; i < devs_.size(); ++i) health_[i].store(devs_[i].healthy ? 1 : 0);
  stats_ = std::make_shared<RpcStats>();
  for (size_t i = 0; i < devs_.size(); ++i) {
    const auto& d = devs_[i];
    index_.emplace(std::string_view(devs_[i].id), static_cast<int>(i));
    AllocDevice a;
    a.gpu = d.gpu;
    a.partition = d.partition;
    a.numa = d.numa;
    a.base_id = base_of(d.id);
    a.annotated = d.id.find("::") != std::string::npos;
    if (a.annotated) aligned_ok_ = false;
    alloc_devs_.push_back(a);
    std::string frag;
    for (const auto& p : d.host_paths) pb::put_bytes(&frag, 3, device_spec(p, p, cfg_.permissions));
    spec_frag_.push_back(std::move(frag));
  }
  if (cfg_.mount_kfd) pb::put_bytes(&kfd_frag_, 3, device_spec(cfg_.kfd_path, cfg_.kfd_path, cfg_.permissions));
  for (const auto& kv : cfg_.extra_envs) pb::put_bytes(&env_extra_frag_, 1, map_entry(kv.first, kv.second));
  std::lock_guard<std::mutex> lk(wmu_);
  publish_law_locked();
}

std::vector<std::string> DeviceTable::ids() const {
  std::vector<std::string> out;
  out.reserve(devs_.size());
  for (const auto& d : devs_) out.push_back(d.id);
  return out;
}

int DeviceTable::index_of(std::string_view id) const {
  auto it = index_.find(id);
  return it == index_.end() ? -1 : it->second;
}

bool DeviceTable::contains(const std::vector<std::string>& ids) const {
  for (const auto& id : ids)
    if (index_of(id) < 0) return false;
  return true;
}

void DeviceTable::publish_law_locked() {
  std::string out;
  for (size_t i = 0; i < devs_.size(); ++i) {
    const auto& d = devs_[i];
    std::string dev;
    pb::put_string_nz(&dev, 1, d.id);
    pb::put_string_nz(&dev, 2, is_healthy(static_cast<int>(i)) ? "Healthy" : "Unhealthy");
    if (d.numa >= 0) {
      std::string node, topo;
      pb::put_int_nz(&node, 1, d.numa);
      pb::put_bytes(&topo, 1, node);
      pb::put_bytes(&dev, 3, topo);
    }
    pb::put_bytes(&out, 1, dev);
  }
  std::atomic_store_explicit(&law_, std::shared_ptr<const std::string>(std::make_shared<std::string>(std::move(out))),
                             std::memory_order_release);
}

void DeviceTable::add_listener(std::weak_ptr<TableListener> l) {
  std::lock_guard<std::mutex> lk(lmu_);
  listeners_.erase(std::remove_if(listeners_.begin(), listeners_.end(),
                                  [](const std::weak_ptr<TableListener>& w) { return w.expired(); }),
                   listeners_.end());
  listeners_.push_back(std::move(l));
}

uint64_t DeviceTable::wait_change(uint64_t seen, int timeout_ms) const {
  std::unique_lock<std::mutex> lk(vmu_);
  const uint64_t w0 = wakes_;
  cv_wait_ms(vcv_, lk, timeout_ms, [&] { return version() != seen || wakes_ != w0; });
  return version();
}

void DeviceTable::wake() const {
  {
    std::lock_guard<std::mutex> lk(vmu_);
    ++wakes_;
  }
  vcv_.notify_all();
}

void DeviceTable::notify_listeners() {
  {
    std::lock_guard<std::mutex> lk(vmu_);  // pairs with wait_change's predicate check
  }
  vcv_.notify_all();
  std::vector<std::shared_ptr<TableListener>> live;
  {
    std::lock_guard<std::mutex> lk(lmu_);
    for (const auto& w : listeners_)
      if (auto sp = w.lock()) live.push_back(std::move(sp));
  }
  for (const auto& l : live) l->on_table_change();
}

bool DeviceTable::set_health(std::string_view id, bool healthy) {
  {
    std::lock_guard<std::mutex> lk(wmu_);
    const int i = index_of(id);
    if (i < 0 || is_healthy(i) == healthy) return false;
    health_[i].store(healthy ? 1 : 0, std::memory_order_release);
    publish_law_locked();
    version_.fetch_add(1, std::memory_order_acq_rel);
  }
  notify_listeners();
  return true;
}

int DeviceTable::set_gpu_health(int gpu, int partition, bool healthy) {
  std::unique_lock<std::mutex> lk(wmu_);
  int changed = 0;
  for (size_t i = 0; i < devs_.size(); ++i) {
    const auto& d = devs_[i];
    if (d.gpu != gpu) continue;
    // a partition event hits that partition (and the whole-GPU device containing it)
    if (partition >= 0 && d.partition >= 0 && d.partition != partition) continue;
    if (is_healthy(static_cast<int>(i)) != healthy) {
      health_[i].store(healthy ? 1 : 0, std::memory_order_release);
      ++changed;
    }
  }
  if (changed) {
    publish_law_locked();
    version_.fetch_add(1, std::memory_order_acq_rel);
    lk.unlock();
    notify_listeners();
  }
  return changed;
}

int DeviceTable::set_gpu_health_except(int gpu, const std::vector<int>& held) {
  std::unique_lock<std::mutex> lk(wmu_);
  int changed = 0;
  for (size_t i = 0; i < devs_.size(); ++i) {
    const auto& d = devs_[i];
    if (d.gpu != gpu) continue;
    // a held partition stays as it is, and so does a whole-GPU device that contains one
    if (d.partition < 0 ? !held.empty() : std::find(held.begin(), held.end(), d.partition) != held.end()) continue;
    if (!is_healthy(static_cast<int>(i))) {
      health_[i].store(1, std::memory_order_release);
      ++changed;
    }
  }
  if (changed) {
    publish_law_locked();
    version_.fetch_add(1, std::memory_order_acq_rel);
    lk.unlock();
    notify_listeners();
  }
  return changed;
}

bool DeviceTable::healthy(std::string_view id) const {
  const int i = index_of(id);
  return i >= 0 && is_healthy(i);
}

int DeviceTable::healthy_count() const {
  int n = 0;
  for (size_t i = 0; i < devs_.size(); ++i) n += is_healthy(static_cast<int>(i));
  return n;
}

template <class F>
void DeviceTable::patch_topology(F&& f) {
  std::lock_guard<std::mutex> lk(wmu_);
  auto cur = std::atomic_load_explicit(&topo_, std::memory_order_acquire);
  auto next = std::make_shared<Topology>(*cur);  // copy-on-write: readers keep their snapshot
  if (!f(*next)) return;
  std::atomic_store_explicit(&topo_, std::shared_ptr<const Topology>(std::move(next)), std::memory_order_release);
}

void DeviceTable::set_link_up(int a, int b, bool up) {
  patch_topology([&](Topology& t) {
    if (a < 0 || b < 0 || a >= t.n || b >= t.n) return false;
    t.at(a, b).up = t.at(b, a).up = up;
    return true;
  });
}

void DeviceTable::set_link_bandwidth(int a, int b, double gbps) {
  patch_topology([&](Topology& t) {
    if (a < 0 || b < 0 || a >= t.n || b >= t.n || a == b) return false;
    t.at(a, b).bw_gbps = t.at(b, a).bw_gbps = std::max(0.0, gbps);
    return true;
  });
}

void DeviceTable::set_link_pods(const std::vector<int>& counts) {
  patch_topology([&](Topology& t) {
    const size_t nn = static_cast<size_t>(t.n) * t.n;
    bool changed = false;
    for (size_t i = 0; i < nn; ++i) {
      const int v = i < counts.size() ? std::max(0, counts[i]) : 0;
      changed |= t.links[i].pods != v;
      t.links[i].pods = v;
    }
    return changed;
  });
}

void DeviceTable::set_recent_allocations(std::shared_ptr<RecentAllocations> r) {
  std::lock_guard<std::mutex> lk(wmu_);
  recent_.store(r.get(), std::memory_order_release);
  if (r) recent_owned_.push_back(std::move(r));
}

Topology DeviceTable::topology() const { return *std::atomic_load_explicit(&topo_, std::memory_order_acquire); }

std::string DeviceTable::list_and_watch() const {
  return *std::atomic_load_explicit(&law_, std::memory_order_acquire);
}

std::string DeviceTable::options_bytes() const {
  std::string s;
  pb::put_bool_nz(&s, 1, cfg_.pre_start_required);
  pb::put_bool_nz(&s, 2, true);  // get_preferred_allocation_available
  return s;
}

bool DeviceTable::submit_prestart(std::string_view req, PreStartDone done, std::string* error) {
  PreStartJob job;
  try {
    pb::Reader r(req);  // PreStartContainerRequest{ repeated string devices_ids = 1 }
    uint32_t f, w;
    while (r.next(&f, &w)) {
      if (f == 1 && w == 2) job.ids.emplace_back(r.bytes());
      else r.skip(w);
    }
  } catch (const pb::DecodeError& e) {
    *error = std::string("malformed PreStartContainerRequest: ") + e.what();
    return false;
  }
  for (const auto& id : job.ids)
    if (index_of(id) < 0) {
      *error = "PreStartContainer for '" + cfg_.resource_name + "': unknown device: " + id;
      return false;
    }
  {
    std::lock_guard<std::mutex> lk(pmu_);
    if (pcancel_) {
      *error = "plugin is stopping";
      return false;
    }
    job.id = next_job_++;
    pwait_.emplace(job.id, std::move(done));
    pjobs_.push_back(std::move(job));
  }
  pcv_.notify_all();
  return true;
}

std::vector<PreStartJob> DeviceTable::pop_prestart(int timeout_ms) {
  std::unique_lock<std::mutex> lk(pmu_);
  cv_wait_ms(pcv_, lk, timeout_ms, [&] { return !pjobs_.empty() || pcancel_; });
  std::vector<PreStartJob> out(std::make_move_iterator(pjobs_.begin()), std::make_move_iterator(pjobs_.end()));
  pjobs_.clear();
  return out;
}

void DeviceTable::complete_prestart(uint64_t id, bool ok, const std::string& error) {
  PreStartDone done;
  {
    std::lock_guard<std::mutex> lk(pmu_);
    auto it = pwait_.find(id);
    if (it == pwait_.end()) return;  // cancelled meanwhile
    done = std::move(it->second);
    pwait_.erase(it);
  }
  if (done) done(ok, error);
}

void DeviceTable::cancel_prestart(const std::string& why) {
  std::unordered_map<uint64_t, PreStartDone> waiting;
  {
    std::lock_guard<std::mutex> lk(pmu_);
    pcancel_ = true;
    pjobs_.clear();
    waiting.swap(pwait_);
  }
  pcv_.notify_all();
  for (auto& kv : waiting)
    if (kv.second) kv.second(false, why);
}

void DeviceTable::resume_prestart() {
  std::lock_guard<std::mutex> lk(pmu_);
  pcancel_ = false;
}

size_t DeviceTable::prestart_pending() const {
  std::lock_guard<std::mutex> lk(pmu_);
  return pwait_.size();
}

namespace {

size_t varint_len(uint64_t v) {
  size_t n = 1;
  while (v >= 0x80) {
    v >>= 7;
    ++n;
  }
  return n;
}

// map<string,string> entry (field `field`) written in place, no temporary message
void put_map_entry(std::string* out, uint32_t field, std::string_view k, std::string_view v) {
  const size_t inner = 1 + varint_len(k.size()) + k.size() + 1 + varint_len(v.size()) + v.size();
  pb::put_tag(out, field, 2);
  pb::put_varint(out, inner);
  pb::put_bytes(out, 1, k);
  pb::put_bytes(out, 2, v);
}

}  // namespace

void DeviceTable::encode_container_alloc(const int* idx, size_t n, std::string* c) const {
  thread_local std::string joined;
  joined.clear();
  for (size_t k = 0; k < n; ++k) {
    if (k) joined.push_back(',');
    joined.append(devs_[idx[k]].id);
  }
  if (!cfg_.visible_env.empty()) put_map_entry(c, 1, cfg_.visible_env, joined);
  c->append(env_extra_frag_);
  c->append(kfd_frag_);
  // de-duplicate device nodes (replicas of one partition share its render node)
  for (size_t k = 0; k < n; ++k) {
    const int i = idx[k];
    bool dup = false;
    for (size_t j = 0; j < k && !dup; ++j) dup = spec_frag_[idx[j]] == spec_frag_[i];
    if (!dup) c->append(spec_frag_[i]);
  }
  if (cfg_.cdi) {
    for (size_t k = 0; k < n; ++k) {
      const std::string& base = alloc_devs_[idx[k]].base_id;
      const size_t name_len = cfg_.cdi_prefix.size() + base.size();
      pb::put_tag(c, 5, 2);  // CDIDevice{ name = 1 }
      pb::put_varint(c, 1 + varint_len(name_len) + name_len);
      pb::put_tag(c, 1, 2);
      pb::put_varint(c, name_len);
      c->append(cfg_.cdi_prefix).append(base);
    }
  }
}

bool DeviceTable::allocate(std::string_view req, std::string* out) const {
  // Flat, reused decode state: one pass validates the whole request (a malformed
  // message is reported as such before any lookup), with no per-call allocation.
  thread_local std::vector<std::string_view> ids;
  thread_local std::vector<size_t> ends;  // ids[ends[k-1], ends[k]) belong to container k
  thread_local std::vector<int> idx;
  thread_local std::vector<uint64_t> masks;  // GPUs each container spans
  thread_local std::string c;
  ids.clear();
  ends.clear();
  masks.clear();
  try {
    pb::Reader r(req);
    uint32_t f, w;
    while (r.next(&f, &w)) {
      if (f == 1 && w == 2) {
        pb::Reader cr(r.bytes());
        uint32_t cf, cw;
        while (cr.next(&cf, &cw)) {
          if (cf == 1 && cw == 2) ids.push_back(cr.bytes());
          else cr.skip(cw);
        }
        ends.push_back(ids.size());
      } else {
        r.skip(w);
      }
    }
  } catch (const pb::DecodeError& e) {
    *out = std::string("malformed AllocateRequest: ") + e.what();
    return false;
  }
  out->clear();
  size_t begin = 0;
  for (const size_t end : ends) {
    idx.clear();
    for (size_t k = begin; k < end; ++k) {
      const std::string_view id = ids[k];
      const int i = index_of(id);
      if (i < 0) {
        *out = "invalid allocation request for '" + cfg_.resource_name + "': unknown device: " + std::string(id);
        return false;
      }
      if (cfg_.reject_unhealthy && !is_healthy(i)) {
        *out = "invalid allocation request for '" + cfg_.resource_name + "': device is Unhealthy: " + std::string(id);
        return false;
      }
      idx.push_back(i);
    }
    uint64_t mask = 0;
    for (const int i : idx)
      if (alloc_devs_[i].gpu >= 0 && alloc_devs_[i].gpu < 64) mask |= 1ull << alloc_devs_[i].gpu;
    masks.push_back(mask);
    begin = end;
    c.clear();
    encode_container_alloc(idx.data(), idx.size(), &c);
    pb::put_bytes(out, 1, c);
  }
  // A container that spans GPUs will drive traffic over their links: count it as link
  // load at once (the PodResources map catches up only at its next poll).  Recorded
  // only once the whole request succeeded.
  if (RecentAllocations* ra = recent_.load(std::memory_order_acquire))
    for (const uint64_t mask : masks)
      if (__builtin_popcountll(mask) >= 2) ra->record(mask, mono_ns());
  return true;
}

AllocResult DeviceTable::preferred_core(const std::string_view* avail, size_t n_avail, const std::string_view* must,
                                        size_t n_must, int size) const {
  thread_local std::vector<int> a, m;
  a.clear();
  m.clear();
  bool any_annotated = false;
  for (size_t k = 0; k < n_avail; ++k) {
    const int i = index_of(avail[k]);
    if (i < 0) continue;
    a.push_back(i);
    any_annotated |= alloc_devs_[i].annotated;
  }
  for (size_t k = 0; k < n_must; ++k) {
    const int i = index_of(must[k]);
    if (i < 0) {
      AllocResult r;
      r.ok = false;
      r.error = "unknown device in must_include_deviceIDs: " + std::string(must[k]);
      return r;
    }
    if (std::find(m.begin(), m.end(), i) == m.end()) m.push_back(i);
  }
  // Contract (go-gpuallocator BestEffort): a non-positive size yields no devices; a size
  // below |must_include| cannot be honoured and is an error rather than a larger set.
  if (size <= 0) return AllocResult{};
  if (static_cast<size_t>(size) < m.size()) {
    AllocResult r;
    r.ok = false;
    r.error = "allocation_size " + std::to_string(size) + " is smaller than must_include_deviceIDs (" +
              std::to_string(m.size()) + ")";
    return r;
  }
  if (aligned_ok_ && !any_annotated) {
    const auto topo = std::atomic_load_explicit(&topo_, std::memory_order_acquire);  // snapshot
    RecentAllocations* ra = recent_.load(std::memory_order_acquire);
    const int64_t now = ra ? mono_ns() : 0;
    if (ra && ra->maybe_live(now)) {
      // multi-GPU containers allocated since the last PodResources poll: their links
      // count as used too
      thread_local std::vector<int> extra;
      extra.assign(static_cast<size_t>(topo->n) * topo->n, 0);
      if (ra->add_link_pods(topo->n, now, &extra) > 0) {
        thread_local Topology with_recent;
        with_recent = *topo;
        for (size_t i = 0; i < extra.size(); ++i) with_recent.links[i].pods += extra[i];
        return aligned_alloc(with_recent, alloc_devs_, a, m, size);
      }
    }
    return aligned_alloc(*topo, alloc_devs_, a, m, size);
  }
  return distributed_alloc(alloc_devs_, a, m, size);
}

AllocResult DeviceTable::preferred_ids(const std::vector<std::string>& avail, const std::vector<std::string>& must,
                                       int size, std::vector<std::string>* out_ids) const {
  std::vector<std::string_view> av(avail.begin(), avail.end()), mu(must.begin(), must.end());
  AllocResult r = preferred_core(av.data(), av.size(), mu.data(), mu.size(), size);
  if (r.ok && out_ids) {
    out_ids->clear();
    for (int i : r.chosen) out_ids->push_back(devs_[i].id);
  }
  return r;
}

bool DeviceTable::preferred(std::string_view req, std::string* out) const {
  // One validating pass into flat reused vectors (malformed => error before any work).
  struct Span {
    size_t av_end, mu_end;
    int32_t size;
  };
  thread_local std::vector<std::string_view> av, mu;
  thread_local std::vector<Span> spans;
  thread_local std::string c;
  av.clear();
  mu.clear();
  spans.clear();
  try {
    pb::Reader r(req);
    uint32_t f, w;
    while (r.next(&f, &w)) {
      if (f == 1 && w == 2) {
        pb::Reader cr(r.bytes());
        int32_t size = 0;
        uint32_t cf, cw;
        while (cr.next(&cf, &cw)) {
          if (cf == 1 && cw == 2) av.push_back(cr.bytes());
          else if (cf == 2 && cw == 2) mu.push_back(cr.bytes());
          else if (cf == 3 && cw == 0) size = static_cast<int32_t>(cr.varint());
          else cr.skip(cw);
        }
        spans.push_back({av.size(), mu.size(), size});
      } else {
        r.skip(w);
      }
    }
  } catch (const pb::DecodeError& e) {
    *out = std::string("malformed PreferredAllocationRequest: ") + e.what();
    return false;
  }
  out->clear();
  size_t av0 = 0, mu0 = 0;
  for (const Span& sp : spans) {
    AllocResult ar = preferred_core(av.data() + av0, sp.av_end - av0, mu.data() + mu0, sp.mu_end - mu0, sp.size);
    av0 = sp.av_end;
    mu0 = sp.mu_end;
    if (!ar.ok) {
      *out = "error getting list of preferred allocation devices: " + ar.error;
      return false;
    }
    c.clear();
    for (int i : ar.chosen) pb::put_bytes(&c, 1, devs_[i].id);
    pb::put_bytes(out, 1, c);
  }
  return true;
}

void DeviceTable::observe(int rpc, double seconds, bool error) const {
  if (rpc < 0 || rpc >= kRpcCount) return;
  stats_->hist[rpc]->observe(seconds);
  if (error) stats_->errors[rpc].fetch_add(1, std::memory_order_relaxed);
}

void DeviceTable::render_metric_headers(std::string* out) {
  append_header(out, "amdgpu_device_plugin_rpc_duration_seconds",
                "Latency of kubelet DevicePlugin RPCs served by this plugin.", "histogram");
}

uint64_t DeviceTable::metrics_version() const {
  uint64_t v = 0;
  for (int r = 0; r < kRpcCount; ++r) v += stats_->hist[r]->count();
  return v;
}

void DeviceTable::render_metrics(std::string* out, bool with_headers) const {
  if (with_headers) render_metric_headers(out);
  std::string labels;
  for (int r = 0; r < kRpcCount; ++r) {
    if (stats_->hist[r]->count() == 0) continue;
    labels.assign("resource=\"");
    append_label_value(&labels, cfg_.resource_name);
    labels.append("\",rpc=\"").append(rpc_name(r)).append("\",");
    stats_->hist[r]->render(out, "amdgpu_device_plugin_rpc_duration_seconds", labels);
  }
}

}  // namespace amdgpu_dp
