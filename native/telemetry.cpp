#include "telemetry.h"

#include <zlib.h>

#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <map>
#include <stdexcept>
#include <cstdio>
#include <cstring>
#include <dirent.h>
#include <fstream>
#include <sys/resource.h>

namespace amdgpu_dp {

namespace {

// deflateInit2 allocates and clears ~256 KiB of state; a scrape-path compressor reuses
// one stream per thread (deflateReset) instead.
struct ThreadDeflater {
  z_stream zs{};
  int level = -100;
  bool live = false;
  ~ThreadDeflater() {
    if (live) deflateEnd(&zs);
  }
  z_stream* get(int lvl) {
    if (live && level == lvl) {
      deflateReset(&zs);
      return &zs;
    }
    if (live) deflateEnd(&zs);
    zs = z_stream{};
    live = deflateInit2(&zs, lvl, Z_DEFLATED, 15 + 16, 8, Z_DEFAULT_STRATEGY) == Z_OK;
    if (!live) throw std::runtime_error("deflateInit2 failed");
    level = lvl;
    return &zs;
  }
};

}  // namespace

void gzip_member(const char* data, size_t n, std::string* out, int level) {
  static thread_local ThreadDeflater td;
  z_stream* zs = td.get(level);
  const size_t base = out->size();
  out->resize(base + deflateBound(zs, static_cast<uLong>(n)));
  zs->next_in = reinterpret_cast<Bytef*>(const_cast<char*>(data));
  zs->avail_in = static_cast<uInt>(n);
  zs->next_out = reinterpret_cast<Bytef*>(&(*out)[base]);
  zs->avail_out = static_cast<uInt>(out->size() - base);
  const int rc = deflate(zs, Z_FINISH);
  out->resize(base + zs->total_out);
  if (rc != Z_STREAM_END) throw std::runtime_error("deflate did not finish");
}

namespace {
std::atomic<uint64_t> g_exporter_ids{0};
}  // namespace

Exporter::Exporter()
    : id_(g_exporter_ids.fetch_add(1) + 1),
      sample_hist_({1e-4, 2.5e-4, 5e-4, 1e-3, 2.5e-3, 5e-3, 1e-2, 2.5e-2, 5e-2, 0.1, 0.25, 0.5, 1.0}) {
  start_time_s_ = now_ns() / 1000000000LL;
  extra_ = std::make_shared<const std::string>();
  gpu_text_ = std::make_shared<const std::string>();
  fresh_ = std::make_shared<const Freshness>();
  stalls_ = std::make_shared<const Stalls>();
  std::lock_guard<std::mutex> lk(mu_);
  publish_view_locked();
}

void Exporter::publish_view_locked() {
  auto v = std::make_shared<ScrapeView>();
  auto h = std::make_shared<std::string>();
  h->reserve(build_info_.size() + gpu_text_->size());
  h->append(build_info_).append(*gpu_text_);
  v->head = std::move(h);
  v->extra = extra_;
  v->tables = tables_;
  std::shared_ptr<const ScrapeView> old;
  {
    std::lock_guard<SpinLock> lk(view_lock_);
    old.swap(view_);
    view_ = std::move(v);
  }
  view_gen_.fetch_add(1, std::memory_order_release);
}

Exporter::TlCache& Exporter::tl_cache() const {
  static thread_local TlCache c;
  if (c.exporter != id_) {  // another exporter rendered on this thread last (tests)
    c = TlCache{};
    c.exporter = id_;
  }
  return c;
}

std::shared_ptr<const Exporter::ScrapeView> Exporter::view() const {
  std::lock_guard<SpinLock> lk(view_lock_);
  return view_;
}

Exporter::~Exporter() { stop(); }

void Exporter::set_inventory(const std::vector<GpuInfo>& gpus) {
  std::lock_guard<std::mutex> lk(mu_);
  gpus_ = gpus;
  last_.assign(gpus.size(), GpuSample{});
  ++inventory_gen_;
}

void Exporter::set_partition_labels(const std::vector<PartitionLabel>& labels) {
  std::lock_guard<std::mutex> lk(mu_);
  labels_ = labels;
}

void Exporter::set_build_info(const std::string& rendered) {
  std::lock_guard<std::mutex> lk(mu_);
  build_info_ = rendered;
  publish_view_locked();
}

void Exporter::set_tables(const std::vector<std::shared_ptr<DeviceTable>>& tables) {
  std::lock_guard<std::mutex> lk(mu_);
  tables_ = tables;
  publish_view_locked();
}

void Exporter::set_extra(const std::string& rendered) {
  auto p = std::make_shared<const std::string>(rendered);
  std::lock_guard<std::mutex> lk(mu_);
  extra_ = p;
  publish_view_locked();
}

void Exporter::start(std::shared_ptr<Backend> backend, int interval_ms, std::shared_ptr<HealthMonitor> monitor) {
  stop();
  std::weak_ptr<Exporter> weak = weak_from_this();
  if (weak.expired()) throw std::logic_error("Exporter must be owned by a std::shared_ptr to start sampling");
  // A sampler left behind by an earlier stop() (stuck in a backend call) sees another
  // generation when its call returns and leaves without touching this exporter again;
  // bump it before anything it could read changes.
  const uint64_t gen = sampler_gen_.fetch_add(1) + 1;
  const int interval = interval_ms > 0 ? interval_ms : 1000;
  {
    std::lock_guard<std::mutex> lk(run_mu_);
    backend_ = std::move(backend);
    monitor_ = std::move(monitor);
    interval_ms_ = interval;
  }
  stop_ = false;
  running_ = true;
  started_ns_.store(mono_ns());
  idle_mode_.store(false);
  poke_.store(false);
  current_interval_ms_.store(interval);
  {
    std::lock_guard<std::mutex> lk(first_mu_);
    first_done_ = false;
  }
  sampler_exit_ = std::make_shared<ThreadExit>();
  {
    std::lock_guard<std::mutex> lk(run_mu_);
    waker_ = std::make_shared<Waker>();  // (under run_mu_: a scrape's note_read reads it)
    watchdog_ = std::thread([this, m = monitor_, wk = waker_] { watchdog_loop(m, wk); });  // before the first call
  }
  thread_ = std::thread(sampler_main, std::move(weak), sampler_exit_, waker_, gen, interval);
  // /metrics is normally populated before start() returns.  The first pass waits on the
  // lanes at most its budget (a wedged driver at start-up stalls one lane, not the pass),
  // and start() waits for the first pass at most the stall threshold: the caller - the
  // plugin manager, which has kubelet restarts, /restart and health events to handle -
  // goes on either way.
  const int ms = stall_ms_.load();
  std::unique_lock<std::mutex> lk(first_mu_);
  cv_wait_ms(first_cv_, lk, ms > 0 ? ms : 10000, [&] { return first_done_; });
}

void Exporter::Waker::sleep_ms(int64_t ms, bool pokeable) {
  std::unique_lock<std::mutex> lk(mu);
  cv_wait_ms(cv, lk, static_cast<int>(std::min<int64_t>(ms, 3600000)), [&] { return stopping || (pokeable && poked); });
  if (pokeable) poked = false;
}

void Exporter::Waker::poke() {
  {
    std::lock_guard<std::mutex> lk(mu);
    poked = true;
  }
  cv.notify_all();
}

void Exporter::Waker::wake() {
  {
    std::lock_guard<std::mutex> lk(mu);
    stopping = true;
  }
  cv.notify_all();
}

bool Exporter::ThreadExit::wait(int ms) {
  std::unique_lock<std::mutex> lk(mu);
  if (ms < 0) {
    cv.wait(lk, [&] { return done; });
    return true;
  }
  return cv_wait_ms(cv, lk, ms, [&] { return done; });
}

void Exporter::ThreadExit::mark() {
  {
    std::lock_guard<std::mutex> lk(mu);
    done = true;
  }
  cv.notify_all();
}

void Exporter::stop() {
  if (!running_.exchange(false)) return;
  stop_ = true;
  if (waker_) waker_->wake();
  const auto self_id = std::this_thread::get_id();
  if (watchdog_.joinable()) {
    if (watchdog_.get_id() == self_id) watchdog_.detach();
    else watchdog_.join();
  }
  if (!thread_.joinable()) return;
  if (thread_.get_id() == self_id) {  // the sampler dropped the last reference: it ends by itself
    thread_.detach();
    return;
  }
  // The sampler never blocks in a hardware call (it waits on lane jobs in short slices),
  // so it leaves within one slice; a call wedged on a lane stays with the lane.
  sampler_exit_->wait(-1);
  thread_.join();
}

int Exporter::stalled_gpu() const {
  std::shared_ptr<const Stalls> st;
  {
    std::lock_guard<SpinLock> lk(fresh_lock_);
    st = stalls_;
  }
  return st->stalled.empty() ? -1 : *std::min_element(st->stalled.begin(), st->stalled.end());
}

std::vector<int> Exporter::stalled_gpus() const {
  std::lock_guard<SpinLock> lk(fresh_lock_);
  return stalls_->stalled;
}

std::vector<int> Exporter::blocked_gpus() const {
  std::lock_guard<SpinLock> lk(fresh_lock_);
  return stalls_->blocked;
}

double Exporter::sample_age_s(int gpu) const {
  std::shared_ptr<const Freshness> f;
  {
    std::lock_guard<SpinLock> lk(fresh_lock_);
    f = fresh_;
  }
  for (const auto& kv : f->last_ok)
    if (kv.first == gpu) return kv.second ? (mono_ns() - kv.second) * 1e-9 : -1.0;
  return -1.0;
}

// Lanes whose call has been in flight past the threshold.  The one stuck longest is the
// culprit.  Another is reported as well only if some call completed after its own call
// had been in flight for a grace period - proof that the library is not serialised behind
// the first wedge, so this GPU is stuck on its own; otherwise it is only waiting behind
// the first (a library that serialises every device) and is reported "blocked".  Each
// stuck call is reported once; the GPU recovers through on_sample once a sample returns.
void Exporter::watchdog_loop(std::shared_ptr<HealthMonitor> monitor, std::shared_ptr<Waker> waker) {
  background_thread("dpwatchdog");
  std::map<std::string, int64_t> reported;  // key -> since of the call reported lost
  int64_t sleep_ms = 25;
  while (!stop_.load()) {
    waker->sleep_ms(sleep_ms);
    if (stop_.load()) break;
    const int ms = stall_ms_.load();
    // Checks a quarter of the stall threshold apart (25 ms .. 5 s; 5 s with no threshold),
    // sooner when a call in flight is about to cross it (then it wakes as it crosses): a
    // 10 s threshold costs a wake-up every 2.5 s on an idle node instead of 40 a second.
    const int64_t period = ms > 0 ? std::max<int64_t>(25, std::min<int64_t>(5000, ms / 4)) : 5000;
    sleep_ms = period;
    std::shared_ptr<Backend> be;
    {
      std::lock_guard<std::mutex> lk(run_mu_);
      be = backend_;
    }
    if (ms <= 0 || !be) continue;
    const int64_t now = mono_ns();
    const int64_t threshold = static_cast<int64_t>(ms) * 1000000;
    const int64_t grace = std::min<int64_t>(threshold / 2, 200000000);
    const int64_t last_done = be->last_completion_ns();
    // only GPUs this exporter serves (the `devices` selection) are reported: a GPU left out
    // is never sampled, so nothing would clear a "lost" verdict on it.  Every stuck lane
    // still counts for attribution (a left-out GPU can be the root of a library-wide block).
    std::vector<std::string> served;  // keys (an index may have moved since set_inventory)
    std::vector<int> served_index;
    {
      std::lock_guard<std::mutex> lk(mu_);
      for (const auto& g : gpus_) {
        served.push_back(g.key);
        served_index.push_back(g.index);
      }
    }
    auto is_served = [&](const LaneReport& r) {
      for (size_t i = 0; i < served.size(); ++i)
        if (served[i].empty() ? served_index[i] == r.index : served[i] == r.lane.key) return true;
      return false;
    };
    std::vector<LaneReport> stuck;
    for (auto& r : be->lanes()) {
      if (r.index < 0 || !r.lane.inflight_since_ns) continue;
      const int64_t left = r.lane.inflight_since_ns + threshold - now;
      if (left < 0) stuck.push_back(r);
      else sleep_ms = std::max<int64_t>(25, std::min(sleep_ms, left / 1000000 + 1));  // wake as it crosses
    }
    int64_t root = 0;
    uint64_t root_batch = 0;
    for (const auto& r : stuck)
      if (!root || r.lane.inflight_since_ns < root) {
        root = r.lane.inflight_since_ns;
        root_batch = r.lane.inflight_batch;
      }
    // The root is known only if its call went out on its own (the sampler's walk posts one
    // call at a time).  When the earliest stuck call belongs to a batch posted to several
    // lanes at once (a discovery's describes) and other calls of that batch are stuck too,
    // any of them may hold a library-wide lock the others wait on: blame none of them.
    const bool ambiguous = root_batch != 0 && std::count_if(stuck.begin(), stuck.end(), [&](const LaneReport& r) {
                                                 return r.lane.inflight_batch == root_batch;
                                               }) > 1;
    auto st = std::make_shared<Stalls>();
    std::map<std::string, int64_t> still;
    std::vector<HwEvent> lost;  // fed to the monitor once the stall list below is published
    for (const auto& r : stuck) {
      if (!is_served(r)) continue;
      const int64_t since = r.lane.inflight_since_ns;
      if ((since != root || ambiguous) && last_done <= since + grace) {
        st->blocked.push_back(r.index);
        continue;
      }
      st->stalled.push_back(r.index);
      still[r.lane.key] = since;
      auto it = reported.find(r.lane.key);
      if (it != reported.end() && it->second == since) continue;
      HwEvent e;
      e.kind = kEvtDeviceLost;
      e.gpu = r.index;
      e.key = r.lane.key;  // the GPU the call went to, even if the node was re-enumerated since
      e.message = r.lane.inflight_what + " call in flight for " + std::to_string((now - since) / 1000000) +
                  " ms (health.sampleStallS)";
      lost.push_back(std::move(e));
    }
    reported.swap(still);
    std::sort(st->stalled.begin(), st->stalled.end());
    std::sort(st->blocked.begin(), st->blocked.end());
    {
      std::lock_guard<SpinLock> lk(fresh_lock_);
      stalls_ = std::move(st);
    }
    // whoever sees the lost verdict (the manager, /ready) also sees the stall behind it
    if (monitor)
      for (const auto& e : lost) monitor->process(e);
  }
}

void Exporter::sampler_main(std::weak_ptr<Exporter> weak, std::shared_ptr<ThreadExit> exit,
                            std::shared_ptr<Waker> waker, uint64_t gen, int interval_ms) {
  background_thread("dpsampler");
  // A strong reference only for the duration of each step: the exporter stays alive
  // through a backend call (however long it blocks), and may be destroyed between
  // steps, by whichever thread drops the last reference.  Nothing below touches it
  // after the reference is released.
  int64_t next = 0;  // mono ns of the next pass; 0 = now (first pass)
  for (;;) {
    int sleep_ms;
    {
      std::shared_ptr<Exporter> self = weak.lock();
      if (!self) break;
      sleep_ms = self->sampler_step(&next, gen, interval_ms);
    }
    if (sleep_ms < 0) break;
    if (sleep_ms > 0) waker->sleep_ms(sleep_ms, true);  // until the next pass, a poke, or stop()
  }
  exit->mark();
}

int Exporter::sampler_step(int64_t* next, uint64_t gen, int interval_ms) {
  if (stop_.load() || sampler_gen_.load() != gen) return -1;
  const int64_t now = mono_ns();
  if (*next != 0 && now < *next && poke_.exchange(false)) {
    // the GPU metrics were read while the sampler idled: the next pass is due one
    // interval after the last, as if it had never slowed down
    const int64_t due = last_pass_ns_.load() + static_cast<int64_t>(interval_ms) * 1000000;
    if (due < *next) *next = due;
  }
  if (*next != 0 && now < *next)  // (stop() cuts the sleep short)
    return static_cast<int>((*next - now) / 1000000 + 1);
  const bool first = *next == 0;
  sample_once(gen);
  if (first) {
    {
      std::lock_guard<std::mutex> lk(first_mu_);
      first_done_ = true;
    }
    first_cv_.notify_all();
    *next = mono_ns();
  }
  const int step = next_interval_ms(interval_ms);
  *next += static_cast<int64_t>(step) * 1000000;  // fixed cadence, no drift
  if (*next < mono_ns()) *next = mono_ns() + static_cast<int64_t>(step) * 1000000;
  return 0;
}

int Exporter::next_interval_ms(int interval_ms) {
  const int idle = idle_interval_ms_.load();
  int step = interval_ms;
  bool unread = false;
  if (idle > interval_ms) {
    const int64_t now = mono_ns(), window = static_cast<int64_t>(active_window_ms_.load()) * 1000000;
    const bool starting = now - started_ns_.load() < window;
    const bool read = now - last_read_ns_.load(std::memory_order_relaxed) < window;
    bool settling = false;
    if (!starting) {
      std::shared_ptr<HealthMonitor> mon;
      {
        std::lock_guard<std::mutex> lk(run_mu_);
        mon = monitor_;
      }
      settling = mon && mon->settling();
    }
    if (!starting && !settling) {
      if (!read) {
        step = idle;
        unread = true;
      } else if (const int64_t gap = read_gap_ns_.load(std::memory_order_relaxed); gap > 0) {
        // scraped: about two samples per scrape interval, between the two periods (a
        // Prometheus scraping every 15-30 s gets samples at most idleIntervalMs old)
        step = static_cast<int>(std::max<int64_t>(interval_ms, std::min<int64_t>(idle, gap / 2000000)));
      }
    }
  }
  idle_mode_.store(unread);
  if (step > interval_ms) idle_passes_.fetch_add(1, std::memory_order_relaxed);
  current_interval_ms_.store(step);
  return step;
}

void Exporter::note_read() const {
  // (every scrape comes here: one relaxed load in the common case, a store at most every
  // 100 ms, the sampler woken only on the first read after it slowed down)
  const int64_t now = mono_ns();
  const int64_t prev = last_read_ns_.load(std::memory_order_relaxed);
  if (now - prev < 100000000) return;
  last_read_ns_.store(now, std::memory_order_relaxed);
  read_gap_ns_.store(prev != 0 ? now - prev : 0, std::memory_order_relaxed);
  if (idle_mode_.load(std::memory_order_relaxed) && !poke_.exchange(true)) {
    std::shared_ptr<Waker> w;
    {
      std::lock_guard<std::mutex> lk(run_mu_);
      w = waker_;
    }
    if (w) w->poke();
  }
}

void Exporter::sample_once(uint64_t sampler_gen) {
  std::lock_guard<std::mutex> slk(sample_mu_);
  if (sampler_gen != 0 && sampler_gen_.load() != sampler_gen) return;
  std::shared_ptr<Backend> be;
  std::shared_ptr<HealthMonitor> mon;
  int interval;
  {
    std::lock_guard<std::mutex> lk(run_mu_);
    be = backend_;
    mon = monitor_;
    interval = interval_ms_;
  }
  // The inventory may be a subset of the node (`devices: "4-7"`): sample, report health
  // for and label each GPU by its backend index, never by its position in the subset.
  uint64_t gen;
  std::vector<int> index;
  std::vector<std::string> keys;
  {
    std::lock_guard<std::mutex> lk(mu_);
    for (const auto& g : gpus_) {
      index.push_back(g.index);
      keys.push_back(g.key);
    }
    gen = inventory_gen_;
  }
  if (gen != slots_gen_) {  // a reload: samples in flight belong to the old indices
    slots_.assign(index.size(), Slot{});
    for (size_t g = 0; g < index.size(); ++g) {
      slots_[g].index = index[g];
      slots_[g].key = keys[g];
    }
    slots_gen_ = gen;
  }
  const size_t n = slots_.size();
  const int64_t t0 = mono_ns();
  // One call in flight at a time, GPU after GPU: each sample is waited for a slice of the
  // pass budget, then left pending on its lane (collected by a later pass) while the walk
  // goes on.  A GPU whose sample is still out from an earlier pass is skipped, not waited
  // for again.  Walking instead of posting all at once keeps the stall attribution exact:
  // in a library that serialises devices, a call posted in parallel can start before the
  // one that wedges and then wait behind it, and "stuck longest" would name the wrong GPU.
  // 8 GPUs x ~1-5 ms per amdsmi sample fits a 1 s tick many times over.
  const int stall = stall_ms_.load();
  const int64_t budget_ms = sampler_gen != 0 ? std::max(1, std::min(interval, stall > 0 ? stall : interval))
                                             : (stall > 0 ? stall : (be ? be->call_timeout_ms() : 1000));
  const int64_t slice_ms = std::max<int64_t>(2, budget_ms / std::max<size_t>(1, n));
  for (size_t g = 0; g < n && be; ++g) {
    Slot& sl = slots_[g];
    if (sl.job && !sl.job->done()) continue;
    sl.out = std::make_shared<GpuSample>();
    sl.job = be->sample_async(sl.index, sl.out, sl.key);
    sl.refused = !sl.job;
    sl.posted_ns = mono_ns();
    const int64_t until = mono_ns() + slice_ms * 1000000;
    while (sl.job && !sl.job->done()) {  // in short waits, so stop() stays prompt
      const int64_t left = (until - mono_ns()) / 1000000;
      if (left <= 0) break;
      if (sampler_gen != 0 && (stop_.load() || sampler_gen_.load() != sampler_gen)) return;
      sl.job->wait(std::min<int64_t>(left, 50));
    }
  }
  std::vector<GpuSample> samples(n);
  std::vector<char> ok(n, 0), fresh(n, 0);
  const int64_t now = mono_ns();
  for (size_t g = 0; g < n; ++g) {
    Slot& sl = slots_[g];
    if (sl.job && sl.job->done()) {
      const bool good = !sl.job->dropped() && sl.out->ok;
      sl.last = *sl.out;
      sl.last_ok = good;
      if (good) sl.last_ok_ns = now;
      fresh[g] = 1;
      sl.job.reset();
    }
    // a sample is shown while its GPU's newer call is still within the budget; not once
    // that call is stuck (the values would pass for current)
    // nor when its lane refused the call (another call to that GPU, e.g. a discovery's,
    // is stuck there)
    const bool stuck = sl.refused ||
                       (sl.job && stall > 0 && now - sl.posted_ns > static_cast<int64_t>(stall) * 1000000);
    ok[g] = sl.last_ok && !stuck && sl.last_ok_ns != 0;
    samples[g] = sl.last;
  }
  const double dt = (mono_ns() - t0) * 1e-9;
  if (be) {
    sample_hist_.observe(dt);
    samples_.fetch_add(1, std::memory_order_relaxed);
  }
  auto f = std::make_shared<Freshness>();
  for (const auto& sl : slots_) f->last_ok.emplace_back(sl.index, sl.last_ok_ns);
  {
    std::lock_guard<SpinLock> lk(fresh_lock_);
    fresh_ = std::move(f);
    // a GPU whose call came back is no longer stalled or blocked (the watchdog would say
    // so at its next look; a reader must not see the stale verdict meanwhile)
    auto returned = [&](int gpu) {
      for (size_t g = 0; g < n; ++g)
        if (fresh[g] && slots_[g].index == gpu) return true;
      return false;
    };
    if (std::any_of(stalls_->stalled.begin(), stalls_->stalled.end(), returned) ||
        std::any_of(stalls_->blocked.begin(), stalls_->blocked.end(), returned)) {
      auto st = std::make_shared<Stalls>(*stalls_);
      st->stalled.erase(std::remove_if(st->stalled.begin(), st->stalled.end(), returned), st->stalled.end());
      st->blocked.erase(std::remove_if(st->blocked.begin(), st->blocked.end(), returned), st->blocked.end());
      stalls_ = std::move(st);
    }
  }
  // after the verdicts above are published: a reader woken by this pass's health
  // update must not still see the GPU's stale stall
  for (size_t g = 0; g < n; ++g) {
    if (!fresh[g]) continue;
    const bool good = slots_[g].last_ok;
    if (!good) sample_errors_.fetch_add(1, std::memory_order_relaxed);
    if (mon) mon->on_sample(slots_[g].index, good, slots_[g].last);
  }
  last_pass_ns_.store(mono_ns());
  render_gpu_text(samples, ok, gen);
}

namespace {

void gpu_labels(std::string* out, int gpu) {
  out->append("gpu=\"");
  append_u64(out, static_cast<uint64_t>(gpu));
  out->append("\"");
}

void line(std::string* out, const char* name, const std::string& labels, double v) {
  out->append(name).append("{").append(labels).append("} ");
  append_float(out, v);
  out->push_back('\n');
}

}  // namespace

void Exporter::render_gpu_text(const std::vector<GpuSample>& samples, const std::vector<char>& ok, uint64_t gen) {
  std::vector<GpuInfo> gpus;
  std::vector<PartitionLabel> labels;
  {
    std::lock_guard<std::mutex> lk(mu_);
    // A reload replaced the inventory while this pass sampled the old one: its samples
    // belong to other GPUs (or more/fewer of them).  Drop the pass; the next tick renders.
    if (gen != inventory_gen_) return;
    gpus = gpus_;
    labels = labels_;
    for (size_t g = 0; g < samples.size() && g < last_.size(); ++g)
      if (ok[g]) last_[g] = samples[g];
  }
  std::string o;
  o.reserve(4096 + gpus.size() * 4096);
  std::vector<std::string> gl(gpus.size());
  for (size_t g = 0; g < gpus.size(); ++g) gpu_labels(&gl[g], gpus[g].index);

  append_header(&o, "amdgpu_info", "Static inventory of each physical AMD GPU (value is always 1).", "gauge");
  for (size_t g = 0; g < gpus.size(); ++g) {
    const GpuInfo& gi = gpus[g];
    std::string l = gl[g];
    l.append(",uuid=\"");
    append_label_value(&l, gi.uuid);
    l.append("\",bdf=\"");
    append_label_value(&l, gi.bdf);
    l.append("\",name=\"");
    append_label_value(&l, gi.market_name);
    l.append("\",gfx_target=\"");
    append_label_value(&l, gi.gfx_target);
    l.append("\",compute_partition=\"");
    append_label_value(&l, gi.compute_partition);
    l.append("\",memory_partition=\"");
    append_label_value(&l, gi.memory_partition);
    l.append("\",numa_node=\"").append(std::to_string(gi.numa_node));
    l.append("\",driver_version=\"");
    append_label_value(&l, gi.driver_version);
    l.append("\",vbios_version=\"");
    append_label_value(&l, gi.vbios_version);
    l.append("\",oam_id=\"").append(std::to_string(gi.oam_id)).append("\"");
    line(&o, "amdgpu_info", l, 1);
  }
  {  // partition profiles the GPU supports, one series per (profile, memory mode)
    static const char* kNps[] = {"NPS1", "NPS2", "NPS4", "NPS8"};
    bool hdr = false;
    for (size_t g = 0; g < gpus.size(); ++g) {
      for (const auto& pp : gpus[g].supported_profiles) {
        for (int b = 0; b < 4; ++b) {
          if (!(pp.nps_caps & (1u << b))) continue;
          if (!hdr) {
            append_header(&o, "amdgpu_partition_profile_supported",
                          "Compute partition profile x memory partition mode the GPU supports (value 1); "
                          "source=current when only the current profile could be read.",
                          "gauge");
            hdr = true;
          }
          std::string l = gl[g];
          l.append(",profile=\"");
          append_label_value(&l, pp.type);
          l.append("\",partitions=\"").append(std::to_string(pp.partitions));
          l.append("\",memory_partition=\"").append(kNps[b]);
          l.append("\",source=\"");
          append_label_value(&l, pp.source);
          l.append("\"");
          line(&o, "amdgpu_partition_profile_supported", l, 1);
        }
      }
    }
  }
  append_header(&o, "amdgpu_telemetry_up", "1 if the last telemetry sample of the GPU succeeded.", "gauge");
  for (size_t g = 0; g < gpus.size(); ++g) line(&o, "amdgpu_telemetry_up", gl[g], ok[g] ? 1 : 0);

  auto per_gpu = [&](const char* name, const char* help, const char* type, auto getter) {
    bool hdr = false;
    for (size_t g = 0; g < gpus.size(); ++g) {
      if (!ok[g]) continue;
      const double v = getter(samples[g]);
      if (v < 0) continue;
      if (!hdr) {
        append_header(&o, name, help, type);
        hdr = true;
      }
      line(&o, name, gl[g], v);
    }
  };
  per_gpu("amdgpu_power_watts", "Current socket power in watts.", "gauge",
          [](const GpuSample& s) { return s.power_w; });
  per_gpu("amdgpu_energy_joules_total", "Accumulated socket energy in joules.", "counter",
          [](const GpuSample& s) { return s.energy_j; });
  per_gpu("amdgpu_gfx_activity_percent", "Average graphics/compute engine activity.", "gauge",
          [](const GpuSample& s) { return s.gfx_activity_pct; });
  per_gpu("amdgpu_umc_activity_percent", "Average memory controller (HBM) activity.", "gauge",
          [](const GpuSample& s) { return s.umc_activity_pct; });
  per_gpu("amdgpu_vram_used_bytes", "VRAM in use.", "gauge", [](const GpuSample& s) { return s.vram_used_bytes; });
  per_gpu("amdgpu_vram_total_bytes", "VRAM capacity.", "gauge", [](const GpuSample& s) { return s.vram_total_bytes; });
  per_gpu("amdgpu_throttle_status", "Raw throttle status bitmask.", "gauge",
          [](const GpuSample& s) { return static_cast<double>(s.throttle_status); });
  per_gpu("amdgpu_xgmi_link_width", "Current xGMI link width of the GPU, lanes (16 when fully trained).", "gauge",
          [](const GpuSample& s) { return s.xgmi_link_width; });
  per_gpu("amdgpu_xgmi_link_speed_gbps", "Current xGMI per-lane rate of the GPU, Gb/s.", "gauge",
          [](const GpuSample& s) { return s.xgmi_link_speed; });
  per_gpu("amdgpu_xgmi_error_status", "xGMI error state of the GPU: 0 none, 1 an error, 2 multiple errors.", "gauge",
          [](const GpuSample& s) { return static_cast<double>(s.xgmi_error_status); });
  per_gpu("amdgpu_pcie_link_width", "Current PCIe link width to the host, lanes.", "gauge",
          [](const GpuSample& s) { return s.pcie_link_width; });
  per_gpu("amdgpu_pcie_link_speed_gtps", "Current PCIe link rate to the host, GT/s per lane.", "gauge",
          [](const GpuSample& s) { return s.pcie_link_speed_gtps; });
  per_gpu("amdgpu_pcie_replays_total", "PCIe replays issued on the host link.", "counter",
          [](const GpuSample& s) { return s.pcie_replays; });
  per_gpu("amdgpu_pcie_recoveries_total", "PCIe host link transitions from L0 to recovery.", "counter",
          [](const GpuSample& s) { return s.pcie_recoveries; });

  {  // temperatures
    bool hdr = false;
    for (size_t g = 0; g < gpus.size(); ++g) {
      if (!ok[g]) continue;
      const GpuSample& s = samples[g];
      auto emit = [&](const char* sensor, double v) {
        if (v < 0) return;
        if (!hdr) {
          append_header(&o, "amdgpu_temperature_celsius", "Temperature by sensor (edge, hotspot, mem, hbmN).", "gauge");
          hdr = true;
        }
        line(&o, "amdgpu_temperature_celsius", gl[g] + ",sensor=\"" + sensor + "\"", v);
      };
      emit("edge", s.temp_edge_c);
      emit("hotspot", s.temp_hotspot_c);
      emit("mem", s.temp_mem_c);
      for (int h = 0; h < s.num_hbm; ++h) emit(("hbm" + std::to_string(h)).c_str(), s.temp_hbm_c[h]);
    }
  }
  {  // clocks
    bool hdr = false;
    for (size_t g = 0; g < gpus.size(); ++g) {
      if (!ok[g]) continue;
      const GpuSample& s = samples[g];
      for (int k = 0; k < 2; ++k) {
        const double v = k == 0 ? s.gfxclk_mhz : s.uclk_mhz;
        if (v < 0) continue;
        if (!hdr) {
          append_header(&o, "amdgpu_clock_mhz", "Current clock frequency in MHz.", "gauge");
          hdr = true;
        }
        line(&o, "amdgpu_clock_mhz", gl[g] + (k == 0 ? ",clock=\"gfx\"" : ",clock=\"mem\""), v);
      }
    }
  }
  {  // ECC
    bool hdr = false;
    for (size_t g = 0; g < gpus.size(); ++g) {
      if (!ok[g] || samples[g].ecc_correctable < 0) continue;
      if (!hdr) {
        append_header(&o, "amdgpu_ecc_errors_total", "Accumulated ECC error counts.", "counter");
        hdr = true;
      }
      line(&o, "amdgpu_ecc_errors_total", gl[g] + ",type=\"correctable\"",
           static_cast<double>(samples[g].ecc_correctable));
      line(&o, "amdgpu_ecc_errors_total", gl[g] + ",type=\"uncorrectable\"",
           static_cast<double>(samples[g].ecc_uncorrectable));
    }
  }
  {  // RAS retired pages (+ the threshold that makes a GPU Unhealthy)
    bool hdr = false;
    for (size_t g = 0; g < gpus.size(); ++g) {
      const GpuSample& s = samples[g];
      if (!ok[g] || s.retired_pages < 0) continue;
      if (!hdr) {
        append_header(&o, "amdgpu_retired_pages", "RAS retired (bad) HBM pages by status.", "gauge");
        hdr = true;
      }
      line(&o, "amdgpu_retired_pages", gl[g] + ",status=\"reserved\"", static_cast<double>(s.retired_pages));
      line(&o, "amdgpu_retired_pages", gl[g] + ",status=\"pending\"", static_cast<double>(std::max<int64_t>(0, s.pending_pages)));
      line(&o, "amdgpu_retired_pages", gl[g] + ",status=\"unreservable\"",
           static_cast<double>(std::max<int64_t>(0, s.unreservable_pages)));
    }
    hdr = false;
    for (size_t g = 0; g < gpus.size(); ++g) {
      if (gpus[g].bad_page_threshold <= 0) continue;
      if (!hdr) {
        append_header(&o, "amdgpu_retired_pages_threshold",
                      "Retired + pending pages at which the GPU is advertised Unhealthy.", "gauge");
        hdr = true;
      }
      line(&o, "amdgpu_retired_pages_threshold", gl[g], gpus[g].bad_page_threshold);
    }
  }
  {  // xGMI
    std::string up, rd, wr, rate, maxr;
    for (size_t g = 0; g < gpus.size(); ++g) {
      if (!ok[g]) continue;
      const GpuSample& s = samples[g];
      for (int k = 0; k < s.num_links; ++k) {
        const std::string l = gl[g] + ",link=\"" + std::to_string(k) + "\",peer=\"" +
                              (s.link_peer[k] >= 0 ? std::to_string(s.link_peer[k]) : std::string("unknown")) + "\"";
        if (s.link_up[k] >= 0) line(&up, "amdgpu_xgmi_link_up", l, s.link_up[k]);
        line(&rd, "amdgpu_xgmi_read_bytes_total", l, s.link_read_kb[k] * 1024.0);
        line(&wr, "amdgpu_xgmi_write_bytes_total", l, s.link_write_kb[k] * 1024.0);
        if (s.link_trained_gbps[k] > 0) {  // a link trained slower than its peers shows here
          line(&rate, "amdgpu_xgmi_link_bitrate_gbps", l, s.link_bitrate_gbps[k]);
          line(&maxr, "amdgpu_xgmi_link_bandwidth_gbps", l, s.link_trained_gbps[k]);
        }
      }
    }
    if (!up.empty()) {
      append_header(&o, "amdgpu_xgmi_link_up", "1 if the xGMI link to the peer GPU is up.", "gauge");
      o.append(up);
    }
    if (!rd.empty()) {
      append_header(&o, "amdgpu_xgmi_read_bytes_total", "Bytes received over the xGMI link.", "counter");
      o.append(rd);
      append_header(&o, "amdgpu_xgmi_write_bytes_total", "Bytes sent over the xGMI link.", "counter");
      o.append(wr);
    }
    if (!rate.empty()) {
      append_header(&o, "amdgpu_xgmi_link_bitrate_gbps", "xGMI per-lane signalling rate (Gb/s).", "gauge");
      o.append(rate);
      append_header(&o, "amdgpu_xgmi_link_bandwidth_gbps", "xGMI link bandwidth over all lanes (Gb/s).", "gauge");
      o.append(maxr);
    }
  }
  {  // partitions
    std::string info, busy, vram;
    std::vector<int> pos;  // backend GPU index -> position in this (possibly subset) inventory
    for (size_t g = 0; g < gpus.size(); ++g) {
      if (gpus[g].index < 0) continue;
      if (static_cast<size_t>(gpus[g].index) >= pos.size()) pos.resize(gpus[g].index + 1, -1);
      pos[gpus[g].index] = static_cast<int>(g);
    }
    for (const auto& pl : labels) {
      if (pl.gpu < 0 || pl.gpu >= static_cast<int>(pos.size()) || pos[pl.gpu] < 0) continue;
      const int g = pos[pl.gpu];
      std::string l = gl[g];
      l.append(",partition=\"").append(std::to_string(pl.partition < 0 ? 0 : pl.partition)).append("\",device_id=\"");
      append_label_value(&l, pl.device_id);
      l.append("\",resource=\"");
      append_label_value(&l, pl.resource);
      l.append("\"");
      std::string il = l;
      il.append(",hip_ids=\"");
      append_label_value(&il, pl.hip_ids);
      il.append("\"");
      line(&info, "amdgpu_partition_info", il, 1);
      if (!ok[g]) continue;
      const GpuSample& s = samples[g];
      const int p = pl.partition < 0 ? 0 : pl.partition;
      if (p < s.num_partitions && s.partition_gfx_busy_pct[p] >= 0)
        line(&busy, "amdgpu_partition_gfx_busy_percent",
             l + (s.partition_busy_source[p] == 1 ? ",source=\"partition_metrics\"" : ",source=\"xcp_stats\""),
             s.partition_gfx_busy_pct[p]);
      if (p < s.num_partitions && s.partition_vram_used_bytes[p] > 0)
        line(&vram, "amdgpu_partition_vram_used_bytes", l, s.partition_vram_used_bytes[p]);
    }
    if (!info.empty()) {
      append_header(&o, "amdgpu_partition_info",
                    "Advertised compute partition -> kubelet device id / resource (value 1).", "gauge");
      o.append(info);
    }
    if (!busy.empty()) {
      append_header(&o, "amdgpu_partition_gfx_busy_percent",
                    "Per-partition (XCP) compute busy: from the partition's own metrics "
                    "(amdsmi_get_gpu_partition_metrics_info) or the socket blob's xcp_stats.",
                    "gauge");
      o.append(busy);
    }
    if (!vram.empty()) {
      append_header(&o, "amdgpu_partition_vram_used_bytes", "Per-partition VRAM in use.", "gauge");
      o.append(vram);
    }
  }
  auto p = std::make_shared<const std::string>(std::move(o));
  std::lock_guard<std::mutex> lk(mu_);
  gpu_text_ = p;
  publish_view_locked();
}

std::shared_ptr<const std::string> Exporter::gpu_text() const {
  std::lock_guard<std::mutex> lk(mu_);
  return gpu_text_;
}

GpuSample Exporter::last_sample(int gpu) const {
  std::lock_guard<std::mutex> lk(mu_);  // `gpu` is the backend (node) index
  for (size_t g = 0; g < gpus_.size() && g < last_.size(); ++g)
    if (gpus_[g].index == gpu) return last_[g];
  return GpuSample{};
}

void Exporter::render_process_cached(std::string* out) const {
  TlCache& c = tl_cache();
  const int64_t now = mono_ns();
  if (c.proc.empty() || now - c.proc_ns >= 1000000000LL) {  // /proc reads cached 1 s
    c.proc.clear();
    render_process(&c.proc);
    c.proc_ns = now;
  }
  out->append(c.proc);
}

void Exporter::render_process(std::string* out) const {
  std::string& o = *out;
  double utime = 0, stime = 0, vsize = 0, rss = 0;
  long long starttime = 0;
  {
    std::ifstream f("/proc/self/stat");
    std::string s((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
    const size_t rp = s.rfind(')');
    if (rp != std::string::npos) {
      std::vector<std::string> fields;
      size_t i = rp + 2;
      while (i < s.size()) {
        size_t j = s.find(' ', i);
        if (j == std::string::npos) j = s.size();
        fields.push_back(s.substr(i, j - i));
        i = j + 1;
      }
      // fields[0] = state (field 3); utime=14, stime=15, starttime=22, vsize=23, rss=24
      if (fields.size() > 22) {
        const double hz = static_cast<double>(sysconf(_SC_CLK_TCK));
        utime = std::stod(fields[11]) / hz;
        stime = std::stod(fields[12]) / hz;
        starttime = std::stoll(fields[19]);
        vsize = std::stod(fields[20]);
        rss = std::stod(fields[21]) * sysconf(_SC_PAGESIZE);
        (void)starttime;
      }
    }
  }
  int fds = 0;
  if (DIR* d = opendir("/proc/self/fd")) {
    while (readdir(d)) ++fds;
    closedir(d);
    fds -= 3;  // ., .., the dir fd itself
  }
  struct rlimit rl {};
  getrlimit(RLIMIT_NOFILE, &rl);
  append_header(&o, "process_cpu_seconds_total", "Total user and system CPU time spent in seconds.", "counter");
  o.append("process_cpu_seconds_total ");
  append_float(&o, utime + stime);
  o.push_back('\n');
  append_header(&o, "process_resident_memory_bytes", "Resident memory size in bytes.", "gauge");
  o.append("process_resident_memory_bytes ");
  append_float(&o, rss);
  o.push_back('\n');
  append_header(&o, "process_virtual_memory_bytes", "Virtual memory size in bytes.", "gauge");
  o.append("process_virtual_memory_bytes ");
  append_float(&o, vsize);
  o.push_back('\n');
  append_header(&o, "process_open_fds", "Number of open file descriptors.", "gauge");
  o.append("process_open_fds ");
  append_float(&o, fds);
  o.push_back('\n');
  append_header(&o, "process_max_fds", "Maximum number of open file descriptors.", "gauge");
  o.append("process_max_fds ");
  append_float(&o, static_cast<double>(rl.rlim_cur));
  o.push_back('\n');
  append_header(&o, "process_start_time_seconds", "Start time of the process since unix epoch in seconds.", "gauge");
  o.append("process_start_time_seconds ");
  append_float(&o, static_cast<double>(start_time_s_));
  o.push_back('\n');
}

// The exposition is assembled from segments so the gzip path can cache the big,
// slowly-changing ones: [inventory + per-tick GPU text] changes once per sampling
// tick, [device health] once per table version; the rest is small and per-scrape.
void Exporter::render_parts(std::string_view* head, std::string* counters, std::string_view* health,
                            std::string* tail, std::shared_ptr<const std::string>* head_sp,
                            std::shared_ptr<const std::string>* health_sp) const {
  note_read();
  TlCache& c = tl_cache();
  const uint64_t gen = view_gen_.load(std::memory_order_acquire);
  if (!c.view || c.view_gen != gen) {
    c.view = view();
    c.view_gen = gen;
  }
  const ScrapeView& v = *c.view;
  const auto& tables = v.tables;
  *head = *v.head;
  if (head_sp) *head_sp = v.head;
  append_header(counters, "amdgpu_telemetry_samples_total", "Telemetry sampling passes completed.", "counter");
  counters->append("amdgpu_telemetry_samples_total ");
  append_u64(counters, samples_.load());
  counters->push_back('\n');
  append_header(counters, "amdgpu_telemetry_sample_errors_total", "Per-GPU telemetry sample failures.", "counter");
  counters->append("amdgpu_telemetry_sample_errors_total ");
  append_u64(counters, sample_errors_.load());
  counters->push_back('\n');
  if (const int cur = current_interval_ms_.load()) {
    append_header(counters, "amdgpu_telemetry_interval_seconds",
                  "The sampler's current period (telemetry.intervalMs, or idleIntervalMs while unread and settled).",
                  "gauge");
    counters->append("amdgpu_telemetry_interval_seconds ");
    append_float(counters, cur * 1e-3);
    counters->push_back('\n');
  }
  if (const int64_t last = last_pass_ns_.load()) {
    append_header(counters, "amdgpu_telemetry_last_pass_age_seconds",
                  "Seconds since the sampler last completed a pass over all GPUs.", "gauge");
    counters->append("amdgpu_telemetry_last_pass_age_seconds ");
    append_float(counters, (mono_ns() - last) * 1e-9);
    counters->push_back('\n');
  }
  {
    std::shared_ptr<const Freshness> f;
    std::shared_ptr<const Stalls> st;
    {
      std::lock_guard<SpinLock> lk(fresh_lock_);
      f = fresh_;
      st = stalls_;
    }
    if (!f->last_ok.empty()) {
      append_header(counters, "amdgpu_telemetry_sample_age_seconds",
                    "Seconds since the GPU's last successful telemetry sample.", "gauge");
      const int64_t now = mono_ns();
      for (const auto& kv : f->last_ok) {
        if (!kv.second) continue;
        counters->append("amdgpu_telemetry_sample_age_seconds{gpu=\"");
        append_u64(counters, static_cast<uint64_t>(kv.first));
        counters->append("\"} ");
        append_float(counters, (now - kv.second) * 1e-9);
        counters->push_back('\n');
      }
    }
    if (!st->stalled.empty()) {
      append_header(counters, "amdgpu_telemetry_sample_stalled",
                    "1 while a hardware call of the GPU has been in flight longer than health.sampleStallS.", "gauge");
      for (int g : st->stalled) {
        counters->append("amdgpu_telemetry_sample_stalled{gpu=\"");
        append_u64(counters, static_cast<uint64_t>(g));
        counters->append("\"} 1\n");
      }
    }
    if (!st->blocked.empty()) {
      append_header(counters, "amdgpu_telemetry_sample_blocked",
                    "1 while the GPU's hardware call waits behind another GPU's stalled call.", "gauge");
      for (int g : st->blocked) {
        counters->append("amdgpu_telemetry_sample_blocked{gpu=\"");
        append_u64(counters, static_cast<uint64_t>(g));
        counters->append("\"} 1\n");
      }
    }
  }
  if (sample_hist_.count()) {
    append_header(counters, "amdgpu_telemetry_sample_duration_seconds", "Wall time of one sampling pass over all GPUs.",
                  "histogram");
    sample_hist_.render(counters, "amdgpu_telemetry_sample_duration_seconds", "");
  }
  *health = std::string_view();
  if (health_sp) health_sp->reset();
  if (!tables.empty()) {
    // device-health block: re-rendered only when a table's version moves
    bool same = c.health && c.health_key.size() == tables.size() * 2;
    for (size_t i = 0; same && i < tables.size(); ++i)
      same = c.health_key[2 * i] == reinterpret_cast<uintptr_t>(tables[i].get()) &&
             c.health_key[2 * i + 1] == tables[i]->version();
    if (!same) {
      c.health_key.clear();
      for (const auto& t : tables) {  // versions read before the text: never newer than it
        c.health_key.push_back(reinterpret_cast<uintptr_t>(t.get()));
        c.health_key.push_back(t->version());
      }
      std::shared_ptr<const HealthShared> shared;
      {
        std::lock_guard<SpinLock> lk(health_lock_);
        shared = health_shared_;
      }
      if (shared && shared->key == c.health_key) {
        c.health = shared->text;  // another thread rendered this version already
        same = true;
      }
    }
    if (!same) {
      auto hc = std::make_shared<std::string>();
      append_header(hc.get(), "amdgpu_device_plugin_device_health",
                    "1 if the advertised device is Healthy, 0 if Unhealthy.", "gauge");
      std::string l;
      for (const auto& t : tables) {
        for (size_t i = 0; i < t->size(); ++i) {
          const TableDevice& d = t->device(i);
          l.assign("resource=\"");
          append_label_value(&l, t->config().resource_name);
          l.append("\",device_id=\"");
          append_label_value(&l, d.id);
          l.append("\"");
          line(hc.get(), "amdgpu_device_plugin_device_health", l, t->healthy(d.id) ? 1 : 0);
        }
      }
      c.health = std::move(hc);
      auto fresh = std::make_shared<HealthShared>();
      fresh->key = c.health_key;
      fresh->text = c.health;
      std::shared_ptr<const HealthShared> old;
      std::lock_guard<SpinLock> lk(health_lock_);
      old.swap(health_shared_);
      health_shared_ = std::move(fresh);
    }
    *health = *c.health;
    if (health_sp) *health_sp = c.health;
    // RPC histograms: between kubelet RPCs (scrapes come far more often) their text does
    // not change; it is rendered again only when a table's observation count moves
    // (versions read before the text, so a cached text is never older than its key)
    bool same_tables = c.tables_key.size() == tables.size() * 2;
    for (size_t i = 0; same_tables && i < tables.size(); ++i)
      same_tables = c.tables_key[2 * i] == reinterpret_cast<uintptr_t>(tables[i].get()) &&
                    c.tables_key[2 * i + 1] == tables[i]->metrics_version();
    if (!same_tables) {
      c.tables_key.clear();
      for (const auto& t : tables) {
        c.tables_key.push_back(reinterpret_cast<uintptr_t>(t.get()));
        c.tables_key.push_back(t->metrics_version());
      }
      c.tables_text.clear();
      bool any = false;
      for (const auto& t : tables) {
        const size_t before = c.tables_text.size();
        if (!any) DeviceTable::render_metric_headers(&c.tables_text);
        const size_t body = c.tables_text.size();
        t->render_metrics(&c.tables_text, false);
        if (c.tables_text.size() == body) {
          c.tables_text.resize(before);  // nothing observed yet: no headers either
          continue;
        }
        any = true;
      }
    }
    tail->append(c.tables_text);
  }
  tail->append(*v.extra);
  render_process_cached(tail);
}

void Exporter::render(std::string* out) const {
  Exposition e;
  render(&e);
  e.append_to(out);
}

void Exporter::render(Exposition* e) const { render_parts(&e->head, &e->counters, &e->health, &e->tail); }

void Exporter::render_gzip(std::string* out, std::string_view trailer) const {
  std::shared_ptr<const std::string> head, health;
  std::string_view hv, lv;
  std::string dyn, tail, gz_health;
  render_parts(&hv, &dyn, &lv, &tail, &head, &health);
  {
    std::lock_guard<std::mutex> lk(gz_mu_);
    if (gz_head_src_ != head) {
      gz_head_.clear();
      gzip_member(head->data(), head->size(), &gz_head_);
      gz_head_src_ = head;
    }
    out->append(gz_head_);
    if (health) {
      if (gz_health_src_ != health) {
        gz_health_.clear();
        gzip_member(health->data(), health->size(), &gz_health_);
        gz_health_src_ = health;
      }
      gz_health = gz_health_;  // the member of this scrape's health text, not a later one's
    }
  }
  // members must follow the plain-text order: head, counters, health, tail + trailer
  gzip_member(dyn.data(), dyn.size(), out);
  out->append(gz_health);
  tail.append(trailer.data(), trailer.size());
  gzip_member(tail.data(), tail.size(), out);
}

}  // namespace amdgpu_dp
