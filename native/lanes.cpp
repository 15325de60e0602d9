#include "lanes.h"

#include <algorithm>
#include <chrono>

#include "backend.h"

namespace amdgpu_dp {

// ---------------------------------------------------------------- LaneJob

void LaneJob::run() {
  started_ns_.store(mono_ns());
  // a throwing call must not take the lane thread (and with it the process) down
  try {
    fn_();
  } catch (const std::exception& e) {
    error_ = e.what()[0] ? e.what() : "exception";
  } catch (...) {
    error_ = "unknown exception";
  }
  fn_ = nullptr;  // captures (and what they keep alive) go with the call, not with the job
  finish();
}

void LaneJob::drop() {
  fn_ = nullptr;
  dropped_.store(true, std::memory_order_release);
  finish();
}

void LaneJob::finish() {
  finished_ns_.store(mono_ns());
  {
    std::lock_guard<std::mutex> lk(mu_);
    done_.store(true, std::memory_order_release);
  }
  cv_.notify_all();
}

bool LaneJob::wait(int64_t ms) {
  if (done()) return true;
  std::unique_lock<std::mutex> lk(mu_);
  if (ms < 0) {
    cv_.wait(lk, [&] { return done(); });
    return true;
  }
  return cv_wait_ms(cv_, lk, ms, [&] { return done(); });
}

// ---------------------------------------------------------------- Lane

Lane::Lane(std::string key) : key_(std::move(key)), s_(std::make_shared<Shared>()) {
  thread_ = std::thread(loop, s_);
}

Lane::~Lane() {
  bool stuck;
  std::deque<std::shared_ptr<LaneJob>> left;
  {
    std::lock_guard<std::mutex> lk(s_->mu);
    s_->stop = true;
    stuck = s_->inflight != nullptr;
    left.swap(s_->queue);
  }
  s_->cv.notify_all();
  for (auto& j : left) j->drop();
  if (!thread_.joinable()) return;
  // The last reference to a lane can be dropped by a job's captures on the lane thread
  // itself; and a call that never returns must not hang whoever destroys the lane.  Either
  // way the thread owns its state (Shared) and ends on its own.
  if (stuck || thread_.get_id() == std::this_thread::get_id()) thread_.detach();
  else thread_.join();
}

void Lane::loop(std::shared_ptr<Shared> s) {
  background_thread("dplane");
  for (;;) {
    std::shared_ptr<LaneJob> job;
    {
      std::unique_lock<std::mutex> lk(s->mu);
      s->cv.wait(lk, [&] { return s->stop || !s->queue.empty(); });
      if (s->stop) return;
      job = std::move(s->queue.front());
      s->queue.pop_front();
      s->inflight = job;
      s->inflight_since = mono_ns();
    }
    job->run();
    std::lock_guard<std::mutex> lk(s->mu);
    s->inflight.reset();
    s->inflight_since = 0;
    ++s->completed;
    s->last_done = mono_ns();
  }
}

bool Lane::post(const std::shared_ptr<LaneJob>& job, int64_t busy_ns) {
  {
    std::lock_guard<std::mutex> lk(s_->mu);
    const bool wedged = busy_ns > 0 && s_->inflight && mono_ns() - s_->inflight_since > busy_ns;
    if (!s_->stop && !wedged && s_->queue.size() < kMaxQueued) {
      s_->queue.push_back(job);
      s_->cv.notify_one();
      return true;
    }
  }
  job->drop();
  return false;
}

LaneState Lane::state() const {
  LaneState st;
  st.key = key_;
  std::lock_guard<std::mutex> lk(s_->mu);
  st.inflight_since_ns = s_->inflight ? s_->inflight_since : 0;
  if (s_->inflight) {
    st.inflight_what = s_->inflight->what();
    st.inflight_batch = s_->inflight->batch();
  }
  st.completed = s_->completed;
  st.last_done_ns = s_->last_done;
  st.queued = s_->queue.size();
  return st;
}

// ---------------------------------------------------------------- LaneSet

std::shared_ptr<Lane> LaneSet::get(const std::string& key) {
  std::lock_guard<std::mutex> lk(mu_);
  auto& l = lanes_[key];
  if (!l) l = std::make_shared<Lane>(key);
  return l;
}

std::shared_ptr<Lane> LaneSet::find(const std::string& key) const {
  std::lock_guard<std::mutex> lk(mu_);
  auto it = lanes_.find(key);
  return it == lanes_.end() ? nullptr : it->second;
}

void LaneSet::prune(const std::vector<std::string>& keep) {
  std::vector<std::shared_ptr<Lane>> gone;  // destroyed outside mu_
  {
    std::lock_guard<std::mutex> lk(mu_);
    for (auto it = lanes_.begin(); it != lanes_.end();) {
      const bool kept = std::find(keep.begin(), keep.end(), it->first) != keep.end();
      if (!kept) {
        const LaneState st = it->second->state();
        if (st.inflight_since_ns == 0 && st.queued == 0) {
          gone.push_back(std::move(it->second));
          it = lanes_.erase(it);
          continue;
        }
      }
      ++it;
    }
  }
}

std::vector<LaneState> LaneSet::states() const {
  std::vector<std::shared_ptr<Lane>> ls;
  {
    std::lock_guard<std::mutex> lk(mu_);
    for (const auto& kv : lanes_) ls.push_back(kv.second);
  }
  std::vector<LaneState> out;
  for (const auto& l : ls) out.push_back(l->state());
  return out;
}

size_t LaneSet::size() const {
  std::lock_guard<std::mutex> lk(mu_);
  return lanes_.size();
}

// ---------------------------------------------------------------- SessionGate

bool SessionGate::enter(uint64_t session) {
  std::unique_lock<std::mutex> lk(mu_);
  cv_.wait(lk, [&] { return !closing_; });
  if (session != 0 && session != session_.load()) return false;
  ++active_;
  return true;
}

void SessionGate::leave() {
  {
    std::lock_guard<std::mutex> lk(mu_);
    --active_;
  }
  cv_.notify_all();
}

bool SessionGate::close(int64_t ms) {
  std::unique_lock<std::mutex> lk(mu_);
  if (closing_) return false;  // one re-initialisation at a time
  closing_ = true;
  if (cv_wait_ms(cv_, lk, ms, [&] { return active_ == 0; })) return true;
  closing_ = false;
  lk.unlock();
  cv_.notify_all();
  return false;
}

uint64_t SessionGate::reopen() {
  uint64_t s;
  {
    std::lock_guard<std::mutex> lk(mu_);
    closing_ = false;
    s = session_.fetch_add(1) + 1;
  }
  cv_.notify_all();
  return s;
}

int SessionGate::active() const {
  std::lock_guard<std::mutex> lk(mu_);
  return active_;
}

}  // namespace amdgpu_dp
