// Per-device owner threads for hardware calls (SURVEY.md §7.5 hard parts 5 and 6).
//
// The reference calls NVML straight from whichever goroutine needs it (device/device.go:
// 37-181, plugin/plugin.go:259-264); nothing bounds a call that never returns.  Here
// every call that touches one GPU runs on that GPU's *lane*: one owner thread per
// physical GPU, keyed by the GPU's identity.  Callers post a job and wait for it with a
// bound of their own; a caller that stops waiting leaves the job to finish (or not) on
// the lane, never on its own stack.  So:
//   * a wedged driver call blocks one lane, not the sampler, the discovery or the manager;
//   * calls to different GPUs run in parallel (an 8-GPU sampling pass costs one GPU's);
//   * per-GPU caches are touched by one thread only;
//   * a lane whose call has been in flight past the stall threshold takes no more work:
//     nothing piles up behind a wedge, and every caller learns at once that the GPU is
//     unresponsive (LaneState says since when, and in which call).
#pragma once

#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace amdgpu_dp {

int64_t mono_ns();

// One posted call.  The submitter keeps a reference and may wait for it (bounded); the
// lane keeps one until the call has run.  Everything the call reads or writes must be
// owned by the closure (shared_ptr captures), never by the submitter's stack.
class LaneJob {
 public:
  // batch: jobs posted to several lanes at once by one caller (a discovery's describes)
  // share a nonzero batch; 0 = a job posted on its own
  LaneJob(std::string what, std::function<void()> fn, uint64_t batch = 0)
      : what_(std::move(what)), fn_(std::move(fn)), batch_(batch) {}
  // true once the call has run (or was dropped, see dropped()); waits at most ms (< 0: forever)
  bool wait(int64_t ms);
  bool done() const { return done_.load(std::memory_order_acquire); }
  // the lane shut down (or refused it) before the call ran: its outputs were never written
  bool dropped() const { return dropped_.load(std::memory_order_acquire); }
  const std::string& what() const { return what_; }
  uint64_t batch() const { return batch_; }
  int64_t started_ns() const { return started_ns_.load(); }
  int64_t finished_ns() const { return finished_ns_.load(); }
  // the call threw (the lane caught it and carried on); valid once done()
  bool failed() const { return !error_.empty(); }
  const std::string& error() const { return error_; }

 private:
  friend class Lane;
  void run();
  void drop();
  void finish();
  std::string what_;
  std::function<void()> fn_;
  const uint64_t batch_;
  std::string error_;  // written before done_ is released
  std::mutex mu_;
  std::condition_variable cv_;
  std::atomic<bool> done_{false};
  std::atomic<bool> dropped_{false};
  std::atomic<int64_t> started_ns_{0}, finished_ns_{0};
};

struct LaneState {
  std::string key;
  int64_t inflight_since_ns = 0;  // 0 = idle
  std::string inflight_what;
  uint64_t inflight_batch = 0;    // LaneJob::batch of the call in flight
  uint64_t completed = 0;         // calls run to completion
  int64_t last_done_ns = 0;       // mono ns the last call ended
  size_t queued = 0;
  int64_t age_ns(int64_t now) const { return inflight_since_ns ? now - inflight_since_ns : 0; }
};

class Lane {
 public:
  explicit Lane(std::string key);
  ~Lane();  // ends the thread; a thread stuck in a call is left to end with it
  Lane(const Lane&) = delete;
  Lane& operator=(const Lane&) = delete;

  // Queues `job`.  Refused (false, job marked dropped) when the lane's current call has
  // been in flight longer than busy_ns (> 0): the device is unresponsive and a job queued
  // behind it would only wait too; or when kMaxQueued jobs already wait.
  static constexpr size_t kMaxQueued = 16;
  bool post(const std::shared_ptr<LaneJob>& job, int64_t busy_ns);
  LaneState state() const;
  const std::string& key() const { return key_; }

 private:
  struct Shared {
    std::mutex mu;
    std::condition_variable cv;
    std::deque<std::shared_ptr<LaneJob>> queue;
    bool stop = false;
    std::shared_ptr<LaneJob> inflight;
    int64_t inflight_since = 0;
    uint64_t completed = 0;
    int64_t last_done = 0;
  };
  static void loop(std::shared_ptr<Shared> s);
  std::string key_;
  std::shared_ptr<Shared> s_;
  std::thread thread_;
};

// Lanes by device identity, created on first use.  A GPU that left the inventory keeps
// its lane (a call may still be stuck on it) until prune() finds it idle.
class LaneSet {
 public:
  std::shared_ptr<Lane> get(const std::string& key);
  std::shared_ptr<Lane> find(const std::string& key) const;  // null if none
  // Drops idle lanes whose key is not in `keep`.
  void prune(const std::vector<std::string>& keep);
  std::vector<LaneState> states() const;
  size_t size() const;

 private:
  mutable std::mutex mu_;
  std::map<std::string, std::shared_ptr<Lane>> lanes_;
};

// Gate around a hardware-library session: calls enter() and leave(); a re-initialisation
// (amdsmi_shut_down + amdsmi_init, which invalidates every handle) closes the gate, waits
// a bounded time for the calls inside to leave, and fails instead of waiting behind a call
// that never returns.  Each successful close ends a session: a call carrying the number
// of an older session is refused (its handles belong to the old one).
class SessionGate {
 public:
  // false: the gate belongs to another session than `session` (stale handles)
  bool enter(uint64_t session);
  void leave();
  // Closes the gate once no call is inside (waits at most ms).  false: a call stayed
  // inside, the gate is open again and the session unchanged.
  bool close(int64_t ms);
  // Reopens a closed gate as a new session; returns its number.
  uint64_t reopen();
  uint64_t session() const { return session_.load(); }
  int active() const;

 private:
  mutable std::mutex mu_;
  std::condition_variable cv_;
  bool closing_ = false;
  int active_ = 0;
  std::atomic<uint64_t> session_{1};
};

}  // namespace amdgpu_dp
