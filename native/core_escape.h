// Core-contention escape for the gRPC workers (grpc.coreEscape, off by default).
//
// A busy-polling worker that the scheduler woke on the SMT sibling of its client's CPU
// shares one core with it for the rest of the burst: on the MI355X hosts an Allocate then
// takes ~4.6 us instead of ~2.6, and the bare exchange 2.7 instead of 2.2
// (scripts/smt_probe.py).  ContentionDetector watches the worker's service time (request
// read -> answer sent) per 32-call window against its own best window, which drifts up
// 0.4 % a window so that a host that got slower for good is learnt.  Two windows in a row
// 35 % over it, at most once per 10 ms, and peer_on_sibling checks whether a thread of
// the client process last ran on the worker's SMT sibling; only then does the worker
// move itself to another core of its L3 (escape_core): pinned there for the move, then
// given its whole allowed set back, which leaves it where it is.  docs/ROUND6.md has the
// measurements, and why it stays off.
#pragma once

#include <cstdint>
#include <vector>

namespace amdgpu_dp {

class ContentionDetector {
 public:
  static constexpr int kWindow = 32;
  static constexpr int kRatioPct = 135;
  static constexpr int kStrikes = 2;
  static constexpr int64_t kMinGapNs = 10'000'000;
  // One call's service time; true when the worker should move now.
  bool note(int64_t svc_ns, int64_t now_ns);
  int64_t best_ns() const { return best_; }
  int64_t last_median_ns() const { return last_median_; }

 private:
  int64_t ring_[kWindow] = {};
  int n_ = 0;
  int64_t best_ = 0;
  int64_t last_median_ = 0;
  int strikes_ = 0;
  int64_t last_move_ = -kMinGapNs;  // (the first move is never held back)
};

// Tells the client's SMT sibling apart from other slowdowns before a move: does a thread
// of the process at the other end of unix socket `fd` (SO_PEERCRED) last run on an SMT
// sibling of `cpu`?  False when the peer is not visible in this PID namespace (kubelet
// seen from an unprivileged pod), so the check, and the move, never happen there.
bool peer_on_sibling(int fd, int cpu, int64_t now_ns = 0);

// Moves the calling thread to another core of its current CPU's L3 (an allowed CPU that
// is not an SMT sibling of the current one; `rotate` picks among them).  Returns the CPU
// moved to, or -1 (no SMT on this CPU, no other core allowed, or the move failed).
int escape_core(unsigned rotate);

// sysfs cpu list ("0-3,8,10-11") -> CPUs
std::vector<int> parse_cpu_list(const char* s);

}  // namespace amdgpu_dp
