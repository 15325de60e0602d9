#include <fcntl.h>
#include <pthread.h>
#include <sched.h>
#include <sys/socket.h>
#include <time.h>
#include <unistd.h>

#include <atomic>
#include <cerrno>
#include <ctime>

#include "backend.h"

namespace amdgpu_dp {

int64_t now_ns() {
  struct timespec ts;
  clock_gettime(CLOCK_REALTIME, &ts);
  return static_cast<int64_t>(ts.tv_sec) * 1000000000LL + ts.tv_nsec;
}

int accept_or_shed(int lfd, struct sockaddr* addr, socklen_t* len, int* spare, bool* shed) {
  *shed = false;
  if (*spare < 0) *spare = open("/dev/null", O_RDONLY | O_CLOEXEC);
  const int fd = accept4(lfd, addr, len, SOCK_NONBLOCK | SOCK_CLOEXEC);
  if (fd >= 0 || (errno != EMFILE && errno != ENFILE)) return fd;
  if (*spare < 0) {  // no reserve to give up (ENFILE): back off instead of spinning
    struct timespec ts {0, 1000000};
    nanosleep(&ts, nullptr);
    errno = EAGAIN;
    return -1;
  }
  close(*spare);
  *spare = -1;
  const int victim = accept4(lfd, nullptr, nullptr, SOCK_CLOEXEC);
  if (victim >= 0) close(victim);
  *spare = open("/dev/null", O_RDONLY | O_CLOEXEC);
  *shed = victim >= 0;
  errno = victim >= 0 ? ECONNABORTED : EAGAIN;
  return -1;
}

int64_t mono_ns() {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return static_cast<int64_t>(ts.tv_sec) * 1000000000LL + ts.tv_nsec;
}

namespace {
std::atomic<bool> g_background_batch{false};
std::atomic<int64_t> g_background_batched{0};
}  // namespace

void set_background_batch(bool on) { g_background_batch.store(on, std::memory_order_relaxed); }
bool background_batch() { return g_background_batch.load(std::memory_order_relaxed); }
int64_t background_batched_threads() { return g_background_batched.load(std::memory_order_relaxed); }

void background_thread(const char* name) {
  if (name && *name) pthread_setname_np(pthread_self(), name);
  if (!g_background_batch.load(std::memory_order_relaxed)) return;
  struct sched_param sp {};
  sp.sched_priority = 0;
  // a non-real-time policy change needs no privilege; failure leaves SCHED_OTHER
  if (pthread_setschedparam(pthread_self(), SCHED_BATCH, &sp) == 0)
    g_background_batched.fetch_add(1, std::memory_order_relaxed);
}

void foreground_thread() {
  // threads inherit the creator's policy: a server started from a batch thread must not
  // serve as one
  if (sched_getscheduler(0) != SCHED_BATCH) return;
  struct sched_param sp {};
  pthread_setschedparam(pthread_self(), SCHED_OTHER, &sp);
}

const char* event_kind_name(int kind) {
  switch (kind) {
    case kEvtPreReset: return "gpu_pre_reset";
    case kEvtPostReset: return "gpu_post_reset";
    case kEvtEccUncorrectable: return "ecc_uncorrectable";
    case kEvtLinkDown: return "xgmi_link_down";
    case kEvtLinkUp: return "xgmi_link_up";
    case kEvtThermal: return "thermal_throttle";
    case kEvtVmFault: return "vm_fault";
    case kEvtDeviceLost: return "device_lost";
    case kEvtDeviceRecovered: return "device_recovered";
    case kEvtRetiredPagesExceeded: return "retired_pages_threshold";
    case kEvtRetiredPagesCleared: return "retired_pages_below_threshold";
    case kEvtLinkQuality: return "xgmi_link_bandwidth_changed";
    case kEvtPcieDegraded: return "pcie_link_degraded";
    case kEvtPcieRestored: return "pcie_link_restored";
    case kEvtResetObserved: return "gpu_reset_observed";
    case kEvtResetCandidate: return "gpu_reset_candidate";
    case kEvtLatchCleared: return "health_latch_cleared";
    default: return "none";
  }
}

}  // namespace amdgpu_dp
