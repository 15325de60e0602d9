#include <fcntl.h>
#include <sys/socket.h>
#include <time.h>
#include <unistd.h>

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
    default: return "none";
  }
}

}  // namespace amdgpu_dp
