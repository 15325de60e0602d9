#include <time.h>

#include "backend.h"

namespace amdgpu_dp {

int64_t now_ns() {
  struct timespec ts;
  clock_gettime(CLOCK_REALTIME, &ts);
  return static_cast<int64_t>(ts.tv_sec) * 1000000000LL + ts.tv_nsec;
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
    default: return "none";
  }
}

}  // namespace amdgpu_dp
