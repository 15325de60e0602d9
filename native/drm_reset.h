// GPU reset counter an unprivileged reader can poll: the amdgpu driver's own count of the
// resets it performed on a device, through an amdgpu context on the device's render node.
//
// AMDGPU_CTX_OP_QUERY_STATE answers whether the device's reset counter moved since the
// previous query on that context (and re-arms), for every reset the driver performs -
// mode-1 and mode-2 ASIC resets and the engine resets that keep the power-management
// firmware running (whose clock, GpuSample::fw_clock_s, therefore does not restart).
// Opening a render node needs no privileges, only the node in the container's device
// cgroup (CDI-injected, or a privileged pod); the default DaemonSet's hostPath mount of
// /dev/dri does not grant it, and then the watch reports "unavailable" (-1) and retries
// once a minute.
#pragma once

#include <cstdint>
#include <string>

namespace amdgpu_dp {

class DrmResetWatch {
 public:
  explicit DrmResetWatch(std::string render_path) : path_(std::move(render_path)) {}
  ~DrmResetWatch();
  DrmResetWatch(const DrmResetWatch&) = delete;
  DrmResetWatch& operator=(const DrmResetWatch&) = delete;
  // Resets seen since the watch first opened the node (monotonic), or -1 while the node
  // cannot be opened or queried.  One ioctl when open.
  int64_t poll();
  const std::string& path() const { return path_; }
  const std::string& error() const { return err_; }

 private:
  bool open_node();
  void close_node();
  std::string path_;
  int fd_ = -1;
  uint32_t ctx_ = 0;
  int64_t count_ = 0;
  int64_t retry_at_ns_ = 0;
  std::string err_;
};

}  // namespace amdgpu_dp
