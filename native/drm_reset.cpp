#include "drm_reset.h"

#include <drm/amdgpu_drm.h>
#include <errno.h>
#include <fcntl.h>
#include <sys/ioctl.h>
#include <unistd.h>

#include <cstring>

#include "backend.h"

namespace amdgpu_dp {

namespace {
constexpr int64_t kRetryNs = 60'000'000'000LL;  // a node that cannot be opened: try again in a minute

int ctx_ioctl(int fd, union drm_amdgpu_ctx* a) {
  int r;
  do {
    r = ioctl(fd, DRM_IOCTL_AMDGPU_CTX, a);
  } while (r != 0 && (errno == EINTR || errno == EAGAIN));
  return r;
}
}  // namespace

DrmResetWatch::~DrmResetWatch() { close_node(); }

bool DrmResetWatch::open_node() {
  fd_ = ::open(path_.c_str(), O_RDWR | O_CLOEXEC);
  if (fd_ < 0) {
    err_ = "open " + path_ + ": " + std::strerror(errno);
    return false;
  }
  union drm_amdgpu_ctx a;
  std::memset(&a, 0, sizeof(a));
  a.in.op = AMDGPU_CTX_OP_ALLOC_CTX;
  a.in.priority = AMDGPU_CTX_PRIORITY_NORMAL;
  if (ctx_ioctl(fd_, &a) != 0) {
    err_ = "amdgpu context on " + path_ + ": " + std::strerror(errno);
    ::close(fd_);
    fd_ = -1;
    return false;
  }
  ctx_ = a.out.alloc.ctx_id;  // its reset baseline is the device's counter now
  err_.clear();
  return true;
}

void DrmResetWatch::close_node() {
  if (fd_ < 0) return;
  union drm_amdgpu_ctx a;
  std::memset(&a, 0, sizeof(a));
  a.in.op = AMDGPU_CTX_OP_FREE_CTX;
  a.in.ctx_id = ctx_;
  (void)ctx_ioctl(fd_, &a);
  ::close(fd_);
  fd_ = -1;
}

int64_t DrmResetWatch::poll() {
  if (fd_ < 0) {
    const int64_t now = mono_ns();
    if (now < retry_at_ns_) return -1;
    if (!open_node()) {
      retry_at_ns_ = now + kRetryNs;
      return -1;
    }
  }
  union drm_amdgpu_ctx a;
  std::memset(&a, 0, sizeof(a));
  a.in.op = AMDGPU_CTX_OP_QUERY_STATE;  // "a reset since the last query", re-armed by the query
  a.in.ctx_id = ctx_;
  if (ctx_ioctl(fd_, &a) != 0) {
    err_ = "query on " + path_ + ": " + std::strerror(errno);
    close_node();
    retry_at_ns_ = mono_ns() + kRetryNs;
    return -1;
  }
  if (a.out.state.reset_status != AMDGPU_CTX_NO_RESET) ++count_;
  return count_;
}

}  // namespace amdgpu_dp
