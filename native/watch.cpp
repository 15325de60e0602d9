#include "watch.h"

#include <errno.h>
#include <poll.h>
#include <sys/inotify.h>
#include <unistd.h>

#include <cstring>
#include <stdexcept>

namespace amdgpu_dp {

bool FsEvent::create() const { return mask & (IN_CREATE | IN_MOVED_TO); }
bool FsEvent::remove() const { return mask & (IN_DELETE | IN_MOVED_FROM); }

DirWatcher::DirWatcher(const std::string& dir) : dir_(dir) {
  fd_ = inotify_init1(IN_NONBLOCK | IN_CLOEXEC);
  if (fd_ < 0) throw std::runtime_error(std::string("inotify_init1: ") + strerror(errno));
  wd_ = inotify_add_watch(fd_, dir.c_str(), IN_CREATE | IN_DELETE | IN_MOVED_TO | IN_MOVED_FROM);
  if (wd_ < 0) {
    const int e = errno;
    ::close(fd_);
    fd_ = -1;
    throw std::runtime_error("inotify_add_watch(" + dir + "): " + strerror(e));
  }
}

DirWatcher::~DirWatcher() { close(); }

void DirWatcher::close() {
  if (fd_ >= 0) ::close(fd_);
  fd_ = -1;
}

std::vector<FsEvent> DirWatcher::read(int timeout_ms) {
  std::vector<FsEvent> out;
  if (fd_ < 0) return out;
  struct pollfd p {fd_, POLLIN, 0};
  if (poll(&p, 1, timeout_ms) <= 0) return out;
  alignas(struct inotify_event) char buf[8192];
  for (;;) {
    const ssize_t n = ::read(fd_, buf, sizeof(buf));
    if (n <= 0) break;
    for (char* q = buf; q < buf + n;) {
      auto* ev = reinterpret_cast<struct inotify_event*>(q);
      FsEvent e;
      e.mask = ev->mask;
      if (ev->len) e.name = ev->name;
      out.push_back(std::move(e));
      q += sizeof(struct inotify_event) + ev->len;
    }
  }
  return out;
}

}  // namespace amdgpu_dp
