#include "watch.h"

#include <dirent.h>
#include <errno.h>
#include <poll.h>
#include <sys/eventfd.h>
#include <sys/inotify.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cstring>
#include <stdexcept>

namespace amdgpu_dp {

bool FsEvent::create() const { return mask & (IN_CREATE | IN_MOVED_TO); }
bool FsEvent::remove() const { return mask & (IN_DELETE | IN_MOVED_FROM); }

namespace {
constexpr uint32_t kWatchMask = IN_CREATE | IN_DELETE | IN_MOVED_TO | IN_MOVED_FROM | IN_DELETE_SELF | IN_MOVE_SELF;
}  // namespace

DirWatcher::DirWatcher(const std::string& dir) : dir_(dir) {
  fd_ = inotify_init1(IN_NONBLOCK | IN_CLOEXEC);
  if (fd_ < 0) throw std::runtime_error(std::string("inotify_init1: ") + strerror(errno));
  efd_ = eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);
  wd_ = inotify_add_watch(fd_, dir.c_str(), kWatchMask);
  struct stat st;
  if (wd_ >= 0 && ::stat(dir.c_str(), &st) == 0) {
    dev_ = st.st_dev;
    ino_ = st.st_ino;
  }
  if (wd_ < 0) {
    const int e = errno;
    ::close(fd_);
    fd_ = -1;
    if (efd_ >= 0) ::close(efd_);
    efd_ = -1;
    throw std::runtime_error("inotify_add_watch(" + dir + "): " + strerror(e));
  }
}

DirWatcher::~DirWatcher() { close(); }

void DirWatcher::close() {
  if (fd_ >= 0) ::close(fd_);
  fd_ = -1;
  std::lock_guard<std::mutex> lk(efd_mu_);
  if (efd_ >= 0) ::close(efd_);
  efd_ = -1;
}

void DirWatcher::wake() {
  std::lock_guard<std::mutex> lk(efd_mu_);
  if (efd_ < 0) return;
  const uint64_t one = 1;
  (void)!::write(efd_, &one, sizeof(one));
}

// The watched directory itself can go away (a node agent that wipes
// /var/lib/kubelet/device-plugins, a kubelet that recreates it), and the watch then sees
// nothing that happens in the new directory.  The kernel's IN_DELETE_SELF cannot be
// relied on to say so: it fires only when the last reference to the old directory goes,
// and the plugin's own bound socket in it (unlinked, still listening) is such a
// reference until the plugin re-registers, which it would only do after seeing the new
// kubelet.sock.  So whenever a read times out the watcher checks that the path still
// names the inode it watches (one stat per timeout), and after a removal or rename
// re-adds the watch once the directory exists again, reporting everything already in it
// as created so that a kubelet.sock that appeared in between is not missed.
bool DirWatcher::same_dir() const {
  struct stat st;
  return ::stat(dir_.c_str(), &st) == 0 && static_cast<uint64_t>(st.st_dev) == dev_ &&
         static_cast<uint64_t>(st.st_ino) == ino_;
}

bool DirWatcher::rewatch(std::vector<FsEvent>* out) {
  struct stat st;
  if (::stat(dir_.c_str(), &st) != 0 || !S_ISDIR(st.st_mode)) return false;
  wd_ = inotify_add_watch(fd_, dir_.c_str(), kWatchMask);
  if (wd_ < 0) return false;
  dev_ = st.st_dev;
  ino_ = st.st_ino;
  if (DIR* d = opendir(dir_.c_str())) {
    while (struct dirent* de = readdir(d)) {
      if (std::strcmp(de->d_name, ".") == 0 || std::strcmp(de->d_name, "..") == 0) continue;
      FsEvent e;
      e.mask = IN_CREATE;
      e.name = de->d_name;
      out->push_back(std::move(e));
    }
    closedir(d);
  }
  return true;
}

std::vector<FsEvent> DirWatcher::read(int timeout_ms) {
  std::vector<FsEvent> out;
  if (fd_ < 0) return out;
  if (wd_ < 0 && rewatch(&out)) return out;
  struct pollfd p[2] = {{fd_, POLLIN, 0}, {efd_, POLLIN, 0}};
  const int np = poll(p, efd_ >= 0 ? 2 : 1, timeout_ms);
  if (np > 0 && efd_ >= 0 && (p[1].revents & POLLIN)) {  // wake()
    uint64_t x;
    while (::read(efd_, &x, sizeof(x)) > 0) {
    }
    return out;
  }
  if (np <= 0) {  // (watch gone: this is the retry pause)
    if (wd_ >= 0 && !same_dir()) {
      inotify_rm_watch(fd_, wd_);  // its IN_IGNORED is skipped below
      wd_ = -1;
      rewatch(&out);
    }
    return out;
  }
  alignas(struct inotify_event) char buf[8192];
  for (;;) {
    const ssize_t n = ::read(fd_, buf, sizeof(buf));
    if (n <= 0) break;
    for (char* q = buf; q < buf + n;) {
      auto* ev = reinterpret_cast<struct inotify_event*>(q);
      q += sizeof(struct inotify_event) + ev->len;
      if (ev->wd == wd_ && (ev->mask & (IN_IGNORED | IN_DELETE_SELF | IN_MOVE_SELF))) {
        if (ev->mask & IN_MOVE_SELF) {
          // renamed away: the watch would follow the old inode, not the path
          inotify_rm_watch(fd_, wd_);
          wd_ = -1;
        }
        if (ev->mask & IN_IGNORED) wd_ = -1;  // the kernel dropped the watch
        continue;
      }
      if (ev->mask & IN_IGNORED) continue;  // a watch we already gave up
      FsEvent e;
      e.mask = ev->mask;
      if (ev->len) e.name = ev->name;
      out.push_back(std::move(e));
    }
  }
  return out;
}

}  // namespace amdgpu_dp
