// inotify directory watcher (reference: modules/watch/watch.go:11-26 via fsnotify;
// consumed at plugin/manager.go:80-84 to detect kubelet restarts by the CREATE of
// kubelet.sock).  Blocking reads with a timeout, cut short by wake().  The
// watch survives the directory being removed and created again (see watch.cpp).
#pragma once

#include <cstdint>
#include <mutex>
#include <string>
#include <utility>
#include <vector>

namespace amdgpu_dp {

struct FsEvent {
  std::string name;  // file name inside the watched directory
  uint32_t mask = 0;
  bool create() const;
  bool remove() const;
};

class DirWatcher {
 public:
  explicit DirWatcher(const std::string& dir);  // throws on failure
  ~DirWatcher();
  std::vector<FsEvent> read(int timeout_ms);
  // Ends a read() in progress (or the next one) at once, with no events: lets the reading
  // thread sleep long between events and still stop promptly.  Safe from any thread, also
  // after close().
  void wake();
  void close();
  const std::string& dir() const { return dir_; }

 private:
  bool rewatch(std::vector<FsEvent>* out);  // re-adds a lost watch; reports existing entries
  bool same_dir() const;                     // the path still names the watched inode

  std::string dir_;
  int fd_ = -1;
  int wd_ = -1;
  int efd_ = -1;     // wake(): an eventfd read() polls next to the inotify descriptor
  std::mutex efd_mu_;  // wake() against close()
  uint64_t dev_ = 0, ino_ = 0;  // identity of the watched directory
};

}  // namespace amdgpu_dp
