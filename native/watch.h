// inotify directory watcher (reference: modules/watch/watch.go:11-26 via fsnotify;
// consumed at plugin/manager.go:80-84 to detect kubelet restarts by the CREATE of
// kubelet.sock).  Blocking reads with a timeout so the caller's thread can stop.
#pragma once

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
  void close();
  const std::string& dir() const { return dir_; }

 private:
  std::string dir_;
  int fd_ = -1;
  int wd_ = -1;
};

}  // namespace amdgpu_dp
