#include "core_escape.h"

#include <dirent.h>
#include <fcntl.h>
#include <sched.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

namespace amdgpu_dp {

bool ContentionDetector::note(int64_t svc_ns, int64_t now_ns) {
  ring_[n_++] = svc_ns;
  if (n_ < kWindow) return false;
  n_ = 0;
  int64_t w[kWindow];
  std::copy(ring_, ring_ + kWindow, w);
  std::nth_element(w, w + kWindow / 2, w + kWindow);
  const int64_t m = w[kWindow / 2];
  last_median_ = m;
  if (best_ == 0 || m < best_) {
    best_ = m;
  } else {
    best_ = std::min(m, best_ + best_ / 256);  // drifts up 0.4 % a window: a host that got slower is learnt
  }
  if (m * 100 > best_ * kRatioPct) {
    ++strikes_;
  } else {
    strikes_ = 0;
  }
  if (strikes_ < kStrikes || now_ns - last_move_ < kMinGapNs) return false;
  strikes_ = 0;
  last_move_ = now_ns;
  return true;
}

std::vector<int> parse_cpu_list(const char* s) {
  std::vector<int> out;
  while (s && *s) {
    char* end = nullptr;
    const long a = std::strtol(s, &end, 10);
    if (end == s) break;
    long b = a;
    s = end;
    if (*s == '-') {
      ++s;
      b = std::strtol(s, &end, 10);
      if (end == s) break;
      s = end;
    }
    for (long c = a; c <= b && c - a < 4096; ++c) out.push_back(static_cast<int>(c));
    while (*s == ',' || *s == '\n' || *s == ' ') ++s;
  }
  return out;
}

namespace {

std::vector<int> read_list(const std::string& path) {
  char buf[4096];
  const int fd = ::open(path.c_str(), O_RDONLY | O_CLOEXEC);
  if (fd < 0) return {};
  const ssize_t r = ::read(fd, buf, sizeof(buf) - 1);
  ::close(fd);
  if (r <= 0) return {};
  buf[r] = 0;
  return parse_cpu_list(buf);
}

std::vector<int> l3_of(int cpu) {
  const std::string base = "/sys/devices/system/cpu/cpu" + std::to_string(cpu) + "/cache/index";
  for (int i = 0; i < 8; ++i) {
    char lvl[8] = {};
    const int fd = ::open((base + std::to_string(i) + "/level").c_str(), O_RDONLY | O_CLOEXEC);
    if (fd < 0) continue;
    const ssize_t r = ::read(fd, lvl, sizeof(lvl) - 1);
    ::close(fd);
    if (r > 0 && lvl[0] == '3') return read_list(base + std::to_string(i) + "/shared_cpu_list");
  }
  return {};
}

// the CPU a thread (its /proc/<pid>/task/<tid> directory) last ran on: field 39 of its
// stat, -1 unknown
long last_cpu_of(const std::string& task_dir) {
  char buf[1024];
  const int sfd = ::open((task_dir + "/stat").c_str(), O_RDONLY | O_CLOEXEC);
  if (sfd < 0) return -1;
  const ssize_t r = ::read(sfd, buf, sizeof(buf) - 1);
  ::close(sfd);
  if (r <= 0) return -1;
  buf[r] = 0;
  const char* p = std::strrchr(buf, ')');  // the command name may hold spaces
  if (!p) return -1;
  int field = 2;  // state is field 3
  for (const char* q = p + 1; *q; ++q)
    if (*q == ' ' && ++field == 39) return std::strtol(q + 1, nullptr, 10);
  return -1;
}

}  // namespace

bool peer_on_sibling(int fd, int cpu, int64_t now_ns) {
  thread_local int64_t last_scan = -1'000'000'000'000LL;
  if (fd < 0 || cpu < 0) return false;
  struct ucred cr {};
  socklen_t len = sizeof(cr);
  if (getsockopt(fd, SOL_SOCKET, SO_PEERCRED, &cr, &len) != 0 || cr.pid <= 0) return false;
  std::vector<int> sib = read_list("/sys/devices/system/cpu/cpu" + std::to_string(cpu) + "/topology/thread_siblings_list");
  sib.erase(std::remove(sib.begin(), sib.end(), cpu), sib.end());
  if (sib.empty()) return false;
  auto on_sib = [&](long c) { return c >= 0 && std::find(sib.begin(), sib.end(), static_cast<int>(c)) != sib.end(); };
  const std::string base = "/proc/" + std::to_string(cr.pid) + "/task";
  if (on_sib(last_cpu_of(base + "/" + std::to_string(cr.pid)))) return true;  // the main thread
  // every thread (kubelet-like clients call from any of theirs): at most every 100 ms
  if (now_ns != 0 && now_ns - last_scan < 100'000'000) return false;
  last_scan = now_ns;
  DIR* d = opendir(base.c_str());
  if (!d) return false;
  bool found = false;
  int seen = 0;
  while (const dirent* e = readdir(d)) {
    if (e->d_name[0] < '0' || e->d_name[0] > '9') continue;
    if (++seen > 1024) break;
    if (on_sib(last_cpu_of(base + "/" + e->d_name))) {
      found = true;
      break;
    }
  }
  closedir(d);
  return found;
}

int escape_core(unsigned rotate) {
  const int cpu = sched_getcpu();
  if (cpu < 0) return -1;
  const std::vector<int> sib =
      read_list("/sys/devices/system/cpu/cpu" + std::to_string(cpu) + "/topology/thread_siblings_list");
  if (sib.size() < 2) return -1;  // no SMT: no core to share
  cpu_set_t allowed;
  CPU_ZERO(&allowed);
  if (sched_getaffinity(0, sizeof(allowed), &allowed) != 0) return -1;
  std::vector<int> cand;
  for (const int c : l3_of(cpu))
    if (c >= 0 && c < CPU_SETSIZE && CPU_ISSET(c, &allowed) && std::find(sib.begin(), sib.end(), c) == sib.end())
      cand.push_back(c);
  if (cand.empty()) return -1;
  const int target = cand[rotate % cand.size()];
  cpu_set_t one;
  CPU_ZERO(&one);
  CPU_SET(target, &one);
  if (sched_setaffinity(0, sizeof(one), &one) != 0) return -1;  // moves this thread now
  (void)!sched_setaffinity(0, sizeof(allowed), &allowed);       // and leaves it there
  return target;
}

}  // namespace amdgpu_dp
