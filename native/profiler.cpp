#include "profiler.h"

#include <dlfcn.h>
#include <signal.h>
#include <sys/time.h>
#include <time.h>
#include <ucontext.h>

#include <algorithm>
#include <atomic>
#include <cstring>
#include <mutex>
#include <unordered_map>

namespace amdgpu_dp {
namespace prof {

namespace {

constexpr size_t kCapacity = 1u << 20;  // ~17 min at 1 kHz of one busy core
// Slots are atomics: the handler may still be writing one (a signal in flight while stop()
// runs, or histogram() read while sampling) - relaxed atomics are lock-free and
// async-signal-safe, and a reader sees either a whole slot or an empty one (pc 0).
std::atomic<uintptr_t> g_buf[kCapacity];
std::atomic<uint32_t> g_weight[kCapacity];  // 1 + expirations merged into this signal (overrun)
std::atomic<size_t> g_next{0};
timer_t g_timer{};
std::atomic<bool> g_on{false};
std::mutex g_mu;  // start/stop/histogram (never taken in the handler)
struct sigaction g_old {};

void on_sigprof(int, siginfo_t*, void* uc) {
  if (!g_on.load(std::memory_order_relaxed)) return;
  const auto* u = static_cast<const ucontext_t*>(uc);
#if defined(__x86_64__)
  const uintptr_t pc = static_cast<uintptr_t>(u->uc_mcontext.gregs[REG_RIP]);
#else
  const uintptr_t pc = static_cast<uintptr_t>(u->uc_mcontext.pc);
#endif
  // Expirations while a SIGPROF is still pending collapse into one signal; the timer's
  // overrun count says how many, so the sample carries their weight (several busy
  // threads would otherwise be under-counted).
  const int over = timer_getoverrun(g_timer);
  const size_t i = g_next.fetch_add(1, std::memory_order_relaxed);
  if (i < kCapacity) {
    g_weight[i].store(1u + static_cast<uint32_t>(over > 0 ? over : 0), std::memory_order_relaxed);
    g_buf[i].store(pc, std::memory_order_release);  // publishes the weight with it
  }
}

}  // namespace

bool start(int hz) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (g_on.load() || hz <= 0) return false;
  const size_t used = std::min(g_next.load(), kCapacity);
  for (size_t i = 0; i < used; ++i) g_buf[i].store(0, std::memory_order_relaxed);
  g_next.store(0);
  struct sigaction sa {};
  sa.sa_sigaction = on_sigprof;
  sa.sa_flags = SA_SIGINFO | SA_RESTART;
  sigemptyset(&sa.sa_mask);
  if (sigaction(SIGPROF, &sa, &g_old) != 0) return false;
  struct sigevent sev {};
  sev.sigev_notify = SIGEV_SIGNAL;
  sev.sigev_signo = SIGPROF;
  if (timer_create(CLOCK_PROCESS_CPUTIME_ID, &sev, &g_timer) != 0) {
    sigaction(SIGPROF, &g_old, nullptr);
    return false;
  }
  g_on.store(true);
  struct itimerspec it {};
  it.it_interval.tv_nsec = std::max(1000L, 1000000000L / hz);
  it.it_value = it.it_interval;
  if (timer_settime(g_timer, 0, &it, nullptr) != 0) {
    g_on.store(false);
    timer_delete(g_timer);
    sigaction(SIGPROF, &g_old, nullptr);
    return false;
  }
  return true;
}

void stop() {
  std::lock_guard<std::mutex> lk(g_mu);
  if (!g_on.load()) return;
  struct itimerspec it {};
  timer_settime(g_timer, 0, &it, nullptr);
  g_on.store(false);
  // A signal already in flight still finds g_on false or a valid handler: restoring the
  // old disposition only after the timer is disarmed keeps SIGPROF from killing us.
  sigaction(SIGPROF, &g_old, nullptr);
  timer_delete(g_timer);
}

bool running() { return g_on.load(); }

std::vector<std::pair<uintptr_t, uint64_t>> histogram() {
  std::lock_guard<std::mutex> lk(g_mu);
  const size_t n = std::min(g_next.load(), kCapacity);
  std::unordered_map<uintptr_t, uint64_t> counts;
  for (size_t i = 0; i < n; ++i) {
    const uintptr_t pc = g_buf[i].load(std::memory_order_acquire);
    if (pc != 0) counts[pc] += g_weight[i].load(std::memory_order_relaxed);  // 0: not written yet
  }
  std::vector<std::pair<uintptr_t, uint64_t>> out(counts.begin(), counts.end());
  std::sort(out.begin(), out.end(), [](const auto& a, const auto& b) {
    return a.second != b.second ? a.second > b.second : a.first < b.first;
  });
  return out;
}

uint64_t dropped() {
  const size_t n = g_next.load();
  return n > kCapacity ? n - kCapacity : 0;
}

bool module_of(uintptr_t pc, std::string* path, uintptr_t* base, std::string* symbol) {
  Dl_info info{};
  if (dladdr(reinterpret_cast<void*>(pc), &info) == 0 || info.dli_fname == nullptr) return false;
  *path = info.dli_fname;
  *base = reinterpret_cast<uintptr_t>(info.dli_fbase);
  symbol->assign(info.dli_sname ? info.dli_sname : "");
  return true;
}

}  // namespace prof
}  // namespace amdgpu_dp
