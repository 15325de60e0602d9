// Whole-process CPU sampling profiler for the `benchmark: true` harness.
//
// Reference: benchmark/benchmark.go:54-89 starts Go's pprof CPU profile, which samples
// every goroutine.  A Python-level profiler (cProfile) sees only the thread that
// enabled it and none of the native code this plugin spends its time in (epoll servers,
// exposition, amdsmi sampling), so the analogue here is a SIGPROF sampler: a POSIX timer
// on CLOCK_PROCESS_CPUTIME_ID signals every `1/hz` s of process CPU time (all threads),
// the signal lands on a running thread, and the async-signal-safe handler records the
// interrupted program counter, weighted by the timer overrun, into a fixed lock-free
// buffer.  Symbolisation (module + offset, then llvm-symbolizer
// or dladdr) happens after stop(), outside the signal context.
#pragma once

#include <cstdint>
#include <string>
#include <utility>
#include <vector>

namespace amdgpu_dp {
namespace prof {

// Installs the handler and starts sampling at `hz` (per second of CPU time).  Returns
// false if a profile is already running or the timer cannot be armed.
bool start(int hz);
// Stops sampling and restores the previous SIGPROF disposition (idempotent).
void stop();
bool running();
// Samples recorded since start(): (pc, count), most frequent first.
std::vector<std::pair<uintptr_t, uint64_t>> histogram();
uint64_t dropped();  // samples beyond the buffer capacity

// Module (shared object / executable) path and load base of a pc; false if unknown.
bool module_of(uintptr_t pc, std::string* path, uintptr_t* base, std::string* symbol);

}  // namespace prof
}  // namespace amdgpu_dp
