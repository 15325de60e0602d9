// Preferred-allocation policies (GetPreferredAllocation).
//
// Reference (plugin/plugin.go:248-326): `alignedAlloc` rebuilds go-gpuallocator's
// NVLink graph through NVML on EVERY call and runs BestEffortPolicy; `distributedAlloc`
// spreads time-sliced replicas ("<id>::<n>") over the least-used GPUs.
//
// MI355X design: the node is a full xGMI mesh (7 links per GPU), so
// every k-subset of a healthy mesh is hop-equivalent.  The aligned policy therefore
// scores sets by (1) packing partitions of one physical GPU (on-package fabric, no
// xGMI), (2) complete cliques over links that are UP, scored by the bandwidth each link
// trained at relative to the node's best (RCCL rings run at their slowest hop) and its
// amdsmi weight, (3) NUMA locality, (4) not stacking a pod's cross-GPU traffic on links
// other multi-GPU pods already use (from the kubelet PodResources map) or on busy GPUs,
// and (5) fragmentation of what stays free.  The topology is captured once at discovery (and
// patched on link events), never per call.
#pragma once

#include <atomic>
#include <cstdint>
#include <string>
#include <vector>

#include "backend.h"

namespace amdgpu_dp {

struct AllocDevice {
  int gpu = -1;        // physical GPU
  int partition = -1;  // partition index, -1 = whole GPU
  int numa = -1;
  std::string base_id;  // id without "::<replica>"
  bool annotated = false;
};

struct AllocResult {
  bool ok = true;
  std::string error;
  std::vector<int> chosen;  // indices into the device vector, in response order
};

// Node-wide references for the link terms of pair_score: the best trained xGMI
// bandwidth and the lowest xGMI link weight on the node (0 = unknown).
struct LinkRefs {
  double best_bw_gbps = 0;
  uint64_t min_weight = 0;
};
LinkRefs link_refs(const Topology& topo);

// Pairwise placement score (higher is better); exposed for tests/metrics.  Integer by
// construction (the allocator's incremental and direct pair sums must agree exactly).
int pair_score(const Topology& topo, const AllocDevice& a, const AllocDevice& b, const LinkRefs& refs);
int pair_score(const Topology& topo, const AllocDevice& a, const AllocDevice& b);

// `avail` / `required` are device indices.  Contract (same as gpuallocator's
// BestEffortPolicy): result ⊆ avail ∪ required, ⊇ required, |result| = size when
// satisfiable, deterministic for identical inputs.
AllocResult aligned_alloc(const Topology& topo, const std::vector<AllocDevice>& devs,
                          const std::vector<int>& avail, const std::vector<int>& required, int size);

// Multi-GPU allocations this plugin answered recently, as link load the allocator adds
// on top of the kubelet PodResources map until that map covers them.  The PodResources
// poll runs every podResources.intervalS (10 s), while a job's pods are admitted within
// a second or two of each other: without this, every pod of a burst would see the links
// as free and pile onto the same GPU pairs.  One tracker is shared by all of a node's
// tables (pods of different resources share the links too).  Allocate records into a
// fixed ring with one atomic increment; readers take a seqlock-style snapshot.
class RecentAllocations {
 public:
  static constexpr int kSlots = 64;
  RecentAllocations();
  // Allocate answered a container request spanning these GPUs (bit g = GPU g < 64).
  void record(uint64_t gpu_mask, int64_t now_ns);
  // Entries allocated before this (mono ns) are in the PodResources map already.
  void set_covered_until(int64_t mono_ns) { covered_.store(mono_ns, std::memory_order_release); }
  void set_ttl_ms(int64_t ms) { ttl_ns_.store(ms > 0 ? ms * 1000000 : 0, std::memory_order_release); }
  // Adds, for every live entry, one pod to each GPU pair it spans (n x n row-major).
  // Returns the number of live entries (0: nothing added, the caller can skip a copy).
  int add_link_pods(int n, int64_t now_ns, std::vector<int>* pods) const;
  int live(int64_t now_ns) const;
  // False when no entry can be live (one load; the common case on the Allocate path).
  bool maybe_live(int64_t now_ns) const;

 private:
  bool fresh(int64_t ts, int64_t now_ns) const;
  struct alignas(64) Slot {
    std::atomic<uint64_t> seq{0};  // odd while being written
    std::atomic<int64_t> ts{0};
    std::atomic<uint64_t> mask{0};
  };
  Slot slots_[kSlots];
  std::atomic<uint64_t> next_{0};
  std::atomic<int64_t> newest_{0};  // lets readers skip the scan when nothing can be live
  std::atomic<int64_t> covered_{0};
  std::atomic<int64_t> ttl_ns_{30'000'000'000LL};
};

// Replica-spreading policy (reference distributedAlloc, plugin/plugin.go:284-326) with a
// stable, deterministic tie-break (fixes defect D14).
AllocResult distributed_alloc(const std::vector<AllocDevice>& devs, const std::vector<int>& avail,
                              const std::vector<int>& required, int size);

}  // namespace amdgpu_dp
