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

// Replica-spreading policy (reference distributedAlloc, plugin/plugin.go:284-326) with a
// stable, deterministic tie-break (fixes defect D14).
AllocResult distributed_alloc(const std::vector<AllocDevice>& devs, const std::vector<int>& avail,
                              const std::vector<int>& required, int size);

}  // namespace amdgpu_dp
