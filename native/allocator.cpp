#include "allocator.h"

#include "metrics.h"  // cpu_relax

#include <algorithm>
#include <cmath>
#include <map>
#include <numeric>
#include <set>
#include <unordered_map>

namespace amdgpu_dp {

LinkRefs link_refs(const Topology& topo) {
  LinkRefs r;
  for (int a = 0; a < topo.n; ++a)
    for (int b = a + 1; b < topo.n; ++b) {
      const Link& l = topo.at(a, b);
      if (l.type != kLinkXgmi) continue;
      if (l.bw_gbps > r.best_bw_gbps) r.best_bw_gbps = l.bw_gbps;
      if (l.weight > 0 && (r.min_weight == 0 || l.weight < r.min_weight)) r.min_weight = l.weight;
    }
  return r;
}

int pair_score(const Topology& topo, const AllocDevice& a, const AllocDevice& b, const LinkRefs& refs) {
  const bool same_numa = a.numa >= 0 && a.numa == b.numa;
  if (a.gpu == b.gpu) return 100 + 5;  // partitions of one GPU: on-package fabric
  if (a.gpu < 0 || b.gpu < 0 || a.gpu >= topo.n || b.gpu >= topo.n) return 5;
  const Link& l = topo.at(a.gpu, b.gpu);
  int s;
  switch (l.type) {
    case kLinkXgmi:
      if (l.up) {
        // A link that trained below the node's best scores in proportion, between a
        // full-rate link and a down one: an RCCL ring runs at its slowest hop.
        const double q = (l.bw_gbps > 0 && refs.best_bw_gbps > 0) ? std::min(1.0, l.bw_gbps / refs.best_bw_gbps) : 1.0;
        s = 10 + static_cast<int>(std::floor((l.hops <= 1 ? 50 : 30) * q + 0.5));
        if (l.weight > 0 && refs.min_weight > 0 && l.weight > refs.min_weight)
          s -= std::min(10, static_cast<int>(std::floor(5 * std::log2(static_cast<double>(l.weight) / refs.min_weight) + 0.5)));
      } else {
        s = 10;
      }
      break;
    case kLinkPcie:
      s = 20;
      break;
    default:
      s = 5;
  }
  s -= 8 * std::min(std::max(l.pods, 0), 4);  // other multi-GPU pods already drive traffic over it
  return s + (same_numa ? 5 : 0);
}

int pair_score(const Topology& topo, const AllocDevice& a, const AllocDevice& b) {
  return pair_score(topo, a, b, link_refs(topo));
}

namespace {

// The vectors of one allocation's context live in the calling thread and keep their
// capacity between calls: a context is built per GetPreferredAllocation, and its ~15
// vectors were as many heap allocations per request.
struct CtxScratch {
  std::vector<char> is_avail;
  std::vector<int> gpu_total, gpu_avail, gpu_numa, numa_ids, gpu_numa_slot, taken, cnt, cls, cls_rep, cls_pair;
  std::vector<uint64_t> adj, whole_free, base_free;
  std::vector<int> touched;
  std::vector<std::pair<int, int>> keys;
};
CtxScratch& ctx_scratch() {
  static thread_local CtxScratch s;
  return s;
}

struct Ctx {
  const Topology& topo;
  const std::vector<AllocDevice>& devs;
  CtxScratch& sc = ctx_scratch();
  std::vector<char>& is_avail = sc.is_avail;    // device index -> available
  std::vector<int>& gpu_total = sc.gpu_total;   // devices per gpu (all)
  std::vector<int>& gpu_avail = sc.gpu_avail;   // available devices per gpu
  std::vector<int>& gpu_numa = sc.gpu_numa;
  std::vector<uint64_t>& adj = sc.adj;                 // healthy direct-link adjacency bitmask per GPU
  std::vector<int>& numa_ids = sc.numa_ids;            // distinct NUMA nodes
  std::vector<int>& gpu_numa_slot = sc.gpu_numa_slot;  // gpu -> index into numa_ids
  int ngpu = 0;
  int parts_per_gpu = 1;
  // score() scratch, reused across the (up to thousands of) candidate evaluations
  std::vector<int>& taken = sc.taken;
  std::vector<uint64_t>& whole_free = sc.whole_free;
  std::vector<int>& cnt = sc.cnt;  // per-class counts of the set being scored
  // pair_score depends only on (gpu, numa) of the two devices: one matrix over those
  // classes replaces the per-pair topology lookups in score()
  std::vector<int>& cls = sc.cls;            // device -> class
  std::vector<int>& cls_rep = sc.cls_rep;    // class -> a device of it
  std::vector<int>& cls_pair = sc.cls_pair;  // nclass x nclass pair scores, filled on first use
  int ncls = 0;
  // set_terms() starts from the pool as it is and adjusts only the GPUs a candidate
  // touches: the fragmentation sum with nothing taken, and the whole-free GPUs per NUMA node
  double base_frag = 0;
  std::vector<uint64_t>& base_free = sc.base_free;
  static constexpr int kUnset = -1;

  int class_pair(int a, int b) const {
    int& v = cls_pair[static_cast<size_t>(a) * ncls + b];
    if (v == kUnset)
      v = cls_pair[static_cast<size_t>(b) * ncls + a] = pair_score(topo, devs[cls_rep[a]], devs[cls_rep[b]], refs);
    return v;
  }

  LinkRefs refs;

  Ctx(const Topology& t, const std::vector<AllocDevice>& d, const std::vector<int>& avail)
      : topo(t), devs(d), refs(link_refs(t)) {
    is_avail.assign(d.size(), 0);
    for (int i : avail) is_avail[i] = 1;
    for (auto& x : d) ngpu = std::max(ngpu, x.gpu + 1);
    gpu_total.assign(ngpu, 0);
    gpu_avail.assign(ngpu, 0);
    gpu_numa.assign(ngpu, -1);
    for (size_t i = 0; i < d.size(); ++i) {
      if (d[i].gpu < 0) continue;
      gpu_total[d[i].gpu]++;
      gpu_avail[d[i].gpu] += is_avail[i];
      gpu_numa[d[i].gpu] = d[i].numa;
    }
    for (int g = 0; g < ngpu; ++g) parts_per_gpu = std::max(parts_per_gpu, gpu_total[g]);
    adj.assign(ngpu, 0);
    for (int a = 0; a < ngpu && a < 64; ++a)
      for (int b = 0; b < ngpu && b < 64; ++b)
        if (a != b && a < t.n && b < t.n && t.at(a, b).up &&
            (t.at(a, b).type == kLinkXgmi || t.at(a, b).type == kLinkPcie))
          adj[a] |= 1ull << b;
    gpu_numa_slot.assign(ngpu, 0);
    numa_ids.clear();
    for (int g = 0; g < ngpu; ++g) {
      auto it = std::find(numa_ids.begin(), numa_ids.end(), gpu_numa[g]);
      if (it == numa_ids.end()) it = numa_ids.insert(numa_ids.end(), gpu_numa[g]);
      gpu_numa_slot[g] = static_cast<int>(it - numa_ids.begin());
    }
    taken.assign(ngpu, 0);
    whole_free.assign(numa_ids.size(), 0);
    base_free.assign(numa_ids.size(), 0);
    for (int g = 0; g < ngpu; ++g) {
      base_frag += static_cast<double>(gpu_avail[g]) * gpu_avail[g] / parts_per_gpu;
      if (gpu_total[g] > 0 && gpu_avail[g] == gpu_total[g] && g < 64) base_free[gpu_numa_slot[g]] |= 1ull << g;
    }
    std::vector<std::pair<int, int>>& keys = sc.keys;
    keys.clear();
    std::vector<int>& rep = cls_rep;
    rep.clear();
    cls.assign(d.size(), 0);
    for (size_t i = 0; i < d.size(); ++i) {
      const std::pair<int, int> key(d[i].gpu, d[i].numa);
      auto it = std::find(keys.begin(), keys.end(), key);
      if (it == keys.end()) {
        keys.push_back(key);
        rep.push_back(static_cast<int>(i));
        it = keys.end() - 1;
      }
      cls[i] = static_cast<int>(it - keys.begin());
    }
    ncls = static_cast<int>(keys.size());
    cls_pair.assign(static_cast<size_t>(ncls) * ncls, kUnset);
    cnt.assign(ncls, 0);
  }

  // Largest set of GPUs in `mask` that are pairwise connected by healthy links.
  int max_clique(uint64_t mask) const {
    const int all = __builtin_popcountll(mask);
    int best = 0;
    // enumerate subsets of mask (callers pass <= 8-16 GPUs of one NUMA node); the first
    // is the whole mask, which on a healthy mesh is a clique: then nothing can beat it
    for (uint64_t sub = mask; sub; sub = (sub - 1) & mask) {
      const int pc = __builtin_popcountll(sub);
      if (pc <= best) continue;
      bool ok = true;
      for (uint64_t rest = sub; rest && ok; rest &= rest - 1) {
        const int v = __builtin_ctzll(rest);
        ok = (sub & ~(adj[v] | (1ull << v))) == 0;
      }
      if (ok) best = pc;
      if (best == all) break;
    }
    return best;
  }

  // score of choosing set S (device indices) out of the available pool
  double score(const std::vector<int>& S) const {
    std::fill(cnt.begin(), cnt.end(), 0);
    for (int i : S) cnt[cls[i]]++;
    const size_t n = S.size();
    if (n * (n - 1) >= static_cast<size_t>(ncls) * (ncls + 1)) return score_counts(cnt);
    // small sets (the exhaustive path): summing the pairs directly is cheaper
    double s = 0;
    for (size_t i = 0; i < n; ++i)
      for (size_t j = i + 1; j < n; ++j) s += class_pair(cls[S[i]], cls[S[j]]);
    return s + set_terms(cnt);
  }

  // Same score from per-class counts: devices of one (gpu, numa) class are
  // interchangeable for every term, so a candidate costs O(classes^2 + gpus) instead of
  // O(|S|^2) - the multi-GPU greedy/local search evaluates hundreds of candidates.
  // (Pair scores are integers, so both pair sums are exact and identical.)
  double score_counts(const std::vector<int>& cn) const { return pair_sum(cn) + set_terms(cn); }

  // the pair-score part of score_counts (an integer: every sum below is exact)
  double pair_sum(const std::vector<int>& cn) const {
    double s = 0;
    for (int a = 0; a < ncls; ++a) {
      if (!cn[a]) continue;
      s += 0.5 * cn[a] * (cn[a] - 1) * class_pair(a, a);
      for (int b = a + 1; b < ncls; ++b)
        if (cn[b]) s += static_cast<double>(cn[a]) * cn[b] * class_pair(a, b);
    }
    return s;
  }
  // how pair_sum(cn) grows when one device of class a joins: sum over b of cn[b] * P(a, b)
  double pair_gain(const std::vector<int>& cn, int a) const {
    double s = 0;
    for (int b = 0; b < ncls; ++b)
      if (cn[b]) s += static_cast<double>(cn[b]) * class_pair(a, b);
    return s;
  }

  // every term but the pair scores: packing, link sharing, fragmentation
  double set_terms(const std::vector<int>& cn) const {
    double s = 0;
    // the GPUs this candidate takes devices from (taken[] is all zero between calls)
    std::vector<int>& touched = sc.touched;
    touched.clear();
    int first_gpu = -2;
    bool multi_gpu = false;
    for (int a = 0; a < ncls; ++a) {
      if (!cn[a]) continue;
      const int g = devs[cls_rep[a]].gpu;
      if (first_gpu == -2) first_gpu = g;
      else if (g != first_gpu) multi_gpu = true;
      if (g < 0) continue;
      if (!taken[g]) touched.push_back(g);
      taken[g] += cn[a];
    }
    // fragmentation of the remainder: concentrate leftovers, and keep the largest
    // healthy-link clique of whole free GPUs per NUMA node (what a future multi-GPU
    // RCCL job needs) - on a healthy mesh this is just the whole-free count.  Only the
    // touched GPUs differ from the pool as it is (every term is a multiple of
    // 1/parts_per_gpu: exact in any order for the power-of-two partition counts, and off
    // by far less than the 1e-9 tie tolerance otherwise).
    double frag = base_frag;
    std::copy(base_free.begin(), base_free.end(), whole_free.begin());
    for (const int g : touched) {
      const bool busy = gpu_avail[g] < gpu_total[g];  // other pods already on this GPU
      if (busy && gpu_total[g] > 1) s += 6.0 * taken[g];  // pack into partially used GPUs
      if (busy && multi_gpu) s -= 4.0;  // cross-GPU traffic would share this GPU's links
      const int f = gpu_avail[g] - taken[g];
      frag += (static_cast<double>(f) * f - static_cast<double>(gpu_avail[g]) * gpu_avail[g]) / parts_per_gpu;
      if (g < 64) whole_free[gpu_numa_slot[g]] &= ~(1ull << g);  // no longer whole and free
      taken[g] = 0;
    }
    for (uint64_t m : whole_free) {
      const int c = __builtin_popcountll(m) <= 16 ? max_clique(m) : __builtin_popcountll(m);
      frag += static_cast<double>(c) * c;
    }
    return s + frag;
  }
};

double n_choose_k(int n, int k) {
  if (k < 0 || k > n) return 0;
  double r = 1;
  for (int i = 1; i <= k; ++i) r = r * (n - k + i) / i;
  return r;
}

}  // namespace

AllocResult aligned_alloc(const Topology& topo, const std::vector<AllocDevice>& devs, const std::vector<int>& avail_in,
                          const std::vector<int>& required_in, int size) {
  AllocResult res;
  const int ndev = static_cast<int>(devs.size());
  std::vector<int> avail, required;
  std::vector<char> seen(ndev, 0);
  for (int i : required_in)
    if (i >= 0 && i < ndev && !seen[i]) {
      seen[i] = 1;
      required.push_back(i);
    }
  std::vector<char> in_avail(ndev, 0);
  for (int i : avail_in)
    if (i >= 0 && i < ndev && !in_avail[i]) {
      in_avail[i] = 1;
      avail.push_back(i);
    }
  for (int i : required)
    if (!in_avail[i]) {
      in_avail[i] = 1;
      avail.push_back(i);
    }
  std::sort(avail.begin(), avail.end());
  const int need = size - static_cast<int>(required.size());
  if (size <= 0 || need <= 0) {
    res.chosen = required;
    return res;
  }
  std::vector<int> cand;
  for (int i : avail)
    if (!seen[i]) cand.push_back(i);
  if (static_cast<int>(cand.size()) < need) {
    res.ok = false;
    res.error = "not enough available devices to satisfy allocation";
    return res;
  }
  std::vector<int> best;
  if (static_cast<int>(cand.size()) == need) {
    best = cand;
  } else {
    Ctx ctx(topo, devs, avail);
    double best_score = -1e300;
    auto consider = [&](std::vector<int>& S) {
      const double sc = ctx.score(S);
      if (sc > best_score + 1e-9) {
        best_score = sc;
        best.assign(S.begin() + required.size(), S.end());
      }
    };
    // Partition packing shortcut: if one GPU can hold the whole request (together with
    // every required device), a single-GPU set dominates - each split pair loses >= 40
    // pair-score points while the fragmentation/packing terms move by < 40 in total.
    // candidates grouped by GPU (ascending GPU, then device index): runs in `grouped`
    thread_local std::vector<int> grouped;
    grouped.assign(cand.begin(), cand.end());
    std::stable_sort(grouped.begin(), grouped.end(), [&](int x, int y) { return devs[x].gpu < devs[y].gpu; });
    int req_gpu = -2;
    for (int i : required) req_gpu = (req_gpu == -2 || req_gpu == devs[i].gpu) ? devs[i].gpu : -3;
    bool single_gpu_done = false;
    if (need >= 1 && req_gpu != -3) {
      std::vector<int> S;
      for (size_t b = 0; b < grouped.size();) {
        size_t e = b;
        while (e < grouped.size() && devs[grouped[e]].gpu == devs[grouped[b]].gpu) ++e;
        const int gpu = devs[grouped[b]].gpu;
        if (static_cast<int>(e - b) >= need && !(req_gpu >= 0 && gpu != req_gpu)) {
          S.assign(required.begin(), required.end());
          S.insert(S.end(), grouped.begin() + b, grouped.begin() + b + need);
          consider(S);
          single_gpu_done = true;
        }
        b = e;
      }
    }
    if (single_gpu_done && ctx.parts_per_gpu > 1) {
      // best single-GPU placement already chosen
    } else if (n_choose_k(static_cast<int>(cand.size()), need) <= 4000) {
      // exhaustive, lexicographic order => deterministic tie-break (first best wins)
      std::vector<int> idx(need);
      std::iota(idx.begin(), idx.end(), 0);
      const int m = static_cast<int>(cand.size());
      std::vector<int> S(required);
      S.resize(required.size() + need);
      for (;;) {
        for (int k = 0; k < need; ++k) S[required.size() + k] = cand[idx[k]];
        consider(S);
        int k = need - 1;
        while (k >= 0 && idx[k] == m - need + k) --k;
        if (k < 0) break;
        ++idx[k];
        for (int j = k + 1; j < need; ++j) idx[j] = idx[j - 1] + 1;
      }
    } else {
      std::vector<int> S(required);
      std::vector<char> used(ndev, 0);
      for (int i : required) used[i] = 1;
      // Devices with the same (gpu, numa) are interchangeable for the score (pair
      // scores and every per-GPU term depend on nothing else), so each step evaluates
      // only the first unused one of each class - the one the full scan would have
      // kept on a tie anyway.  A 64-partition CPX node: 8 evaluations per step, not 64.
      // (a class is exactly a (gpu, numa) pair)
      std::vector<char> seen(ctx.ncls, 0);
      auto first_of_class = [&](int c) {
        char& s = seen[ctx.cls[c]];
        if (s) return false;
        s = 1;
        return true;
      };
      // class counts of S, updated in place around each candidate evaluation; the pair
      // part of a candidate's score is the current sum plus what the device adds (all
      // integers, so exactly score_counts' value)
      std::vector<int> cn(ctx.ncls, 0);
      for (int i : required) cn[ctx.cls[i]]++;
      double pairs = ctx.pair_sum(cn);
      while (static_cast<int>(S.size()) < size) {
        int pick = -1;
        double ps = -1e300, pick_gain = 0;
        std::fill(seen.begin(), seen.end(), 0);
        for (int c : cand) {
          if (used[c] || !first_of_class(c)) continue;
          const int a = ctx.cls[c];
          const double gain = ctx.pair_gain(cn, a);
          cn[a]++;
          const double sc = pairs + gain + ctx.set_terms(cn);
          cn[a]--;
          if (sc > ps + 1e-9) {
            ps = sc;
            pick = c;
            pick_gain = gain;
          }
        }
        S.push_back(pick);
        cn[ctx.cls[pick]]++;
        pairs += pick_gain;
        used[pick] = 1;
      }
      // 1-swap local search (bounded)
      double cur = pairs + ctx.set_terms(cn);
      // classes whose positions found no improving swap since the last change: another
      // position of the same class would see exactly the same candidates and scores
      std::vector<char> tried(ctx.ncls, 0);
      for (int pass = 0; pass < 4; ++pass) {
        bool improved = false;
        for (size_t k = required.size(); k < S.size(); ++k) {
          const int k_cls = ctx.cls[S[k]];
          if (tried[k_cls]) continue;
          bool changed = false;
          std::fill(seen.begin(), seen.end(), 0);
          for (int c : cand) {
            if (used[c] || !first_of_class(c)) continue;
            const int old = S[k];
            if (ctx.cls[old] == ctx.cls[c]) continue;  // same class: same score
            // pairs without `old`, then with `c` in its place
            cn[ctx.cls[old]]--;
            const double without = pairs - ctx.pair_gain(cn, ctx.cls[old]);
            const double with_c = without + ctx.pair_gain(cn, ctx.cls[c]);
            cn[ctx.cls[c]]++;
            const double sc = with_c + ctx.set_terms(cn);
            if (sc > cur + 1e-9) {
              cur = sc;
              pairs = with_c;
              S[k] = c;
              used[old] = 0;
              used[c] = 1;
              improved = changed = true;
            } else {
              cn[ctx.cls[c]]--;
              cn[ctx.cls[old]]++;
            }
          }
          if (changed) std::fill(tried.begin(), tried.end(), 0);
          else tried[k_cls] = 1;
        }
        if (!improved) break;
      }
      consider(S);
    }
  }
  std::sort(best.begin(), best.end());
  res.chosen = required;
  res.chosen.insert(res.chosen.end(), best.begin(), best.end());
  return res;
}

RecentAllocations::RecentAllocations() = default;

void RecentAllocations::record(uint64_t gpu_mask, int64_t now_ns) {
  if (__builtin_popcountll(gpu_mask) < 2 || ttl_ns_.load(std::memory_order_relaxed) == 0) return;
  // Each writer owns its slot: it claims it by moving seq from even to odd with a CAS.  A
  // slot another writer still holds (one preempted while the ring wrapped) is skipped;
  // two writers in one slot could otherwise leave seq odd for good.
  for (int tries = 0; tries < kSlots; ++tries) {
    Slot& s = slots_[next_.fetch_add(1, std::memory_order_relaxed) % kSlots];
    uint64_t q = s.seq.load(std::memory_order_relaxed);
    if ((q & 1) || !s.seq.compare_exchange_strong(q, q + 1, std::memory_order_relaxed)) continue;
    std::atomic_thread_fence(std::memory_order_release);
    s.mask.store(gpu_mask, std::memory_order_relaxed);
    s.ts.store(now_ns, std::memory_order_relaxed);
    s.seq.store(q + 2, std::memory_order_release);
    break;
  }
  int64_t cur = newest_.load(std::memory_order_relaxed);
  while (cur < now_ns && !newest_.compare_exchange_weak(cur, now_ns, std::memory_order_release)) {
  }
}

bool RecentAllocations::fresh(int64_t ts, int64_t now_ns) const {
  const int64_t ttl = ttl_ns_.load(std::memory_order_acquire);
  return ts > 0 && ttl > 0 && ts > covered_.load(std::memory_order_acquire) && now_ns - ts < ttl;
}

int RecentAllocations::add_link_pods(int n, int64_t now_ns, std::vector<int>* pods) const {
  if (!fresh(newest_.load(std::memory_order_acquire), now_ns)) return 0;  // the common case: nothing recent
  int live = 0;
  for (const Slot& s : slots_) {
    uint64_t mask;
    int64_t ts;
    // seqlock read: retry while a writer is in the slot, but never wait on a writer that
    // was preempted there (the entry is then left out of this one answer)
    bool got = false;
    for (int spin = 0; spin < 256 && !got; ++spin) {
      const uint64_t q0 = s.seq.load(std::memory_order_acquire);
      if (q0 & 1) {
        cpu_relax();
        continue;
      }
      mask = s.mask.load(std::memory_order_relaxed);
      ts = s.ts.load(std::memory_order_relaxed);
      std::atomic_thread_fence(std::memory_order_acquire);
      got = s.seq.load(std::memory_order_relaxed) == q0;
    }
    if (!got || !fresh(ts, now_ns)) continue;
    ++live;
    if (!pods) continue;
    for (uint64_t a = mask; a; a &= a - 1) {
      const int ga = __builtin_ctzll(a);
      for (uint64_t b = a & (a - 1); b; b &= b - 1) {
        const int gb = __builtin_ctzll(b);
        if (ga < n && gb < n) {
          (*pods)[static_cast<size_t>(ga) * n + gb]++;
          (*pods)[static_cast<size_t>(gb) * n + ga]++;
        }
      }
    }
  }
  return live;
}

int RecentAllocations::live(int64_t now_ns) const { return add_link_pods(0, now_ns, nullptr); }

bool RecentAllocations::maybe_live(int64_t now_ns) const { return fresh(newest_.load(std::memory_order_acquire), now_ns); }

AllocResult distributed_alloc(const std::vector<AllocDevice>& devs, const std::vector<int>& avail,
                              const std::vector<int>& required, int size) {
  AllocResult res;
  const int ndev = static_cast<int>(devs.size());
  std::vector<char> is_req(ndev, 0);
  for (int i : required)
    if (i >= 0 && i < ndev) is_req[i] = 1;
  std::vector<int> cand;
  std::vector<char> seen(ndev, 0);
  for (int i : avail)
    if (i >= 0 && i < ndev && !is_req[i] && !seen[i]) {
      seen[i] = 1;
      cand.push_back(i);
    }
  const int needed = size - static_cast<int>(required.size());
  if (static_cast<int>(cand.size()) < needed) {
    res.ok = false;
    res.error = "not enough available devices to satisfy allocation";
    return res;
  }
  // replica accounting per base device id (plugin/plugin.go:292-306)
  std::unordered_map<std::string, std::pair<int, int>> rep;  // base -> (total, available)
  for (int c : cand) rep[devs[c].base_id].second++;
  for (const auto& d : devs) {
    auto it = rep.find(d.base_id);
    if (it != rep.end()) it->second.first++;
  }
  res.chosen = required;
  for (int i = 0; i < needed; ++i) {
    std::stable_sort(cand.begin(), cand.end(), [&](int a, int b) {
      const auto& ra = rep[devs[a].base_id];
      const auto& rb = rep[devs[b].base_id];
      return (ra.first - ra.second) < (rb.first - rb.second);
    });
    const int pick = cand.front();
    rep[devs[pick].base_id].second--;
    res.chosen.push_back(pick);
    cand.erase(cand.begin());
  }
  return res;
}

}  // namespace amdgpu_dp
