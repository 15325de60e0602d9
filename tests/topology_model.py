"""xGMI node topology view + a pure-Python reference model of the placement policy.

The production policy is native (``native/allocator.cpp``); this module restates it in
plain Python so it can be read, and so ``tests/test_topology_model.py`` can
differentially test the C++ implementation on random small inputs (identical choices
wherever the C++ side runs its exhaustive search).

MI355X node facts used: 8 GPUs, 7 xGMI links per GPU, one direct link
to every peer (full mesh, ~153 GB/s per link).  A k-GPU RCCL job gets at most k-1 links
per GPU, every k-subset of a *healthy* mesh is hop-equivalent, so preference comes from
(1) partitions sharing one GPU, (2) links that are up and trained at full rate, (3) NUMA
locality, (4) not stacking a pod's cross-GPU traffic on links other multi-GPU pods
already use (and not on busy GPUs), (5) keeping healthy cliques free for future jobs.
"""
from __future__ import annotations

import itertools
import math
from dataclasses import dataclass

LINK_XGMI, LINK_PCIE = 2, 1


@dataclass(frozen=True)
class Dev:
    gpu: int
    partition: int = -1
    numa: int = -1


def _link(links: dict, a: int, b: int) -> tuple:
    """(type, hops, up, bw_gbps, pods, weight) of the a-b link; links may hold the short
    (type, hops, up) form, the rest then default to unknown bandwidth/weight, no pods."""
    v = links.get((min(a, b), max(a, b)), (4, 0, True))
    return tuple(v) + (0.0, 0, 0)[len(v) - 3:]


def link_refs(links: dict) -> tuple:
    """Node-wide references for the link terms: the best xGMI bandwidth and the lowest
    xGMI weight seen on any link (0 = unknown)."""
    bws = [_link(links, a, b)[3] for a, b in links if _link(links, a, b)[0] == LINK_XGMI]
    ws = [_link(links, a, b)[5] for a, b in links if _link(links, a, b)[0] == LINK_XGMI]
    return max([x for x in bws if x > 0], default=0.0), min([x for x in ws if x > 0], default=0)


def pair_score(links: dict, a: Dev, b: Dev, refs: tuple | None = None) -> int:
    """Mirror of native ``pair_score``.  links[(i, j)] = (type, hops, up[, bw_gbps, pods,
    weight]) for i < j."""
    same_numa = a.numa >= 0 and a.numa == b.numa
    if a.gpu == b.gpu:
        return 105
    t, hops, up, bw, pods, weight = _link(links, a.gpu, b.gpu)
    ref_bw, min_w = refs if refs is not None else link_refs(links)
    if t == LINK_XGMI:
        if up:
            # a link trained below the node's best scores in proportion (RCCL rings run at
            # the slowest hop): between a full-rate link and a down one
            q = min(1.0, bw / ref_bw) if bw > 0 and ref_bw > 0 else 1.0
            s = 10 + int(math.floor((50 if hops <= 1 else 30) * q + 0.5))
            if weight > 0 and min_w > 0 and weight > min_w:
                s -= min(10, int(math.floor(5 * math.log2(weight / min_w) + 0.5)))
        else:
            s = 10
    elif t == LINK_PCIE:
        s = 20
    else:
        s = 5
    s -= 8 * min(max(int(pods), 0), 4)  # other multi-GPU pods already drive traffic over this link
    return s + (5 if same_numa else 0)


def _max_clique(gpus, links) -> int:
    gpus = sorted(gpus)
    for k in range(len(gpus), 0, -1):
        for sub in itertools.combinations(gpus, k):
            if all(links.get((a, b), (4, 0, False))[2] and links.get((a, b), (4, 0, False))[0] in (LINK_XGMI, LINK_PCIE)
                   for a, b in itertools.combinations(sub, 2)):
                return k
    return 0


def set_score(links: dict, devs: list, avail: list, chosen: list) -> float:
    ngpu = max(d.gpu for d in devs) + 1
    total = [0] * ngpu
    free = [0] * ngpu
    numa_of = {}
    for i, d in enumerate(devs):
        total[d.gpu] += 1
        free[d.gpu] += i in avail
        numa_of[d.gpu] = d.numa
    ppg = max(total)
    refs = link_refs(links)
    s = sum(pair_score(links, devs[a], devs[b], refs) for a, b in itertools.combinations(chosen, 2))
    taken = [0] * ngpu
    for i in chosen:
        taken[devs[i].gpu] += 1
    multi = len({devs[i].gpu for i in chosen}) > 1
    for g in range(ngpu):
        if not taken[g]:
            continue
        busy = free[g] < total[g]
        if busy and total[g] > 1:
            s += 6.0 * taken[g]
        if busy and multi:
            s -= 4.0
    frag = 0.0
    whole_free = {}
    for g in range(ngpu):
        f = free[g] - taken[g]
        frag += f * f / ppg
        if total[g] > 0 and f == total[g]:
            whole_free.setdefault(numa_of[g], []).append(g)
    for numa in dict.fromkeys(numa_of[g] for g in range(ngpu)):
        c = _max_clique(whole_free.get(numa, []), links)
        frag += c * c
    return s + frag


def best_set(links: dict, devs: list, avail: list, required: list, size: int) -> list:
    """Exhaustive reference search (first best in lexicographic order wins)."""
    avail = sorted(set(avail) | set(required))
    need = size - len(required)
    if need <= 0:
        return list(required)
    cand = [i for i in avail if i not in required]
    if len(cand) < need:
        raise ValueError("not enough available devices to satisfy allocation")
    best, best_s = None, None
    for combo in itertools.combinations(cand, need):
        sc = set_score(links, devs, avail, list(required) + list(combo))
        if best_s is None or sc > best_s + 1e-9:
            best, best_s = list(combo), sc
    return list(required) + sorted(best)


class NodeTopology:
    """Read-only view over the native Topology (debug dumps, cliques, NUMA groups)."""

    def __init__(self, gpus, topo) -> None:
        self.gpus = list(gpus)
        self.topo = topo

    def links(self) -> dict:
        out = {}
        for a in range(self.topo.n):
            for b in range(a + 1, self.topo.n):
                lk = self.topo.link(a, b)
                out[(a, b)] = (lk.type, lk.hops, lk.up, lk.bw_gbps, lk.pods, lk.weight)
        return out

    def numa_groups(self) -> dict:
        groups = {}
        for g in self.gpus:
            groups.setdefault(g.numa_node, []).append(g.index)
        return groups

    def healthy_cliques(self) -> dict:
        """Largest all-links-up clique per NUMA node."""
        links = self.links()
        return {n: _max_clique(gs, links) for n, gs in self.numa_groups().items()}

    def down_links(self) -> list:
        return [(a, b) for (a, b), v in self.links().items() if not v[2]]

    def degraded_links(self, below: float = 0.9) -> list:
        """Up xGMI links trained below ``below`` x the node's best link bandwidth."""
        links = self.links()
        ref, _ = link_refs(links)
        return [(a, b) for (a, b), v in links.items() if v[0] == LINK_XGMI and v[2] and ref > 0 and 0 < v[3] < below * ref]

    def to_dict(self) -> dict:
        return {"gpus": [{"index": g.index, "bdf": g.bdf, "numa": g.numa_node, "partitions": len(g.partitions),
                          "mode": "%s/%s" % (g.compute_partition, g.memory_partition)} for g in self.gpus],
                "links": [{"a": a, "b": b, "type": t, "hops": h, "up": up, "bw_gbps": bw, "pods": pods, "weight": w}
                          for (a, b), (t, h, up, bw, pods, w) in sorted(self.links().items())],
                "healthy_cliques_per_numa": self.healthy_cliques()}
