"""xGMI-aware GetPreferredAllocation policies.

Contract (go-gpuallocator BestEffortPolicy, used at reference plugin/plugin.go:276):
result ⊆ available ∪ required, ⊇ required, |result| = size, deterministic.
MI355X specifics: partition packing, healthy-link cliques, NUMA,
fragmentation.  The distributed (replica) policy mirrors plugin/plugin.go:284-326."""
import itertools

import pytest
from hypothesis import given, settings, strategies as st

from k8s_gpu_device_plugin_amd.models import fixtures


def _topo(n, ngpu, down=()):
    t = n.Topology(ngpu)
    for a in range(ngpu):
        for b in range(a + 1, ngpu):
            t.set_link(a, b, n.Link(type=n.LINK_XGMI, hops=1, up=(a, b) not in down))
    return t


def _whole(n, ngpu, per_numa=4):
    return [n.AllocDevice(g, -1, g // per_numa, "g%d" % g) for g in range(ngpu)]


def _parts(n, ngpu, nparts, per_numa=4):
    return [n.AllocDevice(g, p, g // per_numa, "g%dp%d" % (g, p)) for g in range(ngpu) for p in range(nparts)]


def test_pair_scores(n):
    t = _topo(n, 8, down={(0, 5)})
    d = _whole(n, 8)
    same_gpu = n.pair_score(t, n.AllocDevice(0, 0, 0, "a"), n.AllocDevice(0, 1, 0, "b"))
    xgmi_same_numa = n.pair_score(t, d[0], d[1])
    xgmi_cross_numa = n.pair_score(t, d[0], d[4])
    down = n.pair_score(t, d[0], d[5])
    assert same_gpu > xgmi_same_numa > xgmi_cross_numa > down


def test_whole_gpu_numa_packing_sequence(n):
    """2+2 requests fill NUMA node 0 first, leaving node 1's four GPUs for a 4-GPU job."""
    t, d = _topo(n, 8), _whole(n, 8)
    avail = list(range(8))
    a = n.aligned_alloc(t, d, avail, [], 2)
    assert a == [0, 1]
    avail = [x for x in avail if x not in a]
    b = n.aligned_alloc(t, d, avail, [], 2)
    assert b == [2, 3]
    avail = [x for x in avail if x not in b]
    c = n.aligned_alloc(t, d, avail, [], 4)
    assert c == [4, 5, 6, 7]


def test_avoids_down_links(n):
    t, d = _topo(n, 8, down={(0, 1), (0, 2), (0, 3)}), _whole(n, 8)
    r = n.aligned_alloc(t, d, [0, 1, 2, 3], [0], 2)
    assert r[0] == 0 and len(r) == 2  # forced: 0 plus someone (all links from 0 down)
    r = n.aligned_alloc(t, d, list(range(8)), [], 4)
    assert 0 not in r or all(x not in r for x in (1, 2, 3))
    r = n.aligned_alloc(t, d, [0, 1, 2, 3], [], 3)
    assert r == [1, 2, 3]


def test_partition_packing_best_fit(n):
    t, d = _topo(n, 8), _parts(n, 8, 8)
    # GPU 0 has 3 free partitions, GPU 1 is completely free: a 2-partition job goes to GPU 0
    avail = [i for i in range(len(d)) if (d[i].gpu == 0 and d[i].partition >= 5) or d[i].gpu >= 1]
    r = n.aligned_alloc(t, d, avail, [], 2)
    assert {d[i].gpu for i in r} == {0}
    # a 4-partition job cannot fit GPU 0 (3 free) -> one whole other GPU, not split across two
    r = n.aligned_alloc(t, d, avail, [], 4)
    assert len({d[i].gpu for i in r}) == 1 and d[r[0]].gpu != 0


def test_must_include_is_honoured_and_first(n):
    t, d = _topo(n, 8), _parts(n, 8, 8)
    r = n.aligned_alloc(t, d, list(range(64)), [17], 4)
    assert r[0] == 17 and len(r) == 4 and {d[i].gpu for i in r} == {2}


def test_errors_and_edge_cases(n):
    t, d = _topo(n, 4), _whole(n, 4)
    with pytest.raises(RuntimeError, match="not enough"):
        n.aligned_alloc(t, d, [0, 1], [], 3)
    assert n.aligned_alloc(t, d, [0, 1, 2], [2, 1], 2) == [2, 1]
    assert n.aligned_alloc(t, d, [0, 1, 2], [], 0) == []
    assert n.aligned_alloc(t, d, [3, 1], [], 2) == [1, 3]


@settings(max_examples=150, deadline=None)
@given(st.data())
def test_aligned_invariants(n, data):
    ngpu = data.draw(st.integers(1, 8))
    nparts = data.draw(st.sampled_from([1, 2, 4, 8]))
    d = _parts(n, ngpu, nparts) if nparts > 1 else _whole(n, ngpu)
    down = set(data.draw(st.lists(st.tuples(st.integers(0, 7), st.integers(0, 7)), max_size=4)))
    down = {tuple(sorted(x)) for x in down if x[0] != x[1]}
    t = _topo(n, ngpu, down)
    avail = sorted(data.draw(st.sets(st.integers(0, len(d) - 1), min_size=1)))
    req = data.draw(st.lists(st.sampled_from(avail), max_size=min(3, len(avail)), unique=True))
    size = data.draw(st.integers(len(req), len(avail)))
    r = n.aligned_alloc(t, d, avail, req, size)
    assert len(r) == size == len(set(r))
    assert set(r) <= set(avail) and r[:len(req)] == req
    assert n.aligned_alloc(t, d, avail, req, size) == r  # deterministic


def test_exhaustive_matches_bruteforce_optimum(n):
    """For small sets the chosen set has the best pairwise link score."""
    t, d = _topo(n, 6, down={(0, 1), (2, 3), (1, 4)}), _whole(n, 6, per_numa=3)
    r = n.aligned_alloc(t, d, list(range(6)), [], 3)

    def pairs(s):
        return sum(n.pair_score(t, d[a], d[b]) for a, b in itertools.combinations(s, 2))
    best = max(pairs(s) for s in itertools.combinations(range(6), 3))
    assert pairs(r) == best


def test_large_partition_pool_is_fast_and_packed(n):
    import time
    t, d = _topo(n, 8), _parts(n, 8, 8)
    t0 = time.perf_counter()
    r = n.aligned_alloc(t, d, list(range(64)), [], 8)
    dt = time.perf_counter() - t0
    assert len({d[i].gpu for i in r}) == 1   # a whole GPU's partitions, not 8 GPUs
    assert dt < 0.5, dt


def test_distributed_policy_spreads_replicas(n):
    # 3 GPUs x 2 replicas; replicas of g0 are already in use by someone else
    d = [n.AllocDevice(g, -1, 0, "g%d" % g, True) for g in range(3) for _ in range(2)]
    avail = [2, 3, 4, 5]  # g0's replicas (0, 1) are taken
    r = n.distributed_alloc(d, avail, [], 2)
    assert sorted({d[i].base_id for i in r}) == ["g1", "g2"]  # one replica on each free GPU
    r2 = n.distributed_alloc(d, [1, 2, 3, 4, 5], [], 1)
    assert d[r2[0]].base_id in ("g1", "g2")  # least-used GPUs first
    assert n.distributed_alloc(d, avail, [4], 2)[0] == 4
    with pytest.raises(RuntimeError):
        n.distributed_alloc(d, [2], [], 2)


def test_table_switches_policy_on_annotations(n):
    from k8s_gpu_device_plugin_amd.device import build_device_map
    from k8s_gpu_device_plugin_amd.plugin.plugin import make_table
    from k8s_gpu_device_plugin_amd.resource import new_resources
    g, topo = fixtures.build_backend("4gpu_spx").discover()
    dm = build_device_map(g, new_resources(g, "single"), "single", replicas=2)
    t = make_table("amd.com/gpu", dm["amd.com/gpu"], topo, None)
    assert not t.aligned_supported
    ids = t.ids()
    got = t.preferred_ids(ids[2:], [], 2)
    assert len({x.split("::")[0] for x in got}) == 2
    dm2 = build_device_map(g, new_resources(g, "single"), "single")
    t2 = make_table("amd.com/gpu", dm2["amd.com/gpu"], topo, None)
    assert t2.aligned_supported
    t2.set_link_up(0, 1, False)
    assert t2.preferred_ids(t2.ids()[:3], [], 2) != t2.ids()[:2]


def test_large_cpx_requests_pack_whole_gpus_fast(n):
    """Requests larger than one GPU's partitions on a CPX node take the greedy path:
    whole GPUs first, the remainder on one more GPU of the same NUMA node, never spread
    thin - and quickly (each step scores one device per (gpu, numa) class)."""
    import time
    from collections import Counter
    topo = n.Topology(8)
    for a in range(8):
        for b in range(a + 1, 8):
            topo.set_link(a, b, n.Link(type=n.LINK_XGMI, hops=1, up=True))
    devs = [n.AllocDevice(g, p, g // 4, "g%dp%d" % (g, p)) for g in range(8) for p in range(8)]
    cases = [(12, list(range(64)), {8, 4}), (16, list(range(64)), {8}), (12, list(range(4, 64)), {8, 4}),
             (24, list(range(64)), {8})]
    for size, avail, shape in cases:
        t0 = time.perf_counter()
        chosen = n.aligned_alloc(topo, devs, avail, [], size)
        dt = time.perf_counter() - t0
        per_gpu = Counter(c // 8 for c in chosen)
        assert len(chosen) == size and set(chosen) <= set(avail)
        assert set(per_gpu.values()) == shape, (size, per_gpu)
        if size <= 16:
            assert len({g // 4 for g in per_gpu}) == 1, per_gpu  # one NUMA node
        assert dt < 0.02, dt


def test_pod_link_load_steers_cross_gpu_pods_apart(n):
    """CPX: GPUs 0, 1 and 2 each have 4 free partitions, a pod of 8 must span two GPUs.
    With no other pod on any link the first pair wins (0+1); once a multi-GPU pod is
    known to span GPUs 0 and 1 (kubelet PodResources), the new pod avoids sharing that
    link."""
    topo = n.Topology(4)
    for a in range(4):
        for b in range(a + 1, 4):
            topo.set_link(a, b, n.Link(type=n.LINK_XGMI, hops=1, bw_gbps=608.0))
    devs = [n.AllocDevice(g, p, 0, "g%dp%d" % (g, p)) for g in range(4) for p in range(8)]
    avail = [g * 8 + p for g in range(3) for p in range(4, 8)]
    gpus = lambda chosen: sorted({devs[i].gpu for i in chosen})  # noqa: E731
    assert gpus(n.aligned_alloc(topo, devs, avail, [], 8)) == [0, 1]
    topo.set_link(0, 1, n.Link(type=n.LINK_XGMI, hops=1, bw_gbps=608.0, pods=1))
    assert gpus(n.aligned_alloc(topo, devs, avail, [], 8)) in ([0, 2], [1, 2])


def test_table_link_setters_are_copy_on_write(n):
    t = n.DeviceTable(n.TableConfig(), [n.TableDevice("a", 0), n.TableDevice("b", 1)], n.Topology(2))
    before = t.topology()
    t.set_link_bandwidth(0, 1, 304.0)
    t.set_link_pods([0, 2, 2, 0])
    after = t.topology()
    assert after.link(0, 1).bw_gbps == after.link(1, 0).bw_gbps == 304.0
    assert after.link(0, 1).pods == 2 and before.link(0, 1).pods == 0 and before.link(0, 1).bw_gbps == 0
    t.set_link_pods([])
    assert t.topology().link(0, 1).pods == 0


def test_cpx_churn_shares_fewer_links_with_pod_link_load():
    """BASELINE round-3 protocol (8x8 CPX, 400 steps): feeding the live pods' link load
    to the allocator lowers the number of GPU pairs a new multi-GPU pod shares with
    another one, without rejecting more pods."""
    from k8s_gpu_device_plugin_amd.benchmark.suite import _churn_cpx
    seeds = range(100, 115)
    runs = {vis: [_churn_cpx(vis, seed=s) for s in seeds] for vis in ("none", "podresources", "podresources+allocate")}
    shared = {vis: sum(r["shared_link_pairs"] for r in rs) for vis, rs in runs.items()}
    # the lagged PodResources map helps; adding the plugin's own recent Allocates helps more
    assert shared["podresources+allocate"] < shared["podresources"] < shared["none"], shared
    assert [r["rejected"] for r in runs["none"]] == [r["rejected"] for r in runs["podresources+allocate"]]


def _cpx_table(n, ngpu=4, parts=8):
    topo = n.Topology(ngpu)
    for a in range(ngpu):
        for b in range(a + 1, ngpu):
            topo.set_link(a, b, n.Link(type=n.LINK_XGMI, hops=1, bw_gbps=608.0))
    devs = [n.TableDevice("g%dp%d" % (g, p), g, p, 0, -1, ["/dev/dri/renderD%d" % (128 + g * parts + p)], True)
            for g in range(ngpu) for p in range(parts)]
    return n.DeviceTable(n.TableConfig(), devs, topo)


def test_recent_multi_gpu_allocate_counts_as_link_load(n):
    """A burst of pods is admitted faster than the PodResources poll: a container the
    plugin just allocated across GPUs 0 and 1 already steers the next pod off link 0-1.
    Once a poll covers it (the map has it now) or its TTL passes, it no longer counts."""
    from k8s_gpu_device_plugin_amd.api import v1beta1
    t = _cpx_table(n)
    rec = n.RecentAllocations()
    t.set_recent_allocations(rec)
    ids = t.ids()
    avail = ids[4:8] + ids[12:16] + ids[20:24]  # 4 free partitions on each of GPUs 0, 1, 2
    gpus = lambda got: sorted({ids.index(x) // 8 for x in got})  # noqa: E731
    first = t.preferred_ids(avail, [], 8)
    assert gpus(first) == [0, 1]
    req = v1beta1.AllocateRequest(container_requests=[
        v1beta1.ContainerAllocateRequest(devices_ids=ids[0:4] + ids[8:12])]).SerializeToString()
    ok, _ = t.allocate(req)
    assert ok and rec.live() == 1 and rec.link_pods(4)[0 * 4 + 1] == 1
    second = t.preferred_ids(avail, [], 8)
    assert gpus(second) in ([0, 2], [1, 2])
    rec.set_covered_until(n.mono_ns())  # a PodResources poll now reports that pod
    assert rec.live() == 0
    third = t.preferred_ids(avail, [], 8)
    assert gpus(third) == [0, 1]
    # single-GPU containers and failed requests record nothing; the TTL ends an entry
    bad = v1beta1.AllocateRequest(container_requests=[
        v1beta1.ContainerAllocateRequest(devices_ids=ids[0:2] + ids[8:10]),
        v1beta1.ContainerAllocateRequest(devices_ids=["nope"])]).SerializeToString()
    assert not t.allocate(bad)[0] and rec.live() == 0
    assert t.allocate(v1beta1.AllocateRequest(container_requests=[
        v1beta1.ContainerAllocateRequest(devices_ids=ids[0:8])]).SerializeToString())[0]
    assert rec.live() == 0
    rec.set_ttl_ms(50)
    rec.record_gpus([2, 3])
    assert rec.live() == 1
    import time
    time.sleep(0.08)
    assert rec.live() == 0


def test_podresources_coverage_keeps_a_grace_before_the_list(n, monkeypatch):
    """kubelet writes a container's devices into the PodResources map only after the
    plugin's Allocate answer came back, so a List sent just after an Allocate may miss
    it: coverage stops COVER_GRACE_NS before the List's send time, and an
    Allocate answered inside that window keeps counting as link load."""
    from k8s_gpu_device_plugin_amd.plugin import podresources as pr
    w = pr.PodResourcesWatcher("/nonexistent.sock", 1.0, "amd.com/", lambda: None)
    assert w.covered_until() == 0  # no List yet: nothing covered
    rec = n.RecentAllocations()
    rec.record_gpus([0, 1])  # answered just before the List went out
    monkeypatch.setattr(pr, "list_allocations", lambda *a, **k: {})
    assert w.poll_once()
    assert 0 < w.covered_until_ns <= n.mono_ns()
    assert w.covered_until() == w.covered_until_ns - w.COVER_GRACE_NS
    rec.set_covered_until(w.covered_until())
    assert rec.live() == 1, "an Allocate inside the grace window was treated as covered"
    rec.set_covered_until(n.mono_ns() + 1)  # a List sent COVER_GRACE_NS later covers it
    assert rec.live() == 0
