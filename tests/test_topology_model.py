"""Differential tests: native allocator vs the pure-Python reference model
(tests/topology_model.py), and the /metrics contract vs metrics/families.py."""
from hypothesis import given, settings, strategies as st
from prometheus_client.parser import text_string_to_metric_families

from k8s_gpu_device_plugin_amd.metrics import families
from k8s_gpu_device_plugin_amd.models import fixtures
import topology_model as T


def _native_topo(n, ngpu, links):
    t = n.Topology(ngpu)
    for (a, b), v in links.items():
        typ, hops, up, bw, pods, weight = tuple(v) + (0.0, 0, 0)[len(v) - 3:]
        t.set_link(a, b, n.Link(type=typ, hops=hops, up=up, weight=weight, bw_gbps=bw, pods=pods))
    return t


@settings(max_examples=120, deadline=None)
@given(st.data())
def test_native_matches_reference_model(n, data):
    ngpu = data.draw(st.integers(2, 8))
    nparts = data.draw(st.sampled_from([1, 1, 2, 4]))
    per_numa = data.draw(st.sampled_from([2, 4]))
    links = {}
    quality = data.draw(st.booleans())  # bandwidth / pod-load / weight terms in play
    for a in range(ngpu):
        for b in range(a + 1, ngpu):
            links[(a, b)] = (data.draw(st.sampled_from([T.LINK_XGMI, T.LINK_XGMI, T.LINK_PCIE])), 1,
                             data.draw(st.booleans()) or data.draw(st.booleans()))
            if quality:
                links[(a, b)] += (data.draw(st.sampled_from([0.0, 608.0, 608.0, 456.0, 304.0])),
                                  data.draw(st.sampled_from([0, 0, 0, 1, 2])),
                                  data.draw(st.sampled_from([15, 15, 15, 30, 0])))
    devs = [T.Dev(g, p if nparts > 1 else -1, g // per_numa) for g in range(ngpu) for p in range(nparts)]
    ndevs = [n.AllocDevice(d.gpu, d.partition, d.numa, "d%d" % i) for i, d in enumerate(devs)]
    avail = sorted(data.draw(st.sets(st.integers(0, len(devs) - 1), min_size=1, max_size=min(len(devs), 12))))
    req = data.draw(st.lists(st.sampled_from(avail), max_size=min(2, len(avail)), unique=True))
    size = data.draw(st.integers(len(req), min(len(avail), len(req) + 4)))
    got = n.aligned_alloc(_native_topo(n, ngpu, links), ndevs, avail, req, size)
    want = T.best_set(links, devs, avail, req, size)
    assert T.set_score(links, devs, avail, got) == T.set_score(links, devs, avail, want)
    if nparts == 1:
        assert got == want


def test_node_topology_view():
    be = fixtures.build_backend("8gpu_spx_degraded")
    gpus, topo = be.discover()
    view = T.NodeTopology(gpus, topo)
    assert sorted(view.down_links()) == [(0, 5), (2, 3)]
    assert view.numa_groups() == {0: [0, 1, 2, 3], 1: [4, 5, 6, 7]}
    assert view.healthy_cliques() == {0: 3, 1: 4}
    d = view.to_dict()
    assert len(d["links"]) == 28 and d["gpus"][0]["mode"] == "SPX/NPS1"


def test_metrics_contract_both_ways(n):
    from k8s_gpu_device_plugin_amd import config as C
    from k8s_gpu_device_plugin_amd.plugin.manager import PluginManager
    from k8s_gpu_device_plugin_amd.server.web import WebServer
    import http.client
    import time
    cfg = C.validate(C.from_dict({"backend": "fixture", "fixture": "8gpu_cpx_nps2", "migStrategy": "single",
                                  "pluginDir": "/tmp/dp-contract", "webListenAddress": "127.0.0.1:0",
                                  "log": {"fileDir": ""}, "http": {"accessLog": False}}))
    m = PluginManager(cfg)
    m.load_plugins()
    m._start_telemetry()
    m.plugins[0].table.observe(n.RPC_ALLOCATE, 1e-5, False)
    m.canary_results[(0, 0)] = (time.time(), {  # as one canary run would leave it
        "ok": True, "hbm_errors": 0, "mfma_errors": 0, "gemm_errors": 0, "lowp_errors": 0, "lds_errors": 0,
        "write_gbps": 6000.0, "read_gbps": 5900.0, "mfma_tflops": 1800.0, "gemm_tflops": 1400.0,
        "fp8_tflops": 3800.0, "fp4_tflops": 6500.0})
    m._publish_metrics()
    w = WebServer(cfg, m)
    port = w.start()
    try:
        c = http.client.HTTPConnection("127.0.0.1", port, timeout=5)
        c.request("GET", "/health")
        c.getresponse().read()
        time.sleep(0.05)
        c.request("GET", "/metrics")
        text = c.getresponse().read().decode()
    finally:
        w.stop()
        m.exporter.stop()
        m.monitor.stop()
    seen = set()
    for fam in text_string_to_metric_families(text):
        for s in fam.samples:
            f = families.family_of(s.name)
            assert f is not None, "undocumented metric %s" % s.name
            labels = set(s.labels) - {"le"}
            assert labels == set(f.labels), (s.name, labels, f.labels)
            seen.add(f.name)
    missing = {f.name for f in families.FAMILIES} - seen
    # per-partition VRAM needs real usage and the RAS page threshold needs root (or
    # health.badPageThreshold); everything else must be present on the fixture node
    assert missing <= {"amdgpu_partition_vram_used_bytes", "amdgpu_device_plugin_allocation_info",
                       "amdgpu_device_plugin_pod_resources_up", "amdgpu_retired_pages_threshold",
                       "amdgpu_telemetry_sample_stalled", "amdgpu_telemetry_sample_blocked",
                       "amdgpu_xgmi_link_pods"}, missing


def test_metrics_doc_is_generated_from_the_registry():
    import os
    path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "docs", "METRICS.md")
    with open(path, encoding="utf-8") as f:
        assert f.read() == families.markdown(), "regenerate: python -m k8s_gpu_device_plugin_amd.metrics.families"


def test_pair_score_link_terms_match_the_model(n):
    """Each new link term on its own, native vs model: a half-rate link sits between a
    full-rate and a down one; a link other pods already span scores lower; a heavier
    amdsmi weight costs a little."""
    a, b, c = T.Dev(0, -1, 0), T.Dev(1, -1, 0), T.Dev(2, -1, 0)
    na, nb = n.AllocDevice(0, -1, 0, "a"), n.AllocDevice(1, -1, 0, "b")
    cases = {"full": (T.LINK_XGMI, 1, True, 608.0, 0, 15), "half": (T.LINK_XGMI, 1, True, 304.0, 0, 15),
             "down": (T.LINK_XGMI, 1, False, 608.0, 0, 15), "pods": (T.LINK_XGMI, 1, True, 608.0, 2, 15),
             "heavy": (T.LINK_XGMI, 1, True, 608.0, 0, 30)}
    got = {}
    for name, link in cases.items():
        links = {(0, 1): link, (0, 2): cases["full"], (1, 2): cases["full"]}
        got[name] = T.pair_score(links, a, b)
        assert n.pair_score(_native_topo(n, 3, links), na, nb) == got[name], name
    assert got["full"] == 65 and got["down"] < got["half"] < got["full"]
    assert got["pods"] == got["full"] - 16 and got["heavy"] == got["full"] - 5
    assert T.pair_score({(0, 1): cases["full"]}, a, c) == 5 + 5  # no link known: unknown type


def test_degraded_link_is_avoided_by_2_and_4_gpu_requests(n):
    """8-GPU mesh, two NUMA nodes, link 0-1 trained at half rate: a 2-GPU request that
    must include GPU 0 takes another peer, and a 4-GPU request takes the NUMA node
    whose links all run at full rate."""
    links = {(a, b): (T.LINK_XGMI, 1, True, 608.0, 0, 15) for a in range(8) for b in range(a + 1, 8)}
    links[(0, 1)] = (T.LINK_XGMI, 1, True, 304.0, 0, 15)
    topo = _native_topo(n, 8, links)
    devs = [n.AllocDevice(g, -1, g // 4, "g%d" % g) for g in range(8)]
    pick2 = n.aligned_alloc(topo, devs, list(range(8)), [0], 2)
    assert pick2 == [0, 2]
    assert n.aligned_alloc(topo, devs, list(range(8)), [], 4) == [4, 5, 6, 7]
    assert not {0, 1} <= set(n.aligned_alloc(topo, devs, [0, 1, 2, 3], [], 2))
    # without the degradation the 2-GPU pick is the first peer, as before
    ok = _native_topo(n, 8, {k: (T.LINK_XGMI, 1, True, 608.0, 0, 15) for k in links})
    assert n.aligned_alloc(ok, devs, list(range(8)), [0], 2) == [0, 1]
    lat = n.bench_aligned_alloc(topo, devs, list(range(8)), [1], 4, 500)
    assert sorted(lat)[len(lat) // 2] < 10e-6  # size 4 of 8: well under 10 us
