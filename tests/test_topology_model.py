"""Differential tests: native allocator vs the pure-Python reference model
(parallel/topology.py), and the /metrics contract vs metrics/families.py."""
from hypothesis import given, settings, strategies as st
from prometheus_client.parser import text_string_to_metric_families

from k8s_gpu_device_plugin_amd.metrics import families
from k8s_gpu_device_plugin_amd.models import fixtures
from k8s_gpu_device_plugin_amd.parallel import topology as T


def _native_topo(n, ngpu, links):
    t = n.Topology(ngpu)
    for (a, b), (typ, hops, up) in links.items():
        t.set_link(a, b, n.Link(type=typ, hops=hops, up=up))
    return t


@settings(max_examples=120, deadline=None)
@given(st.data())
def test_native_matches_reference_model(n, data):
    ngpu = data.draw(st.integers(2, 8))
    nparts = data.draw(st.sampled_from([1, 1, 2, 4]))
    per_numa = data.draw(st.sampled_from([2, 4]))
    links = {}
    for a in range(ngpu):
        for b in range(a + 1, ngpu):
            links[(a, b)] = (data.draw(st.sampled_from([T.LINK_XGMI, T.LINK_XGMI, T.LINK_PCIE])), 1,
                             data.draw(st.booleans()) or data.draw(st.booleans()))
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
                       "amdgpu_telemetry_sample_stalled"}, missing


def test_metrics_doc_is_generated_from_the_registry():
    import os
    path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "docs", "METRICS.md")
    with open(path, encoding="utf-8") as f:
        assert f.read() == families.markdown(), "regenerate: python -m k8s_gpu_device_plugin_amd.metrics.families"
