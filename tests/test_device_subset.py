"""A plugin that owns a non-prefix subset of the node's GPUs (``devices: "4-7"``, e.g.
two plugin instances splitting one node) must sample, label and health-check each GPU
by its node index, never by its position in the subset."""
import time

from prometheus_client.parser import text_string_to_metric_families

from k8s_gpu_device_plugin_amd.models import fixtures
from k8s_gpu_device_plugin_amd.plugin.kubelet_stub import KubeletStub
from k8s_gpu_device_plugin_amd.plugin.manager import PluginManager


def _families(text):
    return {f.name: f for f in text_string_to_metric_families(text)}


def _ecc_samples(m, gpu, want, timeout=3.0):
    deadline = time.monotonic() + timeout
    while True:
        f = _families(m.exporter.render()).get("amdgpu_ecc_errors")
        samples = f.samples if f else []
        if any(s.labels["gpu"] == gpu and s.labels["type"] == "uncorrectable" and s.value == want for s in samples) \
                or time.monotonic() > deadline:
            return samples
        time.sleep(0.05)


def test_subset_telemetry_labels_and_health_follow_node_index(make_cfg, plugin_dir):
    be = fixtures.build_backend("8gpu_cpx_nps2")
    cfg = make_cfg(fixture="8gpu_cpx_nps2", migStrategy="single", devices="4-7", telemetry={"intervalMs": 40})
    with KubeletStub(plugin_dir) as k:
        m = PluginManager(cfg, backend=be)
        t = m.start_background()
        try:
            w = k.watch(k.wait_for_registrations(1)[0].endpoint)
            _, devs = w.next()
            assert len(devs) == 32 and [g.index for g in m.gpus] == [4, 5, 6, 7]
            time.sleep(0.15)
            fams = _families(m.exporter.render())
            assert sorted(s.labels["gpu"] for s in fams["amdgpu_info"].samples) == ["4", "5", "6", "7"]
            assert {s.labels["gpu"]: s.value for s in fams["amdgpu_telemetry_up"].samples} == \
                {"4": 1.0, "5": 1.0, "6": 1.0, "7": 1.0}
            # every advertised partition keeps its per-partition telemetry
            parts = fams["amdgpu_partition_info"].samples
            assert len(parts) == 32 and {s.labels["gpu"] for s in parts} == {"4", "5", "6", "7"}
            assert len(fams["amdgpu_partition_gfx_busy_percent"].samples) == 32
            # GPU 6's own counters are sampled, not those of GPU 2 (position 2 in the subset)
            be.set_ecc_uncorrectable(6, 2)
            be.set_ecc_uncorrectable(2, 9)
            _, devs = w.next(timeout=5)
            bad = {d for d, h, _ in devs if h == "Unhealthy"}
            want = {d.id for p in m.plugins for d in p.devices() if d.gpu == 6}
            assert bad == want and len(want) == 8
            ecc = {s.labels["gpu"]: s.value for s in _ecc_samples(m, "6", 2.0) if s.labels["type"] == "uncorrectable"}
            assert ecc["6"] == 2.0 and "2" not in ecc
            assert m.exporter.last_sample(6).ok and not m.exporter.last_sample(2).ok
        finally:
            m.stop()
            t.join(10)
