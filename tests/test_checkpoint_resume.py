"""Checkpoint/resume contract: the plugin is stateless and kubelet
checkpoints allocations by device id, so every restart of the plugin process must
advertise the same ids (in the same order, with the same device nodes) for the same
hardware layout - whatever the strategy or partition mode - and a pod's checkpointed
ids must still Allocate afterwards."""
import pytest

from k8s_gpu_device_plugin_amd.models import fixtures
from k8s_gpu_device_plugin_amd.plugin.kubelet_stub import KubeletStub
from k8s_gpu_device_plugin_amd.plugin.manager import PluginManager


def _advertise(cfg, plugin_dir, fixture):
    """One plugin process lifetime: fresh backend + manager; returns {resource: [(id,
    health, numa)]} and {resource: Allocate device nodes of the first two ids}."""
    with KubeletStub(plugin_dir) as k:
        m = PluginManager(cfg, backend=fixtures.build_backend(fixture))
        t = m.start_background()
        try:
            regs = {r.resource_name: r for r in k.wait_for_registrations(len(m.plugins), timeout=10)}
            ads, nodes = {}, {}
            for name, reg in sorted(regs.items()):
                _, devs = k.watch(reg.endpoint).next()
                ads[name] = devs
                ids = [d for d, _, _ in devs][:2]
                resp = k.client(reg.endpoint).allocate(ids)
                nodes[name] = sorted(s.host_path for s in resp.container_responses[0].devices)
            return ads, nodes
        finally:
            m.stop()
            t.join(10)


@pytest.mark.parametrize("fixture,strategy", [("8gpu_spx_mesh", "none"), ("8gpu_cpx_nps2", "single"),
                                              ("8gpu_qpx_nps2", "mixed"), ("4gpu_spx", "single")])
def test_ids_and_device_nodes_survive_plugin_restart(make_cfg, plugin_dir, fixture, strategy):
    cfg = make_cfg(fixture=fixture, migStrategy=strategy, telemetry={"intervalMs": 1000})
    first = _advertise(cfg, plugin_dir, fixture)
    second = _advertise(cfg, plugin_dir, fixture)
    assert first == second
    ads, _ = first
    ids = [d for devs in ads.values() for d, _, _ in devs]
    assert len(ids) == len(set(ids)) and all(h == "Healthy" for devs in ads.values() for _, h, _ in devs)


def test_checkpointed_ids_allocate_after_restart(make_cfg, plugin_dir):
    """A pod admitted before the restart keeps its ids in kubelet's checkpoint; the new
    plugin process must accept exactly those ids."""
    cfg = make_cfg(fixture="8gpu_cpx_nps2", migStrategy="single", telemetry={"intervalMs": 1000})
    ads, _ = _advertise(cfg, plugin_dir, "8gpu_cpx_nps2")
    checkpoint = [d for d, _, _ in ads["amd.com/gpu"]][10:13]
    with KubeletStub(plugin_dir) as k:
        m = PluginManager(cfg, backend=fixtures.build_backend("8gpu_cpx_nps2"))
        t = m.start_background()
        try:
            reg = k.wait_for_registrations(1)[0]
            resp = k.client(reg.endpoint).allocate(checkpoint)
            env = dict(resp.container_responses[0].envs)
            assert env["AMD_VISIBLE_DEVICES"] == ",".join(checkpoint)
        finally:
            m.stop()
            t.join(10)
