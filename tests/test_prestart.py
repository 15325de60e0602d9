"""health.canaryOnPreStart: kubelet's PreStartContainer runs the gfx950 canary on the
allocated partitions before the container starts (reference: a no-op,
plugin/plugin.go:227-229).  The canary itself is replaced by a fake here; the
hardware run is in tests/test_gpu.py."""
import threading
import time

import grpc
import pytest

from k8s_gpu_device_plugin_amd.models import fixtures
from k8s_gpu_device_plugin_amd.ops import canary
from k8s_gpu_device_plugin_amd.plugin.kubelet_stub import KubeletStub
from k8s_gpu_device_plugin_amd.plugin.manager import PluginManager


@pytest.fixture
def fake_canary(monkeypatch):
    state = {"fail_hip": set(), "delay": 0.0, "calls": [], "lock": threading.Lock()}

    def run_isolated(hip, nbytes=0, timeout=0.0):
        with state["lock"]:
            state["calls"].append(hip)
        time.sleep(state["delay"])
        if hip in state["fail_hip"]:
            return {"ok": False, "device": hip, "error": "injected HBM mismatch"}
        return {"ok": True, "device": hip}
    monkeypatch.setattr(canary, "run_isolated", run_isolated)
    return state


def _start(make_cfg, plugin_dir, server, fixture="2gpu_cpx_nps2"):
    k = KubeletStub(plugin_dir).start()
    m = PluginManager(make_cfg(fixture=fixture, migStrategy="single", grpc={"server": server},
                               health={"canaryOnPreStart": True}))
    t = m.start_background()
    reg = k.wait_for_registrations(1)[0]
    return k, m, t, reg


@pytest.mark.parametrize("server", ["native", "python"])
def test_prestart_runs_canary_on_exactly_the_allocated_partitions(make_cfg, plugin_dir, fake_canary, server):
    k, m, t, reg = _start(make_cfg, plugin_dir, server)
    try:
        assert reg.options.pre_start_required and reg.options.get_preferred_allocation_available
        c = k.client(reg.endpoint)
        assert c.get_options().pre_start_required
        ids = m.plugins[0].table.ids()
        c.pre_start([ids[3], ids[9]])
        parts = {p.id: p.hip_id for g in m.gpus for p in g.partitions}
        assert sorted(fake_canary["calls"]) == sorted([parts[ids[3]], parts[ids[9]]])
        fake_canary["fail_hip"].add(parts[ids[9]])
        with pytest.raises(grpc.RpcError) as e:
            c.pre_start([ids[9]])
        assert "canary failed" in e.value.details() and "partition" in e.value.details()
        w = k.watch(reg.endpoint)
        deadline = time.monotonic() + 5
        while time.monotonic() < deadline:
            _, devs = w.next(timeout=5)
            if dict((d, h) for d, h, _ in devs)[ids[9]] == "Unhealthy":
                break
        health = dict((d, h) for d, h, _ in devs)
        assert health[ids[9]] == "Unhealthy" and health[ids[3]] == "Healthy"
        assert m.counters.get("prestart_failures") == 1
        with pytest.raises(grpc.RpcError):
            c.pre_start(["no-such-device"])
    finally:
        m.stop()
        t.join(10)
        k.stop()


def test_slow_prestart_does_not_block_other_rpcs(make_cfg, plugin_dir, fake_canary, n):
    """A canary that runs for a second must not stall Allocate/GetPreferredAllocation on
    the same kubelet connection (the native server answers PreStart asynchronously)."""
    k, m, t, reg = _start(make_cfg, plugin_dir, "native")
    try:
        fake_canary["delay"] = 1.0
        ids = m.plugins[0].table.ids()
        sock = m.plugins[0].socket
        from k8s_gpu_device_plugin_amd.api import v1beta1
        h2 = n.H2Client(sock)
        pre = v1beta1.PreStartContainerRequest(devices_ids=[ids[0]]).SerializeToString()
        alloc = v1beta1.AllocateRequest(container_requests=[
            v1beta1.ContainerAllocateRequest(devices_ids=[ids[1]])]).SerializeToString()
        done = {}

        def slow():
            t0 = time.monotonic()
            done["pre"] = (h2.unary(v1beta1.METHOD_PRE_START, pre)[0], time.monotonic() - t0)
        th = threading.Thread(target=slow)
        th.start()
        time.sleep(0.1)
        h2b = n.H2Client(sock)
        t0 = time.monotonic()
        for _ in range(50):
            assert h2b.unary(v1beta1.METHOD_ALLOCATE, alloc)[0] == 0
        assert time.monotonic() - t0 < 0.5  # not queued behind the 1 s check
        th.join(5)
        assert done["pre"][0] == 0 and done["pre"][1] >= 0.9
        h2.close()
        h2b.close()
    finally:
        m.stop()
        t.join(10)
        k.stop()


def test_prestart_disabled_is_the_reference_no_op(make_cfg, plugin_dir, fake_canary):
    with KubeletStub(plugin_dir) as k:
        m = PluginManager(make_cfg())
        t = m.start_background()
        try:
            reg = k.wait_for_registrations(1)[0]
            assert not reg.options.pre_start_required
            k.client(reg.endpoint).pre_start(m.plugins[0].table.ids()[:1])
            assert fake_canary["calls"] == []
        finally:
            m.stop()
            t.join(10)


def test_prestart_failure_survives_a_reload(make_cfg, plugin_dir, fake_canary):
    """A partition whose PreStartContainer canary failed stays Unhealthy through a
    /restart reload (the monitor's state of its GPU is healthy, so only the manager
    remembers the verdict)."""
    k, m, t, reg = _start(make_cfg, plugin_dir, "native")
    try:
        ids = m.plugins[0].table.ids()
        parts = {p.id: p.hip_id for g in m.gpus for p in g.partitions}
        fake_canary["fail_hip"].add(parts[ids[5]])
        with pytest.raises(grpc.RpcError):
            k.client(reg.endpoint).pre_start([ids[5]])
        deadline = time.monotonic() + 5
        while m.counters.get("prestart_failures") != 1 and time.monotonic() < deadline:
            time.sleep(0.01)
        reloads = m.counters["reloads"]
        m.restart()
        deadline = time.monotonic() + 10
        while m.counters["reloads"] == reloads and time.monotonic() < deadline:
            time.sleep(0.01)
        # the table was swapped in; the restart registered the same socket again
        assert m.counters["reloads"] > reloads and {r.endpoint for r in k.requests} == {reg.endpoint}
        _, devs = k.watch(reg.endpoint).next(timeout=5)
        health = dict((d, h) for d, h, _ in devs)
        assert health[ids[5]] == "Unhealthy"
        assert [h for d, h in health.items() if d != ids[5]] == ["Healthy"] * (len(ids) - 1)
    finally:
        m.stop()
        t.join(10)
        k.stop()
