"""Scope of health.canaryOnStart: the start-up canary runs the first
time this process advertises a GPU, off the manager thread, never on a /restart or a
reload, never on partitions a container holds."""
import json
import os
import threading
import time

from k8s_gpu_device_plugin_amd.models import fixtures
from k8s_gpu_device_plugin_amd.plugin.kubelet_stub import KubeletStub
from k8s_gpu_device_plugin_amd.plugin.manager import PluginManager


def _wait(pred, timeout=5.0, step=0.02):
    deadline = time.monotonic() + timeout
    while time.monotonic() < deadline:
        if pred():
            return True
        time.sleep(step)
    return False


def _fake_canary(monkeypatch, delay=0.0, fail=()):
    from k8s_gpu_device_plugin_amd.ops import canary
    calls = []
    release = threading.Event()
    if delay <= 0:
        release.set()

    def run_isolated(device, nbytes, timeout=120.0):
        calls.append(device)
        release.wait(delay)
        return {"ok": device not in fail, "device": device, "error": "" if device not in fail else "mismatch"}
    monkeypatch.setattr(canary, "run_isolated", run_isolated)
    return calls, release


def _run(make_cfg, **cfg):
    m = PluginManager(make_cfg(health={"canaryOnStart": True}, **cfg))
    t = m.start_background()
    return m, t


def test_restart_and_reload_run_no_start_up_canary(make_cfg, plugin_dir, monkeypatch):
    calls, _ = _fake_canary(monkeypatch)
    with KubeletStub(plugin_dir) as k:
        m, t = _run(make_cfg)
        try:
            k.wait_for_registrations(1)
            assert _wait(lambda: len(calls) == 2 and not m._start_pending)
            for _ in range(3):
                reloads = m.counters["reloads"]
                m.restart()
                assert _wait(lambda: m.counters["reloads"] > reloads)
            k.restart()  # kubelet restart: re-register, no canary
            k.wait_for_registrations(2, timeout=10)
            time.sleep(0.3)
            assert len(calls) == 2, calls
            assert m.plugins[0].table.healthy_count() == 2
        finally:
            m.stop()
            t.join(10)


def test_slow_start_up_canary_does_not_block_the_manager(make_cfg, plugin_dir, monkeypatch):
    """A 5 s canary: the partitions are advertised Unhealthy meanwhile, a kubelet restart
    re-registers within 1 s, /ready keeps answering, then the verdict makes them Healthy."""
    calls, release = _fake_canary(monkeypatch, delay=5.0)
    with KubeletStub(plugin_dir) as k:
        m, t = _run(make_cfg)
        try:
            w = k.watch(k.wait_for_registrations(1)[0].endpoint)
            _, devs = w.next()
            assert [h for _, h, _ in devs] == ["Unhealthy", "Unhealthy"]  # verdicts pending
            assert _wait(lambda: len(calls) == 2)
            assert m.readiness() == (True, "")
            t0 = time.monotonic()
            k.restart()
            k.wait_for_registrations(2, timeout=5)
            assert time.monotonic() - t0 < 1.0, "kubelet restart waited for the canary"
            reloads = m.counters["reloads"]
            m.restart()
            assert _wait(lambda: m.counters["reloads"] > reloads, 2)
            assert m.plugins[0].table.healthy_count() == 0  # still pending through the reload
            release.set()
            assert _wait(lambda: m.plugins[0].table.healthy_count() == 2)
            assert len(calls) == 2
        finally:
            release.set()
            m.stop()
            t.join(10)


def test_failed_start_up_canary_survives_reloads(make_cfg, plugin_dir, monkeypatch):
    calls, _ = _fake_canary(monkeypatch, fail=(1,))
    with KubeletStub(plugin_dir) as k:
        m, t = _run(make_cfg)
        try:
            k.wait_for_registrations(1)
            assert _wait(lambda: not m._start_pending)
            table = lambda: m.plugins[0].table  # noqa: E731
            assert [table().healthy(i) for i in table().ids()] == [True, False]
            m.restart()
            assert _wait(lambda: m.counters["reloads"] >= 2)
            assert [table().healthy(i) for i in table().ids()] == [True, False]
            assert m.counters["canary_failures"] == 1
        finally:
            m.stop()
            t.join(10)


def test_start_up_canary_skips_partitions_a_container_holds(make_cfg, plugin_dir, monkeypatch):
    """A plugin restarting on a busy node: kubelet's checkpoint lists GPU 0 in a pod, so
    only GPU 1 is canaried."""
    calls, _ = _fake_canary(monkeypatch)
    gpus, _ = fixtures.build_backend("2gpu_spx").discover()
    held = gpus[0].partitions[0].id
    os.makedirs(plugin_dir, exist_ok=True)
    with open(os.path.join(plugin_dir, "kubelet_internal_checkpoint"), "w") as f:
        json.dump({"Data": {"PodDeviceEntries": [{"PodUID": "u1", "ContainerName": "c", "ResourceName": "amd.com/gpu",
                                                  "DeviceIDs": {"0": [held]}, "AllocResp": ""}],
                            "RegisteredDevices": {"amd.com/gpu": [held]}}, "Checksum": 1}, f)
    with KubeletStub(plugin_dir) as k:
        m, t = _run(make_cfg)
        try:
            k.wait_for_registrations(1)
            assert _wait(lambda: not m._start_pending)
            assert calls == [1] and m.counters["canary_skipped_in_use"] == 1
            assert m.plugins[0].table.healthy_count() == 2
        finally:
            m.stop()
            t.join(10)


def test_gpu_that_comes_back_is_canaried_again(make_cfg, plugin_dir, monkeypatch):
    calls, _ = _fake_canary(monkeypatch)
    be = fixtures.build_backend("2gpu_spx")
    with KubeletStub(plugin_dir) as k:
        m = PluginManager(make_cfg(health={"canaryOnStart": True}, rediscoverIntervalS=0.2), backend=be)
        t = m.start_background()
        try:
            k.wait_for_registrations(1)
            assert _wait(lambda: len(calls) == 2 and not m._start_pending)
            be.set_gpu_present(1, False)
            assert _wait(lambda: len(m.plugins[0].table.ids()) == 1, timeout=10)
            be.set_gpu_present(1, True)
            assert _wait(lambda: len(m.plugins[0].table.ids()) == 2, timeout=10)
            assert _wait(lambda: len(calls) == 3 and not m._start_pending)
            assert calls[-1] == 1
        finally:
            m.stop()
            t.join(10)


def test_recovery_while_a_start_up_verdict_is_pending_keeps_it_unhealthy(make_cfg, plugin_dir, monkeypatch):
    """with health.canary off the monitor writes Healthy transitions into the
    tables itself.  A reset that ends while a partition's start-up verdict is pending must
    not advertise it Healthy, and a failed verdict is applied to the tables, not assumed."""
    from k8s_gpu_device_plugin_amd import native
    n = native.load()
    calls, release = _fake_canary(monkeypatch, delay=5.0, fail=(0,))
    be = fixtures.build_backend("2gpu_spx")
    with KubeletStub(plugin_dir) as k:
        m = PluginManager(make_cfg(health={"canaryOnStart": True}), backend=be)
        t = m.start_background()
        try:
            k.wait_for_registrations(1)
            assert _wait(lambda: len(calls) == 2)
            ids = m.plugins[0].table.ids()
            be.inject_event(n.HwEvent(n.EVT_PRE_RESET, 0, message="test reset"))
            assert _wait(lambda: m.counters["health_events"] >= 1)
            be.inject_event(n.HwEvent(n.EVT_POST_RESET, 0, message="test reset"))
            assert _wait(lambda: m.counters["health_events"] >= 2)
            time.sleep(0.3)
            assert not m.plugins[0].table.healthy(ids[0])  # its verdict is still pending
            release.set()  # GPU 0 fails, GPU 1 passes
            assert _wait(lambda: not m._start_pending)
            time.sleep(0.2)
            assert not m.plugins[0].table.healthy(ids[0]) and m.plugins[0].table.healthy(ids[1])
            assert m.counters.get("canary_failures") == 1
        finally:
            m.stop()
            t.join(10)
