"""Plugin manager lifecycle: registration, kubelet restart, /restart, retries, health
events (fault injection via the fixture backend), idempotent stop, no busy loop."""
import os
import threading
import time

import pytest

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


@pytest.fixture
def run_manager():
    started = []

    def _run(cfg, backend=None):
        m = PluginManager(cfg, backend=backend)
        t = m.start_background()
        started.append((m, t))
        return m
    yield _run
    for m, t in started:
        m.stop()
        t.join(10)
        assert not t.is_alive()


@pytest.mark.parametrize("grpc_server", ["native", "python"])
def test_starts_registers_and_serves(make_cfg, plugin_dir, run_manager, grpc_server):
    with KubeletStub(plugin_dir) as k:
        m = run_manager(make_cfg(grpc={"server": grpc_server}))
        regs = k.wait_for_registrations(1)
        assert regs[0].resource_name == "amd.com/gpu"
        assert m.ready.closed and m.running
        _, devs = k.watch(regs[0].endpoint).next()
        assert len(devs) == 2
        text = m.exporter.render()
        assert 'amdgpu_device_plugin_registered{resource="amd.com/gpu"} 1' in text


def test_kubelet_restart_triggers_reregistration(make_cfg, plugin_dir, run_manager):
    k = KubeletStub(plugin_dir).start()
    try:
        m = run_manager(make_cfg())
        k.wait_for_registrations(1)
        k.restart()  # deletes + recreates kubelet.sock -> inotify CREATE
        k.wait_for_registrations(2, timeout=10)
        assert _wait(lambda: m.counters["restarts_kubelet"] >= 1)
        c = k.client("amd-gpu.sock")
        assert c.get_options().get_preferred_allocation_available
    finally:
        k.stop()


def _drain_until(w, pred, timeout=5.0):
    deadline = time.monotonic() + timeout
    seen = []
    while time.monotonic() < deadline:
        seen += w.read(100)
        if any(pred(e) for e in seen):
            return seen
    raise AssertionError("no matching event in %r" % (seen,))


@pytest.mark.parametrize("how", ["remove", "rename"])
def test_dir_watcher_survives_directory_recreation(tmp_path, how):
    """The watched directory goes away and comes back (a node agent wiping
    /var/lib/kubelet/device-plugins): the watcher re-arms, and a kubelet.sock that was
    created before it re-armed is still reported."""
    import shutil
    from k8s_gpu_device_plugin_amd import native
    d = tmp_path / "device-plugins"
    d.mkdir()
    w = native.load().DirWatcher(str(d))
    (d / "a").write_text("")
    _drain_until(w, lambda e: e[0] == "a" and e[2])
    if how == "remove":
        shutil.rmtree(d)
    else:
        os.rename(d, tmp_path / "old")
    for _ in range(3):
        w.read(50)  # watch gone; reads just pause
    d.mkdir()
    (d / "kubelet.sock").write_text("")
    _drain_until(w, lambda e: e[0] == "kubelet.sock" and e[2])
    # and it keeps following the new directory
    (d / "kubelet.sock").unlink()
    (d / "kubelet.sock").write_text("")
    _drain_until(w, lambda e: e[0] == "kubelet.sock" and e[3])
    if how == "rename":
        (tmp_path / "old" / "stale").write_text("")  # the old inode is no longer watched
        assert not [e for e in w.read(100) if e[0] == "stale"]


def test_plugin_dir_recreated_triggers_reregistration(make_cfg, plugin_dir, run_manager):
    import shutil
    k = KubeletStub(plugin_dir).start()
    try:
        m = run_manager(make_cfg())
        k.wait_for_registrations(1)
        k.stop()
        # (the plugin serves its socket again when it sees it removed: it may land while
        # the tree is being deleted)
        for _ in range(20):
            shutil.rmtree(plugin_dir, ignore_errors=True)
            if not os.path.exists(plugin_dir):
                break
            time.sleep(0.05)
        time.sleep(0.3)
        k = KubeletStub(plugin_dir).start()  # recreates the directory and kubelet.sock
        k.wait_for_registrations(1, timeout=10)
        assert _wait(lambda: m.counters["restarts_kubelet"] >= 1)
        assert k.client("amd-gpu.sock").get_options().get_preferred_allocation_available
    finally:
        k.stop()


@pytest.mark.parametrize("grpc_server", ["native", "python"])
def test_removed_plugin_socket_is_served_again(make_cfg, plugin_dir, run_manager, grpc_server):
    """Someone deletes amd-gpu.sock while the plugin serves: kubelet could no longer
    reach it.  The plugin binds a fresh socket and registers again; its own reloads
    (which keep the socket) do not trigger this."""
    with KubeletStub(plugin_dir) as k:
        m = run_manager(make_cfg(grpc={"server": grpc_server}))
        k.wait_for_registrations(1)
        reloads = m.counters["reloads"]
        m.restart()  # own reload: swaps the table, keeps the socket, registers it again
        assert _wait(lambda: m.counters["reloads"] > reloads)
        k.wait_for_registrations(2, timeout=10)
        time.sleep(0.5)
        assert m.counters.get("restarts_socket", 0) == 0 and len(k.requests) == 2
        os.remove(os.path.join(plugin_dir, "amd-gpu.sock"))
        k.wait_for_registrations(3, timeout=10)
        assert _wait(lambda: m.counters.get("restarts_socket", 0) == 1)
        assert k.client("amd-gpu.sock").get_options().get_preferred_allocation_available
        # (the handler counts the restart before it publishes the metrics)
        assert _wait(lambda: 'amdgpu_device_plugin_events_total{event="restarts_socket"} 1' in m.exporter.render())


@pytest.mark.parametrize("grpc_server", ["native", "python"])
def test_restart_api_reloads_without_dropping_kubelet(make_cfg, plugin_dir, run_manager, grpc_server):
    """GET /restart re-reads the hardware and swaps the new device table into the
    running server: kubelet's connection, its ListAndWatch stream and the registration
    stay (the reference stops every server first, plugin/manager.go:177-194)."""
    with KubeletStub(plugin_dir) as k:
        m = run_manager(make_cfg(grpc={"server": grpc_server}))
        reg = k.wait_for_registrations(1)[0]
        c = k.client(reg.endpoint)
        w = k.watch(reg.endpoint)
        _, devs = w.next()
        ids = [d for d, _, _ in devs]
        calls, reloads = m.backend.discover_calls, m.counters["reloads"]
        m.restart()
        m.restart()
        assert _wait(lambda: m.backend.discover_calls >= calls + 1)
        assert _wait(lambda: m.counters["restarts_api"] == 2)
        assert _wait(lambda: m.counters["reloads"] > reloads)
        # the stream that was open before the reload is sent the new table's list
        _, again = w.next(timeout=5)
        assert [d for d, _, _ in again] == ids
        assert c.allocate([ids[0]]).container_responses[0].devices  # same connection
        # the restart ends in a Register on the same socket (reference router/api.go:50-54)
        assert _wait(lambda: len(k.requests) >= 2) and m.counters.get("table_swaps", 0) >= 1
        assert all(r.endpoint == reg.endpoint for r in k.requests)
        assert len(k.requests) == 1 + m.counters["reregistrations_restart"]


@pytest.mark.parametrize("grpc_server", ["native", "python"])
def test_restart_api_registers_again_on_the_running_socket(make_cfg, plugin_dir, run_manager, grpc_server):
    """The reference's /restart always ends in a fresh Register (router/api.go:50-54 ->
    plugin/manager.go:177-194 -> plugin/plugin.go:140-162): the operator's way out when
    kubelet's view of the plugin went wrong while its stream is open.  One /restart ->
    exactly one new Register per resource, for the same socket file (never unbound), and a
    kubelet that re-dials on it gets a fresh stream and working Allocates."""
    from k8s_gpu_device_plugin_amd.plugin.plugin import _socket_ident
    be = fixtures.build_backend("2gpu_spx")
    with KubeletStub(plugin_dir, redial=True) as k:
        m = run_manager(make_cfg(migStrategy="mixed", grpc={"server": grpc_server}), backend=be)
        fixtures.set_gpu_mode(be, 1, "CPX", "NPS1")
        regs = k.wait_for_registrations(1)
        time.sleep(0.3)
        m.restart()  # picks up GPU 1 in CPX: two resources from here on
        assert _wait(lambda: len(m.plugins) == 2, 10)
        # that restart: the new resource registers, the kept one registers again
        assert _wait(lambda: len(k.requests) == 3 and m.counters.get("reregistrations_restart") == 1, 10)
        time.sleep(0.3)
        base = len(k.requests)
        idents = {p.resource: _socket_ident(p.socket) for p in m.plugins}
        old = k.watch(regs[0].endpoint)
        m.restart()
        assert _wait(lambda: len(k.requests) == base + 2, 10)
        time.sleep(0.5)
        assert len(k.requests) == base + 2  # exactly one per resource
        assert sorted(r.endpoint for r in k.requests[base:]) == sorted(os.path.basename(p.socket)
                                                                      for p in m.plugins)
        assert {p.resource: _socket_ident(p.socket) for p in m.plugins} == idents  # never unbound
        assert m.counters["reregistrations_restart"] >= 2
        # kubelet re-dialled: a new stream with the device list, Allocate on the new connection
        assert _wait(lambda: k.reopened >= 1, 10)  # (the one endpoint it watched)
        w = k.watch(regs[0].endpoint)
        assert w is not old
        _, devs = w.next(timeout=5)
        ids = [d for d, _, _ in devs]
        assert ids and k.client(regs[0].endpoint).allocate([ids[0]]).container_responses[0].devices
        assert m.plugins[0].list_and_watch_streams() >= 1


def test_restart_registers_again_when_discovery_fails(make_cfg, plugin_dir, run_manager):
    """A /restart whose discovery fails leaves the plugins serving (make-before-break)
    and still points kubelet at them again."""
    be = fixtures.build_backend("2gpu_spx")
    with KubeletStub(plugin_dir) as k:
        m = run_manager(make_cfg(retrySeconds=30.0), backend=be)
        k.wait_for_registrations(1)
        be.set_fail_discovery(True)
        m.restart()
        k.wait_for_registrations(2, timeout=10)
        assert m.counters["load_failures"] >= 1 and m.plugins[0].serving
        be.set_fail_discovery(False)


def test_retry_until_kubelet_appears(make_cfg, plugin_dir, run_manager):
    m = run_manager(make_cfg(retrySeconds=0.3))
    assert m.ready.wait(5)  # ready even though registration failed (D20)
    time.sleep(0.5)
    assert m.plugins and not m.plugins[0].registered
    with KubeletStub(plugin_dir) as k:
        k.wait_for_registrations(1, timeout=10)  # kubelet CREATE event or the retry timer


def test_discovery_failure_is_retried(make_cfg, plugin_dir, run_manager):
    be = fixtures.build_backend("2gpu_spx")
    be.set_fail_discovery(True)
    with KubeletStub(plugin_dir) as k:
        m = run_manager(make_cfg(retrySeconds=0.2), backend=be)
        assert m.ready.wait(5)
        assert _wait(lambda: m.counters["load_failures"] >= 1)
        be.set_fail_discovery(False)
        k.wait_for_registrations(1, timeout=10)


def test_scripted_reset_marks_unhealthy_then_healthy(make_cfg, plugin_dir, run_manager):
    model = fixtures.mi355x_node(4, events=[{"at": 0.3, "kind": "pre_reset", "gpu": 2},
                                            {"at": 0.8, "kind": "post_reset", "gpu": 2}])
    be = fixtures.build_backend(model)
    with KubeletStub(plugin_dir) as k:
        run_manager(make_cfg(), backend=be)
        w = k.watch(k.wait_for_registrations(1)[0].endpoint)
        _, devs = w.next()
        assert all(h == "Healthy" for _, h, _ in devs)
        _, devs = w.next(timeout=5)
        assert [h for _, h, _ in devs] == ["Healthy", "Healthy", "Unhealthy", "Healthy"]
        _, devs = w.next(timeout=5)
        assert all(h == "Healthy" for _, h, _ in devs)


def test_ecc_uncorrectable_via_telemetry_polling(make_cfg, plugin_dir, run_manager):
    be = fixtures.build_backend("2gpu_spx")
    with KubeletStub(plugin_dir) as k:
        m = run_manager(make_cfg(telemetry={"intervalMs": 50}), backend=be)
        w = k.watch(k.wait_for_registrations(1)[0].endpoint)
        w.next()
        time.sleep(0.2)  # baseline ECC sample
        be.set_ecc_uncorrectable(1, 3)
        _, devs = w.next(timeout=5)
        assert [h for _, h, _ in devs] == ["Healthy", "Unhealthy"]
        # the table flips on the native fast path; the manager records the transition after
        assert _wait(lambda: any("ecc_uncorrectable" in r for _, _, _, r in list(m.health_log)))
        assert 'amdgpu_ecc_errors_total{gpu="1",type="uncorrectable"} 3' in m.exporter.render()


def test_device_lost_and_recovered(make_cfg, plugin_dir, run_manager):
    be = fixtures.build_backend("2gpu_spx")
    with KubeletStub(plugin_dir) as k:
        run_manager(make_cfg(telemetry={"intervalMs": 30}, health={"lostAfterFailures": 2}), backend=be)
        w = k.watch(k.wait_for_registrations(1)[0].endpoint)
        w.next()
        be.set_gpu_present(0, False)
        _, devs = w.next(timeout=5)
        assert devs[0][1] == "Unhealthy"
        be.set_gpu_present(0, True)
        _, devs = w.next(timeout=5)
        assert devs[0][1] == "Healthy"


def test_link_down_updates_allocator_topology(make_cfg, plugin_dir, run_manager):
    be = fixtures.build_backend("4gpu_spx")
    with KubeletStub(plugin_dir) as k:
        m = run_manager(make_cfg(telemetry={"intervalMs": 50}), backend=be)
        reg = k.wait_for_registrations(1)[0]
        c = k.client(reg.endpoint)
        ids = m.plugins[0].table.ids()
        assert list(c.preferred(ids, [ids[0]], 2).container_responses[0].deviceIDs) == ids[:2]
        be.set_link_up(0, 1, False)
        assert _wait(lambda: not m.plugins[0].table.topology().link(0, 1).up)
        got = list(c.preferred(ids, [ids[0]], 2).container_responses[0].deviceIDs)
        assert got[0] == ids[0] and got[1] != ids[1]


def test_stop_is_idempotent_and_quick(make_cfg, plugin_dir):
    with KubeletStub(plugin_dir):
        m = PluginManager(make_cfg())
        t = m.start_background()
        m.stop()
        m.stop()
        t.join(5)
        assert not t.is_alive() and m.wait_stopped(1)
        assert not os.path.exists(os.path.join(plugin_dir, "amd-gpu.sock"))


def test_event_loop_does_not_spin(make_cfg, plugin_dir, run_manager):
    """Reference defect D4: the manager's `default:` branch pins a CPU core."""
    with KubeletStub(plugin_dir) as k:
        run_manager(make_cfg(telemetry={"intervalMs": 1000}))
        k.wait_for_registrations(1)
        t0, c0 = time.monotonic(), time.process_time()
        time.sleep(1.0)
        cpu = (time.process_time() - c0) / (time.monotonic() - t0)
        assert cpu < 0.25, cpu  # the whole process, all threads


def test_device_filter(make_cfg, plugin_dir, run_manager):
    with KubeletStub(plugin_dir) as k:
        m = run_manager(make_cfg(fixture="8gpu_spx_mesh", devices="0-3"))
        _, devs = k.watch(k.wait_for_registrations(1)[0].endpoint).next()
        assert len(devs) == 4 and [g.index for g in m.gpus] == [0, 1, 2, 3]


def test_mixed_strategy_registers_one_plugin_per_resource(make_cfg, plugin_dir, run_manager):
    model = fixtures.mi355x_node(2)
    model["gpus"].append({"compute_partition": "CPX", "memory_partition": "NPS2", "numa_node": 1})
    with KubeletStub(plugin_dir) as k:
        run_manager(make_cfg(migStrategy="mixed"), backend=fixtures.build_backend(model))
        regs = k.wait_for_registrations(2)
        assert sorted((r.resource_name, r.endpoint) for r in regs) == [
            ("amd.com/cpx_nps2", "amd-cpx_nps2.sock"), ("amd.com/gpu", "amd-gpu.sock")]
        _, devs = k.watch("amd-cpx_nps2.sock").next()
        assert len(devs) == 8


def test_no_devices_waits(make_cfg, plugin_dir, run_manager, n):
    with KubeletStub(plugin_dir) as k:
        m = run_manager(make_cfg(), backend=n.FixtureBackend(1))
        assert m.ready.wait(5)
        time.sleep(0.3)
        assert not k.requests and m.running


def test_concurrent_restart_requests_are_serialized(make_cfg, plugin_dir, run_manager):
    with KubeletStub(plugin_dir) as k:
        m = run_manager(make_cfg())
        k.wait_for_registrations(1)
        ts = [threading.Thread(target=m.restart) for _ in range(10)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        assert _wait(lambda: m.counters["restarts_api"] == 10, timeout=20)
        # reloads run behind the requests (discovery on its worker, then the swap)
        assert _wait(lambda: m.events.empty() and not m._discoverer.pending(), timeout=20)
        assert _wait(lambda: m.plugins and m.plugins[0].registered, timeout=20)
        assert k.client("amd-gpu.sock").get_options().get_preferred_allocation_available


def test_startup_canary_marks_failing_partition_unhealthy(make_cfg, plugin_dir, run_manager, monkeypatch):
    from k8s_gpu_device_plugin_amd.ops import canary
    calls = []

    def fake_run_isolated(device, nbytes, timeout=120.0):
        calls.append(device)
        return {"ok": device != 9, "device": device, "error": "" if device != 9 else "hbm mismatch"}
    monkeypatch.setattr(canary, "run_isolated", fake_run_isolated)
    with KubeletStub(plugin_dir) as k:
        m = run_manager(make_cfg(fixture="2gpu_cpx_nps2", migStrategy="single", health={"canaryOnStart": True}))
        w = k.watch(k.wait_for_registrations(1)[0].endpoint)
        assert _wait(lambda: not m._start_pending)  # verdicts arrive off the manager thread
        devs = w.last(timeout=5)
        assert sorted(calls) == list(range(16))
        bad = [i for i, (_, h, _) in enumerate(devs) if h == "Unhealthy"]
        assert bad == [9]  # GPU 1, partition 1 (hip id 9)
        assert m.counters["canary_failures"] == 1 and m.counters["canary_runs"] == 16


def test_partition_mode_change_is_rediscovered(make_cfg, plugin_dir, run_manager):
    be = fixtures.build_backend("2gpu_spx")
    with KubeletStub(plugin_dir) as k:
        m = run_manager(make_cfg(migStrategy="single", rediscoverIntervalS=0.2), backend=be)
        _, devs = k.watch(k.wait_for_registrations(1)[0].endpoint).next()
        assert len(devs) == 2
        fixtures.set_gpu_mode(be, 1, "CPX", "NPS2")  # operator switches GPU 1 to CPX
        assert _wait(lambda: m.counters.get("restarts_inventory", 0) >= 1, timeout=10)
        assert _wait(lambda: len(m.plugins[0].table.ids()) == 9)
        assert len(k.requests) == 1  # same registration: the new table went into the running server
        c = k.client("amd-gpu.sock")
        ids = m.plugins[0].table.ids()
        assert len(ids) == 9 and ids[1].endswith("-xcp0")
        r = c.allocate([ids[4]])
        assert [s.host_path for s in r.container_responses[0].devices] == ["/dev/kfd", "/dev/dri/renderD203"]


def test_cdi_spec_written_and_allocate_names(make_cfg, plugin_dir, run_manager, tmp_path):
    import json
    with KubeletStub(plugin_dir) as k:
        m = run_manager(make_cfg(cdi=True, cdiSpecDir=str(tmp_path / "cdi")))
        k.wait_for_registrations(1)
        spec = json.load(open(tmp_path / "cdi" / "amd.com-gpu.json"))
        assert spec["kind"] == "amd.com/gpu" and spec["cdiVersion"] == "0.6.0"
        assert spec["containerEdits"]["deviceNodes"][0]["path"] == "/dev/kfd"
        ids = m.plugins[0].table.ids()
        assert [d["name"] for d in spec["devices"]] == ids
        assert spec["devices"][1]["containerEdits"]["deviceNodes"][0]["path"] == "/dev/dri/renderD129"
        r = k.client("amd-gpu.sock").allocate([ids[1]])
        assert [d.name for d in r.container_responses[0].cdi_devices] == ["amd.com/gpu=" + ids[1]]


def _gate_canary(monkeypatch, verdicts):
    """Replaces the isolated canary with one that blocks until released."""
    from k8s_gpu_device_plugin_amd.ops import canary
    gate = threading.Event()
    calls = []

    def fake_run_isolated(device, nbytes, timeout=120.0):
        calls.append(device)
        gate.wait(10)
        return {"ok": verdicts.pop(0) if verdicts else True, "device": device}
    monkeypatch.setattr(canary, "run_isolated", fake_run_isolated)
    return gate, calls


def test_recovery_canary_runs_off_the_event_loop(make_cfg, plugin_dir, run_manager, monkeypatch):
    """post_reset with health.canary: the GPU stays Unhealthy until the canary passes,
    and the manager keeps serving other events (here /restart) while it runs."""
    gate, calls = _gate_canary(monkeypatch, [True])
    be = fixtures.build_backend("2gpu_spx")
    with KubeletStub(plugin_dir) as k:
        m = run_manager(make_cfg(health={"canary": True}), backend=be)
        w = k.watch(k.wait_for_registrations(1)[0].endpoint)
        w.next()
        be.inject_event(be_event(m, "EVT_PRE_RESET", 1))
        _, devs = w.next(timeout=5)
        assert [h for _, h, _ in devs] == ["Healthy", "Unhealthy"]
        be.inject_event(be_event(m, "EVT_POST_RESET", 1))
        assert _wait(lambda: calls == [1])
        m.restart()  # handled while the canary is still blocked
        assert _wait(lambda: m.counters["restarts_api"] == 1)
        assert _wait(lambda: m.counters["reloads"] >= 2, timeout=10)
        time.sleep(0.2)
        assert m.plugins[0].table.healthy_count() == 1  # reloaded, GPU 1 still held until verified
        gate.set()
        assert _wait(lambda: m.plugins and m.plugins[0].table.healthy_count() == 2)


def test_stale_canary_verdict_is_dropped(make_cfg, plugin_dir, run_manager, monkeypatch):
    """A new Unhealthy event while the recovery canary runs wins over its (passing) verdict."""
    gate, calls = _gate_canary(monkeypatch, [True])
    be = fixtures.build_backend("2gpu_spx")
    with KubeletStub(plugin_dir) as k:
        m = run_manager(make_cfg(health={"canary": True}), backend=be)
        k.wait_for_registrations(1)
        be.inject_event(be_event(m, "EVT_PRE_RESET", 0))
        assert _wait(lambda: m.plugins[0].table.healthy_count() == 1)
        be.inject_event(be_event(m, "EVT_POST_RESET", 0))
        assert _wait(lambda: calls == [0])
        be.inject_event(be_event(m, "EVT_PRE_RESET", 0))
        assert _wait(lambda: m.counters["health_events"] >= 3)
        gate.set()
        time.sleep(0.3)
        assert m.plugins[0].table.healthy_count() == 1
        assert list(m.health_log)[-1][2] == 0


def be_event(m, kind, gpu):
    from k8s_gpu_device_plugin_amd import native
    n = native.load()
    return n.HwEvent(getattr(n, kind), gpu, -1, -1, "test")


def test_node_feature_file_tracks_partition_mode(make_cfg, plugin_dir, run_manager, tmp_path):
    """Optional NFD local-feature labels; rewritten when the partition mode changes."""
    path = tmp_path / "features.d" / "amd-gpu"
    be = fixtures.build_backend("2gpu_spx")
    with KubeletStub(plugin_dir) as k:
        m = run_manager(make_cfg(migStrategy="single", rediscoverIntervalS=0.2, nodeFeatureFile=str(path)),
                        backend=be)
        k.wait_for_registrations(1)
        labels = dict(ln.split("=", 1) for ln in path.read_text().splitlines())
        assert labels["amd.com/gpu.count"] == "2" and labels["amd.com/gpu.compute-partition"] == "SPX"
        assert labels["amd.com/gpu.product"] == "AMD_Instinct_MI355X" and labels["amd.com/gpu.family"] == "gfx950"
        assert labels["amd.com/gpu.vram-gb"] == "288" and labels["amd.com/gpu.partitions"] == "2"
        assert labels["amd.com/gpu.device-id"] == "75a3"
        assert labels["amd.com/gpu.driver-version"] == fixtures.FIXTURE_DRIVER_VERSION
        assert labels["amd.com/gpu.vbios-version"] == fixtures.FIXTURE_VBIOS_VERSION
        fixtures.set_gpu_mode(be, 0, "CPX", "NPS2")
        fixtures.set_gpu_mode(be, 1, "CPX", "NPS2")
        assert _wait(lambda: "gpu.compute-partition=CPX" in path.read_text(), timeout=10)
        labels = dict(ln.split("=", 1) for ln in path.read_text().splitlines())
        assert labels["amd.com/gpu.partitions"] == "16" and labels["amd.com/gpu.memory-partition"] == "NPS2"
        assert m.counters.get("restarts_inventory", 0) >= 1


def test_reset_state_survives_a_reload(make_cfg, plugin_dir, run_manager):
    """A GPU mid-reset when kubelet restarts (full reload) must still come back Healthy
    on POST_RESET: the monitor keeps per-GPU state across reloads."""
    be = fixtures.build_backend("2gpu_spx")
    with KubeletStub(plugin_dir) as k:
        m = run_manager(make_cfg(), backend=be)
        k.wait_for_registrations(1)
        be.inject_event(be_event(m, "EVT_PRE_RESET", 1))
        assert _wait(lambda: m.plugins[0].table.healthy_count() == 1)
        m.restart()
        assert _wait(lambda: m.counters["reloads"] >= 2, timeout=10)
        assert _wait(lambda: m.counters["restarts_api"] == 1)
        assert m.plugins[0].table.healthy_count() == 1  # still held Unhealthy after the reload
        be.inject_event(be_event(m, "EVT_POST_RESET", 1))
        assert _wait(lambda: m.plugins[0].table.healthy_count() == 2)


def test_pod_resources_allocation_metric(make_cfg, plugin_dir, run_manager, tmp_path):
    """podResources.enabled: the kubelet PodResources List is polled and every held
    device of ours appears as allocation_info{namespace,pod,container}; other vendors'
    resources are ignored; a kubelet outage flips pod_resources_up to 0."""
    from k8s_gpu_device_plugin_amd.plugin.kubelet_stub import PodResourcesStub
    sock = str(tmp_path / "pod-resources" / "kubelet.sock")
    stub = PodResourcesStub(sock).start()
    try:
        with KubeletStub(plugin_dir) as k:
            m = run_manager(make_cfg(podResources={"enabled": True, "socket": sock, "intervalS": 0.05}))
            k.wait_for_registrations(1)
            ids = m.plugins[0].table.ids()
            stub.set_pods([("ml", "trainer-0", [("main", "amd.com/gpu", ids[:1]), ("side", "nvidia.com/gpu", ["x"])]),
                           ("ml", "trainer-1", [("main", "amd.com/gpu", ids[1:2])])])
            want0 = ('amdgpu_device_plugin_allocation_info{resource="amd.com/gpu",device_id="%s",namespace="ml",'
                     'pod="trainer-0",container="main"} 1' % ids[0])
            assert _wait(lambda: want0 in m.exporter.render())
            text = m.exporter.render()
            assert "amdgpu_device_plugin_pod_resources_up 1" in text
            assert 'pod="trainer-1"' in text and "nvidia.com" not in text
            stub.set_pods([("ml", "trainer-1", [("main", "amd.com/gpu", ids[1:2])])])  # trainer-0 finished
            assert _wait(lambda: 'pod="trainer-0"' not in m.exporter.render())
            stub.stop()
            assert _wait(lambda: "amdgpu_device_plugin_pod_resources_up 0" in m.exporter.render())
            assert 'pod="trainer-1"' in m.exporter.render()  # last known map is kept
    finally:
        stub.stop()


class _InjectOnCall:
    """Delegating proxy that runs ``hook`` once, the first time ``method`` is called
    while armed."""

    def __init__(self, target, method, hook):
        self._target, self._method, self._hook, self.armed = target, method, hook, False

    def __getattr__(self, name):
        attr = getattr(self._target, name)
        if name != self._method:
            return attr

        def wrapped(*a, **kw):
            if self.armed:
                self.armed = False
                self._hook()
            return attr(*a, **kw)
        return wrapped


@pytest.mark.parametrize("canary", [False, True])
@pytest.mark.parametrize("where", ["plugin_build", "exporter_inventory"])
def test_health_event_during_reload_reaches_new_tables(make_cfg, plugin_dir, monkeypatch, where, canary):
    """a PRE_RESET processed while load_plugins builds the new plugins
    must reach the new tables whatever the point of the reload it lands on - before the
    monitor adopts them (written in at adoption) or after (fast path).  The old code read
    the monitor state, then installed the fast tables later: an event in between went
    only to the outgoing tables, and the GPU stayed advertised Healthy."""
    from k8s_gpu_device_plugin_amd.plugin import manager as manager_mod
    be = fixtures.build_backend("2gpu_spx")
    m = PluginManager(make_cfg(health={"canary": canary}), backend=be)
    inject = lambda: m.monitor.process(be_event(m, "EVT_PRE_RESET", 1))  # noqa: E731
    if where == "exporter_inventory":
        proxy = _InjectOnCall(m.exporter, "set_inventory", inject)
        m.exporter = proxy
    else:
        real = manager_mod.AmdDevicePlugin

        class proxy:  # noqa: N801 - stands in for the class
            armed = False

        def build(*a, **kw):
            p = real(*a, **kw)
            if proxy.armed:
                proxy.armed = False
                inject()
            return p
        monkeypatch.setattr(manager_mod, "AmdDevicePlugin", build)
    with KubeletStub(plugin_dir) as k:
        t = m.start_background()
        try:
            k.wait_for_registrations(1)
            assert m.plugins[0].table.healthy_count() == 2
            proxy.armed = True
            m.restart()
            assert _wait(lambda: m.counters["reloads"] >= 2, timeout=10)
            assert _wait(lambda: m.counters["restarts_api"] == 1)
            assert not proxy.armed, "the hook did not run during the reload"
            assert _wait(lambda: m.plugins[0].table.healthy_count() == 1), "GPU 1 advertised Healthy after reload"
            assert not m.plugins[0].table.healthy(m.plugins[0].table.ids()[1])
            w = k.watch("amd-gpu.sock")
            _, devs = w.next()
            assert [h for _, h, _ in devs] == ["Healthy", "Unhealthy"]
        finally:
            m.stop()
            t.join(10)


def _full_canary_result(device, ok=True, read=5900.0, tflops=1800.0):
    return {"ok": ok, "device": device, "error": "", "hbm_errors": 0, "mfma_errors": 0, "gemm_errors": 0,
            "lowp_errors": 0, "lds_errors": 0, "write_gbps": 6100.0, "read_gbps": read, "mfma_tflops": tflops,
            "gemm_tflops": 1400.0, "fp8_tflops": 3800.0, "fp4_tflops": 6500.0}


def test_canary_results_are_exported_per_partition(make_cfg, plugin_dir, run_manager, monkeypatch):
    """Every canary run (start-up here) leaves its verdict, HBM bandwidth and matrix-core
    rates in /metrics, labelled with the GPU and hardware partition it ran on."""
    from prometheus_client.parser import text_string_to_metric_families

    from k8s_gpu_device_plugin_amd.ops import canary
    monkeypatch.setattr(canary, "run_isolated",
                        lambda device, nbytes, timeout=120.0: _full_canary_result(device, read=5000.0 + device))
    with KubeletStub(plugin_dir) as k:
        m = run_manager(make_cfg(fixture="2gpu_cpx_nps2", migStrategy="single", health={"canaryOnStart": True}))
        k.wait_for_registrations(1)
        assert _wait(lambda: 'partition="7",direction="read"' in m.exporter.render())
        fams = {f.name: f for f in text_string_to_metric_families(m.exporter.render())}
        ok = [s for s in fams["amdgpu_canary_last_ok"].samples]
        assert len(ok) == 16 and all(s.value == 1 for s in ok)
        reads = {(s.labels["gpu"], s.labels["partition"]): s.value for s in fams["amdgpu_canary_hbm_gbps"].samples
                 if s.labels["direction"] == "read"}
        assert reads[("1", "1")] == 5009.0  # GPU 1 partition 1 is HIP device 9 on this fixture
        paths = {s.labels["path"] for s in fams["amdgpu_canary_matrix_tflops"].samples}
        assert paths == {"mfma_bf16", "gemm_bf16", "mxfp8", "mxfp4"}
        checks = {s.labels["check"] for s in fams["amdgpu_canary_errors"].samples}
        assert checks == {"hbm", "mfma", "gemm", "lowp", "lds"}


def test_canary_performance_floor_marks_slow_partition_unhealthy(make_cfg, plugin_dir, run_manager, monkeypatch):
    """health.canaryMinHbmGbps / canaryMinTflops: exact but slow (throttled, degraded HBM)
    partitions fail the canary like wrong ones do."""
    from k8s_gpu_device_plugin_amd.ops import canary
    monkeypatch.setattr(canary, "run_isolated", lambda device, nbytes, timeout=120.0: _full_canary_result(
        device, read=2500.0 if device == 3 else 5900.0, tflops=900.0 if device == 12 else 1800.0))
    with KubeletStub(plugin_dir) as k:
        m = run_manager(make_cfg(fixture="2gpu_cpx_nps2", migStrategy="single",
                                 health={"canaryOnStart": True, "canaryMinHbmGbps": 4000, "canaryMinTflops": 1500}))
        _, devs = k.watch(k.wait_for_registrations(1)[0].endpoint).next()
        bad = [i for i, (_, h, _) in enumerate(devs) if h == "Unhealthy"]
        assert bad == [3, 12]
        assert m.counters["canary_failures"] == 2
        _, r = m.canary_results[(0, 3)]
        assert not r["ok"] and "HBM 2500 GB/s < 4000" in r["error"]
        _, r = m.canary_results[(1, 4)]
        assert "bf16 MFMA 900 TFLOP/s < 1500" in r["error"]


def test_restart_burst_is_coalesced(make_cfg, plugin_dir, run_manager, monkeypatch):
    """100 /restart calls that arrive while a discovery runs are served by the next one,
    not by 100 reloads: every request is counted, a handful of reloads happen, and the
    plugin ends registered and serving."""
    with KubeletStub(plugin_dir) as k:
        m = run_manager(make_cfg())
        k.wait_for_registrations(1)
        orig = m.backend.discover
        reloads0 = m.counters["reloads"]

        class SlowBackend:  # the burst lands while each discovery runs
            def __getattr__(self, name):
                return getattr(m.backend_real, name)

            def discover(self):
                time.sleep(0.05)
                return orig()
        m.backend_real = m.backend
        m._discoverer._backend = SlowBackend()
        for _ in range(100):
            m.restart()
        assert _wait(lambda: m.counters["restarts_api"] == 100, timeout=20)
        assert _wait(lambda: m.events.empty() and not m._discoverer.pending(), timeout=10)
        time.sleep(0.1)
        reloads = m.counters["reloads"] - reloads0
        assert 1 <= reloads <= 5, reloads
        assert k.client("amd-gpu.sock").get_options().get_preferred_allocation_available


@pytest.mark.skipif(bool(os.environ.get("AMDGPU_DP_NATIVE_SO")),
                    reason="sanitizer runs: ASan's quarantine holds freed memory, TSan is too slow for a soak")
def test_soak_reloads_under_traffic_do_not_grow_the_daemon():
    """scripts/soak.py on the fixture backend: Allocate + scrapes + a /restart every 50 ms
    for 10 s.  Every reload swaps its table into the running server - no Allocate fails,
    the Allocate connection and the ListAndWatch stream never drop, the plugin registers
    once - and the daemon does not grow (per-reload leaks, e.g. render caches of replaced
    tables, showed up here as ~10 KB per reload)."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    p = subprocess.run([sys.executable, os.path.join(root, "scripts", "soak.py"), "--seconds", "10",
                        "--restart-every", "0.05", "--backend", "fixture"], stdout=subprocess.PIPE,
                       stderr=subprocess.DEVNULL, text=True, timeout=120)
    r = json.loads(p.stdout.strip().splitlines()[-1])
    assert r["ok"], r
    # bursts of /restart coalesce into fewer reloads; every reload swapped its table in
    assert r["restarts"] >= 50 and r["reloads"] >= 10 and r["table_swaps"] >= r["reloads"] - 1
    assert r["reconnects"] == 0 and r["law_reopens"] == 1
    assert r["registrations"] == 1 + r["reregistrations_restart"] and r["reregistrations_restart"] >= 1
    assert r["law_updates"] >= r["table_swaps"] // 2
    assert r["rss_growth_second_half_kb"] < 600, r["rss_kb"]


def test_kubelet_restart_that_wipes_plugin_sockets(make_cfg, plugin_dir, run_manager):
    """What a kubelet restart does on disk: kubelet.sock goes, kubelet clears the
    plugin sockets from the directory, then binds a new kubelet.sock.  The plugin is
    registered again promptly (no retry-timer wait) and serves on a socket that exists."""
    with KubeletStub(plugin_dir) as k:
        m = run_manager(make_cfg(retrySeconds=30.0))
        k.wait_for_registrations(1)
        k.stop()
        os.remove(os.path.join(plugin_dir, "amd-gpu.sock"))
        time.sleep(0.05)
        t0 = time.monotonic()
        k.start()
        k.wait_for_registrations(2, timeout=10)
        assert time.monotonic() - t0 < 5.0
        time.sleep(0.5)
        assert os.path.exists(os.path.join(plugin_dir, "amd-gpu.sock"))
        assert k.client("amd-gpu.sock").get_options().get_preferred_allocation_available
        print("registrations", len(k.requests), m.counters)


def test_health_follows_gpu_identity_through_rediscovery(make_cfg, plugin_dir, run_manager):
    """GPU 0 enters a reset and falls off the bus; the periodic re-discovery re-advertises
    the node with GPU 1 at index 0.  That GPU stays Healthy (state is keyed by identity,
    not index); when GPU 0 returns it is advertised Unhealthy until its POST_RESET."""
    from k8s_gpu_device_plugin_amd import native
    n = native.load()
    be = fixtures.build_backend("2gpu_spx")
    gpus, _ = be.discover()
    ids = [g.partitions[0].id for g in gpus]
    with KubeletStub(plugin_dir) as k:
        m = run_manager(make_cfg(telemetry={"intervalMs": 30}, rediscoverIntervalS=0.2,
                                 health={"lostAfterFailures": 2}), backend=be)
        k.wait_for_registrations(1)
        table = lambda: m.plugins[0].table  # noqa: E731 - replaced by every reload
        be.inject_event(n.HwEvent(n.EVT_PRE_RESET, 0, message="fixture reset"))
        assert _wait(lambda: not table().healthy(ids[0]))
        be.set_gpu_present(0, False)
        assert _wait(lambda: table().ids() == [ids[1]], timeout=10)
        time.sleep(0.4)  # several sampling passes and re-discoveries over the new indices
        assert table().healthy(ids[1])
        reg = k.requests[-1]  # the reload kept the registration
        _, devs = k.watch(reg.endpoint).next()
        assert [(d, h) for d, h, _ in devs] == [(ids[1], "Healthy")]
        be.set_gpu_present(0, True)
        assert _wait(lambda: table().ids() == ids, timeout=10)
        assert not table().healthy(ids[0]) and table().healthy(ids[1])
        time.sleep(0.3)  # its telemetry answers again: still mid-reset, still Unhealthy
        assert not table().healthy(ids[0])
        be.inject_event(n.HwEvent(n.EVT_POST_RESET, 0))
        assert _wait(lambda: table().healthy(ids[0]) and table().healthy(ids[1]))
        assert _wait(lambda: m.monitor.unhealthy_keys() == [])


def test_canary_result_does_not_pass_to_the_gpu_that_takes_its_index(make_cfg, plugin_dir, run_manager):
    """A canary result is the GPU's, not the index's: when GPU 0 falls off the bus and
    GPU 1 moves to index 0, /metrics stops showing GPU 0's result under index 0."""
    be = fixtures.build_backend("2gpu_spx")
    with KubeletStub(plugin_dir) as k:
        m = run_manager(make_cfg(rediscoverIntervalS=0.2), backend=be)
        k.wait_for_registrations(1)
        with m._canary_lock:  # as a canary run on GPU 0 and one on GPU 1 would leave them
            for g in (0, 1):
                m.canary_results[(g, 0)] = (time.time(), {"ok": g == 1})
                m._canary_owner[(g, 0)] = m._key_of[g]
        be.set_gpu_present(0, False)
        assert _wait(lambda: len(m.plugins) == 1 and m.plugins[0].table.ids() != [], timeout=10)
        assert _wait(lambda: len(m.gpus) == 1, timeout=10)

        def pruned():  # the reload prunes them just after it installs the new inventory
            with m._canary_lock:
                return m.canary_results == {}  # (0, 0) was GPU 0's, (1, 0) no longer exists
        assert _wait(pruned, timeout=5), m.canary_results


def test_link_retrain_reaches_the_allocator(make_cfg, plugin_dir, run_manager):
    """An up xGMI link re-trains at half its rate: the telemetry poll reports it, the
    table's topology takes the new bandwidth, and a 2-GPU request that must include
    GPU 0 moves off that link."""
    be = fixtures.build_backend("4gpu_spx")
    with KubeletStub(plugin_dir) as k:
        m = run_manager(make_cfg(telemetry={"intervalMs": 30}), backend=be)
        c = k.client(k.wait_for_registrations(1)[0].endpoint)
        ids = m.plugins[0].table.ids()
        assert m.plugins[0].table.topology().link(0, 1).bw_gbps == 608.0  # from discovery
        assert list(c.preferred(ids, [ids[0]], 2).container_responses[0].deviceIDs) == ids[:2]
        be.set_link_bandwidth(0, 1, 304.0)
        assert _wait(lambda: m.plugins[0].table.topology().link(0, 1).bw_gbps == 304.0)
        assert list(c.preferred(ids, [ids[0]], 2).container_responses[0].deviceIDs) == [ids[0], ids[2]]
        be.set_link_bandwidth(0, 1, 608.0)
        assert _wait(lambda: m.plugins[0].table.topology().link(0, 1).bw_gbps == 608.0)


def test_link_state_is_resynced_after_a_reload(make_cfg, plugin_dir, run_manager):
    """Found by the chaos test: a link re-trains at a quarter rate while it is down, and
    a reload's discovery puts that rate into the new tables.  The link then comes back up
    at full rate - the value the monitor last reported, so it saw no change and the
    tables kept the stale rate.  Every link is now reported once more after a reload."""
    be = fixtures.build_backend("4gpu_spx")
    with KubeletStub(plugin_dir) as k:
        m = run_manager(make_cfg(fixture="4gpu_spx", telemetry={"intervalMs": 30}), backend=be)
        k.wait_for_registrations(1)
        topo = lambda: m.plugins[0].table.topology()  # noqa: E731 - replaced by every reload
        be.set_link_up(0, 1, False)
        assert _wait(lambda: not topo().link(0, 1).up)
        be.set_link_bandwidth(0, 1, 152.0)
        m.restart()
        assert _wait(lambda: m.counters["reloads"] >= 2, timeout=10)
        assert _wait(lambda: m.plugins and topo().link(0, 1).bw_gbps == 152.0 and not topo().link(0, 1).up)
        be.set_link_bandwidth(0, 1, 608.0)
        be.set_link_up(0, 1, True)
        assert _wait(lambda: topo().link(0, 1).up and topo().link(0, 1).bw_gbps == 608.0), \
            (topo().link(0, 1).up, topo().link(0, 1).bw_gbps)
        # a link that flapped down between the last sample and the reload's discovery
        be.set_link_up(2, 3, False)
        m.restart()  # may or may not see it down; either way the tables converge
        be.set_link_up(2, 3, True)
        assert _wait(lambda: m.plugins and topo().link(2, 3).up)


def test_halfrate_fixture_is_discovered_degraded(n):
    gpus, topo = fixtures.build_backend("8gpu_spx_halfrate").discover()
    from topology_model import NodeTopology
    assert NodeTopology(gpus, topo).degraded_links() == [(0, 1)]


def test_pod_resources_feed_link_load_to_the_allocator(make_cfg, plugin_dir, run_manager, tmp_path):
    """CPX: a running pod holds partitions on GPUs 0 and 1 (PodResources).  The tables'
    topology counts it on link 0-1, /metrics shows it, and a new 2-GPU pod is placed off
    that link."""
    from k8s_gpu_device_plugin_amd.plugin.kubelet_stub import PodResourcesStub
    sock = str(tmp_path / "pod-resources" / "kubelet.sock")
    stub = PodResourcesStub(sock).start()
    try:
        with KubeletStub(plugin_dir) as k:
            m = run_manager(make_cfg(fixture="4gpu_cpx", migStrategy="single",
                                     podResources={"enabled": True, "socket": sock, "intervalS": 0.05}))
            c = k.client(k.wait_for_registrations(1)[0].endpoint)
            ids = m.plugins[0].table.ids()  # 8 partitions per GPU, GPU-major
            held = ids[0:4] + ids[8:12]
            stub.set_pods([("ml", "ring-0", [("main", "amd.com/gpu", held)])])
            assert _wait(lambda: m.plugins[0].table.topology().link(0, 1).pods == 1)
            assert 'amdgpu_xgmi_link_pods{gpu="0",peer="1"} 1' in m.exporter.render()
            avail = ids[4:8] + ids[12:16] + ids[20:24]  # 4 free on each of GPUs 0, 1, 2
            got = list(c.preferred(avail, [], 8).container_responses[0].deviceIDs)
            gpus = sorted({ids.index(x) // 8 for x in got})
            assert gpus in ([0, 2], [1, 2]), gpus
            stub.set_pods([])
            assert _wait(lambda: m.plugins[0].table.topology().link(0, 1).pods == 0)
    finally:
        stub.stop()


def test_pod_link_load_uses_the_whole_node_topology(make_cfg, plugin_dir, run_manager, tmp_path):
    """`devices` advertises GPUs 0-2 of a 4-GPU node: the tables' topology still spans all
    4 GPUs, so a pod on GPUs 1 and 2 must land on link 1-2 (a row stride of 3 put it on
    1-1 and 1-3)."""
    from k8s_gpu_device_plugin_amd.plugin.kubelet_stub import PodResourcesStub
    sock = str(tmp_path / "pod-resources" / "kubelet.sock")
    stub = PodResourcesStub(sock).start()
    try:
        with KubeletStub(plugin_dir) as k:
            m = run_manager(make_cfg(fixture="4gpu_cpx", migStrategy="single", devices="0-2",
                                     podResources={"enabled": True, "socket": sock, "intervalS": 0.05}))
            k.wait_for_registrations(1)
            t = m.plugins[0].table
            assert t.topology().n == 4 and len(t.ids()) == 24
            ids = t.ids()
            stub.set_pods([("ml", "ring-1", [("main", "amd.com/gpu", ids[8:12] + ids[16:20])])])
            assert _wait(lambda: t.topology().link(1, 2).pods == 1)
            topo = t.topology()
            assert topo.link(2, 1).pods == 1
            assert sum(topo.link(a, b).pods for a in range(4) for b in range(4)) == 2
            assert 'amdgpu_xgmi_link_pods{gpu="1",peer="2"} 1' in m.exporter.render()
    finally:
        stub.stop()


def test_devices_selection_stays_on_the_same_gpus(make_cfg, plugin_dir, run_manager):
    """`devices: 0-2` on a 4-GPU node.  GPU 0 drops off the bus and the others move down
    an index: the plugin must advertise GPUs 1 and 2, not take in GPU 3 (an operator may
    have kept it for something else).  UUIDs and BDFs select the same way."""
    be = fixtures.build_backend("4gpu_spx")
    gpus, _ = be.discover()
    uuid = {g.index: g.partitions[0].id for g in gpus}
    with KubeletStub(plugin_dir) as k:
        m = run_manager(make_cfg(fixture="4gpu_spx", devices="0-2", rediscoverIntervalS=0.1), backend=be)
        k.wait_for_registrations(1)
        assert sorted(m.plugins[0].table.ids()) == sorted(uuid[i] for i in (0, 1, 2))
        be.set_gpu_present(0, False)
        assert _wait(lambda: m.plugins and sorted(m.plugins[0].table.ids()) == sorted([uuid[1], uuid[2]]),
                     timeout=10), m.plugins[0].table.ids()
        time.sleep(0.3)
        assert uuid[3] not in m.plugins[0].table.ids()
        be.set_gpu_present(0, True)
        assert _wait(lambda: m.plugins and sorted(m.plugins[0].table.ids()) == sorted(uuid[i] for i in (0, 1, 2)),
                     timeout=10)
    from k8s_gpu_device_plugin_amd.utils.util import parse_device_selector
    assert parse_device_selector("0-1, 5,0000:75:00.0,ABC-def") == ([0, 1, 5], {"0000:75:00.0", "abc-def"})
    assert parse_device_selector("") is None and parse_device_selector("all") is None
    by_name = PluginManager(make_cfg(fixture="4gpu_spx", devices="%s,%s" % (gpus[3].bdf, gpus[1].uuid.upper())),
                            backend=fixtures.build_backend("4gpu_spx"))
    assert sorted(g.index for g in by_name._selected(gpus)) == [1, 3]
    # hip:<n> selects the GPU a HIP ordinal opens (bench.py advertises hip:0-<N-1>), also
    # where HIP numbers GPUs in another order than PCI
    assert parse_device_selector("hip:0-1,2") == ([2], {"hip:0", "hip:1"})
    pbe = fixtures.build_backend("4gpu_spx_hip_permuted")
    pgpus, _ = pbe.discover()
    by_hip = PluginManager(make_cfg(fixture="4gpu_spx_hip_permuted", devices="hip:0-1"), backend=pbe)
    chosen = by_hip._selected(pgpus)
    assert sorted(p.hip_id for g in chosen for p in g.partitions) == [0, 1]
    assert sorted(g.index for g in chosen) != [0, 1], "fixture no longer permutes HIP against BDF order"
    # a driver that reports no HIP ordinals: hip:<n> is BDF rank n
    for g in pgpus:
        for p in g.partitions:
            p.hip_id = -1
    no_hip = PluginManager(make_cfg(fixture="4gpu_spx_hip_permuted", devices="hip:0-1"),
                           backend=fixtures.build_backend("4gpu_spx_hip_permuted"))
    no_hip._note_seen(pgpus)
    by_bdf = sorted(pgpus, key=lambda g: g.bdf.lower())[:2]
    assert sorted(g.index for g in no_hip._selected(pgpus)) == sorted(g.index for g in by_bdf)
    assert sorted(g.index for g in by_bdf) != sorted(g.index for g in chosen)


@pytest.mark.parametrize("fault", ["worker", "listener"])
def test_native_server_fault_is_restarted_and_reregistered(make_cfg, plugin_dir, run_manager, fault):
    """The native gRPC server loses a worker (exception) or its listening socket: the
    manager's supervision poll restarts it on a fresh socket and registers again
    (reference Serve crash-restart loop, plugin/plugin.go:107-129)."""
    with KubeletStub(plugin_dir) as k:
        m = run_manager(make_cfg(grpc={"server": "native"}))
        k.wait_for_registrations(1)
        srv = m.plugins[0]._native_server
        srv.inject_fault(fault)
        assert _wait(lambda: srv.failure() != "", timeout=3)
        k.wait_for_registrations(2, timeout=10)
        assert _wait(lambda: m.counters.get("restarts_server", 0) == 1)
        assert m.plugins[0]._native_server is not srv and not m.plugins[0]._native_server.failure()
        c = k.client("amd-gpu.sock")
        ids = m.plugins[0].table.ids()
        assert c.allocate(ids[:1]).container_responses[0].devices
        assert m.fatal_error is None and m.running


def test_native_server_crash_loop_is_fatal(make_cfg, plugin_dir):
    """More than 5 crashes within an hour: the manager stops with fatal_error set (the
    CLI exits non-zero), like the reference's Logger.Fatal."""
    with KubeletStub(plugin_dir) as k:
        m = PluginManager(make_cfg(grpc={"server": "native"}))
        t = m.start_background()
        try:
            k.wait_for_registrations(1)
            for i in range(6):
                p = m.plugins[0]
                srv = p._native_server
                srv.inject_fault("worker")
                if i < 5:  # restarted and registered again before the next fault
                    k.wait_for_registrations(i + 2, timeout=10)
                    assert _wait(lambda: p._native_server is not srv and p.registered)
            t.join(10)
            assert not t.is_alive()
            assert m.fatal_error and "repeatedly crashed" in m.fatal_error
            assert m.counters["restarts_server"] == 5
        finally:
            m.stop()
            t.join(10)


def test_allocate_counts_as_link_load_until_pod_resources_has_it(make_cfg, plugin_dir, run_manager, tmp_path):
    """The plugin answers a multi-GPU Allocate: the link it spans counts as used at
    once, before the PodResources poll; after the next poll the count comes from the
    kubelet's map instead (not both)."""
    from k8s_gpu_device_plugin_amd.plugin.kubelet_stub import PodResourcesStub
    sock = str(tmp_path / "pod-resources" / "kubelet.sock")
    stub = PodResourcesStub(sock).start()
    try:
        with KubeletStub(plugin_dir) as k:
            m = run_manager(make_cfg(fixture="4gpu_cpx", migStrategy="single",
                                     podResources={"enabled": True, "socket": sock, "intervalS": 0.5}))
            c = k.client(k.wait_for_registrations(1)[0].endpoint)
            ids = m.plugins[0].table.ids()
            held = ids[0:4] + ids[8:12]
            assert _wait(lambda: m.podres.polls >= 1)
            stub.set_pods([("ml", "ring-0", [("main", "amd.com/gpu", held)])])  # kubelet records it at admission
            c.allocate(held)
            assert m.recent_allocations.live() == 1
            avail = ids[4:8] + ids[12:16] + ids[20:24]
            got = list(c.preferred(avail, [], 8).container_responses[0].deviceIDs)
            assert sorted({ids.index(x) // 8 for x in got}) in ([0, 2], [1, 2])
            assert _wait(lambda: m.plugins[0].table.topology().link(0, 1).pods == 1, timeout=5)
            assert _wait(lambda: m.recent_allocations.live() == 0, timeout=5)
            assert m.recent_allocations.link_pods(4)[1] == 0  # not counted twice
    finally:
        stub.stop()


def test_node_labels_leave_out_a_version_the_gpus_disagree_on():
    """Driver / VBIOS labels name the node's one version; GPUs on different firmware (an
    update rolling through the node) give no label rather than GPU 0's."""
    from k8s_gpu_device_plugin_amd.labels import node_labels
    be = fixtures.build_backend("2gpu_spx")
    gpus, _ = be.discover()
    gpus[1].vbios_version = "OTHER"
    labels = node_labels(gpus)
    assert "amd.com/gpu.vbios-version" not in labels
    assert labels["amd.com/gpu.driver-version"] == fixtures.FIXTURE_DRIVER_VERSION
    gpus[0].device_id = 0
    assert "amd.com/gpu.device-id" not in node_labels(gpus)


@pytest.mark.parametrize("reported,want", [
    ("6.14.14", "6.14.14"),
    # amdgpu built into the kernel: amdsmi hands back the /proc/version banner, blanks removed
    # (what the MI355X box reports)
    ("Linuxversion6.18.54-ant.1(nixbld@localhost)(gcc(GCC)15.3.0,GNUld(GNUBinutils)2.46)#1-ant-ociSMP", "6.18.54-ant.1"),
    ("amdgpu 6.10.5-2109964.24.04", "6.10.5-2109964.24.04"),
    ("", ""),
    ("unknown", "unknown"),
])
def test_driver_version_is_normalised(reported, want):
    from k8s_gpu_device_plugin_amd import native
    assert native.load().normalize_driver_version(reported) == want


@pytest.mark.parametrize("grpc_server", ["native", "python"])
def test_allocate_never_fails_through_restarts_and_inventory_changes(make_cfg, plugin_dir, run_manager,
                                                                     grpc_server):
    """Allocate in a tight loop on one connection through 50 /restart
    reloads and partition-mode flips of another GPU (inventory changes): zero failed calls,
    one connection, one registration, and the open ListAndWatch stream follows the new
    device lists."""
    from k8s_gpu_device_plugin_amd import native
    from k8s_gpu_device_plugin_amd.api import v1beta1
    be = fixtures.build_backend("2gpu_spx")
    with KubeletStub(plugin_dir) as k:
        m = run_manager(make_cfg(migStrategy="single", grpc={"server": grpc_server}, rediscoverIntervalS=0.05),
                        backend=be)
        reg = k.wait_for_registrations(1)[0]
        w = k.watch(reg.endpoint)
        w.next()
        dev0 = m.plugins[0].table.ids()[0]  # GPU 0 keeps its device through every change
        req = v1beta1.AllocateRequest(container_requests=[v1beta1.ContainerAllocateRequest(
            devices_ids=[dev0])]).SerializeToString()
        stop = threading.Event()
        stats = {"ok": 0, "failed": [], "connections": 0}

        def loop():
            n = native.load()
            c = n.H2Client(os.path.join(plugin_dir, reg.endpoint))
            stats["connections"] += 1
            while not stop.is_set():
                try:
                    st, _, msg = c.unary(v1beta1.METHOD_ALLOCATE, req)
                except Exception as e:  # the connection dropped
                    stats["failed"].append(repr(e))
                    c = n.H2Client(os.path.join(plugin_dir, reg.endpoint))
                    stats["connections"] += 1
                    continue
                if st == 0:
                    stats["ok"] += 1
                else:
                    stats["failed"].append(msg)
            c.close()

        t = threading.Thread(target=loop, daemon=True)
        t.start()
        try:
            for i in range(50):
                reloads = m.counters["reloads"]
                m.restart()
                assert _wait(lambda: m.counters["reloads"] > reloads, 10)
                if i % 10 == 5:  # an operator re-partitions GPU 1: the inventory re-check reloads
                    fixtures.set_gpu_mode(be, 1, "CPX" if i % 20 == 5 else "SPX", "NPS1")
                    inv = m.counters.get("restarts_inventory", 0)
                    assert _wait(lambda: m.counters.get("restarts_inventory", 0) > inv, 10)
        finally:
            stop.set()
            t.join(10)
        assert not stats["failed"], stats["failed"][:5]
        assert stats["ok"] > 100 and stats["connections"] == 1
        # one Register per /restart on the same socket, none for the inventory reloads
        assert len(k.requests) == 1 + m.counters["reregistrations_restart"]
        assert all(r.endpoint == reg.endpoint for r in k.requests)
        assert m.counters.get("table_swaps", 0) >= 50
        assert m.counters.get("restarts_inventory", 0) >= 5
        devs = w.last(timeout=5)
        assert len(devs) == len(m.plugins[0].table.ids())


def test_grpcio_reloads_do_not_accumulate_threads(make_cfg, plugin_dir, run_manager):
    """Each hitless reload of the grpcio server hands its supervisor thread over instead
    of starting another one (one thread per server, whatever the number of reloads)."""
    with KubeletStub(plugin_dir) as k:
        m = run_manager(make_cfg(grpc={"server": "python"}))
        k.wait_for_registrations(1)
        names = lambda: [t.name for t in threading.enumerate() if t.name.startswith("dp-supervise-")]  # noqa: E731
        assert len(names()) == 1
        for _ in range(20):
            reloads = m.counters["reloads"]
            m.restart()
            assert _wait(lambda: m.counters["reloads"] > reloads)
        time.sleep(0.2)
        assert len(names()) == 1, names()
        assert k.client("amd-gpu.sock").get_options().get_preferred_allocation_available


def _thread_policies(exclude=frozenset()):
    """{comm: {policy, ...}} of this process's threads not in `exclude` (stat field 41:
    0 OTHER, 3 BATCH)."""
    out: dict = {}
    for tid in set(os.listdir("/proc/self/task")) - exclude:
        try:
            with open("/proc/self/task/%s/stat" % tid) as f:
                stat = f.read()
        except OSError:
            continue
        comm = stat[stat.index("(") + 1:stat.rindex(")")]
        policy = int(stat[stat.rindex(")") + 2:].split()[38])
        out.setdefault(comm.rstrip("0123456789-"), set()).add(policy)
    return out


@pytest.mark.parametrize("sched", ["batch", "normal"])
def test_background_threads_never_preempt_grpc_workers(make_cfg, plugin_dir, run_manager, sched):
    """Sampler, watchdog, lanes and the event thread run SCHED_BATCH (a waking batch
    thread does not preempt a worker mid-request); the gRPC and HTTP workers stay
    SCHED_OTHER even when started from a batch thread."""
    from k8s_gpu_device_plugin_amd import native
    before = frozenset(os.listdir("/proc/self/task"))  # earlier tests' lanes may linger
    with KubeletStub(plugin_dir) as k:
        m = run_manager(make_cfg(backgroundSched=sched, grpc={"server": "native"}, http={"server": "native"}))
        k.wait_for_registrations(1)
        assert m.running
        want = 3 if sched == "batch" else 0
        assert _wait(lambda: {"dpsampler", "dpwatchdog", "dplane", "dpevents", "dpgrpc"} <= set(_thread_policies(before)))
        pol = _thread_policies(before)
        for name in ("dpsampler", "dpwatchdog", "dplane", "dpevents"):
            assert pol[name] == {want}, (name, pol)
        assert pol["dpgrpc"] == {0}, pol
        if "dphttp" in pol:
            assert pol["dphttp"] == {0}, pol
        assert native.load().background_batch() == (sched == "batch")


@pytest.mark.parametrize("grpc_server", ["native", "python"])
def test_plugin_registers_again_when_kubelet_ends_its_stream(make_cfg, plugin_dir, run_manager, grpc_server,
                                                            monkeypatch):
    """kubelet ends its ListAndWatch stream (its side failed) without restarting: it drops
    the endpoint and waits for a Register.  The plugin sees no stream for the grace
    period and registers again; a plugin kubelet never opened a stream to is left alone."""
    from k8s_gpu_device_plugin_amd.plugin import manager as manager_mod
    monkeypatch.setattr(manager_mod, "LAW_LOST_GRACE_S", 0.5)
    with KubeletStub(plugin_dir) as k:
        m = run_manager(make_cfg(grpc={"server": grpc_server}))
        regs = k.wait_for_registrations(1)
        time.sleep(2.5)  # no stream opened yet: nothing to recover
        assert len(k.requests) == 1 and m.counters.get("reregistrations_stream_lost", 0) == 0
        w = k.watch(regs[0].endpoint)
        assert len(w.next()[1]) == 2
        p = m.plugins[0]
        assert _wait(lambda: p.list_and_watch_streams() == 1)
        assert _wait(lambda: p.law_had, timeout=3)
        w.cancel()
        assert _wait(lambda: p.list_and_watch_streams() == 0, timeout=5)
        regs = k.wait_for_registrations(2, timeout=10)
        assert _wait(lambda: m.counters.get("reregistrations_stream_lost") == 1)
        w2 = k.watch(regs[1].endpoint, new=True)  # the same socket serves the new stream
        assert len(w2.next()[1]) == 2
        assert _wait(lambda: p.list_and_watch_streams() == 1)
        time.sleep(1.5)
        assert len(k.requests) == 2  # an open stream: no further Register
        w2.cancel()


@pytest.mark.parametrize("grpc_server", ["native", "python"])
def test_quiet_node_supervises_less_often_and_times_stream_loss_from_its_end(make_cfg, plugin_dir, run_manager,
                                                                            grpc_server, monkeypatch):
    """once every plugin is registered with kubelet's stream open, the
    manager thread supervises every SERVER_CHECK_QUIET_S instead of every second.  A stream
    that ends is timed from its end (the server stamps it), not from the late poll that
    notices it, and the manager is back to 1 s passes until it is resolved."""
    from k8s_gpu_device_plugin_amd.plugin import manager as manager_mod
    monkeypatch.setattr(manager_mod, "SERVER_CHECK_QUIET_S", 3.0)
    monkeypatch.setattr(manager_mod, "LAW_LOST_GRACE_S", 60.0)  # no re-registration in this test
    with KubeletStub(plugin_dir) as k:
        m = run_manager(make_cfg(grpc={"server": grpc_server}))
        regs = k.wait_for_registrations(1)
        assert m._check_period() == manager_mod.SERVER_CHECK_S  # no stream yet
        w = k.watch(regs[0].endpoint)
        w.next()
        p = m.plugins[0]
        assert _wait(lambda: p.law_had, timeout=3)
        assert m._check_period() == 3.0
        assert p.list_and_watch_closed_at() == 0
        time.sleep(1.2)  # a poll falls due later than a 1 s one would
        t_cancel = time.monotonic()
        w.cancel()
        assert _wait(lambda: p.list_and_watch_streams() == 0, timeout=5)
        closed = p.list_and_watch_closed_at()
        assert t_cancel - 0.05 <= closed <= time.monotonic()
        assert _wait(lambda: p.law_lost_since is not None, timeout=5)
        assert p.law_lost_since == closed  # timed from the stream's end
        assert m._check_period() == manager_mod.SERVER_CHECK_S


def test_native_server_fault_wakes_a_quiet_manager(make_cfg, plugin_dir, run_manager, monkeypatch):
    """A native server fault runs the supervision pass at once (the server's failure hook
    posts it) rather than at the quiet node's next poll."""
    from k8s_gpu_device_plugin_amd.plugin import manager as manager_mod
    monkeypatch.setattr(manager_mod, "SERVER_CHECK_QUIET_S", 60.0)
    with KubeletStub(plugin_dir) as k:
        m = run_manager(make_cfg(grpc={"server": "native"}))
        regs = k.wait_for_registrations(1)
        k.watch(regs[0].endpoint).next()
        p = m.plugins[0]
        assert _wait(lambda: p.law_had, timeout=3)
        assert _wait(lambda: m._check_period() == 60.0, timeout=3)
        time.sleep(1.5)  # the manager is now waiting out its 60 s quiet period
        srv = p._native_server
        t0 = time.monotonic()
        srv.inject_fault("worker")
        k.wait_for_registrations(2, timeout=10)
        assert time.monotonic() - t0 < 5.0
        assert _wait(lambda: m.counters.get("restarts_server", 0) == 1)
        assert p._native_server is not srv and not p._native_server.failure()


def test_stream_watchdog_leaves_a_socket_another_instance_took(make_cfg, plugin_dir, run_manager, monkeypatch):
    """an overlapping new instance re-bound the plugin's socket path and kubelet's
    stream went to it.  The old process must not re-register every grace period (kubelet
    would re-dial the path and tear down the new instance's stream each time)."""
    import socket as socket_mod
    from k8s_gpu_device_plugin_amd.plugin import manager as manager_mod
    monkeypatch.setattr(manager_mod, "LAW_LOST_GRACE_S", 0.3)
    with KubeletStub(plugin_dir) as k:
        m = run_manager(make_cfg())
        regs = k.wait_for_registrations(1)
        w = k.watch(regs[0].endpoint)
        w.next()
        p = m.plugins[0]
        assert _wait(lambda: p.law_had, timeout=3)
        # the "new pod": its own socket at the same path (bound aside and renamed over it,
        # so the manager's socket-removed handler never sees the path missing)
        other = socket_mod.socket(socket_mod.AF_UNIX, socket_mod.SOCK_STREAM)
        other.bind(p.socket + ".new")
        other.listen(4)
        os.rename(p.socket + ".new", p.socket)
        try:
            w.cancel()
            assert _wait(lambda: m.counters.get("stream_watch_socket_taken", 0) == 1, timeout=10)
            time.sleep(1.5)  # several grace periods
            assert len(k.requests) == 1 and m.counters.get("reregistrations_stream_lost", 0) == 0
        finally:
            other.close()
