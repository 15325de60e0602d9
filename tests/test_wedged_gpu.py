"""A GPU whose driver call never returns (SURVEY.md §7.5 hard parts
5 and 6).

The fixture models the lock a wedged call holds: one driver lock per GPU (rocm_smi's
per-device mutex, the default) or one for the whole library (``set_serialised``).  Every
hardware call runs on its GPU's lane (native/lanes.h), so the manager, the sampler and
discovery wait on a wedged GPU at most one bound, once.

What must hold while GPU 3 of an 8-GPU node is wedged:
  * the manager keeps handling events: a kubelet restart re-registers the plugin within
    2 s, advertising GPU 3 Unhealthy and the other 7 Healthy, and ``/restart`` reloads;
  * ``GET /ready`` answers 503 and names the GPU discovery could not reach;
  * the other GPUs' telemetry stays fresh and their health checks keep running (an ECC
    error on GPU 5 is seen within two sampling intervals) - in the per-device model; in
    the serialised model they are reported "blocked" behind GPU 3, not lost;
  * a reload whose discovery fails leaves the current plugins serving (make-before-break).
Reference: plugin/manager.go:80-84 (kubelet restart), :177-194 (restartPlugins).
"""
import os
import time

import pytest

from k8s_gpu_device_plugin_amd.models import fixtures
from k8s_gpu_device_plugin_amd.plugin.kubelet_stub import DevicePluginClient, KubeletStub
from k8s_gpu_device_plugin_amd.plugin.manager import PluginManager

# instrumented builds (test_sanitized_suite) run several times slower
SLOW = 4.0 if os.environ.get("AMDGPU_DP_NATIVE_SO") else 1.0


def _wait(pred, timeout=5.0, step=0.01):
    deadline = time.monotonic() + timeout * SLOW
    while time.monotonic() < deadline:
        if pred():
            return True
        time.sleep(step)
    return False


def _advertised(plugin_dir, k):
    """(id, health) of the first ListAndWatch message of the newest registration, over a
    fresh connection (what a restarted kubelet sees)."""
    c = DevicePluginClient(os.path.join(plugin_dir, k.requests[-1].endpoint))
    try:
        stream = c.list_and_watch(timeout=5 * SLOW)
        first = next(iter(stream))
        stream.cancel()
        return [(d.ID, d.health) for d in first.devices]
    finally:
        c.close()


@pytest.fixture
def run_manager():
    started = []

    def _run(cfg, backend):
        m = PluginManager(cfg, backend=backend)
        t = m.start_background()
        started.append((m, t, backend))
        return m
    yield _run
    for m, t, be in started:
        for g in range(8):
            try:
                be.set_sample_stall(g, False)
            except Exception:  # noqa: BLE001 - fewer GPUs
                pass
        m.stop()
        t.join(10)
        assert not t.is_alive()


@pytest.mark.parametrize("serialised,server", [(False, "native"), (True, "native"), (False, "python")],
                         ids=["per_device_lock", "library_lock", "per_device_lock_grpcio_server"])
def test_wedged_gpu_keeps_the_node_advertised(make_cfg, plugin_dir, run_manager, serialised, server):
    be = fixtures.build_backend("8gpu_spx_mesh")
    be.set_serialised(serialised)
    cfg = make_cfg(fixture="8gpu_spx_mesh", grpc={"server": server}, telemetry={"intervalMs": 50},
                   rediscoverIntervalS=0.3, retrySeconds=0.2,
                   health={"sampleStallS": 0.3, "discoveryTimeoutS": 0.5, "lostAfterFailures": 3})
    with KubeletStub(plugin_dir) as k:
        m = run_manager(cfg, be)
        k.wait_for_registrations(1)
        table = m.plugins[0].table
        ids = list(table.ids())
        assert len(ids) == 8 and m.readiness() == (True, "")

        be.set_sample_stall(3, True)  # GPU 3's next call hangs in the driver
        assert _wait(lambda: not m.plugins[0].table.healthy(ids[3]), 5), "GPU 3 never marked Unhealthy"
        assert all(m.plugins[0].table.healthy(i) for j, i in enumerate(ids) if j != 3)
        assert m.exporter.stalled_gpus == [3]
        if serialised:  # the others wait behind GPU 3's call: blocked, not lost
            assert _wait(lambda: m.exporter.blocked_gpus == [0, 1, 2, 4, 5, 6, 7], 5), m.exporter.blocked_gpus
        # the periodic re-discovery cannot reach GPU 3: /ready says so, naming it
        assert _wait(lambda: "discovery stalled on GPU 3" in m.readiness()[1], 5), m.readiness()
        ready, why = m.readiness()
        assert not ready and "advertising its last known description" in why, why

        # kubelet restarts: re-registered within 2 s, GPU 3 Unhealthy, the other 7 Healthy
        n = len(k.requests)
        t0 = time.monotonic()
        k.restart()
        k.wait_for_registrations(n + 1, timeout=2 * SLOW)
        assert time.monotonic() - t0 < 2 * SLOW
        want = [(i, "Unhealthy" if j == 3 else "Healthy") for j, i in enumerate(ids)]
        assert _wait(lambda: _advertised(plugin_dir, k) == want, 3), _advertised(plugin_dir, k)

        # GET /restart still reloads (GPU 3 from its last description), swapping the
        # tables into the running server, and registers that socket again
        n, reloads = len(k.requests), m.counters["reloads"]
        m.restart()
        assert _wait(lambda: m.counters["reloads"] > reloads, 3 * SLOW)
        k.wait_for_registrations(n + 1, timeout=2 * SLOW)
        assert len(k.requests) == n + 1
        assert _wait(lambda: _advertised(plugin_dir, k) == want, 3), _advertised(plugin_dir, k)
        assert not m.readiness()[0]
        assert m.running and m.fatal_error is None

        # the driver lets go: GPU 3 is sampled again, Healthy, and /ready recovers
        be.set_sample_stall(3, False)
        assert _wait(lambda: m.plugins[0].table.healthy(ids[3]), 5)
        assert _wait(lambda: m.readiness() == (True, ""), 5), m.readiness()
        assert m.exporter.stalled_gpus == [] and m.exporter.blocked_gpus == []
        assert _advertised(plugin_dir, k) == [(i, "Healthy") for i in ids]


@pytest.mark.parametrize("serialised", [False, True], ids=["per_device_lock", "library_lock"])
def test_wedged_gpu_does_not_freeze_the_other_gpus_telemetry(n, serialised):
    """Per-GPU isolation of sampling: with GPU 3 wedged, an ECC error on GPU 5 still turns
    it Unhealthy within two sampling intervals and GPUs 0-2, 4-7 keep fresh sample ages
    (per-device locks).  Behind a library-wide lock nothing can be sampled: GPU 3 is the
    one reported lost, the others are reported blocked and keep their health."""
    interval = 0.1
    be = fixtures.build_backend("8gpu_spx_mesh")
    be.set_serialised(serialised)
    gpus, _ = be.discover()
    be.set_stall_ms(300)
    mon = n.HealthMonitor(be, 3)
    mon.set_gpus([be.gpu_key(g.index) for g in gpus])
    ex = n.Exporter()
    ex.set_inventory(gpus)
    ex.set_stall_ms(300)
    ex.start(be, int(interval * 1000), mon)
    try:
        time.sleep(3 * interval)  # ECC baselines
        be.set_sample_stall(3, True)
        lost = []
        assert _wait(lambda: lost.extend(u for u in mon.pop(20) if u.healthy == 0) or lost, 5)
        assert [u.gpu for u in lost] == [3] and "in flight" in lost[0].reason, lost
        assert ex.stalled_gpus == [3]
        others = [0, 1, 2, 4, 5, 6, 7]
        if not serialised:
            assert ex.blocked_gpus == []
            t0 = time.monotonic()
            be.set_ecc_uncorrectable(5, 1)
            got = []
            assert _wait(lambda: got.extend(u for u in mon.pop(10) if u.healthy == 0) or got, 2)
            elapsed = time.monotonic() - t0
            assert [u.gpu for u in got] == [5] and "ecc" in got[0].reason
            assert elapsed < (2 * interval + 0.1) * SLOW, elapsed  # within two sampling intervals
            for g in others:
                assert 0 <= ex.sample_age_s(g) < 2 * interval * SLOW, (g, ex.sample_age_s(g))
            assert ex.sample_age_s(3) > 0.3
            # the exposition is rendered at the end of each pass: wait for one past the bound
            assert _wait(lambda: 'amdgpu_telemetry_up{gpu="5"} 1' in ex.render()
                         and 'amdgpu_telemetry_up{gpu="3"} 0' in ex.render(), 2), \
                [ln for ln in ex.render().splitlines() if ln.startswith("amdgpu_telemetry_up")]
        else:
            assert _wait(lambda: ex.blocked_gpus == others, 5), ex.blocked_gpus
            assert all(mon.gpu_healthy(g) for g in others)
            assert 'amdgpu_telemetry_sample_blocked{gpu="5"} 1' in ex.render()
        be.set_sample_stall(3, False)
        assert _wait(lambda: mon.gpu_healthy(3), 5)
        assert _wait(lambda: ex.stalled_gpus == [] and ex.blocked_gpus == [], 5)
        assert _wait(lambda: all(0 <= ex.sample_age_s(g) < 2 * interval * SLOW for g in range(8)), 5)
    finally:
        be.set_sample_stall(3, False)
        ex.stop()


def test_discovery_gives_a_wedged_gpu_its_last_description(n):
    """Discovery is bounded per GPU: a wedged GPU costs one call bound once, then its lane
    refuses work and it is described from the last discovery that reached it; a GPU no
    discovery ever reached is left out (and reported)."""
    be = fixtures.build_backend("4gpu_cpx")
    be.set_call_timeout_ms(300)
    be.set_stall_ms(200)
    gpus0, topo0 = be.discover()
    be.set_sample_stall(2, True)
    t0 = time.monotonic()
    gpus, topo = be.discover()
    first = time.monotonic() - t0
    assert 0.25 < first < 1.0 * SLOW, first  # one bound for the wedged GPU, all in parallel
    assert [g.uuid for g in gpus] == [g.uuid for g in gpus0]
    assert [len(g.partitions) for g in gpus] == [8] * 4 and topo.n == 4
    rep = be.last_discovery()
    assert [(i, key) for i, key, _ in rep["stale"]] == [(2, gpus0[2].uuid)] and "300 ms" in rep["stale"][0][2]
    time.sleep(0.25)  # the stuck call is now past the stall threshold: its lane refuses work
    t0 = time.monotonic()
    be.discover()
    assert time.monotonic() - t0 < 0.1 * SLOW
    assert "in flight" in be.last_discovery()["stale"][0][2]
    lanes = {x[0]: x for x in be.lanes()}
    assert lanes[2][2] == "describe" and lanes[2][3] > 0.4  # the call stays stuck on GPU 2's lane
    be.set_sample_stall(2, False)
    assert _wait(lambda: {x[0]: x for x in be.lanes()}[2][2] == "", 3)
    be.discover()
    assert be.last_discovery()["stale"] == []
    # a backend whose first discovery cannot reach GPU 1: left out, reported with index -1
    fresh = n.FixtureBackend(3)
    for g in gpus0[:2]:
        fresh.add_gpu(g)
    fresh.set_call_timeout_ms(200)
    fresh.set_sample_stall(1, True)
    try:
        gpus, _ = fresh.discover()
        assert [g.uuid for g in gpus] == [gpus0[0].uuid]
        assert [(i, key) for i, key, _ in fresh.last_discovery()["stale"]] == [(-1, gpus0[1].uuid)]
    finally:
        fresh.set_sample_stall(1, False)


def test_failed_reload_keeps_serving_and_kubelet_restart_reregisters(make_cfg, plugin_dir, run_manager):
    """Make-before-break: /restart while discovery fails leaves the plugin serving (its
    socket, tables and registration untouched); a kubelet restart meanwhile re-registers
    the plugin that serves within 1 s; ListAndWatch never goes empty."""
    be = fixtures.build_backend("2gpu_spx")
    cfg = make_cfg(grpc={"server": "native"}, retrySeconds=0.2, rediscoverIntervalS=0)
    with KubeletStub(plugin_dir) as k:
        m = run_manager(cfg, be)
        k.wait_for_registrations(1)
        ids = list(m.plugins[0].table.ids())
        c = DevicePluginClient(os.path.join(plugin_dir, "amd-gpu.sock"))
        try:
            be.set_fail_discovery(True)
            failures = m.counters["load_failures"]
            m.restart()
            assert _wait(lambda: m.counters["load_failures"] > failures, 3)
            assert c.allocate([ids[0]]).container_responses[0].devices  # same connection, still served
            assert _wait(lambda: m.readiness()[1].startswith("discovery failed") or not m.readiness()[0], 2)
            assert m.plugins and m.plugins[0].registered
            # kubelet restart while discovery keeps failing
            n = len(k.requests)
            t0 = time.monotonic()
            k.restart()
            k.wait_for_registrations(n + 1, timeout=1 * SLOW)
            assert time.monotonic() - t0 < 1 * SLOW
            assert [h for _, h in _advertised(plugin_dir, k)] == ["Healthy", "Healthy"]
            be.set_fail_discovery(False)  # the retry timer reloads
            assert _wait(lambda: m.readiness() == (True, ""), 5), m.readiness()
        finally:
            c.close()
            be.set_fail_discovery(False)


def test_devices_indices_wait_for_gpus_missing_at_first_discovery(make_cfg, plugin_dir, run_manager):
    """`devices: "0-1"` with no GPU at the first discovery selects
    nothing *yet* and picks the GPUs up when they appear.  ADVICE r4 (low): once an index
    has been advertised it stays pinned to that GPU - a GPU that appears later with a lower
    BDF does not push it out (it may be allocated to pods); the conflict is counted."""
    be = fixtures.build_backend("4gpu_spx")
    uuids = [g.uuid for g in be.discover()[0]]
    for g in range(4):
        be.set_gpu_present(g, False)
    cfg = make_cfg(fixture="4gpu_spx", devices="0-1", rediscoverIntervalS=0.1, retrySeconds=0.2)
    with KubeletStub(plugin_dir) as k:
        m = run_manager(cfg, be)
        assert not any(len(p) for p in m.plugins)
        be.set_gpu_present(0, True)
        be.set_gpu_present(2, True)
        be.set_gpu_present(3, True)  # GPU 1 still missing
        assert _wait(lambda: [g.uuid for g in m.gpus] == [uuids[0], uuids[2]], 5), [g.uuid for g in m.gpus]
        k.wait_for_registrations(1, timeout=5)
        # a pod holds GPU 2 (kubelet's device checkpoint names its device)
        dev2 = [d.id for p in m.plugins for d in p.devices() if d.gpu == 1][0]
        _write_checkpoint(plugin_dir, [("amd.com/gpu", [dev2])])
        be.set_gpu_present(1, True)  # now it shows up, ranking 1 by BDF: GPU 2 keeps index 1
        assert _wait(lambda: m.counters.get("devices_index_conflicts", 0) == 1, 5)
        assert [g.uuid for g in m.gpus] == [uuids[0], uuids[2]]
        # the pod goes: the late GPU takes its index back
        _write_checkpoint(plugin_dir, [])
        assert _wait(lambda: [g.uuid for g in m.gpus] == [uuids[0], uuids[1]], 5), [g.uuid for g in m.gpus]
        assert m.counters.get("devices_index_reresolved") == 1
        # and a GPU that drops off the bus leaves its index empty (no neighbour moves in)
        be.set_gpu_present(0, False)
        assert _wait(lambda: [g.uuid for g in m.gpus] == [uuids[1]], 5), [g.uuid for g in m.gpus]
        time.sleep(0.3)
        assert [g.uuid for g in m.gpus] == [uuids[1]]


def _write_checkpoint(plugin_dir, entries):
    """kubelet's device-manager checkpoint: [(resource, [device ids])], one pod each."""
    import json
    data = {"Data": {"PodDeviceEntries": [{"PodUID": "pod-%d" % i, "ContainerName": "c", "ResourceName": res,
                                           "DeviceIDs": {"-1": ids}, "AllocResp": ""}
                                          for i, (res, ids) in enumerate(entries)],
                     "RegisteredDevices": {}}, "Checksum": 0}
    path = os.path.join(plugin_dir, "kubelet_internal_checkpoint")
    with open(path + ".tmp", "w") as f:
        json.dump(data, f)
    os.replace(path + ".tmp", path)


def test_sampler_refused_by_a_lane_stuck_in_discovery_shows_the_gpu_down(n):
    """The call that wedges a GPU need not be a sample: a discovery's describe can hang on
    its lane while the sampler is between passes.  Past the stall threshold the lane takes
    no new job, and the sampler must then show that GPU as not sampled
    (`amdgpu_telemetry_up` 0, growing sample age), not keep rendering its last values as
    current."""
    import threading
    be = fixtures.build_backend("2gpu_spx")
    gpus, _ = be.discover()
    be.set_stall_ms(150)
    be.set_call_timeout_ms(100)
    ex = n.Exporter()
    ex.set_inventory(gpus)
    ex.set_stall_ms(150)
    ex.start(be, 400, None)  # long interval: the wedge starts between passes
    try:
        assert _wait(lambda: 'amdgpu_telemetry_up{gpu="1"} 1' in ex.render(), 3)
        time.sleep(0.05)  # just after a pass
        be.set_sample_stall(1, True)
        t = threading.Thread(target=be.discover, daemon=True)  # describe(1) hangs on lane 1
        t.start()
        t.join(5)
        assert not t.is_alive(), "discovery waited on the wedged GPU past its bound"
        assert _wait(lambda: 'amdgpu_telemetry_up{gpu="1"} 0' in ex.render(), 3)
        text = ex.render()
        assert 'amdgpu_telemetry_up{gpu="0"} 1' in text
        assert ex.sample_age_s(1) > 0.15 and 0 <= ex.sample_age_s(0) < 1.0
        lanes = {r[0]: r for r in be.lanes()}
        assert lanes[1][2] == "describe", lanes  # the stuck call is the discovery's
    finally:
        be.set_sample_stall(1, False)
        ex.stop()


def test_watchdog_ignores_a_gpu_the_devices_selection_leaves_out(n):
    """A GPU outside `devices` is never sampled, so nothing would ever clear a "lost"
    verdict on it: a call stuck on its lane (a discovery's describe) must not be reported.
    It still roots a library-wide block: the served GPUs are then "blocked", not lost."""
    import threading
    for serialised in (False, True):
        be = fixtures.build_backend("4gpu_spx")
        be.set_serialised(serialised)
        gpus, _ = be.discover()
        be.set_stall_ms(150)
        be.set_call_timeout_ms(100)
        mon = n.HealthMonitor(be, 3)
        served = [g for g in gpus if g.index in (0, 1)]
        mon.set_gpus([be.gpu_key(g.index) for g in served])
        ex = n.Exporter()
        ex.set_inventory(served)
        ex.set_stall_ms(150)
        ex.start(be, 50, mon)
        try:
            be.set_sample_stall(3, True)
            t = threading.Thread(target=be.discover, daemon=True)  # describe(3) hangs on lane 3
            t.start()
            t.join(5)
            time.sleep(0.5)
            assert ex.stalled_gpus == [] and mon.unhealthy_keys() == [], (serialised, ex.stalled_gpus,
                                                                          mon.unhealthy_keys())
            if serialised:  # behind the library-wide lock, the served GPUs wait on GPU 3's call
                assert _wait(lambda: ex.blocked_gpus == [0, 1], 3), ex.blocked_gpus
            else:
                assert _wait(lambda: all(0 <= ex.sample_age_s(g) < 0.5 for g in (0, 1)), 3)
        finally:
            be.set_sample_stall(3, False)
            ex.stop()
        assert _wait(lambda: ex.blocked_gpus == [] or not ex.running, 3)


def test_samples_follow_identity_when_a_rediscovery_moves_the_indices(n):
    """Between a re-discovery and the manager's reload the exporter still holds the old
    indices.  GPU 1 leaves the bus: the backend's index 2 is now slot 3.  The exporter
    must keep sampling the GPU it serves as "2" (by identity), never the one that moved
    into that index, and link peers must name the GPUs the sample saw (found by the chaos
    test: a left-out GPU's stale link view pinned a healed link at half rate)."""
    be = fixtures.build_backend("4gpu_spx")
    gpus, _ = be.discover()
    keys = [g.key for g in gpus]
    assert all(keys) and len(set(keys)) == 4
    served = [g for g in gpus if g.index in (0, 1, 2)]
    mon = n.HealthMonitor(be, 3)
    mon.set_gpus([g.key for g in served])
    ex = n.Exporter()
    ex.set_inventory(served)
    ex.start(be, 30, mon)
    try:
        assert _wait(lambda: ex.last_sample(2).key == keys[2], 3)
        peers = ex.last_sample(0).link_peer_keys
        assert sorted(peers) == sorted(keys[1:]), peers
        be.set_gpu_present(1, False)
        moved, _ = be.discover()
        assert [g.key for g in moved] == [keys[0], keys[2], keys[3]]
        time.sleep(0.3)  # several passes with the old indices
        assert ex.last_sample(2).key == keys[2]  # sampled by identity, not index 2 (slot 3)
        peers = [k for k in ex.last_sample(0).link_peer_keys if k]  # "" = a peer no longer enumerated
        assert set(peers) <= set(keys) and keys[3] in peers and keys[1] not in peers, peers
        assert 'amdgpu_telemetry_up{gpu="1"} 0' in ex.render()  # gone from the bus: not sampled
    finally:
        ex.stop()


def test_wedged_gpu_outside_the_selection_does_not_fail_readiness(make_cfg, plugin_dir, run_manager):
    """a GPU that `devices` leaves out wedges; discovery reports it stale,
    but GET /ready - and so a DaemonSet rolling update - does not wait on a GPU this plugin
    does not serve.  The same wedge on a served GPU fails readiness."""
    be = fixtures.build_backend("4gpu_spx")
    cfg = make_cfg(fixture="4gpu_spx", devices="0-1", telemetry={"intervalMs": 50}, rediscoverIntervalS=0.2,
                   health={"sampleStallS": 0.3, "discoveryTimeoutS": 0.3, "lostAfterFailures": 3})
    with KubeletStub(plugin_dir) as k:
        m = run_manager(cfg, be)
        k.wait_for_registrations(1)
        assert _wait(lambda: m.readiness() == (True, ""), 5)
        be.set_sample_stall(3, True)
        assert _wait(lambda: m._stale and m._stale[0][1] == fixtures.fixture_uuid(1, 3), 5), m._stale
        time.sleep(0.5)
        assert m.readiness() == (True, ""), m.readiness()
        be.set_sample_stall(3, False)
        be.set_sample_stall(1, True)
        assert _wait(lambda: "discovery stalled on GPU 1" in m.readiness()[1], 5), m.readiness()
