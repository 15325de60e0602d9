"""Exporter (per-GPU / per-partition telemetry rendering) and the native health monitor."""
import os
import time

import pytest

from hypothesis import given, settings, strategies as st

from prometheus_client.parser import text_string_to_metric_families

from k8s_gpu_device_plugin_amd import native
from k8s_gpu_device_plugin_amd.models import fixtures


def _families(text):
    return {f.name: f for f in text_string_to_metric_families(text)}


def test_exporter_cpx_64_partitions(n):
    be = fixtures.build_backend("8gpu_cpx_nps2")
    gpus, _ = be.discover()
    ex = n.Exporter()
    ex.set_inventory(gpus)
    ex.set_partition_labels([n.PartitionLabel(g.index, p.index, p.id, "amd.com/gpu") for g in gpus
                             for p in g.partitions])
    ex.set_build_info('# TYPE x_build_info gauge\nx_build_info{v="1"} 1\n')
    ex.start(be, 50, None)
    time.sleep(0.2)
    ex.stop()
    assert ex.samples_total >= 2
    fams = _families(ex.render())
    assert len(fams["amdgpu_info"].samples) == 8
    assert fams["amdgpu_info"].samples[0].labels["compute_partition"] == "CPX"
    assert fams["amdgpu_info"].samples[0].labels["driver_version"] == fixtures.FIXTURE_DRIVER_VERSION
    assert fams["amdgpu_info"].samples[0].labels["vbios_version"] == fixtures.FIXTURE_VBIOS_VERSION
    assert [s.labels["oam_id"] for s in fams["amdgpu_info"].samples] == [str(i) for i in range(8)]
    assert len(fams["amdgpu_partition_info"].samples) == 64
    assert len(fams["amdgpu_partition_gfx_busy_percent"].samples) == 64
    assert len(fams["amdgpu_xgmi_link_up"].samples) == 8 * 7
    hbm = [s for s in fams["amdgpu_temperature_celsius"].samples if s.labels["sensor"].startswith("hbm")]
    assert len(hbm) == 64
    assert fams["amdgpu_ecc_errors"].type == "counter"
    assert "process_cpu_seconds" in fams and "x_build_info" in fams
    assert fams["amdgpu_telemetry_sample_duration_seconds"].type == "histogram"
    s = ex.last_sample(3)
    assert s.ok and s.power_w > 0 and len(s.links) == 7


def test_exporter_device_health_and_rpc_histogram(n):
    tc = n.TableConfig()
    t = n.DeviceTable(tc, [n.TableDevice("a", 0), n.TableDevice("b", 1)], n.Topology(2))
    t.observe(n.RPC_ALLOCATE, 12e-6, False)
    t.set_health("b", False)
    ex = n.Exporter()
    ex.set_tables([t])
    fams = _families(ex.render())
    health = {s.labels["device_id"]: s.value for s in fams["amdgpu_device_plugin_device_health"].samples}
    assert health == {"a": 1.0, "b": 0.0}
    buckets = [s for s in fams["amdgpu_device_plugin_rpc_duration_seconds"].samples if s.name.endswith("_bucket")]
    assert buckets[0].labels["rpc"] == "Allocate" and buckets[-1].value == 1


def test_rpc_histogram_sums_every_observing_thread(n):
    """Observations land in per-thread shards; a render sums exactly the shards that were
    written (the used-shard mask), re-rendering whenever a new thread's shard appears."""
    import threading
    tc = n.TableConfig()
    t = n.DeviceTable(tc, [n.TableDevice("a", 0)], n.Topology(1))
    ex = n.Exporter()
    ex.set_tables([t])

    def counts():
        fams = _families(ex.render())
        samples = fams["amdgpu_device_plugin_rpc_duration_seconds"].samples
        b = [s.value for s in samples if s.name.endswith("_bucket") and s.labels["rpc"] == "Allocate"]
        c = [s.value for s in samples if s.name.endswith("_count") and s.labels["rpc"] == "Allocate"]
        return b, c[0]

    t.observe(n.RPC_ALLOCATE, 3e-6, False)
    assert counts()[1] == 1
    done = []

    def worker(i):
        for k in range(500):
            t.observe(n.RPC_ALLOCATE, (1 + (k % 7)) * 1e-6 * (10 ** (i % 4)), False)
        done.append(i)

    ts = [threading.Thread(target=worker, args=(i,)) for i in range(12)]
    for th in ts:
        th.start()
    for th in ts:
        th.join()
    buckets, count = counts()
    assert count == 1 + 12 * 500
    assert buckets[-1] == count and buckets == sorted(buckets)  # cumulative, +Inf holds all


def _discovered(spec="2gpu_spx"):
    """A fixture node after its first discovery: the monitor names GPUs by the identities
    the backend gives for its current enumeration (an index it does not know is ignored)."""
    from k8s_gpu_device_plugin_amd.models import fixtures
    be = fixtures.build_backend(spec)
    be.discover()
    return be


def test_health_monitor_state_machine(n):
    be = _discovered()
    m = n.HealthMonitor(be, 2)
    m.set_gpu_count(2)
    m.process(n.HwEvent(n.EVT_PRE_RESET, 1, message="x"))
    m.process(n.HwEvent(n.EVT_PRE_RESET, 1))  # duplicate -> no second transition
    u = m.pop(100)
    assert [(x.gpu, x.healthy) for x in u] == [(1, 0)]
    assert not m.gpu_healthy(1) and m.gpu_healthy(0)
    m.process(n.HwEvent(n.EVT_ECC_UNCORRECTABLE, 1))
    # still unhealthy, no transition; the new latch is reported (the manager persists it)
    assert [(x.gpu, x.healthy, "(latched)" in x.reason) for x in m.pop(10)] == [(1, -1, True)]
    m.process(n.HwEvent(n.EVT_ECC_UNCORRECTABLE, 1))
    assert m.pop(10) == []  # the latch was already set: nothing new
    m.process(n.HwEvent(n.EVT_POST_RESET, 1))  # reset clears the ECC latch too
    assert [(x.gpu, x.healthy) for x in m.pop(100)] == [(1, 1)]
    m.process(n.HwEvent(n.EVT_LINK_DOWN, 0, peer=1))
    m.process(n.HwEvent(n.EVT_LINK_DOWN, 1, peer=0))  # same link seen from the peer: deduplicated
    u = m.pop(100)
    assert len(u) == 1 and u[0].link_up == 0 and u[0].healthy == -1
    m.process(n.HwEvent(n.EVT_THERMAL, 0, message="hot"))
    u = m.pop(100)
    assert u[0].healthy == -1 and "thermal" in u[0].reason
    assert m.events_seen >= 7
    m.process(n.HwEvent(n.EVT_PRE_RESET, 7))  # out of range gpu: ignored, no crash


def test_failed_sample_of_an_index_no_gpu_holds_is_ignored(n):
    """A sampler pass that still uses the old inventory after a GPU vanished asks for an
    index the backend no longer has.  That failure is nobody's: no phantom GPU state
    (which used to be kept as "#<index>" and stay Unhealthy for ever)."""
    be = _discovered()
    m = n.HealthMonitor(be, 2)
    m.set_gpu_count(2)
    be.set_gpu_present(1, False)
    be.discover()  # the node is re-enumerated: one GPU, index 0
    assert be.gpu_key(1) == ""
    for _ in range(4):
        m.on_sample(1, False, n.GpuSample())  # what the backend answers for index 1: failed, no key
    assert m.unhealthy_keys() == [] and m.pop(10) == []


def test_health_monitor_fast_tables_both_directions(n):
    """Unhealthy always reaches the tables from the monitor itself; Healthy only with
    fast recovery on (no recovery canary), else it waits for the manager."""
    t = n.DeviceTable(n.TableConfig(), [n.TableDevice("a", 0), n.TableDevice("b", 1)], n.Topology(2))
    m = n.HealthMonitor(_discovered(), 2)
    m.set_gpu_count(2)
    m.set_fast_tables([t])
    m.process(n.HwEvent(n.EVT_PRE_RESET, 1))
    assert not t.healthy("b") and t.healthy("a")
    m.process(n.HwEvent(n.EVT_POST_RESET, 1))
    assert not t.healthy("b")  # held for the manager (canary policy)
    m.set_fast_recover(True)
    m.process(n.HwEvent(n.EVT_PRE_RESET, 1))
    m.process(n.HwEvent(n.EVT_POST_RESET, 1))
    assert t.healthy("b")
    assert [(x.gpu, x.healthy) for x in m.pop(100)] == [(1, 0), (1, 1), (1, 0), (1, 1)]


def test_disabled_health_checks(n):
    """health.disabledChecks: an ignored condition is logged, not acted on; turning a
    check off releases a GPU that only it held, turning it back on re-applies it."""
    from k8s_gpu_device_plugin_amd.config import ConfigError, disabled_checks_mask
    assert disabled_checks_mask("ecc, retiredPages") == 2 | 8 and disabled_checks_mask("all") == 31
    assert disabled_checks_mask("") == 0
    with pytest.raises(ConfigError):
        disabled_checks_mask("xid")
    t = n.DeviceTable(n.TableConfig(), [n.TableDevice("a", 0), n.TableDevice("b", 1)], n.Topology(2))
    m = n.HealthMonitor(_discovered(), 2)
    m.set_gpu_count(2)
    m.set_fast_tables([t])
    m.set_fast_recover(True)
    m.set_disabled_checks(disabled_checks_mask("ecc"))
    m.process(n.HwEvent(n.EVT_ECC_UNCORRECTABLE, 1))
    u = m.pop(100)
    assert [(x.gpu, x.healthy) for x in u] == [(1, -1)] and "disabled" in u[0].reason
    assert t.healthy("b") and m.gpu_healthy(1)
    m.process(n.HwEvent(n.EVT_PRE_RESET, 0))  # other checks still act
    assert [(x.gpu, x.healthy) for x in m.pop(100)] == [(0, 0)] and not t.healthy("a")
    m.set_disabled_checks(0)  # the ECC latch of GPU 1 counts again
    assert [(x.gpu, x.healthy) for x in m.pop(100)] == [(1, 0)] and not t.healthy("b")
    m.set_disabled_checks(disabled_checks_mask("all"))
    assert sorted((x.gpu, x.healthy) for x in m.pop(100)) == [(0, 1), (1, 1)]
    assert t.healthy("a") and t.healthy("b")


def test_disabled_checks_config(make_cfg):
    from k8s_gpu_device_plugin_amd import config
    cfg = config.validate(config.from_dict({"health": {"disabledChecks": ["ecc", "lost"]}}))
    assert config.disabled_checks_mask(cfg.health.disabledChecks) == 2 | 4
    cfg = config.apply_env(config.Config(), {"AMDGPU_DP_DISABLE_HEALTHCHECKS": "all"})
    assert config.disabled_checks_mask(cfg.health.disabledChecks) == 31
    with pytest.raises(config.ConfigError):
        config.validate(config.from_dict({"health": {"disabledChecks": "ecc,xids"}}))


def test_sampler_watchdog_marks_a_wedged_gpu_lost(n):
    """A telemetry call that never returns (wedged driver) produces no error to count:
    the watchdog marks that GPU lost once the call has been in flight for
    health.sampleStallS, and the GPU recovers when the call comes back."""
    be = fixtures.build_backend("2gpu_spx")
    m = n.HealthMonitor(be, 3)
    m.set_gpu_count(2)
    ex = n.Exporter()
    gpus, _ = be.discover()
    ex.set_inventory(gpus)
    ex.set_stall_ms(300)
    ex.start(be, 20, m)
    try:
        assert "amdgpu_telemetry_last_pass_age_seconds " in ex.render()
        be.set_sample_stall(1, True)
        t0 = time.monotonic()
        got = []
        while time.monotonic() - t0 < 5 and not got:
            got = [u for u in m.pop(100) if u.healthy == 0]
        assert got and got[0].gpu == 1 and "in flight" in got[0].reason, got
        assert time.monotonic() - t0 >= 0.25  # not before the threshold
        assert ex.stalled_gpu == 1 and not m.gpu_healthy(1) and m.gpu_healthy(0)
        text = ex.render()
        assert 'amdgpu_telemetry_sample_stalled{gpu="1"} 1' in text
        age = float([ln for ln in text.splitlines()
                     if ln.startswith("amdgpu_telemetry_last_pass_age_seconds ")][0].split()[1])
        assert age < 0.25  # passes go on: the wedge holds GPU 1's lane, not the sampler
        ages = {ln.split('"')[1]: float(ln.split()[1]) for ln in text.splitlines()
                if ln.startswith("amdgpu_telemetry_sample_age_seconds{")}
        assert ages["1"] >= 0.25 and ages["0"] < 0.25, ages  # GPU 0 stays fresh
        # telemetry_up comes with the GPU text of a pass: wait for one past the bound
        assert _wait_for(lambda: 'amdgpu_telemetry_up{gpu="1"} 0' in ex.render()
                         and 'amdgpu_telemetry_up{gpu="0"} 1' in ex.render())
        be.set_sample_stall(1, False)
        deadline = time.monotonic() + 5
        back = []
        while time.monotonic() < deadline and not back:
            back = [u for u in m.pop(100) if u.healthy == 1]
        assert back and back[0].gpu == 1 and m.gpu_healthy(1)
        # cleared with the pass that brought the call back (and the watchdog's next look)
        assert _wait_for(lambda: ex.stalled_gpu == -1 and "amdgpu_telemetry_sample_stalled" not in ex.render())
    finally:
        be.set_sample_stall(1, False)
        ex.stop()


def test_health_monitor_from_samples(n):
    be = fixtures.build_backend("2gpu_spx")
    m = n.HealthMonitor(be, 2)
    m.set_gpu_count(2)
    ex = n.Exporter()
    gpus, _ = be.discover()
    ex.set_inventory(gpus)
    ex.start(be, 30, m)
    try:
        time.sleep(0.1)
        be.set_ecc_uncorrectable(0, 1)
        deadline = time.monotonic() + 3
        got = []
        while time.monotonic() < deadline and not got:
            got = [u for u in m.pop(100) if u.healthy == 0]
        assert got and got[0].gpu == 0 and "ecc" in got[0].reason
    finally:
        ex.stop()


def test_monitor_event_thread_scripted(n):
    model = fixtures.mi355x_node(2, events=[{"at": 0.05, "kind": "pre_reset", "gpu": 0},
                                            {"at": 0.10, "kind": "link_down", "gpu": 0, "peer": 1}])
    be = fixtures.build_backend(model)
    m = n.HealthMonitor(be, 3)
    m.set_gpu_count(2)
    m.start()
    try:
        got = []
        deadline = time.monotonic() + 3
        while time.monotonic() < deadline and len(got) < 2:
            got += m.pop(100)
        assert (got[0].gpu, got[0].healthy) == (0, 0)
        assert got[1].link_up == 0 and got[1].peer == 1
        assert not be.discover()[1].link(0, 1).up
    finally:
        m.stop()
        m.stop()


def test_prometheus_number_formatting(n):
    """Shortest round-trip %g formatting (Go strconv.FormatFloat 'g' -1 as used by
    promhttp) on the Ryu fast path; integers print as integers."""
    import math
    cases = {0.0005: "0.0005", 1e-05: "1e-05", 30.0: "30", 0.1: "0.1", 1.5e-07: "1.5e-07", -0.5: "-0.5",
             2.5: "2.5", 0.0: "0", 1e6: "1000000", -3.0: "-3", float("inf"): "+Inf", float("-inf"): "-Inf",
             123.456: "123.456", 1e-4: "0.0001"}
    for v, want in cases.items():
        assert n.format_float(v) == want, (v, n.format_float(v))
    assert n.format_float(float("nan")) == "NaN"


@settings(max_examples=300, deadline=None)
@given(st.floats(allow_nan=False, allow_infinity=False))
def test_prometheus_number_round_trips(n, v):
    assert float(n.format_float(v)) == v


def test_retired_pages_threshold_state_machine(n):
    """Retired + pending HBM pages at the threshold latch Unhealthy; a reset does not
    clear it (retired pages persist), dropping below the threshold does."""
    be = fixtures.build_backend("2gpu_spx")
    m = n.HealthMonitor(be, 3)
    m.set_gpu_count(2)
    m.set_bad_page_thresholds([10, 0])
    ok = be.sample(1)
    assert ok.retired_pages == 0 and ok.pending_pages == 0
    be.set_retired_pages(0, 8, 2)
    be.set_retired_pages(1, 500, 0)  # threshold 0 on GPU 1: check disabled
    for g in (0, 1):
        m.on_sample(g, True, be.sample(g))
    # the first sample also reports every link's state and bandwidth once
    u = [x for x in m.pop(100) if x.kind not in (n.EVT_LINK_QUALITY, n.EVT_LINK_UP, n.EVT_LINK_DOWN)]
    assert [(x.gpu, x.healthy) for x in u] == [(0, 0)] and "retired" in u[0].reason
    m.process(n.HwEvent(n.EVT_PRE_RESET, 0))
    m.process(n.HwEvent(n.EVT_POST_RESET, 0))
    m.on_sample(0, True, be.sample(0))
    assert m.pop(50) == [] and not m.gpu_healthy(0)
    be.set_retired_pages(0, 9, 0)
    m.on_sample(0, True, be.sample(0))
    assert [(x.gpu, x.healthy) for x in m.pop(100)] == [(0, 1)]


def test_retired_pages_exported_and_gate_advertisement(make_cfg, plugin_dir):
    import time as _t
    from k8s_gpu_device_plugin_amd.plugin.kubelet_stub import KubeletStub
    from k8s_gpu_device_plugin_amd.plugin.manager import PluginManager
    model = fixtures.mi355x_node(2)
    for g in model["gpus"]:
        g["bad_page_threshold"] = 64  # what a root-readable RAS threshold would report
    be = fixtures.build_backend(model)
    with KubeletStub(plugin_dir) as k:
        m = PluginManager(make_cfg(telemetry={"intervalMs": 40}), backend=be)
        t = m.start_background()
        try:
            w = k.watch(k.wait_for_registrations(1)[0].endpoint)
            w.next()
            be.set_retired_pages(1, 60, 4)
            _, devs = w.next(timeout=5)
            assert [h for _, h, _ in devs] == ["Healthy", "Unhealthy"]
            _t.sleep(0.1)
            fams = _families(m.exporter.render())
            pages = {(s.labels["gpu"], s.labels["status"]): s.value for s in fams["amdgpu_retired_pages"].samples}
            assert pages[("1", "reserved")] == 60 and pages[("1", "pending")] == 4 and pages[("0", "reserved")] == 0
            thr = {s.labels["gpu"]: s.value for s in fams["amdgpu_retired_pages_threshold"].samples}
            assert thr == {"0": 64.0, "1": 64.0}
        finally:
            m.stop()
            t.join(10)
    # health.badPageThreshold overrides the hardware value; -1 turns the check off
    be = fixtures.build_backend(model)
    be.set_retired_pages(0, 1000, 0)
    m = PluginManager(make_cfg(health={"badPageThreshold": -1}, telemetry={"intervalMs": 40}), backend=be)
    t = m.start_background()
    try:
        _t.sleep(0.2)
        assert all(p.table.healthy_count() == len(p) for p in m.plugins)
        assert "amdgpu_retired_pages_threshold" not in m.exporter.render()
    finally:
        m.stop()
        t.join(10)


@pytest.mark.skipif("tsan" in os.environ.get("LD_PRELOAD", ""),
                    reason="TSan runs: symbolize forks addr2line from the many-threaded instrumented process, "
                           "which can hang in the sanitizer's fork handling (it did once in a full run)")
def test_native_sampling_profiler_sees_native_threads(n):
    """The benchmark harness's pprof analogue samples every thread, including native
    threads Python cannot see, and resolves internal C++ functions."""
    from k8s_gpu_device_plugin_amd.benchmark.profiling import symbolize
    assert n.prof_start(2000) and n.prof_running()
    assert not n.prof_start(2000)  # one profile at a time
    t0 = time.monotonic()
    while time.monotonic() - t0 < 0.6:
        native.load_bench().uds_pingpong(2000, 0, 128, 256)  # client + epoll server threads, no GIL
    n.prof_stop()
    n.prof_stop()
    assert not n.prof_running()
    rows = symbolize(n.prof_histogram())
    assert sum(c for _, _, c in rows) >= 20
    text = " ".join(fn for fn, _, _ in rows)
    assert any(k in text for k in ("send", "recv", "epoll_wait", "uds_pingpong")), rows[:10]


def test_exporter_and_monitor_stop_right_after_start(n):
    """Sampler, watchdog and monitor threads that have not run yet when stop() comes
    still leave promptly."""
    be = fixtures.build_backend("2gpu_spx")
    gpus, _ = be.discover()
    t0 = time.monotonic()
    for _ in range(10):
        m = n.HealthMonitor(be, 3)
        m.set_gpu_count(2)
        m.start()
        ex = n.Exporter()
        ex.set_inventory(gpus)
        ex.set_stall_ms(1000)
        ex.start(be, 20, m)
        ex.stop()
        m.stop()
    assert time.monotonic() - t0 < 15


def test_health_follows_gpu_identity_across_reenumeration(n):
    """GPU 0 starts a reset and drops off the bus; re-discovery moves GPU 1 to index 0.
    Health is kept per identity, so the healthy GPU does not inherit the vanished one's
    reset latch, and the vanished GPU is Unhealthy again when it returns, until its
    POST_RESET (reference device/devices.go:41-85: device IDs are UUIDs)."""
    be = fixtures.build_backend("2gpu_spx")
    gpus, _ = be.discover()
    keys = [be.gpu_key(g.index) for g in gpus]
    assert keys == [g.uuid for g in gpus] and len(set(keys)) == 2
    m = n.HealthMonitor(be, 3)
    m.set_gpus(keys)
    ids = [g.partitions[0].id for g in gpus]

    def tables(gs):
        return [n.DeviceTable(n.TableConfig(), [n.TableDevice(g.partitions[0].id, g.index) for g in gs],
                              n.Topology(len(gs)))]

    m.start()
    try:
        t = tables(gpus)
        m.attach_tables(t, True, [])
        be.inject_event(n.HwEvent(n.EVT_PRE_RESET, 0, message="fixture reset"))
        deadline = time.monotonic() + 5
        while time.monotonic() < deadline and t[0].healthy(ids[0]):
            time.sleep(0.01)
        assert not t[0].healthy(ids[0]) and t[0].healthy(ids[1])
        u = [x for x in m.pop(100) if x.healthy == 0]
        assert u and u[0].key == keys[0] and u[0].gpu == 0
        # GPU 0 falls off the bus; the node is re-discovered and GPU 1 is now index 0
        be.set_gpu_present(0, False)
        gpus2, _ = be.discover()
        assert [g.uuid for g in gpus2] == [keys[1]] and gpus2[0].index == 0
        assert be.gpu_key(0) == keys[1]
        s = be.sample(0)
        assert s is not None and s.key == keys[1]  # index 0 now samples the old GPU 1
        m.set_gpus([be.gpu_key(0)])
        t2 = tables(gpus2)
        m.attach_tables(t2, True, [])
        assert t2[0].healthy(ids[1]) and m.gpu_healthy(0)
        assert m.unhealthy_keys() == [keys[0]]
        # a sampling pass over the new index space leaves it healthy
        m.on_sample(0, True, be.sample(0))
        assert m.gpu_healthy(0) and not [x for x in m.pop(50) if x.healthy == 0]
        # the vanished GPU returns, still mid-reset: Unhealthy at once
        be.set_gpu_present(0, True)
        gpus3, _ = be.discover()
        m.set_gpus([be.gpu_key(g.index) for g in gpus3])
        t3 = tables(gpus3)
        m.attach_tables(t3, True, [])
        assert not t3[0].healthy(ids[0]) and t3[0].healthy(ids[1])
        assert not m.gpu_healthy(0) and m.gpu_healthy(1)
        be.inject_event(n.HwEvent(n.EVT_POST_RESET, 0))
        deadline = time.monotonic() + 5
        while time.monotonic() < deadline and not t3[0].healthy(ids[0]):
            time.sleep(0.01)
        assert t3[0].healthy(ids[0]) and m.gpu_healthy(0) and m.unhealthy_keys() == []
    finally:
        m.stop()


def test_fixture_events_name_slots_and_arrive_in_discovery_indices(n):
    """Scripted events name a fixture GPU by slot; delivered events carry the slot's
    identity and its index in the latest discovery (-1 while it is not discovered)."""
    be = fixtures.build_backend("4gpu_spx")
    gpus, _ = be.discover()
    uuid = [g.uuid for g in gpus]
    be.set_gpu_present(1, False)
    be.discover()
    be.arm_events()
    m = n.HealthMonitor(be, 3)
    m.set_gpus([be.gpu_key(i) for i in range(3)])
    assert [be.gpu_key(i) for i in range(3)] == [uuid[0], uuid[2], uuid[3]]
    be.inject_event(n.HwEvent(n.EVT_LINK_DOWN, 3, peer=2))
    be.inject_event(n.HwEvent(n.EVT_THERMAL, 1))
    m.start()
    try:
        got = []
        deadline = time.monotonic() + 5
        while time.monotonic() < deadline and len(got) < 2:
            got += m.pop(100)
        link = [u for u in got if u.link_up == 0][0]
        assert (link.gpu, link.peer, link.key, link.peer_key) == (2, 1, uuid[3], uuid[2])
        info = [u for u in got if "thermal" in u.reason][0]
        assert info.gpu == -1 and info.key == uuid[1]  # not advertised right now
    finally:
        m.stop()


def test_exporter_start_and_stop_do_not_hang_on_a_wedged_first_call(n):
    """The driver is already wedged when the plugin starts: start() returns after one
    pass budget (the wedge holds GPU 0's lane, not the sampler; the manager still has an
    event loop to run), the watchdog marks the GPU lost, GPU 1 is sampled meanwhile, and
    stop() joins the sampler at once: the stuck call stays on its lane and ends there."""
    be = fixtures.build_backend("2gpu_spx")
    gpus, _ = be.discover()
    m = n.HealthMonitor(be, 3)
    m.set_gpus([be.gpu_key(g.index) for g in gpus])
    ex = n.Exporter()
    ex.set_inventory(gpus)
    ex.set_stall_ms(300)
    be.set_sample_stall(0, True)
    try:
        t0 = time.monotonic()
        ex.start(be, 50, m)
        assert time.monotonic() - t0 < 0.25
        assert 'amdgpu_telemetry_up{gpu="1"} 1' in ex.render()
        deadline = time.monotonic() + 5
        lost = []
        while time.monotonic() < deadline and not lost:
            lost = [u for u in m.pop(100) if u.healthy == 0]
        assert lost and lost[0].gpu == 0 and "in flight" in lost[0].reason
        assert m.gpu_healthy(1)
        t0 = time.monotonic()
        ex.stop()
        assert time.monotonic() - t0 < 0.5 and not ex.running
        lane0 = [x for x in be.lanes() if x[0] == 0][0]
        assert lane0[2] == "sample" and lane0[3] >= 0.25, lane0  # still stuck, on its lane
    finally:
        be.set_sample_stall(0, False)  # the lane's call returns
    assert _wait_for(lambda: [x for x in be.lanes() if x[0] == 0][0][2] == "")
    del ex


def _wait_for(pred, timeout=5.0):
    deadline = time.monotonic() + timeout
    while time.monotonic() < deadline:
        if pred():
            return True
        time.sleep(0.02)
    return False


def test_watchdog_does_not_report_a_call_that_already_returned(n):
    """Calls that return just under the threshold, over and over: the watchdog's check
    and the sampler's end-of-call are ordered, so no GPU is ever reported lost."""
    be = fixtures.build_backend("2gpu_spx")
    gpus, _ = be.discover()
    m = n.HealthMonitor(be, 3)
    m.set_gpus([be.gpu_key(g.index) for g in gpus])
    ex = n.Exporter()
    ex.set_inventory(gpus)
    ex.set_stall_ms(1000)
    ex.start(be, 5, m)
    try:
        t_end = time.monotonic() + 1.0
        while time.monotonic() < t_end:
            assert not [u for u in m.pop(20) if u.healthy == 0]
        assert m.gpu_healthy(0) and m.gpu_healthy(1)
    finally:
        ex.stop()


def test_exporter_restart_while_a_gpu_call_is_wedged(n):
    """stop() and start() again while GPU 1's call is wedged: the new sampler samples GPU 0
    at once, posts nothing more to GPU 1's busy lane, and picks GPU 1 up again when its
    call returns."""
    be = fixtures.build_backend("2gpu_spx")
    gpus, _ = be.discover()
    ex = n.Exporter()
    ex.set_inventory(gpus)
    ex.set_stall_ms(200)
    be.set_sample_stall(1, True)
    ex.start(be, 20, None)
    time.sleep(0.1)
    ex.stop()
    ex.start(be, 20, None)
    try:
        n0 = ex.samples_total
        assert _wait_for(lambda: ex.samples_total >= n0 + 5, 3)
        text = ex.render()
        assert 'amdgpu_telemetry_up{gpu="0"} 1' in text and 'amdgpu_telemetry_up{gpu="1"} 0' in text
        assert [x for x in be.lanes() if x[0] == 1][0][5] == 0  # nothing queued behind the wedge
        be.set_sample_stall(1, False)
        assert _wait_for(lambda: 'amdgpu_telemetry_up{gpu="1"} 1' in ex.render(), 3)
    finally:
        be.set_sample_stall(1, False)
        t0 = time.monotonic()
        ex.stop()
        assert time.monotonic() - t0 < 1.0


def test_link_bandwidth_first_reading_and_retrain(n):
    """The first telemetry reading of each link is reported once per link (the peer's
    sample of the same link is deduplicated), so a link that re-trained between
    discovery and the first sample still reaches the tables; after that only a change
    of more than 5 % is."""
    be = fixtures.build_backend("2gpu_spx")
    gpus, _ = be.discover()
    m = n.HealthMonitor(be, 3)
    m.set_gpus([be.gpu_key(g.index) for g in gpus])
    for g in (0, 1):
        m.on_sample(g, True, be.sample(g))
    q = [u for u in m.pop(100) if u.kind == n.EVT_LINK_QUALITY]
    assert len(q) == 1 and q[0].link_gbps == 608.0 and {q[0].gpu, q[0].peer} == {0, 1}
    be.set_link_bandwidth(0, 1, 600.0)  # within 5 %: not a re-train
    m.on_sample(0, True, be.sample(0))
    assert not [u for u in m.pop(50) if u.kind == n.EVT_LINK_QUALITY]
    be.set_link_bandwidth(0, 1, 304.0)
    m.on_sample(1, True, be.sample(1))
    q = [u for u in m.pop(100) if u.kind == n.EVT_LINK_QUALITY]
    assert len(q) == 1 and q[0].link_gbps == 304.0 and "re-trained" in q[0].reason


def test_pcie_floor_state_machine(n):
    """health.pcieMinWidth / pcieMinSpeedGTs: a host link that trained narrower or slower
    latches the GPU Unhealthy until it trains back; no floor, no check; the check can be
    disabled (still logged) and removing the floor releases a held GPU."""
    be = fixtures.build_backend("2gpu_spx")
    m = n.HealthMonitor(be, 3)
    m.set_gpu_count(2)

    def health_updates():
        return [(x.gpu, x.healthy, x.kind) for x in m.pop(100)
                if x.kind not in (n.EVT_LINK_QUALITY, n.EVT_LINK_UP, n.EVT_LINK_DOWN)]
    be.set_pcie_link(1, 8, 32.0)
    for g in (0, 1):
        m.on_sample(g, True, be.sample(g))
    assert health_updates() == [] and m.gpu_healthy(1)  # no floor configured
    m.set_pcie_floor(16, 32.0)
    m.on_sample(1, True, be.sample(1))
    u = m.pop(100)
    assert [(x.gpu, x.healthy, x.kind) for x in u] == [(1, 0, n.EVT_PCIE_DEGRADED)] and "x8" in u[0].reason
    m.on_sample(1, True, be.sample(1))
    assert m.pop(50) == [] and not m.gpu_healthy(1)  # latched, reported once
    be.set_pcie_link(1, 16, 16.0)  # full width, but Gen4
    m.on_sample(1, True, be.sample(1))
    assert m.pop(50) == [] and not m.gpu_healthy(1)
    be.set_pcie_link(1, 16, 32.0)
    m.on_sample(1, True, be.sample(1))
    assert health_updates() == [(1, 1, n.EVT_PCIE_RESTORED)]
    # disabled: tracked and logged, never Unhealthy
    m.set_disabled_checks(16)
    be.set_pcie_link(0, 4, 32.0)
    m.on_sample(0, True, be.sample(0))
    u = m.pop(50)
    assert m.gpu_healthy(0) and u and "disabled" in u[0].reason
    m.set_disabled_checks(0)
    assert not m.gpu_healthy(0)
    m.pop(50)
    m.set_pcie_floor(0, 0.0)  # the floor removed: the held GPU is released at once
    assert m.gpu_healthy(0) and [(x.gpu, x.healthy) for x in m.pop(50)] == [(0, 1)]


def test_pcie_floor_is_debounced(n):
    """one low PCIe reading (a link caught in a power-saving state) must not flap
    ListAndWatch: `debounce` consecutive samples below the floor degrade the GPU, as many
    at or above it restore it; an alternating link never degrades."""
    be = fixtures.build_backend("2gpu_spx")
    m = n.HealthMonitor(be, 3)
    m.set_gpu_count(2)
    m.set_pcie_floor(16, 32.0, 3)

    def health():
        return [(x.gpu, x.healthy) for x in m.pop(20)
                if x.kind not in (n.EVT_LINK_QUALITY, n.EVT_LINK_UP, n.EVT_LINK_DOWN)]
    for width in (8, 16, 8, 16, 8, 16):  # flapping: never three low readings in a row
        be.set_pcie_link(1, width, 32.0)
        m.on_sample(1, True, be.sample(1))
    assert health() == [] and m.gpu_healthy(1)
    be.set_pcie_link(1, 8, 32.0)
    for i in range(3):
        m.on_sample(1, True, be.sample(1))
        assert m.gpu_healthy(1) == (i < 2)
    assert health() == [(1, 0)]
    be.set_pcie_link(1, 16, 32.0)
    for i in range(3):
        m.on_sample(1, True, be.sample(1))
        assert m.gpu_healthy(1) == (i == 2)
    assert health() == [(1, 1)]


def test_pcie_floor_from_config(make_cfg, plugin_dir):
    """The manager applies health.pcieMinWidth: a GPU whose host link drops to x8 is
    advertised Unhealthy, and Healthy again when it trains back to x16."""
    from k8s_gpu_device_plugin_amd.plugin.kubelet_stub import KubeletStub
    from k8s_gpu_device_plugin_amd.plugin.manager import PluginManager
    be = fixtures.build_backend("2gpu_spx")
    with KubeletStub(plugin_dir) as k:
        m = PluginManager(make_cfg(health={"pcieMinWidth": 16}, telemetry={"intervalMs": 30}), backend=be)
        t = m.start_background()
        try:
            w = k.watch(k.wait_for_registrations(1)[0].endpoint)
            w.next()
            be.set_pcie_link(0, 8, 32.0)
            _, devs = w.next(timeout=5)
            assert [h for _, h, _ in devs] == ["Unhealthy", "Healthy"]
            be.set_pcie_link(0, 16, 32.0)
            _, devs = w.next(timeout=5)
            assert [h for _, h, _ in devs] == ["Healthy", "Healthy"]
        finally:
            m.stop()
            t.join(10)


def test_sampler_slows_down_while_unread_and_settled(n):
    """VERDICT r5 item 4 (telemetry.idleIntervalMs): once the start window is over, nothing
    has read the GPU metrics for activeWindowS and health is settled, the sampler runs at
    the idle period; the first read wakes it at once and restores the interval; a failing
    GPU keeps it at the interval while it fails."""
    be = fixtures.build_backend("2gpu_spx")
    m = n.HealthMonitor(be, 3)
    m.set_gpu_count(2)
    ex = n.Exporter()
    gpus, _ = be.discover()
    ex.set_inventory(gpus)
    ex.set_idle_interval(600, 300)
    ex.start(be, 30, m)
    try:
        assert ex.current_interval_ms == 30
        assert _wait_for(lambda: ex.current_interval_ms == 600, timeout=3)
        assert ex.idle_passes >= 1
        n0, t0 = ex.samples_total, time.monotonic()
        time.sleep(0.9)  # idle: one or two passes, not thirty
        assert ex.samples_total - n0 <= 3
        text = ex.render()  # a scrape: the sampler wakes now, not at its next idle tick
        assert "amdgpu_telemetry_interval_seconds 0.6" in text
        n1, t1 = ex.samples_total, time.monotonic()
        assert _wait_for(lambda: ex.samples_total > n1, timeout=0.4)
        assert time.monotonic() - t1 < 0.4
        assert _wait_for(lambda: ex.current_interval_ms == 30, timeout=1)
        assert "amdgpu_telemetry_interval_seconds 0.03" in ex.render()
        # unread again, but a GPU's samples fail: health is not settled, the cadence holds
        assert _wait_for(lambda: ex.current_interval_ms == 600, timeout=3)
        be.set_sample_fail(1, True)
        ex.render()  # (wake it: the failure is seen on the next pass)
        assert _wait_for(lambda: not m.gpu_healthy(1), timeout=3)
        time.sleep(0.6)  # past the read window
        assert ex.current_interval_ms == 30
        be.set_sample_fail(1, False)
        assert _wait_for(lambda: m.gpu_healthy(1), timeout=3)
        assert _wait_for(lambda: ex.current_interval_ms == 600, timeout=3)
    finally:
        ex.stop()


def test_idle_interval_off_or_below_the_interval_keeps_the_interval(n):
    be = fixtures.build_backend("2gpu_spx")
    ex = n.Exporter()
    gpus, _ = be.discover()
    ex.set_inventory(gpus)
    for idle in (0, 20):
        ex.set_idle_interval(idle, 50)
        ex.start(be, 30, None)
        try:
            time.sleep(0.3)
            assert ex.current_interval_ms == 30 and ex.idle_passes == 0
        finally:
            ex.stop()


def test_sampler_follows_a_slow_scraper(n):
    """While scraped and settled, the sampler runs about twice per scrape interval,
    between telemetry.intervalMs and idleIntervalMs: a Prometheus scraping every 15-30 s
    does not keep it at the 1 s interval."""
    be = fixtures.build_backend("2gpu_spx")
    m = n.HealthMonitor(be, 3)
    m.set_gpu_count(2)
    ex = n.Exporter()
    gpus, _ = be.discover()
    ex.set_inventory(gpus)
    ex.set_idle_interval(800, 1500)
    ex.start(be, 20, m)
    try:
        assert _wait_for(lambda: ex.current_interval_ms == 800, timeout=4)  # start window over, unread
        for _ in range(4):  # a scraper every 300 ms
            ex.render()
            time.sleep(0.3)
        assert _wait_for(lambda: 120 <= ex.current_interval_ms <= 180, timeout=2), ex.current_interval_ms
        for _ in range(3):  # one every 1.2 s: samples every 600 ms
            ex.render()
            time.sleep(1.2)
        assert 500 <= ex.current_interval_ms <= 700, ex.current_interval_ms
        for _ in range(8):  # fast scrapes never push it below the interval
            ex.render()
            time.sleep(0.11)
        assert _wait_for(lambda: 20 <= ex.current_interval_ms <= 60, timeout=2), ex.current_interval_ms
    finally:
        ex.stop()
