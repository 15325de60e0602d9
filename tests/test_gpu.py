"""Real-hardware tests (MI355X via gpurun): amdsmi discovery/telemetry, the gfx950
canary kernels (incl. an MFMA GEMM numerics check against a PyTorch fp32 reference)
and the full plugin path on the real backend."""
import json
import os
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def amdsmi_backend(n):
    if not n.amdsmi_available():
        pytest.fail("amdsmi sees no AMD GPU on a GPU test run")
    be = n.make_amdsmi_backend()
    yield be
    be.shutdown()


def test_amdsmi_probe_session_ownership(n):
    """A probe-only amdsmi_available() closes its session; keep=True hands it to the next
    backend, and release_probe() drops it when no backend follows."""
    assert n.amdsmi_available()
    assert not n.amdsmi_probe_held()
    assert n.amdsmi_available(keep=True)
    n.amdsmi_release_probe()
    assert not n.amdsmi_probe_held()
    assert n.amdsmi_available(keep=True)
    be = n.make_amdsmi_backend()  # adopts the probe's session
    assert not n.amdsmi_probe_held()
    gpus, _ = be.discover()
    assert gpus
    be.shutdown()
    be2 = n.make_amdsmi_backend()  # the session was closed with be: a fresh init works
    assert be2.discover()[0]
    be2.shutdown()


def test_amdsmi_discovers_mi355x(amdsmi_backend):
    gpus, topo = amdsmi_backend.discover()
    assert len(gpus) >= 1 and topo.n == len(gpus)
    g = gpus[0]
    assert g.gfx_target == "gfx950", g.gfx_target
    assert g.uuid and g.bdf.count(":") == 2
    assert g.vram_total_bytes > 200 * 10**9, g.vram_total_bytes  # 288 GB HBM3E
    assert g.compute_partition in ("SPX", "DPX", "QPX", "CPX")
    assert g.memory_partition.startswith("NPS")
    assert len(g.partitions) >= 1
    for p in g.partitions:
        assert p.render_minor >= 128
        assert os.path.exists("/dev/dri/renderD%d" % p.render_minor)
        assert p.id
    # node-labeller inventory: PCI device id, OAM slot, driver and VBIOS versions
    assert g.device_id != 0 and g.driver_version[:1].isdigit() and "." in g.driver_version, \
        (hex(g.device_id), g.driver_version)
    assert len(g.driver_version) <= 63  # fits a label value
    print("discovered", [(x.index, x.bdf, x.market_name, x.compute_partition, x.memory_partition,
                          len(x.partitions), x.numa_node, x.num_compute_units, hex(x.device_id), x.oam_id,
                          x.driver_version, x.vbios_version) for x in gpus])


def test_partition_profile_comes_from_amdsmi(amdsmi_backend):
    """The partition count is the driver's accelerator partition profile
    (amdsmi_get_gpu_accelerator_partition_profile; reference resources.go:43-51 asks the
    driver for MIG profiles too), and it agrees with the processors amdsmi enumerated
    for the box's current mode."""
    gpus, _ = amdsmi_backend.discover()
    seen = []
    for g in gpus:
        seen.append((g.index, g.compute_partition, g.partition_profile, g.profile_partitions, g.profile_index,
                     len(g.partitions), g.nps_caps))
        if g.profile_partitions:
            assert g.partition_profile == g.compute_partition, seen[-1]
            assert g.profile_partitions == len(g.partitions), seen[-1]
    print("partition profiles", seen)
    assert any(x[3] for x in seen), "amdsmi reported no accelerator partition profile: %s" % seen
    assert amdsmi_backend.gpu_key(0) == (gpus[0].uuid or gpus[0].bdf)
    s = amdsmi_backend.sample(0)
    assert s is not None and s.key == amdsmi_backend.gpu_key(0)


def test_amdsmi_telemetry(amdsmi_backend):
    gpus, _ = amdsmi_backend.discover()
    s = amdsmi_backend.sample(0)
    assert s is not None and s.ok
    assert s.power_w > 0 or s.temp_hotspot_c > 0
    assert s.vram_total_bytes > 0
    # the xGMI error state needs privileges the box's user lacks (-1 then: the family is left out)
    assert s.xgmi_error_status in (-1, 0, 1, 2)
    assert s.pcie_link_width == -1 or 1 <= s.pcie_link_width <= 32
    print("sample", s.power_w, s.temp_hotspot_c, s.temp_hbm_c, s.gfx_activity_pct, s.vram_used_bytes, s.links,
          "xgmi errors", s.xgmi_error_status, "pcie x%g %g GT/s replays %g recoveries %g"
          % (s.pcie_link_width, s.pcie_link_speed_gtps, s.pcie_replays, s.pcie_recoveries))


def test_amdsmi_sample_cost_breakdown(amdsmi_backend):
    """Where one telemetry pass spends its time (it runs once per GPU per tick, off the
    request path, but 8 GPUs x 8 partitions must fit a 1 s tick with room to spare)."""
    gpus, _ = amdsmi_backend.discover()
    before = amdsmi_backend.sample_costs()
    first = amdsmi_backend.sample(0)
    assert first.ok
    samples = [amdsmi_backend.sample(0) for _ in range(19)]
    assert all(x.ok for x in samples)
    after = amdsmi_backend.sample_costs()
    counts = ("xgmi_links_", "partition_busy_", "ecc_count_reads_", "vram_reads_")
    per = {k: (after[k][0] - before[k][0]) / 20 * 1e6 for k in after if not k.startswith(counts)}
    paths = {k: after[k][1] - before[k][1] for k in after if k.startswith(counts)}
    print("amdsmi sample cost per GPU (us):", {k: round(v, 1) for k, v in per.items()},
          "total %.1f us" % sum(per.values()), "link paths", paths)
    assert set(per) == {"gpu_metrics", "partition_metrics", "vram_usage", "ecc_count", "xgmi_links", "bad_pages"}
    assert sum(per.values()) < 50e3
    # ECC totals: amdsmi is asked again only when the RAS event state moved (or every
    # 30 s); one-pool VRAM is read from sysfs once it agreed with amdsmi
    ras = "/sys/bus/pci/devices/%s/ras" % gpus[0].bdf.lower()
    if os.path.exists(ras + "/event_state"):
        assert paths["ecc_count_reads_event_gated"] >= 15, paths
    assert paths["vram_reads_sysfs_disagreed"] == 0, paths
    if gpus[0].memory_partition == "NPS1":
        assert paths["vram_reads_sysfs"] == 20, paths
    # samples served from the gpu_metrics blob report the same links as the full path,
    # with byte counters that never run backwards
    for x in samples:
        assert [lk[0] for lk in x.links] == [lk[0] for lk in first.links]
        assert [lk[1] for lk in x.links] == [lk[1] for lk in first.links]
        assert [lk[4:] for lk in x.links] == [lk[4:] for lk in first.links]
    for prev, cur in zip([first] + samples, samples):
        for a, b in zip(prev.links, cur.links):
            assert b[2] >= a[2] and b[3] >= a[3], (a, b)


def test_ecc_totals_are_amdsmi_s_with_or_without_the_event_gate(amdsmi_backend):
    """health.eccEventGate off: the RAS block files are read each sample and amdsmi is
    asked only when one changed; on: only when ras/event_state moved.  Either way the
    counts a sample carries are amdsmi's own totals."""
    gpus, _ = amdsmi_backend.discover()
    amdsmi_backend.set_ecc_event_gate(False)
    try:
        before = amdsmi_backend.sample_costs()
        off = [amdsmi_backend.sample(0) for _ in range(10)]
        after = amdsmi_backend.sample_costs()
    finally:
        amdsmi_backend.set_ecc_event_gate(True)
    on = [amdsmi_backend.sample(0) for _ in range(10)]
    reads = {k: after[k][1] - before[k][1] for k in after if k.startswith("ecc_count_reads_")}
    print("gate off:", reads, "ecc", [(x.ecc_correctable, x.ecc_uncorrectable) for x in off[:2]],
          "gate on:", [(x.ecc_correctable, x.ecc_uncorrectable) for x in on[:2]])
    assert reads["ecc_count_reads_event_gated"] == 0
    if os.path.isdir("/sys/bus/pci/devices/%s/ras" % gpus[0].bdf.lower()):
        assert reads["ecc_count_reads_unchanged"] >= 8, reads
    # the same counters either way (correctable errors may still be counted meanwhile: they
    # only ever grow)
    assert {x.ecc_uncorrectable for x in off} == {x.ecc_uncorrectable for x in on}
    seq = [x.ecc_correctable for x in off + on]
    assert seq == sorted(seq)
    assert off[0].ecc_uncorrectable >= 0


def test_amdsmi_retired_pages(amdsmi_backend):
    """RAS retired-page records read through amdsmi (0 on a healthy GPU); the threshold
    is root-only, so -1 is accepted for it."""
    gpus, _ = amdsmi_backend.discover()
    s = amdsmi_backend.sample(0)
    print("retired pages", s.retired_pages, s.pending_pages, s.unreservable_pages,
          "threshold", gpus[0].bad_page_threshold)
    assert s.retired_pages >= 0 or s.retired_pages == -1
    assert s.retired_pages <= 0 or s.retired_pages < 10**6
    assert gpus[0].bad_page_threshold == -1 or gpus[0].bad_page_threshold > 0


def test_exporter_renders_real_metrics(n, amdsmi_backend):
    gpus, _ = amdsmi_backend.discover()
    ex = n.Exporter()
    ex.set_inventory(gpus)
    ex.start(amdsmi_backend, 100, None)
    time.sleep(0.5)
    ex.stop()
    text = ex.render()
    assert 'amdgpu_telemetry_up{gpu="0"} 1' in text
    assert "amdgpu_power_watts{" in text or "amdgpu_temperature_celsius{" in text
    assert ex.samples_total >= 2


def test_canary_passes_on_device0():
    from k8s_gpu_device_plugin_amd.ops import canary
    assert canary.device_count() >= 1
    r = canary.run(0, hbm_bytes=512 << 20, passes=2, mfma_iters=4096)
    print("canary", r)
    assert r["ok"], r
    assert r["arch"].startswith("gfx950")
    assert r["hbm_errors"] == 0 and r["mfma_errors"] == 0 and r["gemm_errors"] == 0
    assert r["gemm_tflops"] > 100
    assert r["read_gbps"] > 1000 and r["write_gbps"] > 1000
    assert r["mfma_tflops"] > 100


@pytest.mark.parametrize("shape", [(32, 32, 16), (64, 96, 256), (128, 256, 512)])
def test_mfma_gemm_matches_torch_fp32(shape):
    import torch

    from k8s_gpu_device_plugin_amd.ops import canary
    m, nn, k = shape
    g = torch.Generator().manual_seed(m * 7 + nn + k)
    a = torch.randn(m, k, generator=g).to(torch.bfloat16)
    b = torch.randn(k, nn, generator=g).to(torch.bfloat16)
    bits = lambda t: t.view(torch.int16).numpy().view(np.uint16)  # noqa: E731
    c = canary.mfma_gemm(bits(a), bits(b), device=0)
    ref = (a.float() @ b.float()).numpy()
    err = np.abs(c - ref).max() / max(1e-6, np.abs(ref).max())
    assert err < 1e-5, err  # same bf16 inputs, fp32 accumulate: only summation-order rounding


def test_canary_verifier_catches_injected_corruption():
    from k8s_gpu_device_plugin_amd.ops import canary
    assert canary.detects_corruption(0, 64 << 20, 0) == 0
    assert canary.detects_corruption(0, 64 << 20, 7) == 7


def test_canary_mfma_verifier_catches_injected_fault():
    """One perturbed bf16 operand in 3 of the exactness blocks must surface as wrong
    accumulator registers; none without injection."""
    from k8s_gpu_device_plugin_amd.ops import canary
    assert canary.mfma_detects_corruption(0, 0) == 0
    assert canary.mfma_detects_corruption(0, 3) > 0


def test_canary_isolated_subprocess():
    from k8s_gpu_device_plugin_amd.ops import canary
    r = canary.run_isolated(0, 128 << 20)
    assert r["ok"], r


def test_inspect_on_mi355x(make_cfg):
    """--inspect's view of the real node: the amdsmi inventory and its placements."""
    from k8s_gpu_device_plugin_amd.inspect_node import inspect
    d = inspect(make_cfg(backend="amdsmi", migStrategy="single"), [1])
    assert d["gpus"] and d["gpus"][0]["gfx"] == "gfx950" and d["gpus"][0]["partitions"]
    assert d["gpus"][0]["now"]["ok"] and d["gpus"][0]["now"]["power_w"] > 0
    ids = [x["id"] for x in d["resources"]["amd.com/gpu"]]
    assert d["placement"]["amd.com/gpu"]["1"][0] in ids
    print("inspect", json.dumps(d)[:600])


def test_plugin_end_to_end_on_mi355x(make_cfg, plugin_dir):
    from k8s_gpu_device_plugin_amd.plugin.kubelet_stub import KubeletStub
    from k8s_gpu_device_plugin_amd.plugin.manager import PluginManager
    from k8s_gpu_device_plugin_amd.server.web import WebServer
    import http.client

    cfg = make_cfg(backend="amdsmi", migStrategy="single", webListenAddress="127.0.0.1:0")
    k = KubeletStub(plugin_dir).start()
    mgr = PluginManager(cfg)
    t = mgr.start_background()
    web = WebServer(cfg, mgr)
    port = web.start()
    try:
        regs = k.wait_for_registrations(1, 20)
        assert regs[0].resource_name == "amd.com/gpu"
        w = k.watch(regs[0].endpoint)
        _, devs = w.next(10)
        assert devs and devs[0][1] == "Healthy"
        resp = k.client(regs[0].endpoint).allocate([devs[0][0]])
        paths = [s.host_path for s in resp.container_responses[0].devices]
        assert "/dev/kfd" in paths and any(os.path.exists(p) for p in paths if "renderD" in p), paths
        c = http.client.HTTPConnection("127.0.0.1", port, timeout=5)
        c.request("GET", "/metrics")
        body = c.getresponse().read().decode()
        assert "amdgpu_info{" in body and 'gfx_target="gfx950"' in body
        # GPU event notification (resets) is armed on every advertised GPU of the box
        armed = [ln for ln in body.splitlines() if ln.startswith("amdgpu_device_plugin_health_event_sources ")]
        assert armed and int(armed[0].split()[1]) == len(mgr.gpus) >= 1, armed
        c.request("GET", "/metrics")  # the first scrape is counted once it has been answered
        body = c.getresponse().read().decode()
        assert 'echo_http_requests_total{handler="/metrics",method="GET",status="2xx"}' in body
        # registered with kubelet: the readiness route says so (the manager publishes its
        # state after the registration event has been handled)
        deadline = time.monotonic() + 5
        while True:
            c.request("GET", "/ready")
            r = c.getresponse()
            ready = (r.status, r.read())
            if ready[0] == 200 or time.monotonic() > deadline:
                break
            time.sleep(0.05)
        assert ready == (200, b'{"code":0,"data":"ready","msg":"success"}\n'), ready
    finally:
        web.stop()
        mgr.stop()
        t.join(10)
        k.stop()


def test_restored_latch_on_real_gpu(make_cfg, plugin_dir, n, amdsmi_backend):
    """The persisted uncorrectable-ECC latch end to end on the MI355X: a state file that
    records the GPU's firmware start as it is now (no reset since) keeps the GPU Unhealthy
    through a plugin start; one that records an hour-earlier start (the firmware restarted
    since: a reset) is cleared by the first telemetry sample."""
    import json

    from k8s_gpu_device_plugin_amd.plugin.kubelet_stub import KubeletStub
    from k8s_gpu_device_plugin_amd.plugin.manager import PluginManager
    from k8s_gpu_device_plugin_amd.plugin.state import read_boot_id
    gpus, _ = amdsmi_backend.discover()
    key = amdsmi_backend.gpu_key(0)
    s = amdsmi_backend.sample(0)
    assert s.fw_clock_s > 0
    fw_boot = n.boottime_s() - s.fw_clock_s
    path = os.path.join(plugin_dir, ".amdgpu-device-plugin", "health-state.json")
    os.makedirs(os.path.dirname(path), exist_ok=True)

    def run(recorded):
        with open(path, "w") as f:
            json.dump({"version": 1, "boot_id": read_boot_id(), "gpus": {key: {"ecc": {
                "last_ue": max(0, s.ecc_uncorrectable), "fw_boot_s": recorded, "reason": "gpu test latch",
                "since_ns": 0}}}}, f)
        cfg = make_cfg(backend="amdsmi", migStrategy="none", telemetry={"intervalMs": 100})
        k = KubeletStub(plugin_dir).start()
        mgr = PluginManager(cfg)
        t = mgr.start_background()
        try:
            w = k.watch(k.wait_for_registrations(1, 20)[0].endpoint)
            _, first = w.next(10)
            assert mgr.counters.get("latches_restored") == 1
            time.sleep(1.0)  # ten samples
            return first, mgr.plugins[0].table.healthy_count(), mgr.counters.get("resets_observed", 0)
        finally:
            mgr.stop()
            t.join(10)
            k.stop()

    first, healthy, resets = run(round(fw_boot))
    assert first[0][1] == "Unhealthy" and healthy == 0 and resets == 0, (first, healthy, resets)
    # (the first sample may clear it before the watch opens: only the outcome is checked)
    first, healthy, resets = run(round(fw_boot) - 3600)
    assert healthy == 1 and resets == 1, (first, healthy, resets)


def test_native_grpc_server_on_gpu_box(make_cfg, plugin_dir, n):
    assert hasattr(n, "GrpcServer"), "native gRPC server not built (fail loudly on the GPU box)"
    from k8s_gpu_device_plugin_amd.plugin.kubelet_stub import KubeletStub
    from k8s_gpu_device_plugin_amd.plugin.manager import PluginManager
    cfg = make_cfg(backend="amdsmi", migStrategy="none", grpc={"server": "native"})
    k = KubeletStub(plugin_dir).start()
    mgr = PluginManager(cfg)
    t = mgr.start_background()
    try:
        regs = k.wait_for_registrations(1, 20)
        c = k.client(regs[0].endpoint)
        w = k.watch(regs[0].endpoint)
        _, devs = w.next(10)
        resp = c.allocate([devs[0][0]])
        assert resp.container_responses[0].envs["AMD_VISIBLE_DEVICES"] == devs[0][0]
    finally:
        mgr.stop()
        t.join(10)
        k.stop()


def test_amdsmi_health_monitor_runs_and_stops(n, amdsmi_backend):
    gpus, _ = amdsmi_backend.discover()
    mon = n.HealthMonitor(amdsmi_backend, 3)
    mon.set_gpu_count(len(gpus))
    t0 = time.monotonic()
    mon.start()
    time.sleep(0.5)
    print("amdsmi event sources armed:", amdsmi_backend.armed_event_sources)
    assert mon.running and mon.gpu_healthy(0)
    mon.stop()
    assert not mon.running and time.monotonic() - t0 < 5
    assert [u for u in mon.pop(10) if u.healthy == 0] == []


def test_pcie_floor_on_the_real_link(n, amdsmi_backend):
    """health.pcieMinWidth on real gpu_metrics: the box's x16 Gen5 link passes a 16 /
    32 GT/s floor and fails a floor above it (then passes again once the floor is met)."""
    gpus, _ = amdsmi_backend.discover()
    s = amdsmi_backend.sample(0)
    if s.pcie_link_width <= 0:
        pytest.skip("gpu_metrics reports no PCIe link width on this box")
    mon = n.HealthMonitor(amdsmi_backend, 3)
    mon.set_gpu_count(len(gpus))
    mon.set_pcie_floor(int(s.pcie_link_width), float(s.pcie_link_speed_gtps))
    mon.on_sample(0, True, amdsmi_backend.sample(0))
    assert mon.gpu_healthy(0)
    mon.set_pcie_floor(int(s.pcie_link_width) * 2, 0.0)
    mon.on_sample(0, True, amdsmi_backend.sample(0))
    assert not mon.gpu_healthy(0)
    assert any(u.kind == n.EVT_PCIE_DEGRADED for u in mon.pop(50))
    mon.set_pcie_floor(int(s.pcie_link_width), 0.0)
    mon.on_sample(0, True, amdsmi_backend.sample(0))
    assert mon.gpu_healthy(0)


def test_firmware_clock_reset_signal_on_real_gpu(n, amdsmi_backend, tmp_path):
    """The reset signal an unprivileged pod has (native/health.cpp): the GPU firmware's
    clock, read from gpu_metrics, ticks at one second per second (profiles/r5/
    reset_signal_probe.json: 100.004 MHz); a latch restored with the firmware start it
    recorded holds, and one restored with an earlier start (the firmware restarted since,
    i.e. the GPU was reset) is cleared once this process has seen the clock tick (three
    samples: ADVICE r5, a frozen clock never clears a latch)."""
    gpus, _ = amdsmi_backend.discover()
    a = amdsmi_backend.sample(0)
    time.sleep(0.5)
    b = amdsmi_backend.sample(0)
    assert a.fw_clock_s > 0 and b.fw_clock_s > a.fw_clock_s, (a.fw_clock_s, b.fw_clock_s)
    rate = (b.fw_clock_s - a.fw_clock_s) / ((b.ts_ns - a.ts_ns) * 1e-9)
    assert 0.9 < rate < 1.1, rate
    fw_boot = n.boottime_s() - b.fw_clock_s
    key = amdsmi_backend.gpu_key(0)
    for recorded, stays in ((fw_boot, True), (fw_boot - 3600.0, False)):
        mon = n.HealthMonitor(amdsmi_backend, 3)
        mon.set_gpus([key])
        mon.restore_latches([n.HealthLatch(key, max(0, b.ecc_uncorrectable), recorded, "test latch", 0)])
        assert not mon.gpu_healthy(0)
        mon.on_sample(0, True, amdsmi_backend.sample(0))
        assert not mon.gpu_healthy(0)  # one reading says nothing about the clock ticking
        for _ in range(3):
            time.sleep(0.2)
            mon.on_sample(0, True, amdsmi_backend.sample(0))
        assert mon.gpu_healthy(0) != stays, (recorded, fw_boot)
        assert mon.resets_observed == (0 if stays else 1)
    print("firmware clock %.1f s, rate %.6f s/s, firmware started at boot+%.1f s" % (b.fw_clock_s, rate, fw_boot))


def test_kernel_reset_count_through_the_render_node(n, amdsmi_backend):
    """health.resetQuery on the real GPU: the sample reads the amdgpu driver's reset count
    through a context on the GPU's render node (unprivileged: the box's user can open it).
    No reset happens here, so it reads 0 and stays 0; turned off, no count is read."""
    amdsmi_backend.discover()
    samples = []
    for _ in range(3):
        samples.append(amdsmi_backend.sample(0))
        time.sleep(0.1)
    counts = [s.reset_count for s in samples]
    assert counts == [0, 0, 0], counts
    amdsmi_backend.set_reset_query(False)
    try:
        assert amdsmi_backend.sample(0).reset_count == -1
    finally:
        amdsmi_backend.set_reset_query(True)
    key = amdsmi_backend.gpu_key(0)
    mon = n.HealthMonitor(amdsmi_backend, 3)
    mon.set_gpus([key])
    for _ in range(3):
        mon.on_sample(0, True, amdsmi_backend.sample(0))
    assert mon.gpu_healthy(0) and mon.resets_observed == 0
    print("kernel reset count through the render node: %s" % counts)


def test_amdsmi_inventory_signature_is_stable(amdsmi_backend):
    from k8s_gpu_device_plugin_amd.plugin.manager import inventory_signature
    a = inventory_signature(amdsmi_backend.discover()[0])
    b = inventory_signature(amdsmi_backend.discover()[0])
    assert a == b  # no spurious re-advertisement from periodic re-discovery


def _bdf_of_render_node(path):
    """/dev/dri/renderD<N> -> PCI BDF of the GPU behind it (sysfs, no GPU call)."""
    dev = os.path.realpath("/sys/class/drm/%s/device" % os.path.basename(path))
    return os.path.basename(dev).lower()


def test_allocation_maps_to_the_right_physical_gpu(make_cfg, plugin_dir, amdsmi_backend):
    """SURVEY.md §7.3 minimum-slice validation: Allocate's DeviceSpecs name the render
    node of the advertised GPU (checked through sysfs), and a child process restricted
    to the allocated device (HIP_VISIBLE_DEVICES from the partition's HIP id, as a
    container that only sees that render node would be) runs a GEMM on the GPU whose
    PCI address matches the allocation."""
    import json
    import subprocess
    import sys

    from k8s_gpu_device_plugin_amd.plugin.kubelet_stub import KubeletStub
    from k8s_gpu_device_plugin_amd.plugin.manager import PluginManager

    gpus, _ = amdsmi_backend.discover()
    by_id = {p.id: (g, p) for g in gpus for p in g.partitions}
    cfg = make_cfg(backend="amdsmi", migStrategy="single")
    k = KubeletStub(plugin_dir).start()
    mgr = PluginManager(cfg)
    t = mgr.start_background()
    try:
        regs = k.wait_for_registrations(1, 20)
        _, devs = k.watch(regs[0].endpoint).next(10)
        dev_id = devs[0][0]
        g, part = by_id[dev_id]
        resp = k.client(regs[0].endpoint).allocate([dev_id])
    finally:
        mgr.stop()
        t.join(10)
        k.stop()
    renders = [s.host_path for s in resp.container_responses[0].devices if "renderD" in s.host_path]
    assert renders == ["/dev/dri/renderD%d" % part.render_minor], renders
    assert _bdf_of_render_node(renders[0]) == g.bdf.lower(), (renders[0], g.bdf)
    code = ("import json, torch; p = torch.cuda.get_device_properties(0); "
            "a = torch.randn(512, 512, device='cuda', dtype=torch.bfloat16); "
            "c = (a @ a.T).float(); ref = a.float() @ a.float().T; "
            "print(json.dumps({'n': torch.cuda.device_count(), 'bus': p.pci_bus_id, 'dom': p.pci_domain_id, "
            "'dev': p.pci_device_id, 'err': float((c - ref).abs().max() / ref.abs().max())}))")
    env = dict(os.environ, HIP_VISIBLE_DEVICES=str(part.hip_id))
    out = subprocess.run([sys.executable, "-c", code], env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                         text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-3000:]
    r = json.loads(out.stdout.strip().splitlines()[-1])
    bdf = "%04x:%02x:%02x" % (r["dom"], r["bus"], r["dev"])
    assert r["n"] == 1 and g.bdf.lower().startswith(bdf), (r, g.bdf)
    assert r["err"] < 2e-2, r


_REINIT_CHILD = """
import json, time
from k8s_gpu_device_plugin_amd import native
from k8s_gpu_device_plugin_amd.plugin.manager import inventory_signature
n = native.load()
be = n.make_amdsmi_backend()
gpus, _ = be.discover()
before = inventory_signature(gpus)
mon = n.HealthMonitor(be, 3)
mon.set_gpu_count(len(gpus))
mon.start()
time.sleep(0.3)
armed = be.armed_event_sources
ok = be.reinit()
gpus2, _ = be.discover()
out = {"reinit": ok, "count": be.reinit_count, "same": inventory_signature(gpus2) == before,
       "armed_before": armed, "armed_after": be.armed_event_sources, "sample_ok": be.sample(0).ok}
mon.stop()
be.shutdown()
print(json.dumps(out))
"""


def test_amdsmi_reinit_keeps_inventory_and_events():
    """Stale-handle recovery (a compute-partition switch needs a fresh amdsmi
    enumeration): in a process that solely owns the amdsmi session, re-initialising
    yields the same inventory and event delivery is re-armed on the new handles."""
    import json
    import subprocess
    import sys
    out = subprocess.run([sys.executable, "-c", _REINIT_CHILD], stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                         text=True, timeout=120, cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    assert out.returncode == 0, out.stderr[-3000:]
    r = json.loads(out.stdout.strip().splitlines()[-1])
    print("reinit", r)
    assert r["reinit"] and r["count"] == 1 and r["same"] and r["sample_ok"]
    assert r["armed_after"] == r["armed_before"]


def test_prestart_canary_on_allocated_partition(make_cfg, plugin_dir):
    """health.canaryOnPreStart on the real GPU: PreStartContainer runs the gfx950 canary
    (child process) on the allocated partition and passes; the device stays Healthy."""
    from k8s_gpu_device_plugin_amd.plugin.kubelet_stub import KubeletStub
    from k8s_gpu_device_plugin_amd.plugin.manager import PluginManager
    cfg = make_cfg(backend="amdsmi", migStrategy="single", health={"canaryOnPreStart": True,
                                                                   "canaryBytes": 256 << 20})
    k = KubeletStub(plugin_dir).start()
    mgr = PluginManager(cfg)
    t = mgr.start_background()
    try:
        reg = k.wait_for_registrations(1, 20)[0]
        assert reg.options.pre_start_required
        ids = mgr.plugins[0].table.ids()
        t0 = time.monotonic()
        k.client(reg.endpoint).pre_start(ids[:1], timeout=60)
        dt = time.monotonic() - t0
        print("PreStartContainer with canary: %.2f s" % dt)
        assert mgr.counters.get("canary_runs", 0) >= 1 and not mgr.counters.get("prestart_failures")
        assert mgr.plugins[0].table.healthy(ids[0]) and dt < 30
    finally:
        mgr.stop()
        t.join(10)
        k.stop()


@pytest.mark.parametrize("kernel,shape", [
    ("lds128", (128, 128, 64)), ("lds128", (256, 384, 512)), ("lds128", (512, 256, 1024)),
    ("pingpong256", (256, 256, 64)), ("pingpong256", (256, 512, 128)), ("pingpong256", (512, 768, 1024)),
    ("pingpong256", (768, 256, 320)), ("pingpong256s", (256, 256, 64)), ("pingpong256s", (256, 512, 128)),
    ("pingpong256s", (512, 768, 1024)), ("pingpong256s", (768, 256, 320)), ("pingpong256s", (256, 256, 192))])
def test_lds_gemm_matches_torch_fp32(kernel, shape):
    """The LDS-staged MFMA GEMMs (global_load_lds, XCD remap; 128x128 double buffer and the
    256x256 wave-group ping-pong) against a PyTorch fp32 reference on random bf16
    operands.  K-tile counts 1, 2, 5 (odd) and 16 cover the ping-pong's prologue, its
    peeled first iteration and both buffer parities."""
    import torch

    from k8s_gpu_device_plugin_amd.ops import canary
    m, nn, k = shape
    g = torch.Generator().manual_seed(m + 3 * nn + 7 * k)
    a = torch.randn(m, k, generator=g).to(torch.bfloat16)
    b = torch.randn(k, nn, generator=g).to(torch.bfloat16)
    bits = lambda t: t.contiguous().view(torch.int16).numpy().view(np.uint16)  # noqa: E731
    c = canary.gemm(bits(a), bits(b.t()), device=0, kernel=kernel)
    ref = (a.float() @ b.float()).numpy()
    err = np.abs(c - ref).max() / max(1e-6, np.abs(ref).max())
    assert err < 1e-5, err


def test_lds_gemm_rate_and_abft():
    """Throughput of both matrix-path kernels at 4096^3 and their exactness check: no
    checksum errors on a healthy GPU, and a single corrupted output element is caught
    (its row and its column).  The ping-pong kernel is also screened for staging races
    over several shapes (exact integer data: any early LDS read shows as a checksum
    error).  torch.matmul (hipBLASLt) on the same shape for scale."""
    from k8s_gpu_device_plugin_amd.ops import canary
    rates = {}
    for kernel in ("lds128", "pingpong256", "pingpong256s"):
        r = canary.gemm_rate(0, 4096, 4096, 4096, iters=20, kernel=kernel)
        assert r["errors"] == 0, r
        rates[kernel] = r["tflops"]
    for kernel in ("pingpong256", "pingpong256s"):
        for shape in [(256, 256, 64), (1024, 2048, 640), (2048, 1024, 4096), (8192, 8192, 1024)]:
            r = canary.gemm_rate(0, *shape, iters=3, kernel=kernel)
            assert r["errors"] == 0, r
    bad = canary.gemm_rate(0, 1024, 1024, 1024, iters=1, inject=True)
    assert bad["errors"] == 2, bad
    bad = canary.gemm_rate(0, 1024, 1024, 1024, iters=1, inject=True, kernel="pingpong256")
    assert bad["errors"] == 2, bad
    # torch's bundled HIP runtime and the system one the canary links cannot both own the
    # device in one process: time torch.matmul (hipBLASLt) in a child process
    import subprocess
    import sys
    code = ("import torch,time;x=torch.randn(4096,4096,device='cuda',dtype=torch.bfloat16);"
            "y=torch.randn(4096,4096,device='cuda',dtype=torch.bfloat16);[x@y for _ in range(3)];"
            "torch.cuda.synchronize();t=time.perf_counter();[x@y for _ in range(20)];torch.cuda.synchronize();"
            "print(2*4096**3*20/(time.perf_counter()-t)/1e12)")
    out = subprocess.run([sys.executable, "-c", code], stdout=subprocess.PIPE, text=True, timeout=90)
    blas = float(out.stdout.strip().splitlines()[-1]) if out.returncode == 0 else float("nan")
    rnd = canary.gemm_rate(0, 4096, 4096, 4096, iters=20, random_data=True)
    assert rnd["errors"] is None and rnd["tflops"] > 200, rnd
    print("GEMM canary %s TFLOP/s (integer data), %.0f (auto kernel, random data); torch.matmul %.0f TFLOP/s "
          "(random data)" % (" / ".join("%s %.0f" % kv for kv in rates.items()), rnd["tflops"], blas))
    assert min(rates.values()) > 200
