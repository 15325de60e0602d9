"""Real-hardware checks of the round-4 backend (MI355X via gpurun): per-GPU lanes over
amdsmi without a backend-wide lock, the driver's partition-profile model, and
per-partition telemetry through amdsmi's partition metrics API.
"""
import os
import subprocess
import sys
import threading
import time

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NPS = {1: "NPS1", 2: "NPS2", 4: "NPS4", 8: "NPS8"}


@pytest.fixture(scope="module")
def be(n):
    if not n.amdsmi_available():
        pytest.fail("amdsmi sees no AMD GPU on a GPU test run")
    b = n.make_amdsmi_backend()
    b.set_call_timeout_ms(10000)
    b.set_stall_ms(10000)
    yield b
    b.shutdown()


def test_current_profile_is_in_the_supported_list(be):
    """The current accelerator partition profile is one the GPU supports, with matching
    partition count and memory mode.  The driver's full list needs root
    (amdsmi_get_gpu_accelerator_partition_profile_config -> NO_PERM for an ordinary user,
    profiles/r4/amdsmi_probe.json); then only the current profile is known (source
    "current") and the check is that it is consistent with the enumeration."""
    gpus, _ = be.discover()
    for g in gpus:
        sup = [(p.type, p.partitions, p.nps_caps, p.source) for p in g.supported_profiles]
        print("GPU", g.index, g.compute_partition, g.memory_partition, "profiles_status", g.profiles_status, sup)
        assert sup, "no supported profile known"
        cur = [p for p in g.supported_profiles if p.type == g.compute_partition]
        assert cur and cur[0].partitions == len(g.partitions), (g.compute_partition, sup)
        mem_bit = {v: k for k, v in NPS.items()}[g.memory_partition]
        assert cur[0].nps_caps & mem_bit, (g.memory_partition, sup)
        assert g.nps_caps & mem_bit
        if g.profiles_status == "ok":
            assert {p.source for p in g.supported_profiles} == {"driver"}
        else:
            assert "PERMISSION" in g.profiles_status.upper() or "PERM" in g.profiles_status.upper(), g.profiles_status
            assert [p.source for p in g.supported_profiles] == ["current"]


_LOAD = """
import time, torch
a = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16)
torch.cuda.synchronize()
print("busy", flush=True)
t = time.time()
while time.time() - t < %f:
    for _ in range(8):
        a @ a
    torch.cuda.synchronize()
"""


def test_partition_metrics_agree_with_the_socket_blob(be):
    """Per-partition busy comes from amdsmi_get_gpu_partition_metrics_info on the
    partition's processor (source 1).  In SPX the one partition is the whole GPU: its busy
    figure must agree with the socket blob's activity, idle and under a bf16 GEMM load, and
    its VRAM with the GPU's."""
    gpus, _ = be.discover()
    idle = be.sample(0)
    print("idle: partition busy", idle.partition_gfx_busy_pct, "source", idle.partition_busy_source,
          "gfx", idle.gfx_activity_pct, "vram", idle.partition_vram_used_bytes, idle.vram_used_bytes)
    assert idle.ok and idle.partition_busy_source[0] == 1, idle.partition_busy_source
    if len(gpus[0].partitions) != 1:
        pytest.skip("the box is partitioned; the whole-GPU comparison needs SPX")
    assert abs(idle.partition_vram_used_bytes[0] - idle.vram_used_bytes) <= 64 << 20
    p = subprocess.Popen([sys.executable, "-c", _LOAD % 6.0], stdout=subprocess.PIPE, text=True)
    try:
        assert p.stdout.readline().strip() == "busy"
        time.sleep(1.0)
        pairs = []
        for _ in range(20):
            s = be.sample(0)
            assert s.ok and s.partition_busy_source[0] == 1
            pairs.append((s.partition_gfx_busy_pct[0], s.gfx_activity_pct))
            time.sleep(0.15)
    finally:
        p.wait(60)
    print("under load (partition busy, socket gfx activity):", pairs)
    part = sorted(x for x, _ in pairs)[len(pairs) // 2]
    sock = sorted(y for _, y in pairs)[len(pairs) // 2]
    assert part > 50 and sock > 50, pairs  # the GEMM keeps the GPU busy
    assert abs(part - sock) <= 15, (part, sock)


def test_lanes_run_amdsmi_concurrently_without_a_backend_lock(be, n):
    """The backend no longer holds one mutex across every amdsmi call: samples (on the
    GPU's lane), discoveries, event waits and the exporter's sampler run concurrently.
    Three seconds of that must leave every call answered and the session usable."""
    be.discover()
    errors, counts = [], {"sample": 0, "discover": 0}
    stop = threading.Event()

    def sampler():
        while not stop.is_set():
            s = be.sample(0)
            if s is None or not s.ok:
                errors.append("sample failed")
            counts["sample"] += 1

    def discoverer():
        while not stop.is_set():
            gpus, _ = be.discover()
            if not gpus or be.last_discovery()["stale"]:
                errors.append(("discover", be.last_discovery()))
            counts["discover"] += 1

    mon = n.HealthMonitor(be, 3)
    mon.set_gpu_count(1)
    mon.start()
    ex = n.Exporter()
    ex.set_inventory(be.discover()[0])
    ex.set_stall_ms(5000)
    ex.start(be, 20, mon)
    threads = [threading.Thread(target=f) for f in (sampler, sampler, discoverer)]
    for t in threads:
        t.start()
    time.sleep(3.0)
    stop.set()
    for t in threads:
        t.join(30)
    ex.stop()
    mon.stop()
    print("concurrent calls", counts, "exporter passes", ex.samples_total, "lanes", be.lanes())
    assert not errors, errors[:5]
    assert counts["sample"] > 50 and counts["discover"] > 5 and ex.samples_total > 50
    assert all(x[2] == "" for x in be.lanes())  # nothing left in flight
    assert be.sample(0).ok
