"""Chaos: a seeded random mix of every fault the manager handles, while a kubelet-like
client keeps allocating, then a heal and a check that the node converges.

Faults: GPU reset (PRE_RESET without its POST_RESET for a while), a GPU falling off the
bus and coming back (the periodic re-discovery re-advertises around it), xGMI links going
down and re-training at another rate, ``GET /restart`` reloads, kubelet restarts, and
native gRPC server faults (supervised restart).  Each is covered alone elsewhere; here they
overlap in arbitrary order.  After the heal every GPU must be advertised Healthy through
the last registration's ListAndWatch, the allocator's topology must be whole again, the
manager must still be running (not fatal), and a fresh reset must still reach kubelet -
i.e. no latch, index or generation got stuck on the way.
"""
import os
import random
import threading
import time

import grpc
import pytest

from k8s_gpu_device_plugin_amd import native
from k8s_gpu_device_plugin_amd.models import fixtures
from k8s_gpu_device_plugin_amd.plugin.kubelet_stub import DevicePluginClient, KubeletStub
from k8s_gpu_device_plugin_amd.plugin.manager import PluginManager

NGPU = 4
FULL_GBPS = 608.0


def _wait(pred, timeout=10.0, step=0.02):
    deadline = time.monotonic() + timeout
    while time.monotonic() < deadline:
        if pred():
            return True
        time.sleep(step)
    return False


def _advertised(plugin_dir, k, timeout=5.0):
    """(id, health) pairs of the first ListAndWatch message on the newest registration's
    endpoint, over a fresh connection (what a restarted kubelet would see)."""
    try:  # a connect that times out under load is retried by the caller's wait, as kubelet would
        c = DevicePluginClient(os.path.join(plugin_dir, k.requests[-1].endpoint))
    except grpc.FutureTimeoutError:
        return None
    try:
        stream = c.list_and_watch(timeout=timeout)
        first = next(iter(stream))
        stream.cancel()
        return sorted((d.ID, d.health) for d in first.devices)
    finally:
        c.close()


class _Allocator(threading.Thread):
    """A kubelet-like client (the compiled HTTP/2 one: it redials at once, without grpc's
    reconnect backoff) that keeps calling Allocate through every reload."""

    def __init__(self, sock, m):
        super().__init__(daemon=True)
        self.sock, self.m = sock, m
        self.stop_ev = threading.Event()
        self.ok = 0
        self.failed = 0
        self.errors = {}

    def run(self):
        from k8s_gpu_device_plugin_amd.api import v1beta1
        n = native.load()
        native.load_bench()  # H2Client.bench_unary
        c = None
        i = 0
        while not self.stop_ev.is_set():
            try:
                ids = self.m.plugins[0].table.ids() if self.m.plugins else []
                if ids:
                    if c is None:
                        c = n.H2Client(self.sock)
                    req = v1beta1.AllocateRequest(container_requests=[
                        v1beta1.ContainerAllocateRequest(devices_ids=[ids[i % len(ids)]])]).SerializeToString()
                    try:
                        c.bench_unary(v1beta1.METHOD_ALLOCATE, req, 1)
                        self.ok += 1
                    except RuntimeError as e:
                        if "grpc-status" not in str(e):
                            raise
                        self.failed += 1  # an answer (e.g. an Unhealthy device): the connection is fine
                        key = str(e)[:60]
                        self.errors[key] = self.errors.get(key, 0) + 1
                i += 1
            except Exception as e:  # noqa: BLE001 - sockets come and go during reloads
                self.failed += 1
                key = type(e).__name__ + ": " + str(e)[:60]
                self.errors[key] = self.errors.get(key, 0) + 1
                if c is not None:
                    c.close()
                c = None
                time.sleep(0.005)
            time.sleep(0.002)
        if c is not None:
            c.close()


# CHAOS_SEEDS=N runs seeds 1..N (a longer hunt); the suite runs three
@pytest.mark.parametrize("seed", range(1, 1 + int(os.environ.get("CHAOS_SEEDS", "3"))))
# serialised: the fixture driver takes one library-wide lock for every device call (as a
# driver that serialises devices would), so a wedged call also blocks every other GPU's
# calls and every discovery until it returns
@pytest.mark.parametrize("fixture,strategy,server,devices,serialised", [("4gpu_spx", "none", "native", "", False),
                                                                        ("4gpu_cpx", "single", "native", "", False),
                                                                        ("4gpu_spx", "none", "python", "", False),
                                                                        ("4gpu_spx", "none", "native", "0-2", False),
                                                                        ("4gpu_spx", "none", "native", "", True),
                                                                        ("4gpu_cpx", "single", "native", "0-2", True)])
def test_random_fault_mix_converges(make_cfg, plugin_dir, tmp_path, seed, fixture, strategy, server, devices,
                                    serialised):
    from k8s_gpu_device_plugin_amd.plugin.kubelet_stub import PodResourcesStub
    n = native.load()
    rng = random.Random(seed)
    be = fixtures.build_backend(fixture)
    be.set_serialised(serialised)
    gpus, _ = be.discover()
    assert len(gpus) == NGPU
    shown = range(NGPU - 1) if devices else range(NGPU)  # the GPUs `devices` advertises (all but the last)
    ids = sorted(p.id for g in gpus if g.index in shown for p in g.partitions)  # one device per partition
    id_of_slot = {g.index: g.partitions[0].id for g in gpus}
    podsock = str(tmp_path / "pod-resources" / "kubelet.sock")
    pods = PodResourcesStub(podsock).start()
    cfg = make_cfg(fixture=fixture, migStrategy=strategy, grpc={"server": server}, telemetry={"intervalMs": 30},
                   rediscoverIntervalS=0.2, retrySeconds=0.2, devices=devices,
                   podResources={"enabled": True, "socket": podsock, "intervalS": 0.05},
                   health={"lostAfterFailures": 2, "sampleStallS": 0.3, "badPageThreshold": 10, "pcieMinWidth": 16})
    orig, _ = be.discover()  # untouched descriptions, to undo partition-mode changes
    resetting, present, server_faults = set(), set(range(NGPU)), 0
    links = {}  # (a, b) -> (up, gbps) for the links chaos has touched
    ecc = [0] * NGPU
    stalled, pages_high, remoded, pcie_low = set(), set(), set(), set()
    with KubeletStub(plugin_dir) as k:
        m = PluginManager(cfg, backend=be)
        t = m.start_background()
        client = None
        try:
            k.wait_for_registrations(1)
            client = _Allocator(os.path.join(plugin_dir, "amd-gpu.sock"), m)
            client.start()
            log = []
            for _ in range(60):
                op = rng.choice(["reset", "post_reset", "remove", "restore", "link_down", "link_up", "link_bw",
                                 "api_restart", "kubelet_restart", "server_fault", "ecc", "stall", "unstall",
                                 "pages_high", "pages_low", "discovery_fails", "discovery_ok", "mode_change",
                                 "mode_restore", "pods", "pcie_low", "pcie_ok", "idle"])
                g = rng.randrange(NGPU)
                a, b = sorted(rng.sample(range(NGPU), 2))
                if op == "reset" and g in present:
                    be.inject_event(n.HwEvent(n.EVT_PRE_RESET, g, message="chaos reset"))
                    resetting.add(g)
                elif op == "post_reset" and g in present and g in resetting:
                    be.inject_event(n.HwEvent(n.EVT_POST_RESET, g))
                    resetting.discard(g)
                elif op == "remove" and len(present) > 1 and g in present:
                    be.set_gpu_present(g, False)
                    present.discard(g)
                elif op == "restore" and g not in present:
                    be.set_gpu_present(g, True)
                    present.add(g)
                elif op == "link_down":
                    be.set_link_up(a, b, False)
                    links[(a, b)] = (False, links.get((a, b), (True, FULL_GBPS))[1])
                elif op == "link_up":
                    be.set_link_up(a, b, True)
                    links[(a, b)] = (True, links.get((a, b), (True, FULL_GBPS))[1])
                elif op == "link_bw":
                    bw = rng.choice([FULL_GBPS / 2, FULL_GBPS / 4, FULL_GBPS])
                    be.set_link_bandwidth(a, b, bw)
                    links[(a, b)] = (links.get((a, b), (True, FULL_GBPS))[0], bw)
                elif op == "api_restart":
                    m.restart()
                elif op == "kubelet_restart":
                    k.restart()
                elif op == "server_fault" and server_faults < 2 and m.plugins:
                    srv = m.plugins[0]._native_server
                    if srv is not None:
                        srv.inject_fault("worker")
                        server_faults += 1
                elif op == "ecc":  # an uncorrectable error: latched until the GPU's next reset ends
                    ecc[g] += 1
                    be.set_ecc_uncorrectable(g, ecc[g])
                    resetting.add(g)  # the heal's POST_RESET clears the latch
                elif op == "stall" and not stalled:  # one wedged amdsmi call at a time
                    be.set_sample_stall(g, True)
                    stalled.add(g)
                elif op == "unstall" and stalled:
                    be.set_sample_stall(stalled.pop(), False)
                elif op == "pages_high":
                    be.set_retired_pages(g, 12, 0)
                    pages_high.add(g)
                elif op == "pages_low" and g in pages_high:
                    be.set_retired_pages(g, 0, 0)
                    pages_high.discard(g)
                elif op == "discovery_fails":
                    be.set_fail_discovery(True)
                    log.append(("discovery_fails", g, a, b))
                    time.sleep(0.05)
                    be.set_fail_discovery(False)  # a failed reload waits for its retry
                    continue
                elif op == "mode_change" and len(present) == NGPU and g not in remoded:
                    # an operator re-partitions GPU g (by fixture slot; only
                    # while every GPU is present: slot and index agree)
                    mode = "SPX" if orig[g].compute_partition != "SPX" else "CPX"
                    fixtures.set_gpu_mode(be, g, mode, first_render=300 + 8 * g)
                    remoded.add(g)
                elif op == "pods":  # the kubelet's allocation map changes (PodResources)
                    cur = list(m.plugins[0].table.ids()) if m.plugins else []
                    if len(cur) >= 2:
                        pods.set_pods([("ns", "p%d" % j, [("c", "amd.com/gpu", rng.sample(cur, 2))])
                                       for j in range(rng.randrange(1, 4))])
                elif op == "pcie_low":  # the host link trains at x8: below the x16 floor
                    be.set_pcie_link(g, 8, 32.0)
                    pcie_low.add(g)
                elif op == "pcie_ok" and g in pcie_low:
                    be.set_pcie_link(g, 16, 32.0)
                    pcie_low.discard(g)
                elif op == "mode_restore" and g in remoded and len(present) == NGPU:
                    be.replace_gpu(g, orig[g])
                    remoded.discard(g)
                else:
                    op = "idle"
                log.append((op, g, a, b))
                time.sleep(rng.choice([0.0, 0.01, 0.03, 0.08]))
                assert m.running and m.fatal_error is None, (m.fatal_error, log)

            # ---- heal: everything back, every reset finished ----
            for g in stalled:
                be.set_sample_stall(g, False)
            for g in pages_high:
                be.set_retired_pages(g, 0, 0)
            for g in pcie_low:
                be.set_pcie_link(g, 16, 32.0)
            for g in range(NGPU):
                if g not in present:
                    be.set_gpu_present(g, True)
            for g in remoded:
                be.replace_gpu(g, orig[g])
            for (a, b) in links:
                be.set_link_up(a, b, True)
                be.set_link_bandwidth(a, b, FULL_GBPS)
            time.sleep(0.1)
            for g in sorted(resetting):
                be.inject_event(n.HwEvent(n.EVT_POST_RESET, g))
            # one pod spanning GPUs 1 and 2: only that pair's link carries a pod
            pods.set_pods([("ns", "final", [("c", "amd.com/gpu", [id_of_slot[1], id_of_slot[2]])])])

            def table():  # replaced by every reload; none while a failed start waits for its retry
                ps = m.plugins
                return ps[0].table if ps else None

            def whole():
                t_ = table()
                if t_ is None or sorted(t_.ids()) != ids or not all(t_.healthy(i) for i in ids):
                    return False
                topo = t_.topology()
                if topo.n != NGPU:
                    return False
                return all(topo.link(x, y).up and topo.link(x, y).bw_gbps == FULL_GBPS and
                           topo.link(x, y).pods == (1 if {x, y} == {1, 2} else 0)
                           for x in range(NGPU) for y in range(NGPU) if x != y)

            def links_now():
                t_ = table()
                topo = t_.topology() if t_ is not None else None
                return topo and [(x, y, topo.link(x, y).up, topo.link(x, y).bw_gbps, topo.link(x, y).pods)
                                 for x in range(topo.n) for y in range(x + 1, topo.n)]

            if not _wait(whole, timeout=15):
                detail = (table() and [(i, table().healthy(i)) for i in table().ids()], links_now(), log,
                          [ln for ln in m.exporter.render().splitlines()
                           if ln.startswith("amdgpu_xgmi_link_bandwidth")],
                          {"monitor_unhealthy": m.monitor.unhealthy_keys(), "held": sorted(m._held_unhealthy),
                           "canary_failed": sorted(m._canary_failed), "resetting": sorted(resetting),
                           "health_log": list(getattr(m, "_health_log", []))[-20:]})
                if os.environ.get("CHAOS_DUMP"):  # the full picture; pytest truncates the message
                    with open(os.path.join(os.environ["CHAOS_DUMP"], "chaos_%s_%d.txt" % (fixture, seed)), "w") as f:
                        f.write(repr(detail))
                raise AssertionError(detail)
            assert _wait(lambda: m.monitor.unhealthy_keys() == [], timeout=5), m.monitor.unhealthy_keys()
            assert m.running and m.fatal_error is None
            assert _wait(lambda: _advertised(plugin_dir, k) == [(i, "Healthy") for i in ids], timeout=10), \
                _advertised(plugin_dir, k)
            # and GET /ready says so: every resource is registered again
            assert _wait(lambda: m._readiness == (True, ""), timeout=5), m._readiness

            # still wired end to end: a new reset reaches kubelet, and so does its end
            g = rng.choice(list(shown))
            be.inject_event(n.HwEvent(n.EVT_PRE_RESET, g, message="after chaos"))
            assert _wait(lambda: not table().healthy(id_of_slot[g]))
            be.inject_event(n.HwEvent(n.EVT_POST_RESET, g))
            assert _wait(lambda: table().healthy(id_of_slot[g]))

            client.stop_ev.set()
            client.join(10)
            assert client.ok > 0, client.errors
            print("seed", seed, "ops", sorted({o for o, *_ in log}), "allocates ok/failed", client.ok, client.failed,
                  "registrations", len(k.requests), "counters", dict(m.counters))
            c = DevicePluginClient(os.path.join(plugin_dir, "amd-gpu.sock"))
            try:
                for i in ids:
                    assert c.allocate([i]).container_responses[0].devices
            finally:
                c.close()
        finally:
            if client is not None:
                client.stop_ev.set()
                client.join(10)
            m.stop()
            t.join(10)
            pods.stop()
            assert not t.is_alive()
