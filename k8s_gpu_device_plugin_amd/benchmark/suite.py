"""BASELINE.json measurement suite (all five configs + the 1/2/4/8 scaling curve).

    python -m k8s_gpu_device_plugin_amd.benchmark.suite [--configs 1,2,3,4,5,scaling] [--json out.json]

Method (BASELINE.md "Measurement protocol"):
  * Allocate / GetPreferredAllocation: a persistent client on the plugin's unix socket,
    >= 10k calls after warm-up, p50/p99 per call.  Reported for the compiled HTTP/2
    client (kubelet-like) and for a grpcio client.
  * /metrics: keep-alive load generator (native, open-loop at a fixed rate, so latency
    includes queueing - no coordinated omission) at max rate and at 1k RPS.
  * Placement quality (config 3): a seeded churn of 1/2/4-GPU pods on an 8-GPU xGMI
    node (one degraded variant), xGMI-aware policy vs first-fit.
Configs whose hardware is absent run on fixture node models and say so.
"""
from __future__ import annotations

import argparse
import itertools
import json
import os
import platform
import random
import shutil
import tempfile
import time

from .. import config as config_mod
from .. import native
from ..api import v1beta1
from ..models import fixtures
from ..plugin.kubelet_stub import DevicePluginClient, KubeletStub
from ..plugin.manager import PluginManager
from ..server.web import WebServer


def pct(xs, q):
    xs = sorted(xs)
    return xs[min(len(xs) - 1, int(q * len(xs)))] if xs else None


def us(x):
    return None if x is None else round(x * 1e6, 2)


class Node:
    """A plugin manager + native servers + kubelet stub in a temp dir."""

    def __init__(self, backend: str, fixture: str = "2gpu_spx", strategy: str = "none", http_threads: int = 4):
        self.dir = tempfile.mkdtemp(prefix="dp-suite-", dir="/tmp")
        self.cfg = config_mod.validate(config_mod.from_dict({
            "backend": backend, "fixture": fixture, "migStrategy": strategy, "pluginDir": self.dir,
            "webListenAddress": "127.0.0.1:0", "log": {"fileDir": "", "console": False},
            "http": {"accessLog": False, "threads": http_threads}, "grpc": {"server": "native", "threads": 4},
            "telemetry": {"intervalMs": 1000}}))
        self.kubelet = KubeletStub(self.dir).start()
        self.mgr = PluginManager(self.cfg)
        self.thread = self.mgr.start_background()
        self.web = WebServer(self.cfg, self.mgr)
        self.port = self.web.start()
        self.regs = self.kubelet.wait_for_registrations(1, timeout=30)
        self.socket = os.path.join(self.dir, self.regs[0].endpoint)

    def ids(self):
        return self.mgr.plugins[0].table.ids()

    def close(self):
        self.web.stop()
        self.mgr.stop()
        self.thread.join(10)
        self.kubelet.stop()
        shutil.rmtree(self.dir, ignore_errors=True)


def alloc_req(ids):
    return v1beta1.AllocateRequest(container_requests=[
        v1beta1.ContainerAllocateRequest(devices_ids=list(ids))]).SerializeToString()


def pref_req(avail, must, size):
    return v1beta1.PreferredAllocationRequest(container_requests=[v1beta1.ContainerPreferredAllocationRequest(
        available_deviceIDs=list(avail), must_include_deviceIDs=list(must), allocation_size=size)]).SerializeToString()


def rpc_latency(node, method, req, n_native=10000, n_grpcio=2000):
    nat = native.load()
    native.load_bench()  # H2Client.bench_unary
    c = nat.H2Client(node.socket)
    c.bench_unary(method, req, 500)  # warm-up
    lat = c.bench_unary(method, req, n_native)
    c.close()
    out = {"p50_us": us(pct(lat, 0.5)), "p99_us": us(pct(lat, 0.99)), "calls": n_native}
    if n_grpcio:
        g = DevicePluginClient(node.socket)
        call = g.channel.unary_unary(method)
        for _ in range(200):
            call(req)
        ts = []
        for _ in range(n_grpcio):
            t0 = time.perf_counter()
            call(req)
            ts.append(time.perf_counter() - t0)
        g.close()
        out.update({"grpcio_p50_us": us(pct(ts, 0.5)), "grpcio_p99_us": us(pct(ts, 0.99))})
    return out


def scrape(node, conns=4, seconds=2.0, rate=0.0, gzip=False, path="/metrics"):
    r = native.load_bench().http_load("127.0.0.1", node.port, path, conns, seconds, rate, gzip)
    lat = r["latencies_s"]
    return {"rps": round(r["ok"] / r["elapsed_s"], 1), "errors": r["errors"], "p50_us": us(pct(lat, 0.5)),
            "p99_us": us(pct(lat, 0.99)), "bytes": r["bytes"] // max(1, r["ok"]), "conns": conns,
            "target_rps": rate or "max", "seconds": seconds, "gzip": gzip}


def config1():
    node = Node("fixture", "2gpu_spx")
    try:
        ids = node.ids()
        return {"config": "Mock-device backend (2 fake GPUs), in-process kubelet stub, CPU",
                "backend": "fixture:2gpu_spx",
                "allocate": rpc_latency(node, v1beta1.METHOD_ALLOCATE, alloc_req(ids[:1])),
                "preferred_size1": rpc_latency(node, v1beta1.METHOD_GET_PREFERRED, pref_req(ids, [], 1), 5000, 0),
                "scrape_max": scrape(node, 4, 2.0)}
    finally:
        node.close()


def config2():
    if not native.load().amdsmi_available():
        return {"config": "1xMI355X full GPU (SPX/NPS1)", "skipped": "no amdsmi-visible GPU on this host"}
    node = Node("amdsmi", strategy="none")
    try:
        ids = node.ids()
        g = node.mgr.gpus[0]
        time.sleep(2.5)  # a few 1 s sampling ticks of real amdsmi telemetry
        text = node.mgr.exporter.render()
        sample = [ln for ln in text.splitlines() if ln.startswith("amdgpu_telemetry_sample_duration_seconds_")]
        sums = {ln.split()[0]: float(ln.split()[1]) for ln in sample if "_sum" in ln or "_count" in ln}
        cost = None
        if sums.get("amdgpu_telemetry_sample_duration_seconds_count"):
            cost = sums["amdgpu_telemetry_sample_duration_seconds_sum"] / \
                sums["amdgpu_telemetry_sample_duration_seconds_count"]
        return {"config": "1xMI355X full GPU, amd.com/gpu=1, amdsmi health-watch + /metrics", "backend": "amdsmi",
                "gpu": {"name": g.market_name, "gfx": g.gfx_target, "mode": g.compute_partition + "/" +
                        g.memory_partition, "bdf": g.bdf},
                "advertised": len(ids),
                "allocate": rpc_latency(node, v1beta1.METHOD_ALLOCATE, alloc_req(ids[:1])),
                "scrape_max": scrape(node, 4, 2.0),
                "scrape_1conn": scrape(node, 1, 1.0),
                "health_route_1conn": scrape(node, 1, 1.0, path="/health"),
                "telemetry_sample_cost_us": us(cost)}
    finally:
        node.close()


def _churn(policy, n_gpu=8, steps=400, seed=7, degraded=(), slow=()):
    """Pods of 1/2/4 GPUs arrive/leave; returns placement-quality stats for `policy`.
    ``degraded``: links down; ``slow``: links up but trained at half rate."""
    nat = native.load()
    topo = nat.Topology(n_gpu)
    for a in range(n_gpu):
        for b in range(a + 1, n_gpu):
            topo.set_link(a, b, nat.Link(type=nat.LINK_XGMI, hops=1, up=(a, b) not in degraded,
                                         bw_gbps=304.0 if (a, b) in slow else 608.0))
    devs = [nat.AllocDevice(gi, -1, gi // 4, "g%d" % gi) for gi in range(n_gpu)]
    rng = random.Random(seed)
    free = set(range(n_gpu))
    pods = []
    stats = {"placed": 0, "multi": 0, "numa_local": 0, "down_link": 0, "slow_link": 0, "rejected": 0, "quad_ok": 0,
             "quad_probe": 0}
    for _ in range(steps):
        if pods and (rng.random() < 0.45 or not free):
            free |= set(pods.pop(rng.randrange(len(pods))))
            continue
        size = rng.choice([1, 1, 2, 2, 4])
        if size > len(free):
            stats["rejected"] += 1
            continue
        avail = sorted(free)
        chosen = nat.aligned_alloc(topo, devs, avail, [], size) if policy == "xgmi" else avail[:size]
        stats["placed"] += 1
        if size > 1:
            stats["multi"] += 1
            stats["numa_local"] += len({c // 4 for c in chosen}) == 1
            stats["down_link"] += any(not topo.link(a, b).up for a in chosen for b in chosen if a < b)
            stats["slow_link"] += any((a, b) in slow for a in chosen for b in chosen if a < b)
        free -= set(chosen)
        pods.append(chosen)
        if len(free) >= 4:  # could a 4-GPU NUMA-local, all-links-up job still land right now?
            stats["quad_probe"] += 1
            stats["quad_ok"] += any(all(topo.link(a, b).up for a in q for b in q if a < b)
                                    for q in itertools.combinations(sorted(free), 4) if len({g // 4 for g in q}) == 1)
    m = max(1, stats["multi"])
    return {"numa_local_multi_gpu": round(stats["numa_local"] / m, 3),
            "multi_gpu_on_down_link": round(stats["down_link"] / m, 3),
            "multi_gpu_on_half_rate_link": round(stats["slow_link"] / m, 3),
            "quad_clique_available": round(stats["quad_ok"] / max(1, stats["quad_probe"]), 3),
            "placements": stats["placed"]}


def _churn_cpx(visibility, n_gpu=8, parts=8, steps=400, seed=11, poll_every=10):
    """CPX node (8 GPUs x 8 partitions): pods of 1..16 partitions arrive and leave.  For
    each multi-GPU pod placed, counts the GPU pairs it spans that another live
    multi-GPU pod already spans: both drive RCCL traffic over that one xGMI link.

    ``visibility`` is what link load the allocator is given:
      * ``"none"``: nothing (the round-2 policy);
      * ``"podresources"``: the kubelet PodResources map as of its last poll, one poll
        per ``poll_every`` steps (pods placed since are invisible, pods gone since still
        count);
      * ``"podresources+allocate"``: that map plus the multi-GPU containers the plugin
        allocated since the poll (what the plugin runs: ``RecentAllocations``);
      * ``"oracle"``: exactly the live pods.
    (``True`` / ``False`` are the oracle / none of the first version of this protocol.)"""
    if visibility is True:
        visibility = "oracle"
    elif visibility is False:
        visibility = "none"
    nat = native.load()
    devs = [nat.AllocDevice(g, p, g // 4, "g%dp%d" % (g, p)) for g in range(n_gpu) for p in range(parts)]
    rng = random.Random(seed)
    free = set(range(len(devs)))
    pods = []  # (device indices, set of GPUs, id)
    polled, since_poll, next_id = [], [], 0
    st = {"placed": 0, "multi": 0, "pairs": 0, "shared_pairs": 0, "pods_sharing": 0, "rejected": 0}

    def topology():
        if visibility == "oracle":
            seen = [gs for _, gs, _ in pods]
        elif visibility == "podresources":
            seen = list(polled)
        elif visibility == "podresources+allocate":
            seen = list(polled) + list(since_poll)
        else:
            seen = []
        load = {}
        for gs in seen:
            for a, b in itertools.combinations(sorted(gs), 2):
                load[(a, b)] = load.get((a, b), 0) + 1
        t = nat.Topology(n_gpu)
        for a in range(n_gpu):
            for b in range(a + 1, n_gpu):
                t.set_link(a, b, nat.Link(type=nat.LINK_XGMI, hops=1, bw_gbps=608.0, pods=load.get((a, b), 0)))
        return t

    for step in range(steps):
        if step % poll_every == 0:
            polled, since_poll = [gs for _, gs, _ in pods], []
        if pods and (rng.random() < 0.45 or not free):
            chosen, _, _ = pods.pop(rng.randrange(len(pods)))
            free |= set(chosen)
            continue
        size = rng.choice([1, 2, 4, 4, 8, 12, 16])
        if size > len(free):
            st["rejected"] += 1
            continue
        chosen = nat.aligned_alloc(topology(), devs, sorted(free), [], size)
        gs = {devs[i].gpu for i in chosen}
        st["placed"] += 1
        if len(gs) > 1:
            live = set()
            for _, other, _ in pods:
                if len(other) > 1:
                    live |= set(itertools.combinations(sorted(other), 2))
            mine = set(itertools.combinations(sorted(gs), 2))
            st["multi"] += 1
            st["pairs"] += len(mine)
            st["shared_pairs"] += len(mine & live)
            st["pods_sharing"] += bool(mine & live)
            since_poll.append(gs)
        free -= set(chosen)
        pods.append((chosen, gs, next_id))
        next_id += 1
    m = max(1, st["multi"])
    return {"placements": st["placed"], "multi_gpu_pods": st["multi"], "gpu_pairs_spanned": st["pairs"],
            "shared_link_pairs": st["shared_pairs"], "multi_gpu_pods_sharing_a_link": round(st["pods_sharing"] / m, 3),
            "rejected": st["rejected"]}


def config3():
    node = Node("fixture", "8gpu_spx_mesh")
    try:
        ids = node.ids()
        out = {"config": "8xMI355X, xGMI-topology GetPreferredAllocation for 2- and 4-GPU pod requests",
               "backend": "fixture:8gpu_spx_mesh (full xGMI mesh, 2 NUMA nodes)"}
        for size in (2, 4):
            out["preferred_size%d" % size] = rpc_latency(node, v1beta1.METHOD_GET_PREFERRED,
                                                         pref_req(ids, [], size), 5000, 0)
        out["placement_healthy_mesh"] = {"xgmi_policy": _churn("xgmi"), "first_fit": _churn("first")}
        deg = ((0, 5), (2, 3), (1, 2))
        out["placement_degraded_links"] = {"down": [list(d) for d in deg], "xgmi_policy": _churn("xgmi", degraded=deg),
                                           "first_fit": _churn("first", degraded=deg)}
        slow = ((0, 1), (4, 6))
        out["placement_half_rate_links"] = {"half_rate": [list(d) for d in slow],
                                            "xgmi_policy": _churn("xgmi", slow=slow),
                                            "first_fit": _churn("first", slow=slow)}
        runs = {vis: [_churn_cpx(vis, seed=s) for s in range(100, 130)]
                for vis in ("none", "podresources", "podresources+allocate", "oracle")}
        out["placement_cpx_link_sharing"] = {
            "protocol": "8x8 CPX partitions, 400 arrivals/departures, pods of 1-16 partitions, 30 seeds; "
                        "PodResources polled every 10 steps",
            **{vis: {k: sum(r[k] for r in rs) for k in ("multi_gpu_pods", "gpu_pairs_spanned", "shared_link_pairs",
                                                        "rejected")}
               for vis, rs in runs.items()}}
        return out
    finally:
        node.close()


def config4():
    # BASELINE.json names CPX+NPS4; MI355X exposes NPS1|NPS2 (profiles/r4/amdsmi_probe.json),
    # so the measured mode is CPX+NPS2 (64 devices either way: CPX is 8 partitions per GPU)
    node = Node("fixture", "8gpu_cpx_nps2", strategy="single")
    try:
        ids = node.ids()
        nat = native.load()
        law = []
        for _ in range(200):
            c = nat.H2Client(node.socket)
            t0 = time.perf_counter()
            body = c.first_stream_message(v1beta1.METHOD_LIST_AND_WATCH, b"")
            law.append(time.perf_counter() - t0)
            c.close()
        n_dev = len(v1beta1.ListAndWatchResponse.FromString(body).devices)
        return {"config": "8xMI355X CPX+NPS2 (BASELINE's CPX+NPS4: NPS4 is not exposed by MI355X) -> 64 "
                          "amd.com/gpu sub-devices via ListAndWatch",
                "backend": "fixture:8gpu_cpx_nps2", "advertised": n_dev, "list_and_watch_bytes": len(body),
                "list_and_watch_first_message": {"p50_us": us(pct(law, 0.5)), "p99_us": us(pct(law, 0.99))},
                "allocate": rpc_latency(node, v1beta1.METHOD_ALLOCATE, alloc_req(ids[9:10])),
                "preferred_size8_whole_gpu_pack": rpc_latency(node, v1beta1.METHOD_GET_PREFERRED,
                                                              pref_req(ids, [], 8), 2000, 0),
                "preferred_size16_two_gpus": rpc_latency(node, v1beta1.METHOD_GET_PREFERRED,
                                                         pref_req(ids, [], 16), 1000, 0)}
    finally:
        node.close()


def config5(seconds=10.0):
    node = Node("fixture", "8gpu_cpx_nps2", strategy="single")
    try:
        return {"config": "Sustained /metrics at 1k RPS, 8 GPUs x 8 partitions, per-partition telemetry",
                "backend": "fixture:8gpu_cpx_nps2",
                "sustained_1k": scrape(node, 4, seconds, 1000.0),
                "sustained_1k_gzip": scrape(node, 4, seconds, 1000.0, gzip=True),
                "max_rate_8conns": scrape(node, 8, 3.0),
                "max_rate_8conns_gzip": scrape(node, 8, 3.0, gzip=True)}
    finally:
        node.close()


def scaling():
    rows = []
    for n_gpu in (1, 2, 4, 8):
        node = Node("fixture", "%dgpu_spx" % n_gpu)
        try:
            ids = node.ids()
            a = rpc_latency(node, v1beta1.METHOD_ALLOCATE, alloc_req(ids[:1]), 10000, 0)
            s = scrape(node, 4, 2.0)
            rows.append({"gpus_advertised": n_gpu, "allocate_p50_us": a["p50_us"], "allocate_p99_us": a["p99_us"],
                         "scrape_rps": s["rps"], "scrape_p50_us": s["p50_us"], "metrics_bytes": s["bytes"]})
        finally:
            node.close()
    return {"config": "scaling curve (fixture nodes, strategy none)", "rows": rows}


def health_propagation(events=60):
    """Hardware event -> Unhealthy/Healthy visible to a kubelet-like ListAndWatch watcher.
    Event injection and the watcher are native (no GIL) so only the plugin is measured.
    Unhealthy takes the native fail-fast path (monitor thread -> table -> server push);
    Healthy goes through the manager, which owns recovery policy (canary, held GPUs)."""
    nat = native.load()
    node = Node("fixture", "8gpu_spx_mesh")
    try:
        native.load_bench().health_propagation(node.mgr.backend, node.socket, 3, 2)  # warm-up pair
        res = native.load_bench().health_propagation(node.mgr.backend, node.socket, 3, events)
        down = [t for d, t in res if d == 1]
        up = [t for d, t in res if d == 0]
        both = down + up
        return {"config": "health event -> ListAndWatch update seen by a compiled kubelet-like watcher "
                          "(fixture PRE/POST_RESET on GPU 3)",
                "events": events, "p50_us": us(pct(both, 0.5)), "p99_us": us(pct(both, 0.99)),
                "unhealthy_p50_us": us(pct(down, 0.5)), "unhealthy_p99_us": us(pct(down, 0.99)),
                "healthy_p50_us": us(pct(up, 0.5)), "healthy_p99_us": us(pct(up, 0.99))}
    finally:
        node.close()


def uds_floor():
    """Speed-of-light reference for one kubelet RPC: two threads exchange Allocate-sized
    messages over a unix socket with the server's exact syscalls (epoll_wait, recv, send)
    and no protocol work.  Allocate p50 minus this is the plugin's own cost."""
    lat = native.load_bench().uds_pingpong(20000, 1000, 140, 250)
    return {"config": "unix-socket round trip floor (no HTTP/2, HPACK, protobuf or table work)",
            "p50_us": us(pct(lat, 0.5)), "p99_us": us(pct(lat, 0.99)), "round_trips": len(lat)}


def startup(runs=5):
    """Plugin start-up as kubelet sees it: process spawn -> Registration.Register
    received -> first ListAndWatch answered (fresh process each run, so Python start,
    imports, hardware discovery and the native servers are all inside).  The reference
    publishes no start-up figure."""
    import subprocess
    import sys
    nat = native.load()
    backend = "amdsmi" if nat.amdsmi_available() else "fixture"
    root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    reg_t, law_t = [], []
    for _ in range(runs):
        d = tempfile.mkdtemp(prefix="dp-start-", dir="/tmp")
        kubelet = KubeletStub(d).start()
        env = dict(os.environ, PYTHONPATH=root + os.pathsep + os.environ.get("PYTHONPATH", ""))
        cmd = [sys.executable, "-m", "k8s_gpu_device_plugin_amd", "--configFile", "none", "--backend", backend,
               "--fixture", "8gpu_spx_mesh", "--plugin-dir", d, "--web-listen-address", "127.0.0.1:0",
               "--log-dir", "", "--log-level", "warn"]
        t0 = time.perf_counter()
        proc = subprocess.Popen(cmd, env=env, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL,
                                start_new_session=True)
        try:
            reg = kubelet.wait_for_registrations(1, timeout=60)[0]
            reg_t.append(time.perf_counter() - t0)
            c = nat.H2Client(os.path.join(d, reg.endpoint))
            c.first_stream_message(v1beta1.METHOD_LIST_AND_WATCH, b"")
            law_t.append(time.perf_counter() - t0)
            c.close()
        finally:
            proc.terminate()
            try:
                proc.wait(15)
            except subprocess.TimeoutExpired:
                proc.kill()
            kubelet.stop()
            shutil.rmtree(d, ignore_errors=True)
    # kubelet restart (kubelet.sock re-created) -> inotify -> reload -> Register again
    node = Node(backend, "8gpu_spx_mesh")
    rereg = []
    try:
        for i in range(runs):
            node.kubelet.stop()  # kubelet gone (its socket removed) ...
            time.sleep(0.05)
            t0 = time.perf_counter()  # ... and back: the clock starts when kubelet.sock reappears
            node.kubelet.start()
            node.kubelet.wait_for_registrations(i + 2, timeout=30)
            rereg.append(time.perf_counter() - t0)
            time.sleep(0.05)  # let the plugin's Register call return before the next restart
    finally:
        node.close()
    ms = lambda x: None if x is None else round(x * 1e3, 1)  # noqa: E731
    return {"config": "process spawn -> Register -> first ListAndWatch; kubelet restart -> Register "
                      "(%s backend)" % backend, "runs": runs,
            "register_p50_ms": ms(pct(reg_t, 0.5)), "register_max_ms": ms(max(reg_t)),
            "first_list_and_watch_p50_ms": ms(pct(law_t, 0.5)),
            "kubelet_restart_reregister_p50_ms": ms(pct(rereg, 0.5))}


RUNNERS = {"floor": uds_floor, "startup": startup, "health": health_propagation, "1": config1, "2": config2, "3": config3, "4": config4, "5": config5, "scaling": scaling}


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--configs", default="floor,startup,1,2,3,4,5,scaling,health")
    ap.add_argument("--json", default="")
    a = ap.parse_args(argv)
    from ..utils.log import init_logger
    init_logger("warn", None, console=False)
    results = {"host": platform.node(), "python": platform.python_version(), "cpus": os.cpu_count(),
               "time": time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime()), "results": {}}
    try:
        rocm = open("/opt/rocm/.info/version").read().strip()
    except OSError:
        rocm = "unknown"
    results["rocm"] = rocm
    for key in a.configs.split(","):
        t0 = time.time()
        results["results"][key] = RUNNERS[key]()
        results["results"][key]["wall_s"] = round(time.time() - t0, 1)
        print(json.dumps({key: results["results"][key]}), flush=True)
    if a.json:
        with open(a.json, "w") as f:
            json.dump(results, f, indent=1)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
