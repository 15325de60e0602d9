"""Allocate tail probe: where do the slow (> 2x p50) kubelet Allocates come from?

Runs the bench's client pattern (batches of back-to-back Allocates through the compiled
HTTP/2 client, a /metrics scrape phase between batches) against fresh plugin daemons in
several variants and attributes each slow call:

  default        the bench's daemon config
  no_sampler     telemetry and health off (no amdsmi sampling thread in the daemon)
  pinned_client  the client thread pinned to one CPU (no client migration)
  no_gap         batches back to back, no scrape phase between them
  floor          the bare unix-socket exchange (no daemon, polling server thread)

With --gap-kind: a plain 50 ms sleep between batches instead of the scrape phase, and
the scrape phase with the HTTP workers' busy-poll off.

    python scripts/tail_probe.py [--batches 40] [--out gpurun_out/tail_probe.json]
"""
from __future__ import annotations

import argparse
import json
import os
import shutil
import signal
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402

ALLOCS = bench.ALLOCS


def pct(xs, q):
    xs = sorted(xs)
    return xs[min(len(xs) - 1, int(q * len(xs)))] if xs else None


def analyse(batches):
    lat = [x for _, l, _ in batches for x in l]
    p50 = pct(lat, 0.5)
    thr = 2 * p50
    slow_t, first, migrated, pos = [], 0, 0, []
    for starts, l, cpus in batches:
        for i, x in enumerate(l):
            if x <= thr:
                continue
            slow_t.append(starts[i])
            pos.append(i)
            if i == 0:
                first += 1
            elif cpus[i] != cpus[i - 1]:
                migrated += 1
    slow_t.sort()
    clustered = sum(1 for a, b in zip(slow_t, slow_t[1:]) if b - a < 100_000)
    return {"calls": len(lat), "p50_us": round(p50 * 1e6, 2), "p99_us": round(pct(lat, 0.99) * 1e6, 2),
            "p999_us": round(pct(lat, 0.999) * 1e6, 2), "max_us": round(max(lat) * 1e6, 2),
            "slow": len(slow_t), "slow_fraction": round(len(slow_t) / len(lat), 4), "first_of_batch": first,
            "cpu_migrated": migrated, "within_100us_of_another_slow": clustered,
            "slow_positions_head": sorted(pos)[:40],
            "client_cpus": sorted({c for _, _, cs in batches for c in cs})}


def run_variant(name, batches, overrides=None, pin=False, gap=True, idle_gap_s=0.0):
    from k8s_gpu_device_plugin_amd import native
    from k8s_gpu_device_plugin_amd.api import v1beta1
    from k8s_gpu_device_plugin_amd.plugin.kubelet_stub import DevicePluginClient

    n = native.load()
    native.load_bench()  # the harness extension: load generators, H2Client.bench_unary
    workdir = tempfile.mkdtemp(prefix="tailprobe-", dir="/tmp")
    proc, kubelet, port, reg, backend = bench.start_daemon(1, "native", workdir, overrides=overrides)
    try:
        sock = os.path.join(workdir, "device-plugins", reg.endpoint)
        c = DevicePluginClient(sock)
        law = c.list_and_watch()
        ids = [d.ID for d in next(iter(law)).devices]
        law.cancel()
        c.close()
        req = v1beta1.AllocateRequest(container_requests=[
            v1beta1.ContainerAllocateRequest(devices_ids=ids[:1])]).SerializeToString()
        old_aff = os.sched_getaffinity(0)
        if pin:
            os.sched_setaffinity(0, {sorted(old_aff)[len(old_aff) // 2]})
        h2 = n.H2Client(sock)
        try:
            h2.bench_unary(v1beta1.METHOD_ALLOCATE, req, 2000)  # warm-up
            recs = []
            for _ in range(batches):
                recs.append(h2.bench_unary_ts(v1beta1.METHOD_ALLOCATE, req, ALLOCS)[:4])
                if idle_gap_s:
                    time.sleep(idle_gap_s)
                elif gap:
                    native.load_bench().http_load("127.0.0.1", port, "/metrics", bench.SCRAPE_CONNS, bench.SCRAPE_S, 0.0)
        finally:
            h2.close()
            if pin:
                os.sched_setaffinity(0, old_aff)
        out = analyse(recs)
        out.update({"variant": name, "backend": backend, "overrides": overrides or {}, "pinned": pin, "gap": gap})
        return out
    finally:
        try:
            os.killpg(proc.pid, signal.SIGTERM)
        except ProcessLookupError:
            pass
        try:
            proc.wait(15)
        except subprocess.TimeoutExpired:
            os.killpg(proc.pid, signal.SIGKILL)
        kubelet.stop()
        shutil.rmtree(workdir, ignore_errors=True)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", type=int, default=40)
    ap.add_argument("--out", default="")
    ap.add_argument("--gap-kind", action="store_true", help="A/B idle gaps against scrape-phase gaps instead")
    a = ap.parse_args()
    from k8s_gpu_device_plugin_amd import native
    n = native.load()
    res = {"host_cpus": os.cpu_count(), "affinity_cpus": len(os.sched_getaffinity(0)), "variants": []}
    floor = native.load_bench().uds_pingpong(a.batches * ALLOCS, 500, 140, 190, server_spin=True)
    res["floor"] = {"p50_us": round(pct(floor, 0.5) * 1e6, 2), "p99_us": round(pct(floor, 0.99) * 1e6, 2),
                    "p999_us": round(pct(floor, 0.999) * 1e6, 2), "max_us": round(max(floor) * 1e6, 2),
                    "slow_fraction": round(sum(1 for x in floor if x > 2 * pct(floor, 0.5)) / len(floor), 4)}
    print(json.dumps({"floor": res["floor"]}), flush=True)
    variants = (("default", {}),
                ("no_sampler", {"overrides": {"telemetry": {"enabled": False}, "health": {"enabled": False}}}),
                ("pinned_client", {"pin": True}),
                ("no_gap", {"gap": False}),
                ("default_again", {}))
    if a.gap_kind:  # what about the gap slows the next call: idleness or the scraping next door?
        variants = (("scrape_gap", {}),
                    ("idle_gap_50ms", {"idle_gap_s": 0.05}),
                    ("scrape_gap_http_no_busy_poll", {"overrides": {"http": {"busyPollUs": 0}}}),
                    ("scrape_gap_again", {}))
    for name, kw in variants:
        t0 = time.time()
        r = run_variant(name, a.batches, **kw)
        r["wall_s"] = round(time.time() - t0, 1)
        res["variants"].append(r)
        print(json.dumps({k: r[k] for k in ("variant", "p50_us", "p99_us", "p999_us", "slow_fraction",
                                            "first_of_batch", "cpu_migrated", "within_100us_of_another_slow")}),
              flush=True)
    if a.out:
        os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
