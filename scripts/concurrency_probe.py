"""Daemon concurrency probe: how Allocate latency and /metrics throughput behave as the
number of concurrent kubelet-like clients grows (the per-rank load of bench.py at
N = 1, 2, 4, 8, without the rank processes, RCCL or gloo around it).

One plugin daemon (the bench's config, with as many gRPC and HTTP workers as the largest
client count needs); for k concurrent clients:
  * k threads, each with its own compiled HTTP/2 connection, run batches of back-to-back
    Allocates at the same time: per-call p50/p99 over all of them, aggregate calls/s;
  * 2k /metrics connections scrape for 1 s: aggregate RPS and per-scrape p50/p99.

    python scripts/concurrency_probe.py [--clients 1,2,4,8,16] [--out gpurun_out/concurrency.json]
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
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def pct(xs, q):
    xs = sorted(xs)
    return xs[min(len(xs) - 1, int(q * len(xs)))] if xs else None


def allocate_round(n, sock, req, method, k, batches, per_batch):
    clients = [n.H2Client(sock) for _ in range(k)]
    for c in clients:
        c.bench_unary(method, req, 500)  # warm-up
    go = threading.Barrier(k)
    lat = [[] for _ in range(k)]
    errs = []

    def run(i):
        try:
            go.wait()
            for _ in range(batches):
                lat[i].extend(clients[i].bench_unary(method, req, per_batch))
        except Exception as e:  # noqa: BLE001 - reported, not swallowed
            errs.append(repr(e))

    ts = [threading.Thread(target=run, args=(i,)) for i in range(k)]
    t0 = time.perf_counter()
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    wall = time.perf_counter() - t0
    for c in clients:
        c.close()
    if errs:
        raise RuntimeError(errs[0])
    allx = [x for l in lat for x in l]
    return {"calls": len(allx), "p50_us": round(pct(allx, 0.5) * 1e6, 2), "p99_us": round(pct(allx, 0.99) * 1e6, 2),
            "per_client_p50_us": [round(pct(l, 0.5) * 1e6, 2) for l in lat],
            "calls_per_s": round(len(allx) / wall)}


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--clients", default="1,2,4,8,16")
    ap.add_argument("--batches", type=int, default=20)
    ap.add_argument("--per-batch", type=int, default=256)
    ap.add_argument("--scrape-s", type=float, default=1.0)
    ap.add_argument("--backend", default="auto")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    ks = [int(x) for x in a.clients.split(",")]
    kmax = max(ks)

    from k8s_gpu_device_plugin_amd import native
    from k8s_gpu_device_plugin_amd.api import v1beta1
    from k8s_gpu_device_plugin_amd.plugin.kubelet_stub import DevicePluginClient

    n = native.load()
    native.load_bench()  # the harness extension: load generators, H2Client.bench_unary
    workdir = tempfile.mkdtemp(prefix="concprobe-", dir="/tmp")
    over = {"grpc": {"threads": max(4, kmax)}, "http": {"threads": max(4, 2 * kmax)}}
    proc, kubelet, port, reg, backend = bench.start_daemon(1, "native", workdir, overrides=over, backend=a.backend)
    res = {"backend": backend, "host_cpus": os.cpu_count(), "affinity_cpus": len(os.sched_getaffinity(0)),
           "daemon_overrides": over, "rounds": []}
    try:
        sock = os.path.join(workdir, "device-plugins", reg.endpoint)
        c = DevicePluginClient(sock)
        law = c.list_and_watch()
        ids = [d.ID for d in next(iter(law)).devices]
        law.cancel()
        c.close()
        req = v1beta1.AllocateRequest(container_requests=[
            v1beta1.ContainerAllocateRequest(devices_ids=ids[:1])]).SerializeToString()
        for k in ks:
            al = allocate_round(n, sock, req, v1beta1.METHOD_ALLOCATE, k, a.batches, a.per_batch)
            sc = native.load_bench().http_load("127.0.0.1", port, "/metrics", 2 * k, a.scrape_s, 0.0)
            if sc["errors"]:
                raise RuntimeError("%d scrape errors at k=%d" % (sc["errors"], k))
            sl = sc["latencies_s"]
            row = {"clients": k, "allocate": al,
                   "scrape": {"conns": 2 * k, "rps": round(sc["ok"] / sc["elapsed_s"]),
                              "p50_us": round(pct(sl, 0.5) * 1e6, 2), "p99_us": round(pct(sl, 0.99) * 1e6, 2)}}
            res["rounds"].append(row)
            print(json.dumps({"clients": k, "allocate_p50_us": al["p50_us"], "allocate_p99_us": al["p99_us"],
                              "allocate_calls_per_s": al["calls_per_s"], "scrape_rps": row["scrape"]["rps"],
                              "scrape_p50_us": row["scrape"]["p50_us"]}), flush=True)
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
    if a.out:
        os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
