"""Allocate latency as a function of how long the plugin sat idle before the call.

Kubelet calls the plugin a few times per pod admission, seconds or minutes apart, so
the call it makes almost never finds a warm server.  For idle gaps of 1 ms to 1 s this
measures, on one daemon (bench config, amdsmi backend when present):

  * ``allocate``: one Allocate after the gap (compiled HTTP/2 client, kubelet-like);
  * ``admission``: GetPreferredAllocation after the gap, ~200 us of client work, then
    Allocate (the Allocate is timed: kubelet's admission sequence);
  * ``floor``: the bare unix-socket exchange of the same sizes after the same gap
    between two threads of this process (no HTTP/2, protobuf or table work).

    python scripts/idle_probe.py [--gaps 0.001,0.01,0.1,1] [--calls 40] [--out FILE]

Prints one JSON line per gap, then the whole result.
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


def pct(xs, q):
    xs = sorted(xs)
    return round(xs[min(len(xs) - 1, int(q * len(xs)))] * 1e6, 2) if xs else None


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gaps", default="0.001,0.01,0.1,1")
    ap.add_argument("--calls", type=int, default=40, help="calls per gap (the 1 s gap takes this many seconds)")
    ap.add_argument("--backend", default="auto")
    ap.add_argument("--admission-poll-us", type=int, default=None, help="override grpc.admissionPollUs")
    ap.add_argument("--busy-poll-us", type=int, default=None, help="override grpc.busyPollUs / http.busyPollUs")
    ap.add_argument("--out", default="")
    a = ap.parse_args()

    from k8s_gpu_device_plugin_amd import native
    from k8s_gpu_device_plugin_amd.api import v1beta1
    from k8s_gpu_device_plugin_amd.plugin.kubelet_stub import DevicePluginClient

    n = native.load()
    workdir = tempfile.mkdtemp(prefix="idleprobe-", dir="/tmp")
    proc, kubelet, port, reg, backend = bench.start_daemon(1, "native", workdir, busy_poll_us=a.busy_poll_us,
                                                         admission_poll_us=a.admission_poll_us, backend=a.backend)
    res = {"backend": backend, "calls_per_gap": a.calls, "rows": []}
    try:
        sock = os.path.join(workdir, "device-plugins", reg.endpoint)
        c = DevicePluginClient(sock)
        law = c.list_and_watch()
        ids = [d.ID for d in next(iter(law)).devices]
        law.cancel()
        alloc = v1beta1.AllocateRequest(container_requests=[
            v1beta1.ContainerAllocateRequest(devices_ids=ids[:1])]).SerializeToString()
        pref = v1beta1.PreferredAllocationRequest(container_requests=[
            v1beta1.ContainerPreferredAllocationRequest(available_deviceIDs=ids, must_include_deviceIDs=ids[:1],
                                                        allocation_size=1)]).SerializeToString()
        resp_len = len(c.allocate_raw(alloc))
        c.close()
        sizes = (9 + 80 + 9 + 5 + len(alloc), 9 + 20 + 9 + 5 + resp_len + 9 + 16)
        h2 = n.H2Client(sock)
        h2.bench_unary(v1beta1.METHOD_ALLOCATE, alloc, 2000)  # warm the connection and the code
        perf = time.perf_counter
        for gap in [float(x) for x in a.gaps.split(",")]:
            al, adm = [], []
            for _ in range(a.calls):
                time.sleep(gap)
                al.extend(h2.bench_unary(v1beta1.METHOD_ALLOCATE, alloc, 1))
            for _ in range(a.calls):
                time.sleep(gap)
                h2.bench_unary(v1beta1.METHOD_GET_PREFERRED, pref, 1)
                t_go = perf() + 200e-6
                while perf() < t_go:
                    pass
                adm.extend(h2.bench_unary(v1beta1.METHOD_ALLOCATE, alloc, 1))
            floor = n.uds_pingpong(a.calls, 2, *sizes, gap_us=int(gap * 1e6))
            row = {"gap_s": gap, "allocate_p50_us": pct(al, 0.5), "allocate_p90_us": pct(al, 0.9),
                   "admission_allocate_p50_us": pct(adm, 0.5), "admission_allocate_p90_us": pct(adm, 0.9),
                   "floor_p50_us": pct(floor, 0.5), "floor_p90_us": pct(floor, 0.9)}
            res["rows"].append(row)
            print(json.dumps(row), flush=True)
        h2.close()
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
    print(json.dumps(res), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
