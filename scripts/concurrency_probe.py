"""Concurrency probe: Allocate (compiled HTTP/2 clients on the plugin socket) and
/metrics (keep-alive HTTP) at 1/2/4/8 concurrent clients against one fixture daemon,
closed loop, p50 per call.  Shows whether concurrent kubelet-side clients (the bench's N
ranks) slow each other down inside the plugin.  Prints one JSON line."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from k8s_gpu_device_plugin_amd import native  # noqa: E402
from k8s_gpu_device_plugin_amd.api import v1beta1  # noqa: E402
from k8s_gpu_device_plugin_amd.benchmark import suite  # noqa: E402


def pct(xs, q):
    xs = sorted(xs)
    return xs[min(len(xs) - 1, int(q * len(xs)))] if xs else None


def main():
    n = native.load()
    node = suite.Node("fixture", "8gpu_spx_mesh", http_threads=8)
    out = {}
    try:
        ids = node.ids()
        req = v1beta1.AllocateRequest(container_requests=[v1beta1.ContainerAllocateRequest(
            devices_ids=[ids[0]])]).SerializeToString()
        for conns in (1, 2, 4, 8):
            rows = []
            for _ in range(2):
                r = n.grpc_load(node.socket, v1beta1.METHOD_ALLOCATE, req, conns, 1.0)
                rows.append((round(pct(r["latencies_s"], 0.5) * 1e6, 2), round(r["ok"] / r["elapsed_s"])))
            out["allocate_conns%d" % conns] = rows
        for conns in (1, 2, 4, 8):
            rows = []
            for _ in range(2):
                r = n.http_load("127.0.0.1", node.port, "/metrics", conns, 1.0, 0.0)
                rows.append((round(pct(r["latencies_s"], 0.5) * 1e6, 2), round(r["ok"] / r["elapsed_s"])))
            out["scrape_conns%d" % conns] = rows
    finally:
        node.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
