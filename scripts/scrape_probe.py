"""Scrape-path probe on one box: /metrics latency and throughput of the native HTTP
server at 1/2/4 keep-alive connections, next to the loopback-TCP floor measured with
the same number of concurrent ping-pong pairs (is a slowdown at 2 connections the
server's or the box's?).  Fixture backend, 1 GPU; prints one JSON line."""
import json
import sys
import tempfile
import threading
import time

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from k8s_gpu_device_plugin_amd import config as config_mod, native  # noqa: E402
from k8s_gpu_device_plugin_amd.plugin.manager import PluginManager  # noqa: E402
from k8s_gpu_device_plugin_amd.server.web import WebServer  # noqa: E402


def pct(xs, q):
    xs = sorted(xs)
    return xs[min(len(xs) - 1, int(q * len(xs)))] if xs else None


def floor_parallel(n, pairs, body):
    res = [None] * pairs

    def run(i):
        res[i] = native.load_bench().uds_pingpong(3000, 300, 90, body, server_spin=True, tcp=True)
    ts = [threading.Thread(target=run, args=(i,)) for i in range(pairs)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    return round(pct([x for r in res for x in r], 0.5) * 1e6, 2)


def main():
    n = native.load()
    native.load_bench()  # the harness extension: load generators, H2Client.bench_unary
    out = {}
    for threads in (2, 4):
        d = tempfile.mkdtemp()
        cfg = config_mod.validate(config_mod.from_dict({
            "backend": "fixture", "fixture": "1gpu_spx", "pluginDir": d, "log": {"fileDir": ""},
            "telemetry": {"intervalMs": 1000}, "webListenAddress": "127.0.0.1:0",
            "http": {"server": "native", "accessLog": False, "threads": threads}}))
        m = PluginManager(cfg)
        m.load_plugins()
        m._start_telemetry()
        w = WebServer(cfg, m)
        port = w.start()
        time.sleep(0.3)
        try:
            if threads == 4:  # user-space cost of one exposition, 1/2/4 threads at once, no sockets
                native.load_bench().http_load("127.0.0.1", port, "/metrics", 1, 0.2, 0.0)  # populate the echo_http_* families
                for nt in (1, 2, 4):
                    out["render_ns_threads%d" % nt] = [round(x) for x in native.load_bench().render_bench(m.exporter, w._impl, nt, 20000)]
            for conns in (1, 2, 4):
                rows = []
                for _ in range(3):
                    r = native.load_bench().http_load("127.0.0.1", port, "/metrics", conns, 1.0, 0.0)
                    rows.append((r["ok"] / r["elapsed_s"], pct(r["latencies_s"], 0.5) * 1e6, r["bytes"] // max(1, r["ok"])))
                out["threads%d_conns%d" % (threads, conns)] = {"rps": [round(x[0]) for x in rows],
                                                              "p50_us": [round(x[1], 2) for x in rows],
                                                              "bytes": rows[0][2]}
        finally:
            w.stop()
            m.exporter.stop()
            m.monitor.stop()
    body = out["threads2_conns1"]["bytes"]
    for pairs in (1, 2, 4):
        out["tcp_floor_pairs%d_p50_us" % pairs] = [floor_parallel(n, pairs, body) for _ in range(2)]
    print(json.dumps(out))


if __name__ == "__main__":
    main()
