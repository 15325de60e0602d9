"""Whole-process CPU profile of the /metrics path: a 1-GPU fixture daemon (manager,
exporter, native HTTP server) in this process, scraped on 2 keep-alive connections for
6 s by the native load generator, sampled by the native SIGPROF profiler (every thread,
native symbols).  Shows how much of a scrape is syscalls vs exposition code.

    python scripts/scrape_profile.py [--seconds 6] [--conns 2] [--out FILE]
"""
import argparse
import collections
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from k8s_gpu_device_plugin_amd import config as config_mod, native  # noqa: E402
from k8s_gpu_device_plugin_amd.plugin.manager import PluginManager  # noqa: E402
from k8s_gpu_device_plugin_amd.server.web import WebServer  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=6.0)
    ap.add_argument("--conns", type=int, default=2)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    n = native.load()
    native.load_bench()  # the harness extension: load generators, H2Client.bench_unary
    d = tempfile.mkdtemp(prefix="scrapeprof-")
    cfg = config_mod.validate(config_mod.from_dict({
        "backend": "fixture", "fixture": "1gpu_spx", "pluginDir": d, "log": {"fileDir": ""},
        "telemetry": {"intervalMs": 1000}, "webListenAddress": "127.0.0.1:0",
        "http": {"server": "native", "accessLog": False, "threads": a.conns}}))
    m = PluginManager(cfg)
    m.load_plugins()
    m._start_telemetry()
    w = WebServer(cfg, m)
    port = w.start()
    try:
        time.sleep(0.3)
        native.load_bench().http_load("127.0.0.1", port, "/metrics", a.conns, 0.5, 0.0)  # warm up
        n.prof_start(4999)
        r = native.load_bench().http_load("127.0.0.1", port, "/metrics", a.conns, a.seconds, 0.0)
        n.prof_stop()
        agg = collections.Counter()
        for mod, off, sym, cnt in n.prof_histogram():
            agg[(mod.split("/")[-1], sym or hex(off))] += cnt
        tot = sum(agg.values()) or 1
        lines = ["/metrics, %d conns, %.0f s: %.0f RPS, p50 %.2f us; %d samples" % (
            a.conns, a.seconds, r["ok"] / r["elapsed_s"], r.get("p50_us", float("nan")), tot)]
        lines += ["%5.1f%%  %s  %s" % (100 * c / tot, mod, sym[:110]) for (mod, sym), c in agg.most_common(40)]
    finally:
        w.stop()
        m._shutdown()
    text = "\n".join(lines) + "\n"
    sys.stdout.write(text)
    if a.out:
        with open(a.out, "w") as f:
            f.write(text)
    return 0


if __name__ == "__main__":
    sys.exit(main())
