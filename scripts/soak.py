"""Soak test of the daemon on the real backend: kubelet-like Allocate traffic, /metrics
scrapes and frequent GET /restart reloads at once, with fast telemetry sampling, for a
fixed time.  Checks that the daemon stays up, keeps answering and does not grow (RSS
sampled every few seconds), and that reloads are hitless for kubelet: the Allocate
connection never drops (``reconnects`` 0), the kubelet-like ListAndWatch stream opened at
the start stays open through every reload (``law_reopens`` 1) and is sent each new device
table (``law_updates``), and the plugin registers once.  Prints one JSON line.

    python scripts/soak.py --seconds 90 [--restart-every 0.25] [--backend auto|fixture]
                           [--fault-every 0.1]   # fixture: scripted GPU 1 resets

With ``--fault-every`` (fixture backend) GPU 1 alternates PRE_RESET / POST_RESET on that
period; the run checks that the watcher kept seeing updates and that both GPUs are still
advertised at the end.
"""
import argparse
import http.client
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

from k8s_gpu_device_plugin_amd import native  # noqa: E402
from k8s_gpu_device_plugin_amd.api import v1beta1  # noqa: E402
from k8s_gpu_device_plugin_amd.plugin.kubelet_stub import KubeletStub  # noqa: E402


def rss_kb(pid):
    with open("/proc/%d/status" % pid) as f:
        for line in f:
            if line.startswith("VmRSS:"):
                return int(line.split()[1])
    return 0


def http_get(port, path):
    c = http.client.HTTPConnection("127.0.0.1", port, timeout=5)
    c.request("GET", path)
    r = c.getresponse()
    body = r.read()
    c.close()
    return r.status, body


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=90.0)
    ap.add_argument("--restart-every", type=float, default=0.25)
    ap.add_argument("--backend", default="auto")
    ap.add_argument("--fault-every", type=float, default=0.0)
    a = ap.parse_args()
    n = native.load()
    native.load_bench()  # the harness extension: load generators, H2Client.bench_unary
    backend = a.backend if a.backend != "auto" else ("amdsmi" if n.amdsmi_available() else "fixture")
    work = tempfile.mkdtemp(prefix="dp-soak-")
    plugin_dir = os.path.join(work, "device-plugins")
    os.makedirs(plugin_dir)
    kubelet = KubeletStub(plugin_dir).start()
    s = __import__("socket").socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    fixture = "2gpu_spx"
    if a.fault_every > 0:
        if backend != "fixture":
            raise SystemExit("--fault-every needs the fixture backend")
        from k8s_gpu_device_plugin_amd.models import fixtures
        model = fixtures.load_model("2gpu_spx")
        n_ev = int((a.seconds + 10) / a.fault_every)
        model["events"] = [{"at": 3.0 + i * a.fault_every, "kind": "pre_reset" if i % 2 == 0 else "post_reset",
                            "gpu": 1} for i in range(n_ev)]
        fixture = os.path.join(work, "faults.json")
        with open(fixture, "w") as f:
            json.dump(model, f)
    cfg = os.path.join(work, "soak.yml")
    with open(cfg, "w") as f:
        f.write("webListenAddress: \"127.0.0.1:%d\"\nmigStrategy: none\nbackend: %s\nfixture: \"%s\"\n"
                "pluginDir: \"%s\"\nlog:\n  level: warn\n  fileDir: \"\"\nhttp:\n  accessLog: false\n"
                "telemetry:\n  intervalMs: 100\n" % (port, backend, fixture, plugin_dir))
    env = dict(os.environ, PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""))
    log = open(os.path.join(work, "daemon.log"), "w")
    proc = subprocess.Popen([sys.executable, "-m", "k8s_gpu_device_plugin_amd", "--configFile", cfg], cwd=work,
                            env=env, stdout=log, stderr=subprocess.STDOUT, start_new_session=True)
    stats = {"backend": backend, "allocs": 0, "alloc_errors": 0, "reconnects": 0, "scrapes": 0, "scrape_errors": 0,
             "restarts": 0, "restart_errors": 0, "rss_kb": [], "fds": [], "threads": [], "law_updates": 0,
             "law_reopens": 0}
    stop = threading.Event()
    try:
        regs = kubelet.wait_for_registrations(1, timeout=60)
        sock = os.path.join(plugin_dir, regs[0].endpoint)
        deadline = time.time() + 30
        while time.time() < deadline:
            try:
                if http_get(port, "/health")[0] == 200:
                    break
            except OSError:
                time.sleep(0.1)
        dev = v1beta1.ListAndWatchResponse.FromString(
            n.H2Client(sock).first_stream_message(v1beta1.METHOD_LIST_AND_WATCH, b"")).devices[0].ID
        req = v1beta1.AllocateRequest(container_requests=[v1beta1.ContainerAllocateRequest(
            devices_ids=[dev])]).SerializeToString()

        def allocator():
            c = None
            while not stop.is_set():
                try:
                    if c is None:
                        c = n.H2Client(sock, 2.0)
                    st, _, _ = c.unary(v1beta1.METHOD_ALLOCATE, req)
                    if st == 0:
                        stats["allocs"] += 1
                    else:
                        stats["alloc_errors"] += 1
                except Exception:  # the connection dropped (a reload must not do this)
                    stats["reconnects"] += 1
                    c = None
                    time.sleep(0.005)

        def scraper():
            while not stop.is_set():
                r = native.load_bench().http_load("127.0.0.1", port, "/metrics", 2, 0.2, 0.0)
                stats["scrapes"] += r["ok"]
                stats["scrape_errors"] += r["errors"]

        def restarter():
            while not stop.wait(a.restart_every):
                try:
                    st, _ = http_get(port, "/restart")
                    stats["restarts" if st == 200 else "restart_errors"] += 1
                except OSError:
                    stats["restart_errors"] += 1

        last_law = {}

        def watcher():  # kubelet's ListAndWatch: re-opened only if the stream ends
            c = None
            while not stop.is_set():
                try:
                    if c is None:
                        c = n.H2Client(sock, 2.0)
                        c.open_stream(v1beta1.METHOD_LIST_AND_WATCH, b"")
                        stats["law_reopens"] += 1
                    msg = c.next_stream_message(0.5)
                    if msg is None:
                        c = None
                        continue
                    stats["law_updates"] += 1
                    last_law["devices"] = {d.ID: d.health for d in v1beta1.ListAndWatchResponse.FromString(msg).devices}
                except Exception:
                    c = None
                    time.sleep(0.005)

        workers = [allocator, scraper, restarter, watcher]
        ts = [threading.Thread(target=f, daemon=True) for f in workers]
        for t in ts:
            t.start()
        t0 = time.time()
        while time.time() - t0 < a.seconds:
            time.sleep(min(5.0, a.seconds / 10))
            if proc.poll() is not None:
                break
            stats["rss_kb"].append(rss_kb(proc.pid))
            stats["fds"].append(len(os.listdir("/proc/%d/fd" % proc.pid)))
            stats["threads"].append(len(os.listdir("/proc/%d/task" % proc.pid)))
            print("t=%.0fs allocs=%d scrapes=%d restarts=%d rss=%d KB" % (
                time.time() - t0, stats["allocs"], stats["scrapes"], stats["restarts"], stats["rss_kb"][-1]),
                file=sys.stderr, flush=True)
        stop.set()
        for t in ts:
            t.join(10)
        stats["daemon_alive"] = proc.poll() is None
        stats["health_after"] = http_get(port, "/health")[0] if stats["daemon_alive"] else None
        stats["registrations"] = len(kubelet.requests)
        if stats["daemon_alive"]:
            import re
            body = http_get(port, "/metrics")[1].decode()
            for ev in ("reloads", "table_swaps", "restarts_coalesced", "reregistrations_restart"):
                m = re.search(r'amdgpu_device_plugin_events_total\{event="%s"\} (\d+)' % ev, body)
                stats[ev] = int(m.group(1)) if m else 0
        rs = stats["rss_kb"]
        half = rs[len(rs) // 2:] or rs
        stats["rss_growth_second_half_kb"] = (max(half) - min(half)) if half else None
        # descriptors and threads do not accumulate over reloads.  A sample taken while a
        # reload has the old servers down reads low (a dip, not growth): compare the
        # medians of the second and last quarters instead of max - min.
        def growth(xs):
            q = len(xs) // 4
            if q < 2:
                return None
            mid, last = sorted(xs[q:2 * q]), sorted(xs[-q:])
            return last[len(last) // 2] - mid[len(mid) // 2]

        stats["fd_growth_second_half"] = growth(stats["fds"])
        stats["thread_growth_second_half"] = growth(stats["threads"])
        stats["ok"] = bool(stats["daemon_alive"] and stats["health_after"] == 200 and stats["allocs"] > 0
                           and (stats["fd_growth_second_half"] or 0) <= 8
                           and (stats["thread_growth_second_half"] or 0) <= 8
                           and stats["scrapes"] > 0 and stats["restarts"] > 0 and stats["alloc_errors"] == 0
                           and stats["scrape_errors"] <= stats["restarts"] * 4
                           # hitless reloads: one connection, one stream; every /restart's
                           # reload registers again on the same socket (reference contract)
                           and stats["reconnects"] == 0 and stats["law_reopens"] == 1
                           and stats["registrations"] == 1 + stats.get("reregistrations_restart", 0)
                           and stats.get("reregistrations_restart", 0) >= 1 and stats["law_updates"] > 1)
        stats["law_last"] = last_law.get("devices")
        if a.fault_every > 0:
            # both GPUs still advertised; the stream kept moving (faults + reloads)
            stats["ok"] = stats["ok"] and stats["law_updates"] > a.seconds / a.fault_every / 4 and \
                len(last_law.get("devices", {})) == 2
    finally:
        stop.set()
        try:
            os.killpg(proc.pid, signal.SIGTERM)
            proc.wait(15)
        except (ProcessLookupError, subprocess.TimeoutExpired):
            os.killpg(proc.pid, signal.SIGKILL)
        kubelet.stop()
        shutil.rmtree(work, ignore_errors=True)
    print(json.dumps(stats))
    return 0 if stats.get("ok") else 1


if __name__ == "__main__":
    sys.exit(main())
