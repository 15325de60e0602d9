"""HTTP ops surface parity with the reference (router/api.go, server/server.go,
middleware/echo_metric.go) for the native epoll server and the Python server."""
import http.client
import json
import socket
import time

import pytest
from prometheus_client.parser import text_string_to_metric_families

from k8s_gpu_device_plugin_amd.plugin.manager import PluginManager
from k8s_gpu_device_plugin_amd.server.web import WebServer


@pytest.fixture(params=["native", "python"])
def web(request, make_cfg):
    cfg = make_cfg(webListenAddress="127.0.0.1:0", http={"server": request.param, "accessLog": False})
    mgr = PluginManager(cfg)
    restarts = []
    mgr.restart = lambda: restarts.append(time.monotonic())  # observe, do not reload
    mgr.load_plugins()
    mgr._start_telemetry()  # exporter sampling the fixture backend, health monitor
    w = WebServer(cfg, mgr)
    port = w.start()
    yield port, restarts, request.param
    w.stop()
    mgr.exporter.stop()
    mgr.monitor.stop()


def get(port, path, method="GET", headers=None, body=None):
    c = http.client.HTTPConnection("127.0.0.1", port, timeout=5)
    c.request(method, path, body=body, headers=headers or {})
    r = c.getresponse()
    data = r.read()
    c.close()
    return r.status, dict(r.getheaders()), data


def test_json_routes_byte_exact(web):
    port, restarts, _ = web
    assert get(port, "/")[2] == b'{"code":0,"data":"version : 0.1.0","msg":"success"}\n'
    st, h, body = get(port, "/health")
    assert st == 200 and body == b'{"code":0,"data":"ok","msg":"success"}\n'
    assert h["Content-Type"] == "application/json"
    st, _, body = get(port, "/restart")
    assert st == 200 and json.loads(body) == {"code": 0, "data": "ok", "msg": "success"}
    assert len(restarts) == 1


def test_errors_and_cors(web):
    port, _, _ = web
    st, h, body = get(port, "/nope")
    assert st == 404 and body == b'{"message":"Not Found"}\n'
    assert h["Access-Control-Allow-Origin"] == "*"
    assert h["Access-Control-Allow-Credentials"] == "true"
    assert h["Access-Control-Allow-Methods"] == "POST, GET, OPTIONS, PATCH, PUT, DELETE"
    assert h["Access-Control-Allow-Headers"] == \
        "Content-Type, Content-Length, Accept-Encoding, Authorization, Origin"
    st, h, body = get(port, "/health", headers={"Origin": "https://ops.example"})
    assert h["Access-Control-Allow-Origin"] == "https://ops.example"
    st, h, body = get(port, "/anything", method="OPTIONS")
    assert st == 200 and body == b'{"message":"OK"}\n'
    st, _, body = get(port, "/health", method="POST", body=b"x=1")
    assert st == 405 and body == b'{"message":"Method Not Allowed"}\n'
    st, _, _ = get(port, "/health?probe=1")
    assert st == 200


def test_metrics_exposition_is_valid_and_complete(web):
    port, _, kind = web
    get(port, "/health")
    get(port, "/missing")
    st, h, body = get(port, "/metrics")
    assert st == 200 and h["Content-Type"] == "text/plain; version=0.0.4; charset=utf-8"
    st, h, body = get(port, "/metrics")
    fams = {f.name: f for f in text_string_to_metric_families(body.decode())}
    for name in ("k8s_gpu_device_plugin_build_info", "amdgpu_info", "amdgpu_power_watts",
                 "amdgpu_temperature_celsius", "amdgpu_xgmi_link_up", "amdgpu_partition_info",
                 "amdgpu_device_plugin_device_health", "echo_http_requests", "echo_http_request_duration_seconds"):
        assert name in fams, name
    reqs = {(s.labels["handler"], s.labels["method"], s.labels["status"]): s.value
            for s in fams["echo_http_requests"].samples}
    assert reqs[("/health", "GET", "2xx")] >= 1 and reqs[("/not-found", "GET", "4xx")] >= 1
    assert reqs[("/metrics", "GET", "2xx")] >= 1
    les = [s.labels["le"] for s in fams["echo_http_request_duration_seconds"].samples
           if s.name.endswith("_bucket") and s.labels["handler"] == "/health"]
    assert les == ["0.0005", "0.001", "0.002", "0.005", "0.01", "0.02", "0.05", "0.1", "0.2", "0.5", "1",
                   "2", "5", "10", "15", "20", "30", "+Inf"]  # Go FormatFloat(g, -1)


def test_metrics_gzip_negotiation(web):
    """promhttp compresses /metrics for scrapers sending Accept-Encoding: gzip (Prometheus
    does).  The native server sends a multi-member gzip stream whose large members are
    cached per sampling tick; it must decode to the same exposition as a plain scrape."""
    import gzip
    port, _, kind = web
    get(port, "/health")  # so the echo_http families exist in every scrape below
    volatile = ("echo_http", "process_", "amdgpu_telemetry_last_pass_age", "amdgpu_telemetry_sample_age")  # change between two scrapes
    strip = lambda t: [ln for ln in t.splitlines() if not ln.startswith(volatile)]  # noqa: E731
    ticks = lambda t: [ln for ln in t.splitlines() if ln.startswith("amdgpu_telemetry_samples_total ")]  # noqa: E731
    for ae in ("gzip", "deflate, gzip;q=1.0", "br,gzip"):
        for _ in range(20):  # a plain and a gzip scrape within one sampling tick
            st, h, plain = get(port, "/metrics")
            assert "Content-Encoding" not in h
            st, h, body = get(port, "/metrics", headers={"Accept-Encoding": ae})
            assert st == 200 and h["Content-Encoding"] == "gzip", (ae, h)
            text = gzip.decompress(body).decode()
            if ticks(text) == ticks(plain.decode()):
                break
        fams = {f.name for f in text_string_to_metric_families(text)}
        assert fams == {f.name for f in text_string_to_metric_families(plain.decode())}
        # everything but the per-request counters is identical
        assert strip(text) == strip(plain.decode())
        assert len(body) < len(plain) / 3
    st, h, body = get(port, "/metrics", headers={"Accept-Encoding": "identity, gzipx"})
    assert "Content-Encoding" not in h and body.startswith(b"# HELP")
    if kind == "native":  # cached head member: byte-identical across scrapes within a tick
        a = get(port, "/metrics", headers={"Accept-Encoding": "gzip"})[2]
        b = get(port, "/metrics", headers={"Accept-Encoding": "gzip"})[2]
        head = min(len(a), len(b)) // 2
        assert a[:head] == b[:head]


def test_keepalive_and_pipelining(web):
    port, _, kind = web
    c = http.client.HTTPConnection("127.0.0.1", port, timeout=5)
    for _ in range(20):
        c.request("GET", "/health")
        assert c.getresponse().read().endswith(b'"ok","msg":"success"}\n')
    c.close()
    if kind != "native":
        return
    s = socket.create_connection(("127.0.0.1", port))
    s.sendall(b"GET /health HTTP/1.1\r\nHost: x\r\n\r\nGET / HTTP/1.1\r\nHost: x\r\n\r\n"
              b"GET /health HTTP/1.1\r\nHost: x\r\nConnection: close\r\n\r\n")
    data = b""
    s.settimeout(5)
    while True:
        chunk = s.recv(65536)
        if not chunk:
            break
        data += chunk
    s.close()
    assert data.count(b"HTTP/1.1 200 OK") == 3 and b"Connection: close" in data
    s = socket.create_connection(("127.0.0.1", port))
    s.sendall(b"GET /health HTTP/1.0\r\n\r\n")
    s.settimeout(5)
    data = b""
    while True:
        chunk = s.recv(65536)
        if not chunk:
            break
        data += chunk
    assert data.startswith(b"HTTP/1.0 200 OK")


def test_native_http_rejects_garbage(make_cfg):
    cfg = make_cfg(webListenAddress="127.0.0.1:0", http={"accessLog": False})
    mgr = PluginManager(cfg)
    w = WebServer(cfg, mgr)
    port = w.start()
    try:
        s = socket.create_connection(("127.0.0.1", port))
        s.sendall(b"garbage\r\n\r\n")
        s.settimeout(5)
        assert s.recv(4096).startswith(b"HTTP/1.1 400 Bad Request")
        s.close()
        s = socket.create_connection(("127.0.0.1", port))
        s.sendall(b"GET / HTTP/1.1\r\n" + b"X-Long: " + b"a" * 70000 + b"\r\n")
        assert s.recv(4096).startswith(b"HTTP/1.1 431")
        s.close()
        # a negative or overflowing Content-Length is refused, never read as 0 (the body
        # would otherwise be parsed as the next request)
        for cl in (b"-1", b"99999999999999999999999", b"+2000000"):
            s = socket.create_connection(("127.0.0.1", port))
            s.settimeout(5)
            s.sendall(b"POST /health HTTP/1.1\r\nContent-Length: " + cl + b"\r\n\r\nGET / HTTP/1.1\r\n\r\n")
            assert s.recv(4096).startswith(b"HTTP/1.1 413"), cl
            s.close()
        # header names in any case; a body of the announced length is skipped, the next
        # pipelined request answered; "Connection: CLOSE" closes after the answer
        s = socket.create_connection(("127.0.0.1", port))
        s.settimeout(5)
        s.sendall(b"POST /health HTTP/1.1\r\nCONTENT-LENGTH: 2\r\n\r\nxxGET /health HTTP/1.1\r\n"
                  b"CoNNection: CLOSE\r\n\r\n")
        data = b""
        while True:
            chunk = s.recv(65536)
            if not chunk:
                break
            data += chunk
        assert data.count(b"HTTP/1.1 ") == 2 and b"Connection: close" in data.split(b"HTTP/1.1 ")[2], data
        s.close()
        assert get(port, "/health")[0] == 200  # server still fine
    finally:
        w.stop()


def test_start_stop_start_same_port(make_cfg):
    """D16: the reference registers routes/collectors globally, a 2nd Run panics."""
    cfg = make_cfg(webListenAddress="127.0.0.1:0", http={"accessLog": False})
    mgr = PluginManager(cfg)
    w = WebServer(cfg, mgr)
    port = w.start()
    w.stop()
    cfg.webListenAddress = "127.0.0.1:%d" % port
    w2 = WebServer(cfg, mgr)
    assert w2.start() == port
    assert get(port, "/health")[0] == 200
    w2.stop()


def test_access_log_lines(make_cfg, capfd):
    cfg = make_cfg(webListenAddress="127.0.0.1:0", http={"accessLog": True})
    mgr = PluginManager(cfg)
    w = WebServer(cfg, mgr)
    port = w.start()
    get(port, "/health", headers={"User-Agent": "probe/1"})
    time.sleep(0.3)
    w.stop()
    out = capfd.readouterr().out
    line = [ln for ln in out.splitlines() if '"uri":"/health"' in ln][0]
    rec = json.loads(line)
    assert rec["method"] == "GET" and rec["status"] == 200 and rec["user_agent"] == "probe/1"
    assert rec["remote_ip"] == "127.0.0.1" and rec["bytes_out"] > 0 and "latency" in rec


def test_native_scrapers_spread_over_workers(make_cfg):
    """Concurrent keep-alive scrapers are owned by different HTTP workers (the accepting
    worker hands each connection to the least-loaded one) and all get answers."""
    cfg = make_cfg(webListenAddress="127.0.0.1:0", http={"server": "native", "accessLog": False, "threads": 3})
    mgr = PluginManager(cfg)
    mgr.load_plugins()
    w = WebServer(cfg, mgr)
    port = w.start()
    try:
        conns = [http.client.HTTPConnection("127.0.0.1", port, timeout=5) for _ in range(3)]
        for _ in range(5):
            for c in conns:
                c.request("GET", "/metrics")
                r = c.getresponse()
                assert r.status == 200 and b"process_start_time_seconds" in r.read()
        assert sorted(w._impl.worker_connections) == [1, 1, 1]
        for c in conns:
            c.close()
        deadline = time.time() + 5
        while sum(w._impl.worker_connections) and time.time() < deadline:
            time.sleep(0.02)
        assert w._impl.worker_connections == [0, 0, 0]
    finally:
        w.stop()


def _rss_bytes():
    with open("/proc/self/status") as f:
        for line in f:
            if line.startswith("VmRSS:"):
                return int(line.split()[1]) * 1024
    return 0


def test_pipelining_client_that_does_not_read_is_throttled(make_cfg):
    """A client pipelines 2000 GET /metrics (77 KB answers, 150 MB in all) and reads
    nothing for a second: the server stops reading its socket once 4 MiB of answers are
    pending, so its memory stays flat; then every answer arrives, in order."""
    import threading

    cfg = make_cfg(webListenAddress="127.0.0.1:0", fixture="8gpu_cpx_nps4", migStrategy="single",
                   http={"server": "native", "accessLog": False, "threads": 2})
    mgr = PluginManager(cfg)
    mgr.load_plugins()
    mgr._start_telemetry()  # the full 64-partition exposition
    w = WebServer(cfg, mgr)
    port = w.start()
    try:
        s = socket.create_connection(("127.0.0.1", port), timeout=10)
        s.setsockopt(socket.SOL_SOCKET, socket.SO_RCVBUF, 1 << 16)
        n = 2000
        req = b"GET /metrics HTTP/1.1\r\nHost: x\r\n\r\n"
        rss0 = _rss_bytes()
        sender = threading.Thread(target=lambda: s.sendall(req * n), daemon=True)
        sender.start()
        time.sleep(1.0)
        grown = _rss_bytes() - rss0
        assert grown < 48 << 20, grown  # unthrottled: ~150 MB of queued answers
        buf, got = b"", 0
        while got < n:
            chunk = s.recv(1 << 20)
            assert chunk, "connection closed after %d answers" % got
            buf += chunk
            while True:
                he = buf.find(b"\r\n\r\n")
                if he < 0:
                    break
                head = buf[:he].decode()
                assert head.startswith("HTTP/1.1 200 OK"), head[:80]
                cl = int([h for h in head.split("\r\n") if h.lower().startswith("content-length:")][0].split(":")[1])
                if len(buf) < he + 4 + cl:
                    break
                buf = buf[he + 4 + cl:]
                got += 1
        assert got == n and buf == b""
        sender.join(5)
        s.close()
    finally:
        w.stop()
        mgr.exporter.stop()
        mgr.monitor.stop()


def test_connection_churn_across_workers_leaves_nothing_behind(make_cfg):
    """2000 short connections from 8 threads, each answered by whichever worker the
    accepting one hands it to: every answer arrives, and afterwards no worker still counts
    a connection and the process holds no extra descriptors."""
    import os
    import threading

    cfg = make_cfg(webListenAddress="127.0.0.1:0", http={"server": "native", "accessLog": False, "threads": 4})
    mgr = PluginManager(cfg)
    mgr.load_plugins()
    w = WebServer(cfg, mgr)
    port = w.start()
    try:
        fds0 = len(os.listdir("/proc/self/fd"))
        errors = []

        def churn():
            for _ in range(250):
                try:
                    s = socket.create_connection(("127.0.0.1", port), timeout=5)
                    s.sendall(b"GET /health HTTP/1.1\r\nHost: x\r\n\r\n")
                    if not s.recv(4096).startswith(b"HTTP/1.1 200 OK"):
                        errors.append("bad answer")
                    s.close()
                except OSError as e:
                    errors.append(repr(e))
        ts = [threading.Thread(target=churn) for _ in range(8)]
        for t in ts:
            t.start()
        for t in ts:
            t.join(120)
        assert not errors, errors[:3]
        deadline = time.time() + 5
        while sum(w._impl.worker_connections) and time.time() < deadline:
            time.sleep(0.02)
        assert w._impl.worker_connections == [0, 0, 0, 0]
        assert len(os.listdir("/proc/self/fd")) <= fds0 + 4 + 2  # + one reserve descriptor per worker
    finally:
        w.stop()


def test_native_http_stop_right_after_start(n):
    """Counterpart of the gRPC server's stop-after-start case: workers that have not run
    yet when stop() comes must still leave (no lock held across the join)."""
    ex = n.Exporter()
    for _ in range(50):
        cfg = n.HttpConfig()
        cfg.host, cfg.port, cfg.threads, cfg.access_log = "127.0.0.1", 0, 8, False
        srv = n.HttpServer(cfg, ex)
        srv.start()
        srv.stop()
        assert not srv.running


def test_hostile_clients_do_not_disturb_scrapes(make_cfg):
    """While a Prometheus-like client scrapes /metrics over keep-alive, other clients
    misbehave on the same port: random bytes, requests cut off mid-header, connections
    that send half a request line and go silent, oversized headers, a pipelined burst that
    is closed unread, and resets (RST) at random points.  Every scrape must get its full
    answer and the server must keep answering afterwards."""
    import random
    import struct
    import threading
    cfg = make_cfg(webListenAddress="127.0.0.1:0", http={"server": "native", "accessLog": False, "threads": 3})
    mgr = PluginManager(cfg)
    mgr.load_plugins()
    w = WebServer(cfg, mgr)
    port = w.start()
    stop = threading.Event()
    errs, done, idle = [], [0], []

    def good():
        c = http.client.HTTPConnection("127.0.0.1", port, timeout=5)
        try:
            while not stop.is_set():
                c.request("GET", "/metrics")
                r = c.getresponse()
                body = r.read()
                if r.status != 200 or b"process_start_time_seconds" not in body:
                    errs.append((r.status, len(body)))
                done[0] += 1
        except Exception as e:  # pragma: no cover - reported below
            errs.append(repr(e))
        finally:
            c.close()

    def hostile(seed):
        rng = random.Random(seed)
        req = b"GET /metrics HTTP/1.1\r\nHost: x\r\nAccept-Encoding: gzip\r\n\r\n"
        while not stop.is_set():
            s = socket.socket()
            try:
                s.settimeout(0.5)
                s.connect(("127.0.0.1", port))
                kind = rng.randrange(6)
                if kind == 0:
                    s.sendall(bytes(rng.randrange(256) for _ in range(rng.randrange(1, 300))))
                elif kind == 1:
                    s.sendall(req[:rng.randrange(1, len(req))])
                elif kind == 2:
                    s.sendall(b"GET /metr")
                    idle.append(s)  # slow client: half a request line, then nothing
                    s = None
                    if len(idle) > 16:
                        idle.pop(0).close()
                elif kind == 3:
                    s.sendall(b"GET / HTTP/1.1\r\nX-Big: " + b"b" * 80000 + b"\r\n\r\n")
                    s.recv(64)
                elif kind == 4:
                    s.sendall(req * 50)  # pipelined, closed unread
                else:
                    s.sendall(req)
                    s.setsockopt(socket.SOL_SOCKET, socket.SO_LINGER, struct.pack("ii", 1, 0))  # RST on close
            except OSError:
                pass
            finally:
                if s is not None:
                    s.close()

    ts = [threading.Thread(target=good)] + [threading.Thread(target=hostile, args=(i,)) for i in range(4)]
    try:
        for t in ts:
            t.start()
        time.sleep(3.0)
        stop.set()
        for t in ts:
            t.join(10)
        assert not errs, errs[:3]
        assert done[0] > 50
        assert get(port, "/health")[0] == 200
    finally:
        stop.set()
        for s in idle:
            s.close()
        w.stop()


def _non_loopback_ipv4():
    """An address of this host that is not loopback (None when the host has none)."""
    s = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    try:
        s.connect(("198.51.100.1", 9))  # no packet is sent: this only picks a source address
        ip = s.getsockname()[0]
    except OSError:
        return None
    finally:
        s.close()
    return None if ip.startswith("127.") or ip == "0.0.0.0" else ip


@pytest.mark.parametrize("server", ["native", "python"])
def test_restart_local_only(make_cfg, server):
    """http.restartLocalOnly: /restart from loopback reloads, from another address it is a
    403 (counted as 4xx); /health and /metrics stay open to everyone."""
    ip = _non_loopback_ipv4()
    if ip is None:
        pytest.skip("no non-loopback IPv4 address on this host")
    cfg = make_cfg(webListenAddress="0.0.0.0:0", http={"server": server, "accessLog": False,
                                                       "restartLocalOnly": True})
    mgr = PluginManager(cfg)
    restarts = []
    mgr.restart = lambda: restarts.append(time.monotonic())
    mgr.load_plugins()
    w = WebServer(cfg, mgr)
    port = w.start()
    try:
        def remote(path):
            c = http.client.HTTPConnection(ip, port, timeout=5)
            c.request("GET", path)
            r = c.getresponse()
            out = (r.status, r.read())
            c.close()
            return out
        assert remote("/restart") == (403, b'{"message":"Forbidden"}\n') and restarts == []
        assert remote("/health")[0] == 200
        assert get(port, "/restart")[0] == 200 and len(restarts) == 1
        body = remote("/metrics")[1].decode()
        assert 'echo_http_requests_total{handler="/restart",method="GET",status="4xx"} 1' in body
    finally:
        w.stop()
        mgr.exporter.stop()
        mgr.monitor.stop()


def test_restart_is_open_to_everyone_by_default(make_cfg):
    """The reference's behaviour stays the default."""
    ip = _non_loopback_ipv4()
    if ip is None:
        pytest.skip("no non-loopback IPv4 address on this host")
    cfg = make_cfg(webListenAddress="0.0.0.0:0", http={"accessLog": False})
    mgr = PluginManager(cfg)
    restarts = []
    mgr.restart = lambda: restarts.append(time.monotonic())
    w = WebServer(cfg, mgr)
    port = w.start()
    try:
        c = http.client.HTTPConnection(ip, port, timeout=5)
        c.request("GET", "/restart")
        assert c.getresponse().status == 200 and len(restarts) == 1
        c.close()
    finally:
        w.stop()


def _wait_for(pred, timeout=10.0):
    deadline = time.monotonic() + timeout
    while time.monotonic() < deadline:
        if pred():
            return True
        time.sleep(0.05)
    return False


@pytest.mark.parametrize("server", ["native", "python"])
def test_ready_follows_kubelet_registration(make_cfg, plugin_dir, server):
    """GET /ready: 503 with the reason while a resource is not registered with kubelet
    (no kubelet.sock yet), 200 once it is; /health answers ok throughout (reference)."""
    from k8s_gpu_device_plugin_amd.plugin.kubelet_stub import KubeletStub
    cfg = make_cfg(webListenAddress="127.0.0.1:0", http={"server": server, "accessLog": False}, retrySeconds=0.2)
    mgr = PluginManager(cfg)
    w = WebServer(cfg, mgr)
    port = w.start()  # the web server comes up before the plugins (D20)
    t = mgr.start_background()
    try:
        st, hdrs, body = get(port, "/ready")
        assert st == 503 and json.loads(body) == {"code": -1, "data": None,
                                                 "msg": "not registered with kubelet: amd.com/gpu"}
        assert get(port, "/health")[0] == 200
        with KubeletStub(plugin_dir) as k:
            k.wait_for_registrations(1, timeout=10)
            assert _wait_for(lambda: get(port, "/ready")[0] == 200)
            assert get(port, "/ready")[2] == b'{"code":0,"data":"ready","msg":"success"}\n'
        reqs = {(s.labels["handler"], s.labels["status"]): s.value
                 for f in text_string_to_metric_families(get(port, "/metrics")[2].decode())
                 for s in f.samples if s.name == "echo_http_requests_total"}
        assert reqs[("/ready", "5xx")] >= 1 and reqs[("/ready", "2xx")] >= 1
    finally:
        mgr.stop()
        t.join(10)
        assert get(port, "/ready")[0] == 503  # a stopped manager is not ready
        w.stop()


@pytest.mark.parametrize("server", ["native", "python"])
def test_health_clear_route(make_cfg, plugin_dir, server):
    """GET /health/clear?gpu=...: the operator's latch clear.  The
    util envelope; 400 without a GPU, 404 for one that does not exist; a latched GPU comes
    back Healthy; only loopback peers by default (http.healthClearLocalOnly)."""
    from k8s_gpu_device_plugin_amd.models import fixtures
    from k8s_gpu_device_plugin_amd.plugin.kubelet_stub import KubeletStub
    model = fixtures.mi355x_node(2)
    model["hardware_events"] = False
    be = fixtures.build_backend(model)
    ip = _non_loopback_ipv4()
    cfg = make_cfg(webListenAddress="0.0.0.0:0", http={"server": server, "accessLog": False},
                   telemetry={"intervalMs": 50})
    with KubeletStub(plugin_dir) as k:
        mgr = PluginManager(cfg, backend=be)
        t = mgr.start_background()
        w = WebServer(cfg, mgr)
        port = w.start()
        try:
            k.wait_for_registrations(1)
            st, _, body = get(port, "/health/clear")
            assert st == 400 and json.loads(body)["code"] == -1
            st, _, body = get(port, "/health/clear?gpu=GPU-nope")
            assert st == 404 and json.loads(body) == {"code": -1, "data": None, "msg": "no GPU matches 'GPU-nope'"}
            be.set_ecc_uncorrectable(1, 1)
            ids = mgr.plugins[0].table.ids()
            assert _wait_for(lambda: not mgr.plugins[0].table.healthy(ids[1]))
            st, _, body = get(port, "/health/clear?gpu=" + ids[1])
            reply = json.loads(body)
            assert st == 200 and reply["code"] == 0 and reply["msg"] == "success"
            assert reply["data"]["cleared"] == ["uncorrectable_ecc"] and reply["data"]["index"] == 1
            assert _wait_for(lambda: mgr.plugins[0].table.healthy(ids[1]))
            if ip is not None:
                c = http.client.HTTPConnection(ip, port, timeout=5)
                c.request("GET", "/health/clear?gpu=1")
                r = c.getresponse()
                assert (r.status, r.read()) == (403, b'{"message":"Forbidden"}\n')
                c.close()
            reqs = {(s.labels["handler"], s.labels["status"]): s.value
                    for f in text_string_to_metric_families(get(port, "/metrics")[2].decode())
                    for s in f.samples if s.name == "echo_http_requests_total"}
            assert reqs[("/health/clear", "2xx")] == 1 and reqs[("/health/clear", "4xx")] >= 2
            # (the manager counts the clear, then publishes the metrics)
            assert _wait_for(lambda: 'amdgpu_device_plugin_events_total{event="health_clears"}' in mgr.exporter.render())
        finally:
            w.stop()
            mgr.stop()
            t.join(10)
