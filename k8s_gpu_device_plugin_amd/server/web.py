"""HTTP ops surface: ``GET /``, ``/metrics``, ``/health``, ``/restart``, ``/ready``,
``/health/clear``.

Reference: ``server/server.go`` (echo, middleware Recover->Cros->Logger->Metrics,
30 s read timeout), ``router/api.go:27-54`` (routes), ``router/router.go`` (global
route registry - defect D16: a second ``Run`` re-registers and panics; here every
``WebServer`` owns its routes and metric counters, so start/stop/start works).

``native`` (default): the C++ epoll server in ``native/httpd.cpp`` serves /metrics from
the exporter's pre-rendered bytes without touching the GIL.  ``python``: a
``ThreadingHTTPServer`` with identical routes/bodies/headers, kept as a readable
reference implementation and for hosts where the native core is being debugged.
"""
from __future__ import annotations

import gzip
import http.server
import socketserver
import threading
import time

from .. import native
from ..utils.log import get_logger
from ..utils.util import envelope_bytes, failed, success
from ..utils.version import VERSION

log = get_logger("web")

ROUTES = ("/", "/metrics", "/health", "/restart", "/ready", "/health/clear")
CORS_HEADERS = (
    ("Access-Control-Allow-Credentials", "true"),
    ("Access-Control-Allow-Headers", "Content-Type, Content-Length, Accept-Encoding, Authorization, Origin"),
    ("Access-Control-Allow-Methods", "POST, GET, OPTIONS, PATCH, PUT, DELETE"),
)
METRICS_CTYPE = "text/plain; version=0.0.4; charset=utf-8"
ECHO_BUCKETS = (0.0005, 0.001, 0.002, 0.005, 0.01, 0.02, 0.05, 0.1, 0.2, 0.5, 1.0, 2.0, 5.0, 10.0, 15.0, 20.0, 30.0)


def health_clear(manager, query: str) -> tuple:
    """``GET /health/clear?gpu=<uuid|bdf|index|device id>``: the operator's way to drop a
    GPU's health latches (uncorrectable ECC, a reset that never finished, failed canary
    verdicts) once they know it is fine - e.g. after a reset no signal this deployment can
    see.  Logged, counted (``health_clears``) and persisted like any latch change.
    Returns (status, JSON body) in the envelope of the other routes."""
    import urllib.parse
    gpu = (urllib.parse.parse_qs(query or "").get("gpu") or [""])[0].strip()
    if not gpu:
        return 400, envelope_bytes(failed("missing ?gpu=<uuid|bdf|index|device id>")).decode()
    clear = getattr(manager, "clear_health", None)
    if clear is None:
        return 503, envelope_bytes(failed("no health monitor")).decode()
    try:
        status, data = clear(gpu)
    except TimeoutError:
        return 503, envelope_bytes(failed("the plugin manager did not answer in time")).decode()
    body = success(data) if status == 200 else failed(data)
    return status, envelope_bytes(body).decode()


class WebServer:
    def __init__(self, cfg, manager, kind: str | None = None) -> None:
        self.cfg = cfg
        self.manager = manager
        self.kind = kind or cfg.http.server
        self.host, self.port = cfg.listen_host_port()
        self._impl = None

    def start(self) -> int:
        if self.kind == "native":
            n = native.load()
            hc = n.HttpConfig()
            hc.host, hc.port = self.host, self.port
            hc.threads = max(1, self.cfg.http.threads)
            hc.access_log = bool(self.cfg.http.accessLog)
            hc.read_timeout_s = 30  # server/server.go:45
            hc.busy_poll_us = int(self.cfg.http.busyPollUs)
            hc.restart_local_only = bool(self.cfg.http.restartLocalOnly)
            hc.clear_local_only = bool(self.cfg.http.healthClearLocalOnly)
            hc.version = VERSION
            srv = n.HttpServer(hc, self.manager.exporter)
            srv.set_restart_hook(self.manager.restart)
            srv.set_clear_hook(lambda q: health_clear(self.manager, q))
            self.port = srv.start()
            self._impl = srv
        else:
            self._impl = PyWebServer(self.host, self.port, self.manager, bool(self.cfg.http.restartLocalOnly),
                                     bool(self.cfg.http.healthClearLocalOnly))
            self.port = self._impl.start()
        for r in ROUTES:  # server/server.go:48-54 prints the route table
            log.info("GET  %s", r)
        log.info("web server started on %s:%d (%s)", self.host, self.port, self.kind)
        add = getattr(self.manager, "add_readiness_listener", None)
        if add is not None:  # GET /ready follows the manager's registration state
            add(self._set_ready)
        return self.port

    def _set_ready(self, ready: bool, reason: str) -> None:
        impl = self._impl
        if impl is not None:
            impl.set_ready(bool(ready), reason or "")

    def stop(self) -> None:
        remove = getattr(self.manager, "remove_readiness_listener", None)
        if remove is not None:
            remove(self._set_ready)
        impl, self._impl = self._impl, None
        if impl is not None:
            impl.stop()
            log.info("web server stopped")


def _is_loopback(addr: str) -> bool:
    import ipaddress
    try:
        ip = ipaddress.ip_address(addr)
    except ValueError:
        return False
    if getattr(ip, "ipv4_mapped", None) is not None:
        ip = ip.ipv4_mapped
    return ip.is_loopback


def accepts_gzip(header: str) -> bool:
    """promhttp ``gzipAccepted``: a comma-separated part equal to ``gzip`` or ``gzip;...``."""
    return any(p.strip() == "gzip" or p.strip().startswith("gzip;") for p in header.split(","))


class _Metrics:
    """echo_http_* families for the Python server (middleware/echo_metric.go)."""

    def __init__(self) -> None:
        self.lock = threading.Lock()
        self.counts: dict = {}
        self.hist: dict = {}

    def observe(self, method: str, handler: str, status: int, dt: float) -> None:
        cls = "%dxx" % min(5, max(1, status // 100))
        with self.lock:
            self.counts[(handler, method, cls)] = self.counts.get((handler, method, cls), 0) + 1
            h = self.hist.setdefault((handler, method), [[0] * (len(ECHO_BUCKETS) + 1), 0.0])
            i = 0
            while i < len(ECHO_BUCKETS) and dt > ECHO_BUCKETS[i]:
                i += 1
            h[0][i] += 1
            h[1] += dt

    def render(self) -> str:
        out = []
        with self.lock:
            if self.counts:
                out += ["# HELP echo_http_requests_total Number of HTTP operations",
                        "# TYPE echo_http_requests_total counter"]
                for (h, m, s), v in sorted(self.counts.items()):
                    out.append('echo_http_requests_total{handler="%s",method="%s",status="%s"} %d' % (h, m, s, v))
            if self.hist:
                out += ["# HELP echo_http_request_duration_seconds Spend time by processing a route",
                        "# TYPE echo_http_request_duration_seconds histogram"]
                for (h, m), (b, total) in sorted(self.hist.items()):
                    cum = 0
                    for i, le in enumerate(list(ECHO_BUCKETS) + ["+Inf"]):
                        cum += b[i]
                        les = le if isinstance(le, str) else ("%g" % le)
                        out.append('echo_http_request_duration_seconds_bucket{handler="%s",method="%s",le="%s"} %d'
                                   % (h, m, les, cum))
                    out.append('echo_http_request_duration_seconds_sum{handler="%s",method="%s"} %r' % (h, m, total))
                    out.append('echo_http_request_duration_seconds_count{handler="%s",method="%s"} %d' % (h, m, cum))
        return "\n".join(out) + ("\n" if out else "")


class PyWebServer:
    def __init__(self, host: str, port: int, manager, restart_local_only: bool = False,
                 clear_local_only: bool = True) -> None:
        self.host, self.port, self.manager = host, port, manager
        self.restart_local_only = restart_local_only
        self.clear_local_only = clear_local_only
        self.ready, self.not_ready_reason = True, ""
        self.metrics = _Metrics()
        self._httpd = None
        self._thread = None

    def start(self) -> int:
        outer = self

        class Handler(http.server.BaseHTTPRequestHandler):
            protocol_version = "HTTP/1.1"
            server_version = "amdgpu-device-plugin"
            sys_version = ""

            def log_message(self, fmt, *args):  # access log goes through our logger
                log.debug("%s %s", self.address_string(), fmt % args)

            def _send(self, status: int, body: bytes, ctype: str = "application/json", gz: bool = False) -> None:
                self.send_response_only(status, {200: "OK", 400: "Bad Request", 403: "Forbidden", 404: "Not Found",
                                                 405: "Method Not Allowed", 503: "Service Unavailable"}.get(status))
                for k, v in CORS_HEADERS:
                    self.send_header(k, v)
                self.send_header("Access-Control-Allow-Origin", self.headers.get("Origin") or "*")
                if gz:
                    self.send_header("Content-Encoding", "gzip")
                self.send_header("Content-Length", str(len(body)))
                self.send_header("Content-Type", ctype)
                self.send_header("Date", self.date_time_string())
                self.end_headers()
                self.wfile.write(body)

            def _route(self, method: str) -> None:
                path = self.path.split("?", 1)[0]
                length = int(self.headers.get("Content-Length") or 0)
                if length:
                    self.rfile.read(length)
                if method == "OPTIONS":
                    return self._send(200, b'{"message":"OK"}\n')
                t0 = time.perf_counter()
                gz = False
                handler = path if path in ROUTES else "/not-found"
                if handler == "/not-found":
                    status, body, ctype = 404, b'{"message":"Not Found"}\n', "application/json"
                elif method != "GET":
                    status, body, ctype = 405, b'{"message":"Method Not Allowed"}\n', "application/json"
                elif path == "/":
                    status, body, ctype = 200, envelope_bytes(success("version : " + VERSION)), "application/json"
                elif path == "/health":
                    status, body, ctype = 200, envelope_bytes(success("ok")), "application/json"
                elif path == "/ready":
                    if outer.ready:
                        status, body, ctype = 200, envelope_bytes(success("ready")), "application/json"
                    else:
                        status, body, ctype = 503, envelope_bytes(failed(outer.not_ready_reason)), "application/json"
                elif path == "/health/clear" and outer.clear_local_only and not _is_loopback(self.client_address[0]):
                    status, body, ctype = 403, b'{"message":"Forbidden"}\n', "application/json"
                elif path == "/health/clear":
                    st, text = health_clear(outer.manager, self.path.split("?", 1)[1] if "?" in self.path else "")
                    status, body, ctype = st, text.encode(), "application/json"
                elif path == "/restart" and outer.restart_local_only and not _is_loopback(self.client_address[0]):
                    status, body, ctype = 403, b'{"message":"Forbidden"}\n', "application/json"
                elif path == "/restart":
                    outer.manager.restart()
                    status, body, ctype = 200, envelope_bytes(success("ok")), "application/json"
                else:
                    text = outer.manager.exporter.render() + outer.metrics.render()
                    status, body, ctype = 200, text.encode(), METRICS_CTYPE
                    if accepts_gzip(self.headers.get("Accept-Encoding", "")):
                        body, gz = gzip.compress(body, compresslevel=1), True
                outer.metrics.observe(method, handler, status, time.perf_counter() - t0)
                self._send(status, body, ctype, gz)

            def do_GET(self):
                self._route("GET")

            def do_POST(self):
                self._route("POST")

            def do_PUT(self):
                self._route("PUT")

            def do_DELETE(self):
                self._route("DELETE")

            def do_PATCH(self):
                self._route("PATCH")

            def do_OPTIONS(self):
                self._route("OPTIONS")

        class Server(socketserver.ThreadingMixIn, http.server.HTTPServer):
            daemon_threads = True
            allow_reuse_address = True

        self._httpd = Server((self.host, self.port), Handler)
        self.port = self._httpd.server_address[1]
        self._thread = threading.Thread(target=self._httpd.serve_forever, kwargs={"poll_interval": 0.2},
                                        daemon=True, name="py-httpd")
        self._thread.start()
        return self.port

    def stop(self) -> None:
        if self._httpd is not None:
            self._httpd.shutdown()
            self._httpd.server_close()
            self._httpd = None

    def set_ready(self, ready: bool, reason: str = "") -> None:
        self.ready, self.not_ready_reason = bool(ready), ("" if ready else reason)
