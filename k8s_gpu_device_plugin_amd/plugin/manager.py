"""Plugin lifecycle manager.

Reference ``plugin/manager.go``: owns the NVML handle, resources, device map and
plugins; ``Start`` watches the device-plugin dir, loads + starts plugins, then loops
over restart timer / ``kubelet.sock`` CREATE / watcher errors / ctx done / a
``default:`` branch polling a ``restart`` bool.

Defects fixed here:
  D1  the ready latch is stored and closed once
  D4  no busy loop: a blocking ``queue.Queue`` carries every event
  D5  stop returns from the loop exactly once; stop is idempotent
  D6  restart stops the *old* plugins, then starts the freshly loaded ones
  D7  ``restart()`` is a thread-safe enqueue, not an unsynchronised bool
  D9  a real health producer (native HealthMonitor) feeds ListAndWatch
  D20 a failed load does not end the process; it retries every ``retrySeconds``
Event sources: native inotify thread (kubelet restarts), native health monitor,
HTTP ``/restart``, retry timer, ``stop()``, and the discovery worker.

Discovery never runs on the manager thread (reference ``restartPlugins`` discovers inline,
``plugin/manager.go:177-194``, so one hung NVML call stops its loop).  A worker thread
runs ``backend.discover()`` - itself bounded per GPU by the backend's lanes - and posts
the result back as an event; the manager keeps handling kubelet restarts, ``/restart``,
health events and server supervision meanwhile.  Reloads are make-before-break: the new
device tables are built from a finished discovery before the old plugins stop; a
discovery that fails or stalls leaves the current plugins serving (the reference stops
them first, defect class D6), and ``GET /ready`` says why.  A kubelet restart re-registers
the plugins that serve at once and checks the inventory in the background.
"""
from __future__ import annotations

import collections
import concurrent.futures
import itertools
import os
import platform
import queue
import threading
import time

from .. import native
from ..config import disabled_checks_mask, state_file_path
from ..device import build_device_map
from ..device.backend import make_backend
from ..resource import new_resources
from ..utils.log import get_logger
from ..utils.util import CloseOnce, name_os_thread, parse_device_selector
from ..utils.version import APP_NAME, VERSION
from .plugin import AmdDevicePlugin, _socket_ident
from .state import HealthState

log = get_logger("manager")

EV_STOP, EV_RESTART, EV_RETRY, EV_KUBELET, EV_HEALTH, EV_REDISCOVER, EV_VERIFIED, EV_PODRES, EV_PRESTART_FAIL = (
    "stop", "restart", "retry", "kubelet", "health", "rediscover", "verified", "podresources", "prestart_fail")
EV_METRICS = "metrics"  # state read by /metrics changed off the manager thread (canary results)
EV_SOCKET_GONE = "socket_gone"  # a *.sock other than kubelet.sock was removed from the plugin dir
EV_DISCOVERED = "discovered"  # the discovery worker finished: (purpose, gpus, topo, report, error)
EV_START_CANARY = "start_canary"  # a start-up canary verdict: (identity, partition, ok, why)
EV_CLEAR = "clear"  # GET /health/clear: (gpu selector, concurrent.futures.Future)
EV_SUPERVISE = "supervise"  # a native gRPC server faulted: run the supervision pass now
EV_CANDIDATE_VERIFIED = "candidate_verified"  # recovery canary after a reset candidate: (identity, gen, ok)
DISCOVERY_RELOAD, DISCOVERY_CHECK = "reload", "check"  # rebuild always / only if the inventory changed
HEALTH_LOG_LEN = 4096
SERVER_CHECK_S = 1.0  # gRPC server supervision poll
# ... and once every plugin is registered with kubelet's stream open and readiness holds:
# a quiet node's manager thread wakes every 5 s (a stream that ends is timed from its end,
# so the re-registration below is as prompt as with the 1 s poll)
SERVER_CHECK_QUIET_S = 5.0
# kubelet holds one ListAndWatch stream per registered plugin for the plugin's life; when
# it ends the stream (its side failed) it drops the endpoint and waits for a new Register.
# A plugin whose stream has been gone this long, kubelet.sock still in place, registers again
LAW_LOST_GRACE_S = 5.0


def inventory_signature(gpus) -> tuple:
    """What must stay identical for the advertised device set to stay valid."""
    return tuple((g.index, g.uuid, g.compute_partition, g.memory_partition,
                  tuple((p.id, p.render_minor) for p in g.partitions)) for g in gpus)


def build_info_text() -> str:
    return ("# HELP k8s_gpu_device_plugin_build_info Build information of the MI355X device plugin.\n"
            "# TYPE k8s_gpu_device_plugin_build_info gauge\n"
            'k8s_gpu_device_plugin_build_info{app="%s",version="%s",python="%s",native="%s"} 1\n'
            % (APP_NAME, VERSION, platform.python_version(), "cxx17"))


class DiscoveryStalled(RuntimeError):
    pass


class Discoverer:
    """One thread that runs ``backend.discover()`` for the manager (GIL released), so the
    manager thread never waits on the hardware.  Requests made while a discovery runs are
    merged into one more run (a reload request outranks a check); each finished run is
    handed to ``post(purpose, gpus, topo, report, error)``."""

    def __init__(self, backend, post) -> None:
        self._backend = backend
        self._post = post
        self._cv = threading.Condition()
        self._want: str | None = None
        self._since: float | None = None  # monotonic start of the run in flight
        self._stop = False
        self._runs = 0
        self.first_done = threading.Event()  # set once the first run has been posted
        self._thread = threading.Thread(target=self._run, name="discovery", daemon=True)
        self._thread.start()

    def request(self, purpose: str) -> None:
        with self._cv:
            if self._want != DISCOVERY_RELOAD:
                self._want = purpose
            self._cv.notify_all()

    def inflight_s(self) -> float | None:
        """Seconds the current discovery has been running (None: idle)."""
        since = self._since
        return None if since is None else time.monotonic() - since

    @property
    def runs(self) -> int:
        return self._runs

    def pending(self) -> bool:
        with self._cv:
            return self._want is not None or self._since is not None

    def stop(self) -> None:
        with self._cv:
            self._stop = True
            self._cv.notify_all()
        self._thread.join(1.0)  # a discovery stuck in the driver stays behind (daemon)

    def _run(self) -> None:
        background_thread()
        while True:
            with self._cv:
                while self._want is None and not self._stop:
                    self._cv.wait()
                if self._stop:
                    return
                purpose, self._want = self._want, None
                self._since = time.monotonic()
            gpus = topo = report = err = None
            try:
                gpus, topo = self._backend.discover()
                report = self._backend.last_discovery() if hasattr(self._backend, "last_discovery") else None
            except Exception as e:  # a failed enumeration: the caller keeps what it serves
                err = e
            with self._cv:
                self._since = None
                self._runs += 1
                stopping = self._stop
            if not stopping:
                self._post(purpose, gpus, topo, report, err)
            self.first_done.set()


def background_thread() -> None:
    """The calling helper thread runs SCHED_BATCH (config ``backgroundSched``): it never
    preempts a gRPC worker when it wakes.  Native servers started from it switch their
    workers back to SCHED_OTHER (``foreground_thread`` in native/common.cpp)."""
    name_os_thread()
    if native.load().background_batch():
        try:
            os.sched_setscheduler(0, os.SCHED_BATCH, os.sched_param(0))  # 0: this thread
        except (OSError, AttributeError):
            pass


def _as_background(fn):
    def run():
        background_thread()
        fn()
    return run


class PluginManager:
    def __init__(self, cfg, ready: CloseOnce | None = None, backend=None) -> None:
        n = native.load()
        n.set_background_batch(getattr(cfg, "backgroundSched", "normal") == "batch")
        self.cfg = cfg
        self.ready = ready if ready is not None else CloseOnce()
        self.backend = backend if backend is not None else make_backend(cfg)
        # every hardware call runs on its GPU's lane, waited for at most this long; a lane
        # whose call is older than the stall threshold takes no more work
        if hasattr(self.backend, "set_call_timeout_ms"):
            self.backend.set_call_timeout_ms(int(cfg.health.discoveryTimeoutS * 1000))
            self.backend.set_stall_ms(int(cfg.health.sampleStallS * 1000) if cfg.health.enabled else 0)
        self.exporter = n.Exporter()
        self.exporter.set_build_info(build_info_text())
        self.monitor = n.HealthMonitor(self.backend, cfg.health.lostAfterFailures)
        self.monitor.set_disabled_checks(disabled_checks_mask(cfg.health.disabledChecks))
        self.monitor.set_pcie_floor(int(cfg.health.pcieMinWidth), float(cfg.health.pcieMinSpeedGTs),
                                    int(cfg.health.pcieDebounceSamples))
        if hasattr(self.backend, "set_reset_query"):
            self.backend.set_reset_query(bool(cfg.health.resetQuery))
        if hasattr(self.backend, "set_ecc_event_gate"):
            self.backend.set_ecc_event_gate(bool(cfg.health.eccEventGate))
        self.events: "queue.Queue[tuple]" = queue.Queue()
        self.plugins: list[AmdDevicePlugin] = []
        self.gpus: list = []
        self.topology = None
        # `devices` indices name GPUs by BDF rank among every GPU this process has seen,
        # so a GPU that drops off the bus does not shift the others into the selection
        self._seen_bdfs: dict[str, str] = {}  # bdf -> identity
        self._selection: tuple | None = None
        self._pinned_index: dict[int, str] = {}  # `devices` index -> identity it was first resolved to
        self._index_conflicts: set[tuple[int, str]] = set()
        self._hip_fallback_logged = False
        self.device_map = None
        self._discoverer: Discoverer | None = None
        self._discovery_error: str | None = None
        self._stale: list = []  # [(index, key, reason)] GPUs the last discovery could not reach
        self._retry_timer: threading.Timer | None = None
        self._threads: list[threading.Thread] = []
        self._running = threading.Event()
        self._stopped = threading.Event()
        self._stop_flag = threading.Event()
        self.signature = None
        self._lock = threading.Lock()
        self.fatal_error: str | None = None
        self.counters = {"restarts_api": 0, "restarts_kubelet": 0, "restarts_retry": 0, "registrations": 0,
                         "load_failures": 0, "health_events": 0}
        # (t, gpu, healthy, reason); bounded so a flapping GPU cannot grow it forever
        self.health_log: "collections.deque[tuple[float, int, int, str]]" = collections.deque(maxlen=HEALTH_LOG_LEN)
        # Health state the manager keeps is keyed by GPU identity (Backend.gpu_key: UUID,
        # else BDF), never by index: when a GPU falls off the bus, re-discovery moves
        # every later GPU down one index, and their health must not move with it.
        self._key_of: dict[int, str] = {}   # advertised GPU index -> identity
        self._index_of: dict[str, int] = {}  # identity -> advertised GPU index
        self._node_index_of: dict[str, int] = {}  # identity -> index, every GPU of the node
        # Recovery canaries run off the manager thread; a per-GPU generation drops a
        # verdict that an Unhealthy event overtook while the canary was running.
        self._health_gen: dict[str, int] = {}
        # GPUs the manager holds Unhealthy although the monitor reports them healthy:
        # recovery canary pending or failed.  Survives plugin reloads.
        self._held_unhealthy: set[str] = set()
        # (gpu identity, partition) whose PreStartContainer canary failed.  Re-applied by
        # every reload (a /restart or kubelet restart must not re-advertise them Healthy)
        # until the GPU reports healthy again or a start-up canary re-checks it.
        self._canary_failed: set[tuple[str, int]] = set()
        self._verify_pool: concurrent.futures.ThreadPoolExecutor | None = None
        # health.canaryOnStart: identities canaried by this process, and (identity,
        # partition) whose verdict is pending (advertised Unhealthy until it arrives)
        self._start_canaried: set[str] = set()
        self._start_pending: set[tuple[str, int]] = set()
        self._canary_pool: concurrent.futures.ThreadPoolExecutor | None = None
        self.podres = None  # PodResourcesWatcher when podResources.enabled
        self.link_pods: dict[tuple[int, int], int] = {}  # GPU pair -> multi-GPU pods spanning it
        # multi-GPU containers allocated since the last PodResources poll (shared by all
        # tables, kept across reloads)
        self.recent_allocations = n.RecentAllocations()
        self.recent_allocations.set_ttl_ms(int(cfg.allocator.recentAllocationTtlS * 1000))
        self.multi_gpu_pods = 0
        # GPUs with hardware event notification armed (read when the monitor starts and
        # after each re-discovery, which can re-initialise amdsmi); None = not monitoring
        self._event_sources: int | None = None
        # last canary result per (gpu, hardware partition index): (unix time, result dict);
        # written by canary pool threads, rendered by the manager thread
        # GET /ready: (ready, reason) pushed to listeners (the web server) when it changes
        self._readiness: tuple[bool, str] = (False, "plugins not loaded yet")
        self._readiness_listeners: list = []
        # held while listeners are called, so a listener added during a change cannot
        # end up with the older state (listeners must not call back into the manager)
        self._readiness_lock = threading.Lock()
        self.canary_results: dict[tuple[int, int], tuple[float, dict]] = {}
        self._canary_owner: dict[tuple[int, int], str] = {}  # same keys -> identity of the GPU it ran on
        self._canary_lock = threading.Lock()
        # health latches persisted across plugin restarts (plugin/state.py)
        path = state_file_path(cfg)
        self._state = HealthState(path) if path else None
        self._reverify: set[str] = set()  # restored recovery-canary holds to verify once loaded
        # a /restart (or SIGHUP) is being served: once its reload is done every plugin that
        # kept its server registers again on the same socket (reference contract, see
        # _register_again): the monotonic time it was asked for, else None
        self._register_pending: float | None = None
        # identities whose next Healthy transition was verified already (the recovery canary
        # passed after a reset candidate): no second canary for it
        self._verified_clear: set[str] = set()

    # ------------------------------------------------------------ public API
    def restart(self) -> None:
        """Thread-safe restart request (``GET /restart``; reference ``Restart`` sets a racy bool)."""
        self.events.put((EV_RESTART, "api"))

    def stop(self) -> None:
        self.events.put((EV_STOP,))

    def clear_health(self, gpu: str, timeout: float = 10.0) -> tuple:
        """Thread-safe operator clear (``GET /health/clear?gpu=...``): drops the health
        latches of the GPU ``gpu`` names (identity/UUID, BDF, index or an advertised device
        ID) on the manager thread.  (HTTP status, data or message).  Raises TimeoutError
        when the manager does not answer within ``timeout``."""
        fut = concurrent.futures.Future()
        self.events.put((EV_CLEAR, str(gpu), fut))
        try:
            return fut.result(timeout)
        except concurrent.futures.TimeoutError:
            raise TimeoutError("manager busy") from None

    def add_readiness_listener(self, fn) -> None:
        """fn(ready, reason) now and on every change of the readiness ``GET /ready`` reports."""
        with self._readiness_lock:
            self._readiness_listeners.append(fn)
            fn(*self._readiness)

    def remove_readiness_listener(self, fn) -> None:
        with self._readiness_lock:
            if fn in self._readiness_listeners:
                self._readiness_listeners.remove(fn)

    def readiness(self) -> tuple:
        """Ready when every resource that has devices is registered with kubelet (the
        reference has no such signal: its /health answers ok whatever the plugins do)."""
        if self.fatal_error:
            return False, "fatal: %s" % self.fatal_error
        if not self._running.is_set():
            return False, "plugin manager not running"
        bound = float(self.cfg.health.discoveryTimeoutS)
        inflight = self._discoverer.inflight_s() if self._discoverer is not None else None
        if inflight is not None and inflight > bound + 1.0:
            return False, "discovery stalled: running for %.0f s%s" % (inflight, self._stuck_lanes_text())
        # a wedged GPU that `devices` leaves out is not this plugin's to wait for (ADVICE
        # r4): it is logged, but readiness (and so rolling updates) does not hang on it
        stale = [s for s in self._stale if self._serves(s[1])]
        if stale:
            idx, key, why = stale[0]
            more = " (and %d more GPU(s))" % (len(stale) - 1) if len(stale) > 1 else ""
            where = "GPU %d" % idx if idx >= 0 else "a GPU"
            return False, "discovery stalled on %s (%s): %s%s; %s" % (
                where, key, why, more, "advertising its last known description" if idx >= 0 else "not advertised")
        with_devices = [p for p in self.plugins if len(p)]
        if self._discovery_error:
            return False, "discovery failed: %s%s" % (self._discovery_error, "; the current plugins keep serving"
                                                       if with_devices else "")
        if not with_devices:
            return False, "no devices found" if self.device_map is not None else "plugins not loaded yet"
        missing = [str(p.resource) for p in with_devices if not p.registered]
        if missing:
            return False, "not registered with kubelet: %s" % ", ".join(missing)
        return True, ""

    def _serves(self, key: str) -> bool:
        """Whether the GPU with this identity is (or, before the first load, may be) in
        what this plugin advertises."""
        return parse_device_selector(self.cfg.devices) is None or not self._key_of or key in self._key_of.values()

    def _stuck_lanes_text(self) -> str:
        try:
            stuck = [(i, k, what, age) for i, k, what, age, _, _ in self.backend.lanes()
                     if what and age > float(self.cfg.health.sampleStallS or self.cfg.health.discoveryTimeoutS)]
        except Exception:  # pragma: no cover - every native backend has lanes
            return ""
        if not stuck:
            return ""
        i, k, what, age = max(stuck, key=lambda x: x[3])
        return "; GPU %d (%s): %s call in flight for %.0f s" % (i, k, what, age)

    def _push_readiness(self) -> None:
        state = self.readiness()
        with self._readiness_lock:
            if state == self._readiness:
                return
            self._readiness = state
            for fn in list(self._readiness_listeners):
                try:
                    fn(*state)
                except Exception as e:  # pragma: no cover - a listener must not stop the manager
                    log.error("readiness listener failed: %s", e)
        # an orderly stop is not a fault: only a running (or fatal) manager warns
        quiet = state[0] or (not self._running.is_set() and not self.fatal_error)
        (log.info if quiet else log.warning)("readiness: %s", "ready" if state[0] else state[1])

    @property
    def running(self) -> bool:
        return self._running.is_set()

    def wait_stopped(self, timeout: float | None = None) -> bool:
        return self._stopped.wait(timeout)

    def start(self) -> None:
        """Runs the manager loop in the calling thread until ``stop()``."""
        name_os_thread("manager")
        os.makedirs(self.cfg.pluginDir, exist_ok=True)
        self._running.set()
        try:
            self._restore_state()
            self._start_watch()
            self._discoverer = Discoverer(self.backend, lambda *r: self.events.put((EV_DISCOVERED,) + r))
            self._discoverer.request(DISCOVERY_RELOAD)
            # the first discovery is normally done in milliseconds: wait for it (bounded) and
            # handle what is queued by then, in order, so plugins are registered when start()
            # hands over to the loop; a stalled one is applied by the loop whenever it finishes
            if self._discoverer.first_done.wait(float(self.cfg.health.discoveryTimeoutS) + 1.0):
                while True:
                    try:
                        ev = self.events.get_nowait()
                    except queue.Empty:
                        break
                    if ev[0] == EV_STOP:
                        self.events.put(ev)  # the loop ends on it
                        break
                    self._handle(ev)
            self._start_telemetry()
            self.ready.close()
            self._loop()
        finally:
            self._shutdown()

    def start_background(self) -> threading.Thread:
        t = threading.Thread(target=self.start, name="plugin-manager", daemon=True)
        t.start()
        self.ready.wait(30)
        return t

    # ------------------------------------------------------------ loop
    def _check_servers(self) -> bool:
        """Supervises every plugin's gRPC server (polled about once a second, however
        busy the queue is).  Returns False when a plugin reached its crash limit: the
        manager then stops and the process exits non-zero."""
        restarted = False
        for p in self.plugins:
            try:
                if p.check_server():
                    restarted = True
                    self.counters["restarts_server"] = self.counters.get("restarts_server", 0) + 1
                    self.counters["registrations"] += 1
            except Exception as e:
                self.counters["load_failures"] += 1
                log.error("restarting the gRPC server of %s failed: %s; retrying in %.0fs", p.resource, e,
                          self.cfg.retrySeconds)
                self._arm_retry()
            if p.fatal_error:
                self.fatal_error = p.fatal_error
                log.critical("fatal: %s", p.fatal_error)
                return False
            restarted = self._check_stream(p) or restarted
        if restarted:
            self._publish_metrics()
        return True

    def _check_period(self) -> float:
        """Seconds to the next supervision pass: SERVER_CHECK_S while anything is in flux
        (not ready, a discovery running, a plugin unregistered or without its stream, a
        restart's Register pending, PodResources coverage to move on), else
        SERVER_CHECK_QUIET_S."""
        if (self.podres is not None or not self._readiness[0] or self._register_pending is not None
                or (self._discoverer is not None and self._discoverer.pending())):
            return SERVER_CHECK_S
        for p in self.plugins:
            if len(p) and (not p.registered or not p.serving or not p.law_had or p.law_lost_since is not None):
                return SERVER_CHECK_S
        return SERVER_CHECK_QUIET_S

    def _check_stream(self, p) -> bool:
        """Re-registers a plugin whose kubelet ListAndWatch stream ended and was not
        reopened within LAW_LOST_GRACE_S (kubelet dropped the endpoint without restarting:
        the reference recovered from this only on a /restart, which re-registered every
        plugin).  True if it registered again."""
        if not p.registered or not p.serving:
            return False
        try:
            open_streams = p.list_and_watch_streams()
        except Exception:  # pragma: no cover - a stopping server
            return False
        now = time.monotonic()
        if open_streams > 0:
            p.law_had, p.law_lost_since = True, None
            return False
        if not p.law_had:
            return False  # kubelet has not opened its stream since the last Register yet
        if p.law_lost_since is None:
            closed = p.list_and_watch_closed_at()  # when the stream ended (the poll may be late)
            p.law_lost_since = closed if 0 < closed <= now else now
        if now - p.law_lost_since < LAW_LOST_GRACE_S or not os.path.exists(self.cfg.kubelet_socket):
            return False
        if _socket_ident(p.socket) != p._sock_ident:
            # another instance bound this path since (an overlapping old/new pod): kubelet's
            # stream went to it.  Registering would make kubelet re-dial the path and tear
            # down the new instance's stream every grace period; leave the path to it (a
            # deleted socket is EV_SOCKET_GONE's business)
            if p.law_lost_since is not None and not getattr(p, "_socket_taken_logged", False):
                p._socket_taken_logged = True
                self.counters["stream_watch_socket_taken"] = self.counters.get("stream_watch_socket_taken", 0) + 1
                log.warning("the socket %s of %s is no longer the one this process bound (another instance "
                            "serves it): not registering again", p.socket, p.resource)
            return False
        failures = getattr(p, "_reregister_failures", 0)
        if not failures:
            log.warning("kubelet ended the ListAndWatch stream of %s %.0f s ago and did not open another: "
                        "registering again", p.resource, now - p.law_lost_since)
        try:
            p.register()
        except Exception as e:
            p.law_lost_since = now  # try again after another grace period
            p._reregister_failures = failures + 1
            # a kubelet that is down but left its socket: one error, then quiet retries
            (log.error if not failures else log.debug)("registering %s again failed: %s", p.resource, e)
            return False
        p._reregister_failures = 0
        self.counters["reregistrations_stream_lost"] = self.counters.get("reregistrations_stream_lost", 0) + 1
        self.counters["registrations"] += 1
        return True

    def _loop(self) -> None:
        next_check = time.monotonic() + SERVER_CHECK_S
        while True:
            now = time.monotonic()
            if now >= next_check:
                if not self._check_servers():
                    return
                # readiness follows plugin state and stalls that no event announces (a
                # discovery running past its bound, a server that lost its registration)
                self._push_readiness()
                if self.podres is not None:  # PodResources' coverage moves on with every poll,
                    # changed map or not (its grace keeps a just-answered Allocate counted)
                    self.recent_allocations.set_covered_until(self.podres.covered_until())
                next_check = now + self._check_period()
            try:
                ev = self.events.get(timeout=max(0.0, next_check - now))
            except queue.Empty:
                continue
            if ev[0] == EV_STOP:
                log.info("plugin server stopped")
                return
            if ev[0] == EV_SUPERVISE:
                next_check = 0.0
                continue
            self._handle(ev)

    # ------------------------------------------------------------ persisted latches
    def _restore_state(self) -> None:
        """Re-applies the latches the previous process of this boot persisted, before the
        first discovery: a GPU it held Unhealthy is never advertised Healthy in between."""
        if self._state is None:
            return
        snap = self._state.load()
        if not snap:
            return
        n = native.load()
        latches = [n.HealthLatch(k, e["last_ue"], float("nan") if e["fw_boot_s"] is None else e["fw_boot_s"],
                                 e["reason"], e["since_ns"])
                   for k, e in sorted(snap["ecc"].items())]
        if latches:
            self.monitor.restore_latches(latches)
        self._canary_failed = {(k, p) for k, parts in snap["canary_failed"].items() for p in parts}
        if self.cfg.health.canary:
            self._held_unhealthy |= set(snap["held"])
            self._reverify |= set(snap["held"])
        restored = len(latches) + len(self._canary_failed) + len(snap["held"])
        self.counters["latches_restored"] = restored
        if restored:
            log.warning("restored health latches from %s: uncorrectable ECC on %s; failed canaries on %s; "
                        "recovery canary held on %s", self._state.path,
                        ", ".join(e.key for e in latches) or "none",
                        ", ".join("%s/%d" % kp for kp in sorted(self._canary_failed)) or "none",
                        ", ".join(sorted(snap["held"])) or "none")

    def _state_snapshot(self) -> dict:
        ecc = {}
        for l in self.monitor.latches():
            fw = float(l.fw_boot_s)  # NaN: the firmware clock was never seen advancing
            ecc[l.key] = {"last_ue": int(l.last_ue), "fw_boot_s": None if fw != fw else round(fw),
                          "reason": l.reason, "since_ns": int(l.since_ns)}
        failed: dict = {}
        for k, part in self._canary_failed:
            failed.setdefault(k, set()).add(part)
        return {"ecc": ecc, "canary_failed": {k: sorted(v) for k, v in failed.items()},
                "held": sorted(self._held_unhealthy)}

    def _save_state(self) -> None:
        if self._state is None:
            return
        try:
            if self._state.save(self._state_snapshot()):
                self.counters["state_writes"] = self._state.writes
            elif self._state.write_errors:
                self.counters["state_write_errors"] = self._state.write_errors
        except Exception as e:  # pragma: no cover - persistence never stops the manager
            log.error("persisting health latches failed: %s", e)

    def _handle(self, ev) -> None:
        kind = ev[0]
        try:
            if kind == EV_RESTART:
                self.counters["restarts_" + ev[1]] = self.counters.get("restarts_" + ev[1], 0) + 1
                log.info("restarting plugins (%s)", ev[1])
                kubelet = self._coalesce_restarts()
                if kubelet:
                    self._reregister()
                elif self._register_pending is None:
                    self._register_pending = time.monotonic()
                self._request_discovery(DISCOVERY_RELOAD)
            elif kind == EV_KUBELET:
                self.counters["restarts_kubelet"] += 1
                log.info("kubelet.sock re-created: kubelet restarted; re-registering")
                self._coalesce_restarts()
                self._reregister()
                self._request_discovery(DISCOVERY_CHECK)
            elif kind == EV_DISCOVERED:
                self._apply_discovery(*ev[1:])
            elif kind == EV_RETRY:
                self.counters["restarts_retry"] += 1
                self._retry_timer = None
                if not self.plugins or self._discovery_error:
                    self._request_discovery(DISCOVERY_RELOAD)
                else:
                    self.start_plugins()
            elif kind == EV_HEALTH:
                self._apply_health(ev[1])
            elif kind == EV_VERIFIED:
                self._apply_verified(*ev[1:])
            elif kind == EV_PODRES:
                self._push_link_pods()  # and _publish_metrics below re-renders the allocation map
            elif kind == EV_METRICS:
                pass  # canary results changed: _publish_metrics below re-renders
            elif kind == EV_PRESTART_FAIL:
                self.counters["prestart_failures"] = self.counters.get("prestart_failures", 0) + 1
                self._canary_failed.add((ev[1], ev[2]))  # (identity, partition)
                self._set_health(ev[1], ev[2], False, ev[3])
            elif kind == EV_REDISCOVER:
                self._request_discovery(DISCOVERY_CHECK)
            elif kind == EV_SOCKET_GONE:
                self._socket_gone(ev[1])
            elif kind == EV_START_CANARY:
                self._apply_start_canary(*ev[1:])
            elif kind == EV_CLEAR:
                self._clear_health(*ev[1:])
            elif kind == EV_CANDIDATE_VERIFIED:
                self._apply_candidate_verified(*ev[1:])
        except Exception as e:
            self.counters["load_failures"] += 1
            log.error("event %s failed: %s; retrying in %.0fs", kind, e, self.cfg.retrySeconds)
            self._arm_retry()
            if kind == EV_CLEAR and not ev[2].done():
                ev[2].set_result((500, "clearing failed: %s" % e))
        if kind in (EV_HEALTH, EV_VERIFIED, EV_PRESTART_FAIL, EV_DISCOVERED, EV_START_CANARY, EV_CLEAR,
                    EV_CANDIDATE_VERIFIED):
            self._sync_held()
            self._save_state()
        self._publish_metrics()

    def _coalesce_restarts(self) -> bool:
        """Takes the restart requests (``GET /restart``, kubelet re-creations) that are
        already queued behind the one being handled: one reload serves them all, so a
        burst of /restart calls cannot keep the manager reloading (the reference's
        ``Restart()`` sets a flag, which coalesces too).  Every request is still counted;
        other events keep their order.  True when a kubelet restart was among them."""
        n = 0
        kubelet = False
        with self.events.mutex:  # queue.Queue's own lock: nothing else runs meanwhile
            q = self.events.queue
            keep = collections.deque()
            while q:
                ev = q.popleft()
                if ev[0] == EV_RESTART:
                    key = "restarts_" + ev[1]
                elif ev[0] == EV_KUBELET:
                    key = "restarts_kubelet"
                    kubelet = True
                else:
                    keep.append(ev)
                    continue
                self.counters[key] = self.counters.get(key, 0) + 1
                n += 1
            q.extend(keep)
        if n:
            self.counters["restarts_coalesced"] = self.counters.get("restarts_coalesced", 0) + n
            log.info("%d more restart request(s) served by this reload", n)
        return kubelet

    def _socket_gone(self, name: str) -> None:
        """A plugin's own socket was deleted while it serves (an operator or a cleanup
        job wiping the directory; the reference would keep serving on an unreachable
        socket until the next kubelet restart): serve again on a fresh socket and
        re-register.  The plugin's own stop removes its socket too; by the time this
        event is handled the reload that did so has bound the new one, so the file
        exists and nothing happens."""
        for p in self.plugins:
            if os.path.basename(p.socket) != name or not p.serving or os.path.exists(p.socket):
                continue
            self.counters["restarts_socket"] = self.counters.get("restarts_socket", 0) + 1
            log.warning("plugin socket %s was removed; serving again and re-registering", p.socket)
            p.stop()
            self.start_plugins()

    # ------------------------------------------------------------ plugins
    def load_plugins(self, gpus=None, topo=None) -> None:
        """Builds the plugins for a discovery (``gpus``/``topo``; a synchronous discovery
        when not given), then puts them in service.  Everything that can fail - discovery,
        resources, device map, tables - happens before anything that serves changes: a
        failure leaves the current plugins serving (make-before-break).

        A resource that keeps its name keeps its socket, server and kubelet registration:
        its new table is swapped into the running server, whose ListAndWatch streams push
        the new device list at once (reference ``restartPlugins`` stops every server and
        starts new ones, ``plugin/manager.go:177-194``, so kubelet's endpoint is gone for a
        moment on every reload and an admission landing then fails).  Only resources that
        disappeared stop; only new ones start (``start_plugins``)."""
        if gpus is None:
            gpus, topo = self.backend.discover()
            self._note_report(self.backend.last_discovery() if hasattr(self.backend, "last_discovery") else None)
        self._note_seen(gpus)
        node = gpus
        sel = self._selected(gpus)
        resources = new_resources(sel, self.cfg.strategy, self.cfg.resourcePrefix, self.cfg.resources)
        device_map = build_device_map(sel, resources, self.cfg.strategy, self.cfg.mountCardNodes,
                                      self.cfg.sharing.replicas, self.cfg.sharing.renameByDefault)
        key_of = {g.index: self._identity(g) for g in sel}
        index_of = {k: i for i, k in key_of.items()}
        node_keys = {self._identity(g) for g in node}
        canary_jobs = self._plan_startup_canary(sel, key_of, node_keys, device_map) \
            if self.cfg.health.canaryOnStart else []
        # partitions held Unhealthy by a canary: failed before, or a start-up verdict pending
        held = self._canary_failed | self._start_pending
        failed = {(index_of[k], p) for k, p in held if k in index_of}
        plugins = [AmdDevicePlugin(name, devs, topo, self.cfg) for name, devs in device_map.items()]
        events = self.events  # (the hook holds the queue only: no cycle through the server)
        for p in plugins:
            p.table.set_recent_allocations(self.recent_allocations)
            p.on_server_fault = lambda: events.put((EV_SUPERVISE,))
        if self.cfg.health.canaryOnPreStart:
            for p in plugins:
                p.prestart_check = self._prestart_check
        # canary verdicts are per partition and known only here
        for p in plugins:
            for gpu, part in failed:
                p.set_gpu_health(gpu, part, False)
        # Health state survives a reload.  The monitor installs the new tables and writes
        # its current state into them under the lock that orders its transitions, so an
        # event that lands during the reload reaches the new tables either way (reading
        # gpu_healthy() here and calling set_fast_tables() later left a window in which
        # it reached only the outgoing ones).
        keys = [""] * (max([g.index for g in sel], default=-1) + 1)
        for i, k in key_of.items():
            keys[i] = k
        self.monitor.set_gpus(keys)
        self._sync_held()
        self.monitor.attach_tables([p.table for p in plugins], not self.cfg.health.canary,
                                   sorted(index_of[k] for k in self._held_unhealthy if k in index_of))
        # the new tables carry every health verdict: put them in service.  A resource that
        # stays takes over the running server of its predecessor (table swap, no socket
        # change); readers of self.plugins see the old list until then, never an empty one
        old = {str(p.resource): p for p in self.plugins}
        swapped = 0
        for p in plugins:
            prev = old.pop(str(p.resource), None)
            if prev is not None and prev.serving and not prev.fatal_error:
                try:
                    p.adopt(prev)
                    swapped += 1
                    continue
                except Exception as e:  # the fresh plugin starts in start_plugins instead
                    log.error("swapping the device table of %s into its server failed: %s", p.resource, e)
            if prev is not None:
                self._stop_plugin(prev)
        for prev in old.values():  # resources that are gone
            self._stop_plugin(prev)
        if swapped:
            self.counters["table_swaps"] = self.counters.get("table_swaps", 0) + swapped
        self._node_index_of = {self._identity(g): g.index for g in node}
        self.gpus, self.topology = sel, topo
        self.signature = self._signature(node, sel)
        self.device_map = device_map
        self._key_of, self._index_of = key_of, index_of
        gpus = sel
        self.counters["reloads"] = self.counters.get("reloads", 0) + 1
        self.plugins = plugins
        for job in canary_jobs:
            self._start_canary_pool().submit(self._startup_canary_job, *job)
        for key in [k for k in self._reverify if k in index_of]:
            self._reverify.discard(key)
            self._verify_later(key, -1, "recovery canary held when the previous plugin process stopped")
        n = native.load()
        labels = []
        hips = {(g.index, p.index): p.hip_id for g in gpus for p in g.partitions}
        for name, devs in self.device_map.items():
            for d in devs:
                if d.replica <= 0:
                    spans = sorted(h for (gi, pi), h in hips.items()
                                   if gi == d.gpu and (d.partition < 0 or pi == d.partition) and h >= 0)
                    labels.append(n.PartitionLabel(d.gpu, d.partition, d.get_uuid(), name,
                                                   ",".join(str(h) for h in spans)))
        if self.cfg.cdi:
            from ..cdi import build_spec, write_spec
            for name, devs in self.device_map.items():
                try:
                    write_spec(self.cfg.cdiSpecDir, build_spec(name, devs))
                except OSError as e:
                    log.error("cannot write CDI spec for %s to %s: %s", name, self.cfg.cdiSpecDir, e)
        if self.cfg.nodeFeatureFile:
            from ..labels import node_labels, write_feature_file
            try:
                write_feature_file(self.cfg.nodeFeatureFile, node_labels(gpus))
            except OSError as e:
                log.error("cannot write node feature file %s: %s", self.cfg.nodeFeatureFile, e)
        # retired-page limit per GPU: config override, else the GPU's own RAS threshold
        limit = int(self.cfg.health.badPageThreshold)
        for g in gpus:
            g.bad_page_threshold = limit if limit > 0 else (g.bad_page_threshold if limit == 0 else -1)
        thresholds = [-1] * (max([g.index for g in gpus], default=-1) + 1)
        for g in gpus:
            thresholds[g.index] = g.bad_page_threshold
        self.monitor.set_bad_page_thresholds(thresholds)
        if self._event_sources is not None:
            self._event_sources = getattr(self.backend, "armed_event_sources", None)
        with self._canary_lock:  # results of partitions that no longer exist leave /metrics,
            # and so do those of a GPU whose index another GPU holds after a re-enumeration
            live = {(g.index, p.index) for g in gpus for p in g.partitions}
            for k in [k for k in self.canary_results
                      if k not in live or self._canary_owner.get(k, self._key_of.get(k[0])) != self._key_of.get(k[0])]:
                del self.canary_results[k]
                self._canary_owner.pop(k, None)
        self._push_link_pods()  # the new tables start from the known allocation map
        self.exporter.set_inventory(gpus)
        self.exporter.set_partition_labels(labels)
        self.exporter.set_tables([p.table for p in plugins])
        log.info("loaded %d GPU(s), resources: %s", len(gpus),
                 ", ".join("%s=%d" % (k, len(v)) for k, v in self.device_map.items()) or "none")

    def start_plugins(self) -> None:
        started = 0
        for p in self.plugins:
            if len(p) == 0 or p.registered:
                continue
            try:
                p.start()
                started += 1
                self.counters["registrations"] += 1
            except Exception as e:
                log.error("failed to start plugin %s: %s", p.resource, e)
                log.info("Failed to start one or more plugins. Retrying in %.0fs...", self.cfg.retrySeconds)
                self._arm_retry()
                return
        if not any(len(p) for p in self.plugins):
            log.info("No devices found. Waiting indefinitely.")
        elif started:
            log.info("All plugins started.")

    def stop_plugins(self) -> None:
        for p in self.plugins:
            try:
                p.stop()
            except Exception as e:  # pragma: no cover
                log.error("failed to stop plugin %s: %s", p.resource, e)

    def restart_plugins(self, gpus=None, topo=None) -> None:
        """Reload (make-before-break, see load_plugins) and register the new plugins."""
        self._cancel_retry()
        self.load_plugins(gpus, topo)
        self.start_plugins()

    def _request_discovery(self, purpose: str) -> None:
        if self._discoverer is None:  # not started (direct callers): synchronous
            gpus, topo = self.backend.discover()
            self._apply_discovery(purpose, gpus, topo, self.backend.last_discovery()
                                  if hasattr(self.backend, "last_discovery") else None, None)
            return
        self._discoverer.request(purpose)

    def _note_report(self, report) -> None:
        stale = list(report["stale"]) if report else []
        # the GPU whose own call is stuck first (behind a library-wide lock the others only
        # wait for it)
        stalled = set(self.exporter.stalled_gpus)
        stale.sort(key=lambda x: (x[0] not in stalled, x[0] < 0, x[0]))
        for idx, key, why in stale:
            if (idx, key, why) not in self._stale:
                log.warning("discovery could not reach GPU %s (%s): %s; %s", idx if idx >= 0 else "?", key, why,
                            "serving its last known description" if idx >= 0 else "left out")
        if stale:
            self.counters["discovery_stale"] = self.counters.get("discovery_stale", 0) + 1
        elif self._stale:
            log.info("discovery reaches every GPU again")
        self._stale = stale

    def _apply_discovery(self, purpose, gpus, topo, report, err) -> None:
        """A finished discovery (worker thread, via the queue).  Failure: what serves keeps
        serving.  Success: reload if asked to, or if the inventory changed."""
        if err is not None:
            self.counters["load_failures"] += 1
            self._discovery_error = str(err)
            log.error("discovery failed: %s; %s, retrying in %.0fs", err,
                      "the current plugins keep serving" if self.plugins else "nothing advertised yet",
                      self.cfg.retrySeconds)
            self._arm_retry()
            self._register_again()  # what serves still answers: kubelet is pointed at it again
            return
        self._discovery_error = None
        self._note_report(report)
        self._note_seen(gpus)
        changed = self._signature(gpus, self._selected(gpus)) != self.signature
        if purpose == DISCOVERY_CHECK and self.plugins and not changed:
            if any(not p.registered for p in self.plugins if len(p)):
                self.start_plugins()
            return
        if purpose == DISCOVERY_CHECK and self.plugins:
            self.counters["restarts_inventory"] = self.counters.get("restarts_inventory", 0) + 1
            log.warning("device inventory changed (partition mode or GPU set); re-advertising")
        self.restart_plugins(gpus, topo)
        self._register_again()

    def _register_again(self) -> None:
        """The end of a ``GET /restart`` (or SIGHUP): every plugin that kept its server
        through the reload sends ``Register`` again for its still-served socket.  The
        reference's restart always ends in a fresh Register (``router/api.go:50-54`` ->
        ``plugin/manager.go:177-194`` -> ``plugin/plugin.go:140-162``), which is the
        operator's way out when kubelet's view of a plugin went wrong (allocatable 0, a
        stale endpoint) while its stream may still be open.  The socket is not dropped:
        kubelet dials the same endpoint again and reopens ListAndWatch, so admissions keep
        finding it.  A plugin that registered after the restart was asked for (started by this
        reload, or re-registered by a kubelet restart) is skipped."""
        since = self._register_pending
        if since is None:
            return
        self._register_pending = None
        for p in self.plugins:
            # (one that registered after the restart was asked for has met it already)
            if not len(p) or not p.serving or not p.registered or p.registered_at >= since:
                continue
            try:
                p.register()
            except Exception as e:
                p.registered = False  # start_plugins (the retry timer) registers it later
                log.error("registering %s again after the restart failed: %s; retrying in %.0fs", p.resource, e,
                          self.cfg.retrySeconds)
                self._arm_retry()
                continue
            self.counters["registrations"] += 1
            self.counters["reregistrations_restart"] = self.counters.get("reregistrations_restart", 0) + 1
            log.info("registered %s again on its running socket (restart)", p.resource)

    def _reregister(self) -> None:
        """A kubelet restart drops every registration (and kubelet clears the plugin
        sockets): serve the current plugins on fresh sockets and register them again at
        once - no discovery on this path, so a wedged GPU cannot delay it."""
        self._cancel_retry()
        for p in self.plugins:
            if len(p):
                p.stop()
        self.start_plugins()

    def _signature(self, node, selected) -> tuple:
        """The advertised set, plus which GPUs the node enumerates where: a GPU that
        `devices` leaves out still has links in the tables' topology."""
        return inventory_signature(selected), tuple((self._identity(g), g.index) for g in node)

    def _note_seen(self, gpus) -> None:
        for g in gpus:
            if g.bdf:
                self._seen_bdfs[g.bdf.lower()] = self._identity(g)

    def _selected(self, gpus) -> list:
        """The GPUs `devices` selects.  An index names a GPU by its BDF rank among every
        GPU this process has seen, not by its position in one enumeration, and once an
        index has been advertised it stays pinned to that GPU's identity: a
        GPU that drops off the bus leaves its index empty (the selection does not take in
        the next GPU), and one that appears later with a lower BDF does not push a served
        GPU that a pod holds out of the selection; it is logged and counted
        (``devices_index_conflicts``) instead.  While no pod holds the pinned GPU the late
        one takes its index back (``devices_index_reresolved``): a GPU missing
        from the first discovery does not lose its index for the life of the process.  Indices never resolved are filled as GPUs
        appear.  UUIDs and BDFs are matched as given, and ``hip:<n>`` selects the GPU a
        HIP ordinal opens."""
        sel = parse_device_selector(self.cfg.devices)
        if sel is None:
            return list(gpus)
        indices, names = sel
        hips = {int(x[4:]) for x in names if x.startswith("hip:")}
        if hips and not any(p.hip_id >= 0 for g in gpus for p in g.partitions):
            # the driver reports no HIP ordinals: the HIP runtime numbers GPUs in PCI order
            # unless told otherwise, so hip:<n> falls back to BDF rank n
            if not self._hip_fallback_logged:
                log.warning("devices %r: no HIP ordinals reported; hip:<n> selects by BDF rank", self.cfg.devices)
                self._hip_fallback_logged = True
            indices = sorted(set(indices) | hips)
        rank = {bdf: i for i, bdf in enumerate(sorted(self._seen_bdfs))}
        by_key = {self._identity(g): g for g in gpus}
        picked = set()
        for i in sorted(indices):
            at_rank = [g for g in gpus if rank.get((g.bdf or "").lower(), -1) == i]
            pinned = self._pinned_index.get(i)
            if pinned is not None and at_rank and self._identity(at_rank[0]) != pinned:
                newk = self._identity(at_rank[0])
                if newk not in self._pinned_index.values() and not self._pinned_gpu_in_use(pinned):
                    # a GPU that enumerated late (missing from an earlier discovery) takes
                    # its index back while no pod holds the GPU that stood in for it
                    # 
                    self._pinned_index[i] = newk
                    picked.add(newk)
                    self.counters["devices_index_reresolved"] = self.counters.get("devices_index_reresolved", 0) + 1
                    log.warning("devices %r: index %d now names %s (ranks %d by BDF); %s, which held it, is "
                                "not allocated to any pod", self.cfg.devices, i, newk, i, pinned)
                    continue
            if pinned is not None:
                if pinned in by_key:
                    picked.add(pinned)
                if at_rank and self._identity(at_rank[0]) != pinned:
                    moved = (i, self._identity(at_rank[0]))
                    if moved not in self._index_conflicts:
                        self._index_conflicts.add(moved)
                        self.counters["devices_index_conflicts"] = self.counters.get("devices_index_conflicts", 0) + 1
                        log.warning("devices %r: index %d is pinned to %s, which a pod holds; %s now ranks %d by "
                                    "BDF and is not selected until no pod holds %s", self.cfg.devices, i, pinned,
                                    moved[1], i, pinned)
                continue
            if at_rank:
                k = self._identity(at_rank[0])
                if k not in self._pinned_index.values():
                    self._pinned_index[i] = k
                    picked.add(k)
        out = [g for g in gpus if self._identity(g) in picked
               or (g.uuid or "").lower() in names or (g.bdf or "").lower() in names
               or any(p.hip_id >= 0 and "hip:%d" % p.hip_id in names for p in g.partitions)]
        chosen = tuple(self._identity(g) for g in out)
        if chosen != self._selection:
            log.info("devices %r selects %s", self.cfg.devices, ", ".join(chosen) or "nothing (yet)")
            self._selection = chosen
        return out

    def _pinned_gpu_in_use(self, key: str) -> bool:
        """Whether a pod holds a device of the advertised GPU ``key`` (PodResources when
        polled, else kubelet's device checkpoint).  A GPU never advertised is not held."""
        idx = self._index_of.get(key)
        if idx is None or not self.device_map:
            return False
        return any(g == idx for g, _ in self._in_use_partitions(self.device_map))

    # ------------------------------------------------------------ health
    def _identity(self, g) -> str:
        """The key health state is kept under: the backend's own (the monitor uses the
        same), else the GPU's UUID or BDF."""
        k = ""
        try:
            k = self.backend.gpu_key(g.index)
        except Exception:  # pragma: no cover - every native backend implements it
            pass
        return k or g.uuid or g.bdf or "#%d" % g.index

    def _key(self, u) -> str:
        return getattr(u, "key", "") or self._key_of.get(u.gpu, "#%d" % u.gpu)

    def _gpu_name(self, key: str) -> str:
        i = self._index_of.get(key)
        return "GPU %d (%s)" % (i, key) if i is not None else "GPU %s (not advertised)" % key

    def _apply_health(self, u) -> None:
        n = native.load()
        self.counters["health_events"] += 1
        if u.kind == n.EVT_RESET_OBSERVED:  # a reset seen by polling, not by an event
            self.counters["resets_observed"] = self.counters.get("resets_observed", 0) + 1
        key = self._key(u)
        if u.kind == n.EVT_RESET_CANDIDATE:
            self._reset_candidate(key, u.reason)
            return
        if u.healthy in (0, 1):
            healthy = bool(u.healthy)
            gen = self._health_gen[key] = self._health_gen.get(key, 0) + 1
            if healthy and key in self._verified_clear:
                # the recovery canary that cleared these latches has just passed: no second run
                self._verified_clear.discard(key)
                self._held_unhealthy.discard(key)
                self._set_health(key, u.partition, True, u.reason, apply=self.cfg.health.canary)
                return
            if healthy and self.cfg.health.canary:
                # stay Unhealthy until the canary passes; do not block the event loop on it
                log.info("%s reports healthy (%s); verifying with the canary", self._gpu_name(key), u.reason)
                self._held_unhealthy.add(key)
                if self._verify_pool is None:
                    self._verify_pool = concurrent.futures.ThreadPoolExecutor(max_workers=4,
                                                                              thread_name_prefix="canary",
                                                                              initializer=background_thread)
                self._verify_pool.submit(self._verify_and_post, u, key, gen)
                return
            if healthy:
                self._held_unhealthy.discard(key)
            # without the canary the monitor thread already applied both directions to
            # the tables; re-applying a queued update here could briefly undo a newer one
            self._set_health(key, u.partition, healthy, u.reason, apply=self.cfg.health.canary)
        elif u.link_up in (0, 1):
            a, b = self._link_ends(u, key)
            if a < 0 or b < 0:  # an end the node no longer enumerates
                log.debug("xGMI link %s<->%s %s (GPU gone)", key, getattr(u, "peer_key", "") or u.peer,
                          "up" if u.link_up else "down")
                return
            if not self.plugins or self.plugins[0].table.topology().link(a, b).up == bool(u.link_up):
                return  # the tables agree (every link is reported once more after a reload)
            for p in self.plugins:
                p.set_link_up(a, b, bool(u.link_up))
            log.warning("xGMI link %d<->%d %s", a, b, "up" if u.link_up else "down")
        elif u.kind == native.load().EVT_LINK_QUALITY:
            a, b = self._link_ends(u, key)
            if a < 0 or b < 0 or not self.plugins:
                return
            cur = self.plugins[0].table.topology().link(a, b).bw_gbps
            if cur > 0 and abs(cur - u.link_gbps) <= 0.05 * max(cur, u.link_gbps):
                return  # what discovery found (the first reading of every link lands here)
            for p in self.plugins:
                p.set_link_bandwidth(a, b, u.link_gbps)
            log.warning("xGMI link %d<->%d trains at %.0f Gb/s (was %.0f): %s", a, b, u.link_gbps, cur, u.reason)
        else:
            log.info("GPU event on %s: %s", self._gpu_name(key), u.reason)

    def _link_ends(self, u, key: str) -> tuple:
        """Topology indices of a link event's two GPUs (-1: not in the node)."""
        peer = getattr(u, "peer_key", "") or self._key_of.get(u.peer, "")
        return self._node_index_of.get(key, -1), self._node_index_of.get(peer, -1)

    def _push_link_pods(self) -> None:
        """Which GPU pairs' xGMI links already carry a multi-GPU pod (from the PodResources
        allocation map): the allocator keeps a new pod's cross-GPU traffic off them when it
        can (in CPX/QPX/DPX two pods that each span GPUs A and B
        share the one A-B link)."""
        if self.podres is None or not self.plugins:
            return
        allocs, _ = self.podres.snapshot()
        # allocations answered before that poll are in its map now
        self.recent_allocations.set_covered_until(self.podres.covered_until())
        gpu_of = {}
        for p in self.plugins:
            for d in p.devices():
                gpu_of[(str(p.resource), d.id)] = d.gpu
        spans = {}
        for (res, dev), (ns, pod, _ctr) in allocs.items():
            g = gpu_of.get((res, dev))
            if g is not None and g >= 0:
                spans.setdefault((ns, pod), set()).add(g)
        # the tables' topology spans every discovered GPU, also those `devices` leaves out
        n = self.topology.n if self.topology is not None else max([g.index for g in self.gpus], default=-1) + 1
        load = [0] * (n * n)
        multi = 0
        for gs in spans.values():
            if len(gs) < 2:
                continue
            multi += 1
            for a, b in itertools.combinations(sorted(gs), 2):
                load[a * n + b] += 1
                load[b * n + a] += 1
        for p in self.plugins:
            p.set_link_pods(load)
        self.link_pods = {(a, b): load[a * n + b] for a in range(n) for b in range(a + 1, n) if load[a * n + b]}
        self.multi_gpu_pods = multi

    def _set_health(self, key: str, partition: int, healthy: bool, reason: str, apply: bool = True) -> None:
        if healthy:  # a recovery supersedes earlier canary verdicts on this GPU
            self._canary_failed = {k for k in self._canary_failed if k[0] != key}
            self._sync_held()
        gpu = self._index_of.get(key, -1)
        if gpu >= 0 and apply:  # else the monitor thread has already written the tables
            held = {part for k, part in self._start_pending if k == key} if healthy else ()
            if -1 in held:
                return  # the whole GPU waits for its start-up canary
            for p in self.plugins:
                p.set_gpu_health(gpu, partition, healthy, held)
        self.health_log.append((time.monotonic(), gpu, int(healthy), reason))
        (log.info if healthy else log.warning)("%s marked %s: %s", self._gpu_name(key),
                                               "Healthy" if healthy else "Unhealthy", reason)

    def _verify_and_post(self, u, key: str, gen: int) -> None:
        try:
            ok = self._canary_ok(key)
        except Exception as e:  # a canary that cannot run does not prove health
            log.error("recovery canary on %s could not run: %s", self._gpu_name(key), e)
            ok = False
        self.events.put((EV_VERIFIED, u, key, gen, ok))

    def _apply_verified(self, u, key: str, gen: int, ok: bool) -> None:
        if self._health_gen.get(key) != gen:
            log.info("dropping stale canary verdict for %s (newer health event)", self._gpu_name(key))
            return
        if ok:
            self._held_unhealthy.discard(key)
        self._set_health(key, u.partition, ok, u.reason + ("" if ok else "; canary failed"))

    def _stop_plugin(self, p) -> None:
        try:
            p.stop()
        except Exception as e:  # pragma: no cover
            log.error("failed to stop plugin %s: %s", p.resource, e)

    def _start_canary_pool(self) -> concurrent.futures.ThreadPoolExecutor:
        if self._canary_pool is None:
            self._canary_pool = concurrent.futures.ThreadPoolExecutor(max_workers=8, thread_name_prefix="canary-start",
                                                                      initializer=background_thread)
        return self._canary_pool

    def _in_use_partitions(self, device_map) -> set:
        """(gpu, partition) pairs a container holds, as far as this process can tell: the
        kubelet PodResources map when it is polled, else kubelet's device checkpoint in the
        plugin directory (it lists every device kubelet has handed to a pod)."""
        ids = set()
        if self.podres is not None:
            allocs, up = self.podres.snapshot()
            if up:
                ids |= {(res, dev.split("::")[0]) for res, dev in allocs}
        if not ids:
            from .podresources import checkpoint_allocations
            ids = {(res, dev.split("::")[0]) for res, dev in
                   checkpoint_allocations(os.path.join(self.cfg.pluginDir, "kubelet_internal_checkpoint"),
                                          self.cfg.resourcePrefix)}
        out = set()
        for name, devs in device_map.items():
            for d in devs:
                if (name, d.id.split("::")[0]) in ids:
                    out.add((d.gpu, d.partition))
        return out

    def _plan_startup_canary(self, sel, key_of, node_keys, device_map) -> list:
        """health.canaryOnStart: the partitions to canary before they are advertised
        Healthy - those of each GPU identity this process advertises for the first time
        (a plain /restart or reload runs none; a GPU that left the node and came back runs
        it again), except partitions a container holds already (a plugin restart on a busy
        node must not run the canary next to a job, nor fail it on the memory the job
        holds).  Marked pending: they are advertised Unhealthy until their verdict."""
        self._start_canaried &= node_keys
        in_use = self._in_use_partitions(device_map) if any(key_of[g.index] not in self._start_canaried
                                                               for g in sel) else set()
        jobs = []
        for g in sel:
            key = key_of[g.index]
            if key in self._start_canaried:
                continue
            self._start_canaried.add(key)
            for p in g.partitions:
                part = p.index if len(g.partitions) > 1 else -1
                if (g.index, part) in in_use or (g.index, -1) in in_use:
                    self.counters["canary_skipped_in_use"] = self.counters.get("canary_skipped_in_use", 0) + 1
                    log.info("start-up canary skips GPU %d partition %d: a container holds it", g.index, part)
                    continue
                self._start_pending.add((key, part))
                jobs.append((key, g.index, part, p.index, p.hip_id))
        return jobs

    def _startup_canary_job(self, key: str, gpu: int, part: int, hw_part: int, hip: int) -> None:
        """Pool thread: one partition's start-up canary; the verdict goes back as an event."""
        try:
            res = self._run_canary(gpu, hw_part, hip, key)
            ok, why = bool(res.get("ok")), res.get("error") or ("" if res.get("ok") else str(res))
        except Exception as e:  # a canary that cannot run does not pass the partition
            ok, why = False, "canary could not run: %s" % e
        self.events.put((EV_START_CANARY, key, part, ok, why))

    def _apply_start_canary(self, key: str, part: int, ok: bool, why: str) -> None:
        if (key, part) not in self._start_pending:
            return  # the GPU left the node meanwhile
        self._start_pending.discard((key, part))
        gpu = self._index_of.get(key, -1)
        if not ok:
            self._canary_failed.add((key, part))
            self._sync_held()
            # it was advertised Unhealthy while pending, but a recovery in between may have
            # written the GPU Healthy: the verdict is applied to the tables, not assumed
            if gpu >= 0:
                for p in self.plugins:
                    p.set_gpu_health(gpu, part, False)
            self._count("canary_failures")
            log.error("start-up canary failed on %s partition %d: %s", self._gpu_name(key), part, why)
            return
        self._canary_failed.discard((key, part))  # a fresh verdict replaces an older one
        if gpu >= 0 and self.monitor.gpu_healthy(gpu) and key not in self._held_unhealthy:
            for p in self.plugins:
                p.set_gpu_health(gpu, part, True)
        log.info("start-up canary passed on %s partition %d", self._gpu_name(key), part)

    def _sync_held(self) -> None:
        """Tells the monitor which partitions a recovery must leave Unhealthy: failed
        canary verdicts and start-up verdicts still pending (its fast path writes Healthy
        transitions to the tables itself)."""
        held: dict = {}
        for k, part in self._canary_failed | self._start_pending:
            held.setdefault(k, set()).add(part)
        snap = {k: sorted(v) for k, v in held.items()}
        if snap != getattr(self, "_held_pushed", None):
            self.monitor.set_held_partitions(snap)
            self._held_pushed = snap

    def _reset_candidate(self, key: str, reason: str) -> None:
        """A latched GPU came back from a telemetry outage and nothing confirmed a reset
        (no kernel reset count, no firmware clock restart): re-verify it with the recovery
        canary when one is configured, else leave it latched for an operator."""
        self.counters["reset_candidates"] = self.counters.get("reset_candidates", 0) + 1
        if self.cfg.health.canary:
            log.warning("%s is back from a telemetry outage (%s); verifying it with the canary before its health "
                        "latches are dropped", self._gpu_name(key), reason)
            gen = self._health_gen[key] = self._health_gen.get(key, 0) + 1
            if self._verify_pool is None:
                self._verify_pool = concurrent.futures.ThreadPoolExecutor(max_workers=4, thread_name_prefix="canary",
                                                                         initializer=background_thread)
            self._verify_pool.submit(self._verify_candidate, key, gen)
            return
        log.warning("%s is back from a telemetry outage (%s), but nothing confirms a reset: its health latches hold. "
                    "Once the GPU is known good: GET /health/clear?gpu=%s (or enable health.canary to verify such "
                    "GPUs automatically)", self._gpu_name(key), reason, key)

    def _verify_candidate(self, key: str, gen: int) -> None:
        try:
            ok = self._canary_ok(key)
        except Exception as e:  # a canary that cannot run does not prove health
            log.error("recovery canary on %s could not run: %s", self._gpu_name(key), e)
            ok = False
        self.events.put((EV_CANDIDATE_VERIFIED, key, gen, ok))

    def _apply_candidate_verified(self, key: str, gen: int, ok: bool) -> None:
        if self._health_gen.get(key) != gen:
            log.info("dropping stale canary verdict for %s (newer health event)", self._gpu_name(key))
            return
        if not ok:
            self._count("canary_failures")
            log.error("%s failed the recovery canary after a telemetry outage: its health latches hold",
                      self._gpu_name(key))
            return
        self._verified_clear.add(key)
        cleared = self.monitor.clear_latches(key, "recovery canary passed after a telemetry outage")
        if not cleared:
            self._verified_clear.discard(key)
        self.counters["latches_cleared_verified"] = self.counters.get("latches_cleared_verified", 0) + 1
        log.warning("%s passed the recovery canary after a telemetry outage: cleared %s", self._gpu_name(key),
                    ", ".join(cleared) or "nothing (no latch was set any more)")

    def _resolve_gpu(self, sel: str):
        """The identity ``sel`` names: an identity/UUID, a BDF, a GPU index or an advertised
        device ID (a partition's, or a replica's ``<id>::<n>``).  None when nothing matches."""
        sel = sel.strip()
        known = set(self._node_index_of) | set(self._index_of) | set(self.monitor.unhealthy_keys())
        if sel in known:
            return sel
        low = sel.lower()
        for k in known:
            if k.lower() == low:
                return k
        for bdf in (low, "0000:" + low):  # a BDF, with or without its PCI domain
            if bdf in self._seen_bdfs:
                return self._seen_bdfs[bdf]
        if sel.isdigit() and int(sel) in self._key_of:
            return self._key_of[int(sel)]
        base = sel.split("::")[0]
        for p in self.plugins:
            for d in p.devices():
                if d.id == base or d.id.split("::")[0] == base:
                    return self._key_of.get(d.gpu)
        return None

    def _clear_health(self, sel: str, fut) -> None:
        """GET /health/clear: drops GPU ``sel``'s latches (uncorrectable ECC, a reset that
        never finished, failed canary verdicts, a held recovery canary).  Levels the next
        samples judge again (telemetry lost, retired pages, PCIe) stay, and are reported;
        with health.canary the GPU is verified before it is advertised Healthy again."""
        key = self._resolve_gpu(sel)
        if key is None:
            fut.set_result((404, "no GPU matches %r" % sel))
            return
        reason = "operator: GET /health/clear"
        cleared = list(self.monitor.clear_latches(key, reason))
        failed = sorted(part for k, part in self._canary_failed if k == key)
        if failed:
            self._canary_failed = {kp for kp in self._canary_failed if kp[0] != key}
            cleared.append("canary_failed")
        if key in self._held_unhealthy:
            self._held_unhealthy.discard(key)
            self._reverify.discard(key)
            cleared.append("recovery_canary_held")
        self._health_gen[key] = self._health_gen.get(key, 0) + 1  # a canary verdict in flight is stale now
        self._sync_held()
        holds = list(self.monitor.holds(key))
        gpu = self._index_of.get(key, -1)
        if gpu >= 0 and not holds and (failed or "recovery_canary_held" in cleared) and not self.cfg.health.canary:
            held = {part for k, part in self._start_pending if k == key}
            for p in self.plugins:  # what only the manager held: written here
                p.set_gpu_health(gpu, -1, True, held)
        self.counters["health_clears"] = self.counters.get("health_clears", 0) + 1
        self.health_log.append((time.monotonic(), gpu, -1, "%s (cleared: %s)" % (reason, ", ".join(cleared) or "nothing")))
        log.warning("%s: health latches cleared by an operator: %s%s", self._gpu_name(key),
                    ", ".join(cleared) or "nothing was latched",
                    ("; still Unhealthy: " + ", ".join(holds)) if holds else "")
        fut.set_result((200, {"gpu": key, "index": gpu, "cleared": cleared, "still_unhealthy": holds,
                              "verify_with_canary": bool(self.cfg.health.canary and not holds and cleared)}))

    def _verify_later(self, key: str, partition: int, reason: str) -> None:
        """Holds a GPU Unhealthy and runs the recovery canary on it off the manager thread."""
        import types
        gen = self._health_gen[key] = self._health_gen.get(key, 0) + 1
        if self._verify_pool is None:
            self._verify_pool = concurrent.futures.ThreadPoolExecutor(max_workers=4, thread_name_prefix="canary",
                                                                     initializer=background_thread)
        self._held_unhealthy.add(key)
        self._verify_pool.submit(self._verify_and_post, types.SimpleNamespace(partition=partition, reason=reason),
                                 key, gen)

    def _count(self, key: str, n: int = 1) -> None:
        with self._canary_lock:  # counters touched from canary pool threads too
            self.counters[key] = self.counters.get(key, 0) + n

    def _run_canary(self, gpu: int, hw_part: int, hip: int, owner: str | None = None) -> dict:
        """One isolated canary run on HIP device ``hip`` (GPU ``gpu``, hardware partition
        ``hw_part``): applies the configured performance floors and records the result for
        /metrics.  Thread-safe; runs on canary pool threads."""
        from ..ops import canary
        res = dict(canary.run_isolated(max(0, hip), self.cfg.health.canaryBytes, self.cfg.health.canaryTimeoutS))
        h = self.cfg.health
        if res.get("ok"):
            low = []
            hbm = min(res.get("write_gbps", 0.0), res.get("read_gbps", 0.0))
            if h.canaryMinHbmGbps > 0 and hbm < h.canaryMinHbmGbps:
                low.append("HBM %.0f GB/s < %.0f" % (hbm, h.canaryMinHbmGbps))
            if h.canaryMinTflops > 0 and res.get("mfma_tflops", 0.0) < h.canaryMinTflops:
                low.append("bf16 MFMA %.0f TFLOP/s < %.0f" % (res.get("mfma_tflops", 0.0), h.canaryMinTflops))
            if low:
                res["ok"] = False
                res["error"] = "below the canary performance floor: " + ", ".join(low)
        with self._canary_lock:
            self.counters["canary_runs"] = self.counters.get("canary_runs", 0) + 1
            self.canary_results[(gpu, hw_part)] = (time.time(), res)
            self._canary_owner[(gpu, hw_part)] = owner or self._key_of.get(gpu, "#%d" % gpu)
        self.events.put((EV_METRICS,))
        return res

    def _prestart_check(self, ids) -> str:
        """PreStartContainer verifier (health.canaryOnPreStart): the gfx950 canary on
        every partition the container is about to get, all in parallel child processes,
        right before it starts.  A failing partition is marked Unhealthy and the
        container start is refused.  Runs on the plugin's verifier pool, never on a
        server thread."""
        from ..ops import canary
        want = set(ids)
        gpus = {g.index: g for g in self.gpus}
        targets = {}  # (gpu, partition) -> hardware partitions to check
        for p in self.plugins:
            for d in p.devices():
                if d.id not in want or d.gpu not in gpus:
                    continue
                parts = gpus[d.gpu].partitions
                sel = parts if d.partition < 0 else [x for x in parts if x.index == d.partition]
                targets[(d.gpu, d.partition)] = sel
        jobs = [(key, x) for key, parts in targets.items() for x in parts]
        if not jobs:
            return ""
        failures = {}
        with concurrent.futures.ThreadPoolExecutor(max_workers=min(8, len(jobs))) as ex:
            futs = {ex.submit(self._run_canary, key[0], x.index, x.hip_id): key for key, x in jobs}
            for f in concurrent.futures.as_completed(futs):
                res = f.result()
                if not res.get("ok"):
                    failures.setdefault(futs[f], res.get("error") or "canary reported errors")
        for (gpu, part), why in sorted(failures.items()):
            self.events.put((EV_PRESTART_FAIL, self._key_of.get(gpu, "#%d" % gpu), part,
                             "PreStartContainer canary failed: %s" % why))
        if failures:
            return "PreStartContainer: gfx950 canary failed on %s" % ", ".join(
                "GPU %d%s" % (g, "" if p < 0 else " partition %d" % p) for g, p in sorted(failures))
        return ""

    def _canary_ok(self, key: str) -> bool:
        gpu = self._index_of.get(key)
        if gpu is None:
            raise RuntimeError("GPU %s is not in the advertised inventory" % key)
        for g in self.gpus:
            if g.index != gpu:
                continue
            for part in g.partitions:
                res = self._run_canary(gpu, part.index, part.hip_id)
                if not res.get("ok"):
                    log.error("canary failed on GPU %d partition %d: %s", gpu, part.index, res)
                    return False
        return True

    # ------------------------------------------------------------ threads
    def _start_watch(self) -> None:
        n = native.load()
        try:
            watcher = n.DirWatcher(self.cfg.pluginDir)
        except Exception as e:
            log.error("failed to create FS watcher on %s: %s", self.cfg.pluginDir, e)
            watcher = None

        self._watcher = watcher  # _shutdown wakes its read

        def watch_loop():
            # long reads (inotify wakes it for every change in the directory): an idle node
            # pays one wake-up every 5 s for it, and _shutdown cuts the read short
            # (DirWatcher.wake).  A directory removed and created again is noticed on the
            # timeout, so within 5 s.
            while self._running.is_set() and watcher is not None:
                for name, _mask, created, _removed in watcher.read(5000):
                    if name == "kubelet.sock" and created:
                        self.events.put((EV_KUBELET,))
                    elif _removed and name.endswith(".sock") and name != "kubelet.sock":
                        self.events.put((EV_SOCKET_GONE, name))
            if watcher is not None:
                watcher.close()

        def health_loop():
            while self._running.is_set():
                if not self.monitor.running:
                    time.sleep(0.1)
                    continue
                for u in self.monitor.pop(5000):  # (returns at once on an update or stop)
                    self.events.put((EV_HEALTH, u))

        def rediscover_loop():
            interval = float(self.cfg.rediscoverIntervalS)
            while interval > 0 and not self._stop_flag.wait(interval):
                self.events.put((EV_REDISCOVER,))

        for fn, name in ((watch_loop, "fs-watch"), (health_loop, "health-pump"), (rediscover_loop, "rediscover")):
            t = threading.Thread(target=_as_background(fn), name=name, daemon=True)
            t.start()
            self._threads.append(t)
        if self.cfg.podResources.enabled:
            from .podresources import PodResourcesWatcher
            self.podres = PodResourcesWatcher(self.cfg.podResources.socket, self.cfg.podResources.intervalS,
                                              self.cfg.resourcePrefix, lambda: self.events.put((EV_PODRES,)))
            self.podres.start()

    def _start_telemetry(self) -> None:
        if self.cfg.health.enabled:
            self.monitor.start()
            self._event_sources = getattr(self.backend, "armed_event_sources", None)
            if self.gpus and self._event_sources == 0:
                # amdsmi event notification needs /dev/kfd (device cgroup or privileged pod):
                # without it resets are seen only as failed telemetry samples
                log.warning("no GPU event source armed (GPU reset / thermal events will not be received; "
                            "health falls back to telemetry polling): check access to /dev/kfd")
        if self.cfg.telemetry.enabled:
            self.exporter.set_stall_ms(int(self.cfg.health.sampleStallS * 1000) if self.cfg.health.enabled else 0)
            self.exporter.set_idle_interval(int(self.cfg.telemetry.idleIntervalMs),
                                            int(self.cfg.telemetry.activeWindowS * 1000))
            self.exporter.start(self.backend, self.cfg.telemetry.intervalMs,
                                self.monitor if self.cfg.health.enabled else None)
        self._publish_metrics()

    def _arm_retry(self) -> None:
        with self._lock:
            if self._retry_timer is not None:
                return
            t = threading.Timer(self.cfg.retrySeconds, lambda: self.events.put((EV_RETRY,)))
            t.daemon = True
            self._retry_timer = t
            t.start()

    def _cancel_retry(self) -> None:
        with self._lock:
            if self._retry_timer is not None:
                self._retry_timer.cancel()
                self._retry_timer = None

    def _publish_metrics(self) -> None:
        self._push_readiness()  # runs after every event, like the metrics
        glitches = self.monitor.fw_clock_glitches
        if glitches:
            self.counters["fw_clock_glitches"] = glitches
        lines = ["# HELP amdgpu_device_plugin_events_total Plugin manager lifecycle events.",
                 "# TYPE amdgpu_device_plugin_events_total counter"]
        for k in sorted(self.counters):
            lines.append('amdgpu_device_plugin_events_total{event="%s"} %d' % (k, self.counters[k]))
        lines += ["# HELP amdgpu_device_plugin_devices Devices advertised per resource and health.",
                  "# TYPE amdgpu_device_plugin_devices gauge"]
        for p in self.plugins:
            healthy = p.table.healthy_count()
            lines.append('amdgpu_device_plugin_devices{resource="%s",health="Healthy"} %d' % (p.resource, healthy))
            lines.append('amdgpu_device_plugin_devices{resource="%s",health="Unhealthy"} %d'
                         % (p.resource, len(p) - healthy))
        if self._event_sources is not None:
            lines += ["# HELP amdgpu_device_plugin_health_event_sources GPUs whose hardware event notification "
                      "(reset, thermal, VM fault) is armed.",
                      "# TYPE amdgpu_device_plugin_health_event_sources gauge",
                      "amdgpu_device_plugin_health_event_sources %d" % self._event_sources]
        lines += ["# HELP amdgpu_device_plugin_registered 1 if the resource is registered with kubelet.",
                  "# TYPE amdgpu_device_plugin_registered gauge"]
        for p in self.plugins:
            lines.append('amdgpu_device_plugin_registered{resource="%s"} %d' % (p.resource, int(p.registered)))
        lines += ["# HELP amdgpu_device_plugin_ready 1 if every resource with devices is registered with kubelet "
                  "(GET /ready).",
                  "# TYPE amdgpu_device_plugin_ready gauge",
                  "amdgpu_device_plugin_ready %d" % int(self._readiness[0])]
        if self.podres is not None:
            from .podresources import render
            allocs, up = self.podres.snapshot()
            lines += render(allocs, up)
            if self.link_pods:
                lines += ["# HELP amdgpu_xgmi_link_pods Multi-GPU pods whose devices span this GPU pair (they share "
                          "its xGMI link).",
                          "# TYPE amdgpu_xgmi_link_pods gauge"]
                lines += ['amdgpu_xgmi_link_pods{gpu="%d",peer="%d"} %d' % (a, b, c)
                          for (a, b), c in sorted(self.link_pods.items())]
        lines += self._canary_lines()
        self.exporter.set_extra("\n".join(lines) + "\n")

    def _canary_lines(self) -> list:
        with self._canary_lock:
            runs = sorted(self.canary_results.items())
        if not runs:
            return []
        fams = (("amdgpu_canary_last_run_timestamp_seconds", "Unix time of the partition's last canary run."),
                ("amdgpu_canary_last_ok", "1 if the last canary run passed."),
                ("amdgpu_canary_errors", "Mismatches found by the last canary run, per check."),
                ("amdgpu_canary_hbm_gbps", "HBM bandwidth measured by the last canary run."),
                ("amdgpu_canary_matrix_tflops", "Dense matrix-core rate measured by the last canary run."))
        rows = {name: [] for name, _ in fams}
        for (gpu, part), (t, r) in runs:
            lab = 'gpu="%d",partition="%d"' % (gpu, part)
            rows["amdgpu_canary_last_run_timestamp_seconds"].append("{%s} %.3f" % (lab, t))
            rows["amdgpu_canary_last_ok"].append("{%s} %d" % (lab, int(bool(r.get("ok")))))
            for check, key in (("hbm", "hbm_errors"), ("mfma", "mfma_errors"), ("gemm", "gemm_errors"),
                               ("lowp", "lowp_errors"), ("lds", "lds_errors")):
                if key in r:
                    rows["amdgpu_canary_errors"].append('{%s,check="%s"} %d' % (lab, check, int(r[key])))
            for d, key in (("write", "write_gbps"), ("read", "read_gbps")):
                if key in r:
                    rows["amdgpu_canary_hbm_gbps"].append('{%s,direction="%s"} %.1f' % (lab, d, float(r[key])))
            for path, key in (("mfma_bf16", "mfma_tflops"), ("gemm_bf16", "gemm_tflops"), ("mxfp8", "fp8_tflops"),
                              ("mxfp4", "fp4_tflops")):
                if key in r:
                    rows["amdgpu_canary_matrix_tflops"].append('{%s,path="%s"} %.1f' % (lab, path, float(r[key])))
        out = []
        for name, help_ in fams:
            if rows[name]:
                out += ["# HELP %s %s" % (name, help_), "# TYPE %s gauge" % name]
                out += [name + x for x in rows[name]]
        return out

    def _shutdown(self) -> None:
        self._cancel_retry()
        if self._discoverer is not None:
            self._discoverer.stop()
        if self._verify_pool is not None:
            self._verify_pool.shutdown(wait=False, cancel_futures=True)
        if self._canary_pool is not None:
            self._canary_pool.shutdown(wait=False, cancel_futures=True)
        self._stop_flag.set()
        self._running.clear()
        if getattr(self, "_watcher", None) is not None:
            self._watcher.wake()
        if self.podres is not None:
            self.podres.stop()
        self.stop_plugins()
        self.exporter.stop()
        self.monitor.stop()
        for t in self._threads:
            t.join(2.0)
        self._threads.clear()
        self._push_readiness()
        self._stopped.set()
        self.ready.close()
