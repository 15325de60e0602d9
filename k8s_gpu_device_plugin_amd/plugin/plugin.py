"""One kubelet DevicePlugin endpoint per resource name.

Reference ``plugin/plugin.go`` (``NvidiaDevicePlugin``):
  * socket ``<DevicePluginPath>/nvidia-<name>.sock`` (``:46-51``) -> ``amd-<name>.sock``
  * ``Serve`` (``:100-137``): remove stale socket, listen, serve with a crash-restart
    loop (fatal after >5 crashes within 1 h), then a blocking self-dial check (5 s)
  * ``Register`` (``:140-162``): dial ``kubelet.sock``, ``RegisterRequest{v1beta1,
    endpoint, resource, GetPreferredAllocationAvailable}``
  * RPCs ``GetDevicePluginOptions``/``ListAndWatch``/``GetPreferredAllocation``/
    ``Allocate``/``PreStartContainer`` (``:165-229``)

MI355X design: the device set, health, topology, allocator and the protobuf encoding
of every hot response live in a native ``DeviceTable`` (C++).  Two interchangeable
servers put it on the kubelet socket:
  * ``native`` - C++ HTTP/2 gRPC server (``native/grpc_h2.cpp``): no Python and no
    GIL on the request path.
  * ``python`` - grpcio generic handlers with identity (de)serialisers, so request
    bytes go straight into the native table and its bytes straight back out.
Health changes bump the table version and wake every ListAndWatch stream; devices can
become Healthy again (reference only ever marks Unhealthy, ``:181-186``).
Lifecycle is idempotent: ``stop()`` twice, or after a failed ``start()``, is safe
(defects D5/D6/D10).
"""
from __future__ import annotations

import concurrent.futures
import os
import threading
import time

from .. import native
from ..api import v1beta1
from ..device import Devices
from ..resource import ResourceName
from ..utils.log import get_logger
from ..utils.util import name_os_thread

log = get_logger("plugin")

SERVE_CRASH_LIMIT = 5          # plugin/plugin.go:110
SERVE_CRASH_WINDOW_S = 3600.0  # plugin/plugin.go:122
DIAL_TIMEOUT_S = 5.0           # plugin/plugin.go:130,141


def socket_name(resource: ResourceName, vendor: str = "amd") -> str:
    return "%s-%s.sock" % (vendor, ResourceName(resource).get_resource_name())


def _unix_target(path: str) -> str:
    return "unix://" + os.path.abspath(path)


def dial(path: str, timeout: float = DIAL_TIMEOUT_S) -> "grpc.Channel":
    """Blocking dial of a unix socket (reference ``dial`` ``plugin/plugin.go:231-246``).
    grpcio is imported on demand: the native path (server, Register, self-check) never
    loads it, which keeps ~70 ms of imports out of start-up."""
    import grpc
    ch = grpc.insecure_channel(_unix_target(path), options=[("grpc.enable_http_proxy", 0)])
    try:
        grpc.channel_ready_future(ch).result(timeout=timeout)
    except grpc.FutureTimeoutError:
        ch.close()
        raise TimeoutError("timed out dialing %s after %.1fs" % (path, timeout)) from None
    return ch


def close_async(ch: "grpc.Channel") -> None:
    """grpcio's Channel.close() joins its polling thread, which wakes every 200 ms:
    closing inline would add up to 0.2 s to each start-up and registration."""
    threading.Thread(target=ch.close, name="grpc-channel-close", daemon=True).start()


def native_probe(path: str, timeout: float = DIAL_TIMEOUT_S) -> None:
    """Blocking self-check of a native server: connect, HTTP/2 handshake and one
    GetDevicePluginOptions call (the reference dials its own socket, plugin.go:130-134)."""
    n = native.load()
    c = n.H2Client(path, timeout)
    try:
        status = c.unary(v1beta1.METHOD_GET_OPTIONS, b"")[0]
        if status != 0:
            raise RuntimeError("self-check of %s: grpc-status %d" % (path, status))
    finally:
        c.close()


def _socket_ident(path: str):
    try:
        st = os.stat(path)
    except OSError:
        return None
    return st.st_dev, st.st_ino


def _remove_if_ours(path: str, ident) -> None:
    """Removes the plugin's socket file unless another instance has bound its own at
    that path since (during a rolling update the next pod can start before this one has
    stopped; deleting its socket would cut kubelet off from it)."""
    if ident is None or _socket_ident(path) != ident:
        return
    try:
        os.remove(path)
    except FileNotFoundError:
        pass


def make_table(resource: str, devices: Devices, topology, cfg) -> "object":
    """Builds the native DeviceTable for a resource from the Python device view."""
    n = native.load()
    tc = n.TableConfig()
    tc.resource_name = str(resource)
    tc.visible_env = cfg.visibleDevicesEnv if cfg is not None else "AMD_VISIBLE_DEVICES"
    tc.cdi = bool(cfg.cdi) if cfg is not None else False
    tc.cdi_prefix = str(resource) + "="
    tc.reject_unhealthy = bool(cfg.health.rejectUnhealthyAllocate) if cfg is not None else True
    tc.pre_start_required = bool(cfg.health.canaryOnPreStart) if cfg is not None else False
    tds = [n.TableDevice(d.id, d.gpu, d.partition, d.numa_node if d.numa_node is not None else -1, d.replica,
                         list(d.paths), d.health == v1beta1.HEALTHY) for d in devices]
    table = n.DeviceTable(tc, tds, topology)
    for d in devices:  # from here on the Python view reads health from the table
        d.bind_table(table)
    return table


class AmdDevicePlugin:
    """kubelet DevicePlugin for one ``amd.com/*`` resource."""

    def __init__(self, resource: str, devices: Devices, topology, cfg=None, plugin_dir: str | None = None,
                 server_kind: str | None = None) -> None:
        self.resource = ResourceName(resource)
        self._devices = devices
        self.cfg = cfg
        self.plugin_dir = plugin_dir or (cfg.pluginDir if cfg is not None else v1beta1.DEVICE_PLUGIN_PATH)
        self.socket = os.path.join(self.plugin_dir, socket_name(self.resource))
        self.kubelet_socket = os.path.join(self.plugin_dir, v1beta1.KUBELET_SOCKET_NAME)
        self.server_kind = server_kind or (cfg.grpc.server if cfg is not None else "python")
        self.table = make_table(str(self.resource), devices, topology, cfg)
        self._lock = threading.RLock()
        self._server = None
        self._native_server = None
        self._serving = False
        self._stopping = False
        self._supervisor: threading.Thread | None = None
        self.fatal_error: str | None = None
        # Serve crash accounting (plugin/plugin.go:107-129), shared by both servers
        self._crashes = 0
        self._last_crash = time.monotonic()
        self.server_restarts = 0
        self.registered = False
        self.registered_at = -1.0  # time.monotonic() of the last successful Register
        self._sock_ident = None  # (st_dev, st_ino) of the socket file this plugin bound
        # PreStartContainer verifier: fn(device ids) -> "" (pass) or an error message
        self.prestart_check = None
        # called (on a native worker thread) when the native server faults: the manager
        # supervises at once; must not hold this plugin (the server would keep it alive)
        self.on_server_fault = None
        self._prestart_thread: threading.Thread | None = None
        self._prestart_pool: concurrent.futures.ThreadPoolExecutor | None = None
        self._retiring = False  # a successor took the server over (adopt)
        # the plugin a grpcio server's handlers serve from: shared with (and redirected
        # by) a successor that adopts the server, so requests follow the current table
        self._front = [self]
        # ListAndWatch streams open on the grpcio server (the native server counts its own);
        # shared with a successor that adopts the server, like _front
        self._law = [0, 0.0]  # [open streams, time.monotonic() when one last ended]
        # stream watchdog (PluginManager._check_stream): kubelet opened a stream since the
        # last Register, and since when none is open
        self.law_had = False
        self.law_lost_since: float | None = None

    # ------------------------------------------------------------------ views
    def devices(self) -> Devices:
        return self._devices

    def __len__(self) -> int:
        return len(self._devices)

    # ------------------------------------------------------------------ lifecycle
    def start(self) -> None:
        """Serve then register; on register failure the server is stopped again
        (reference ``Start`` ``plugin/plugin.go:68-83``)."""
        self.serve()
        log.info("Starting to serve", extra={"resourceName": str(self.resource), "socket": self.socket})
        try:
            self.register()
        except Exception as e:
            log.info("Could not register device plugin", extra={"resourceName": str(self.resource), "error": str(e)})
            self.stop()
            raise
        log.info("Registered device plugin", extra={"resourceName": str(self.resource)})

    def _prestart_loop(self) -> None:
        """Pops PreStartContainer jobs from the table (either server enqueues them) and
        runs the verifier off the server threads; several containers verify in parallel."""
        name_os_thread("prestart")
        while not self._stopping:
            for job_id, ids in self.table.pop_prestart(5000):  # (a job or stop() wakes it)
                self._prestart_pool.submit(self._run_prestart, job_id, ids)
            if self._retiring and self.table.prestart_pending == 0:
                # a successor serves now and every check queued here has been answered
                self._prestart_pool.shutdown(wait=False)
                return

    def _run_prestart(self, job_id: int, ids) -> None:
        try:
            err = self.prestart_check(list(ids)) if self.prestart_check else ""
        except Exception as e:  # a verifier that cannot run does not pass the devices
            err = "PreStartContainer check failed to run: %s" % e
        self.table.complete_prestart(job_id, not err, err or "")

    def adopt(self, prev: "AmdDevicePlugin") -> None:
        """Takes over ``prev``'s running server, socket and kubelet registration and
        swaps this plugin's table into it: kubelet's connection stays up, its ListAndWatch
        stream gets the new device list, and no admission finds the endpoint gone.
        ``prev`` is left inert (its stop() does nothing to the server)."""
        self.table.inherit_stats(prev.table)  # RPC histograms continue across the swap
        with prev._lock:
            if not prev._serving or prev._stopping:
                raise RuntimeError("%s is not serving" % prev.resource)
            server, nserver = prev._server, prev._native_server
            prev._server = prev._native_server = None
            prev._serving = False
            prev._retiring = True
            sock_ident, prev._sock_ident = prev._sock_ident, None
            registered, prev.registered = prev.registered, False
        with self._lock:
            self._server, self._native_server = server, nserver
            self._serving, self._stopping = True, False
            self._sock_ident, self.registered = sock_ident, registered
            self.registered_at = prev.registered_at
            self._crashes, self._last_crash = prev._crashes, prev._last_crash
            self.server_restarts = prev.server_restarts
            self._front = prev._front
            self._law = prev._law
            self.law_had, self.law_lost_since = prev.law_had, prev.law_lost_since
            if self.cfg is not None and self.cfg.health.canaryOnPreStart and self._prestart_thread is None:
                self._start_prestart_locked()
        if nserver is not None:
            nserver.set_table(self.table)  # workers switch tables and push ListAndWatch
        self._front[0] = self  # grpcio handlers serve from this plugin's table from now on
        prev.table.wake()      # grpcio ListAndWatch generators waiting on the old table
        # (a grpcio server's supervisor thread follows _front: it now acts for this plugin)
        self._supervisor, prev._supervisor = prev._supervisor, None
        # the predecessor's PreStartContainer loop answers what is queued on its table, then ends
        log.info("device table swapped into the running server", extra={"resourceName": str(self.resource),
                                                                        "devices": len(self)})

    def _start_prestart_locked(self) -> None:
        self.table.resume_prestart()
        self._prestart_pool = concurrent.futures.ThreadPoolExecutor(
            max_workers=4, thread_name_prefix="prestart-" + self.resource.get_resource_name())
        self._prestart_thread = threading.Thread(target=self._prestart_loop, daemon=True,
                                                 name="prestart-" + self.resource.get_resource_name())
        self._prestart_thread.start()

    def stop(self) -> None:
        if self._retiring:  # the server belongs to a successor now
            return
        self.table.cancel_prestart("device plugin for %s is stopping" % self.resource)
        if self._prestart_thread is not None:
            self._stopping = True
            self._prestart_thread.join(2.0)
            self._prestart_thread = None
        if self._prestart_pool is not None:
            self._prestart_pool.shutdown(wait=False, cancel_futures=True)
            self._prestart_pool = None
        with self._lock:
            self._stopping = True
            server, self._server = self._server, None
            nserver, self._native_server = self._native_server, None
            was_serving, self._serving = self._serving, False
        self.notify()
        if server is not None:
            server.stop(grace=0.5).wait(2.0)
        if nserver is not None:
            nserver.stop()
            nserver.set_failure_hook(None)
        if was_serving:
            log.info("Stopped serving", extra={"resourceName": str(self.resource), "socket": self.socket})
        _remove_if_ours(self.socket, self._sock_ident)
        self._sock_ident = None
        self.registered = False

    @property
    def serving(self) -> bool:
        return self._serving

    def serve(self) -> None:
        with self._lock:
            if self._serving:
                return
            self._stopping = False
            os.makedirs(self.plugin_dir, exist_ok=True)
            try:
                os.remove(self.socket)
            except FileNotFoundError:
                pass
            if self.server_kind == "native":
                self._start_native_server()
            else:
                self._start_grpcio_server()
            self._serving = True
            self._sock_ident = _socket_ident(self.socket)
            if self.cfg is not None and self.cfg.health.canaryOnPreStart and self._prestart_thread is None:
                self._start_prestart_locked()
        # blocking self-dial (plugin/plugin.go:130-134)
        try:
            if self.server_kind == "native":
                native_probe(self.socket, DIAL_TIMEOUT_S)
            else:
                close_async(dial(self.socket, DIAL_TIMEOUT_S))
        except Exception:
            self.stop()
            raise

    def _start_native_server(self) -> None:
        n = native.load()
        srv = n.GrpcServer(self.socket, max(1, self.cfg.grpc.threads if self.cfg is not None else 2),
                           self.cfg.grpc.busyPollUs if self.cfg is not None else 0,
                           self.cfg.grpc.admissionPollUs if self.cfg is not None else 0)
        srv.set_table(self.table)
        if self.on_server_fault is not None:
            srv.set_failure_hook(self.on_server_fault)
        if self.cfg is not None:
            srv.set_keep_warm_ms(int(self.cfg.grpc.keepWarmMs))
            srv.set_keep_warm_full(bool(self.cfg.grpc.keepWarmFull))
            srv.set_idle_wake_ms(int(self.cfg.grpc.idleWakeMs))
            srv.set_active_window_ms(int(self.cfg.grpc.activeWindowMs))
            srv.set_peek_reads(bool(self.cfg.grpc.peekReads))
            srv.set_poll_gap_ns(int(self.cfg.grpc.pollGapNs))
            srv.set_core_escape(bool(self.cfg.grpc.coreEscape))
            if self.cfg.grpc.callTraceFile:
                srv.set_call_trace(self.cfg.grpc.callTraceFile.replace("{resource}", self.resource.get_resource_name()),
                                   int(self.cfg.grpc.callTraceEntries))
        srv.start()
        self._native_server = srv

    def _start_grpcio_server(self) -> None:
        import grpc
        server = grpc.server(concurrent.futures.ThreadPoolExecutor(
            max_workers=max(4, self.cfg.grpc.threads if self.cfg is not None else 4),
            thread_name_prefix="dp-" + self.resource.get_resource_name()))
        server.add_generic_rpc_handlers((self._handler(),))
        if server.add_insecure_port(_unix_target(self.socket)) == 0:
            raise OSError("cannot listen on %s" % self.socket)
        server.start()
        self._server = server
        self._supervisor = threading.Thread(target=self._supervise, args=(server,), daemon=True,
                                            name="dp-supervise-" + self.resource.get_resource_name())
        self._supervisor.start()

    def _note_crash(self, why: str) -> bool:
        """Counts a server crash the way the reference's Serve loop does
        (``plugin/plugin.go:107-129``): the count resets when the previous crash is more
        than an hour old; more than 5 is fatal.  Returns True when fatal."""
        now = time.monotonic()
        self._crashes = 0 if now - self._last_crash > SERVE_CRASH_WINDOW_S else self._crashes + 1
        self._last_crash = now
        log.error("gRPC server for '%s' crashed with error: %s", self.resource, why)
        if self._crashes > SERVE_CRASH_LIMIT:
            self.fatal_error = "GRPC server for '%s' has repeatedly crashed recently. Quitting" % self.resource
            log.critical(self.fatal_error)
            return True
        return False

    def check_server(self) -> bool:
        """Supervision of the native server, polled by the manager: a server whose worker
        died or whose listener broke is restarted on a fresh socket and registered with
        kubelet again.  Returns True if it was restarted.  Raises if the restart failed
        (the manager's retry timer takes over); sets ``fatal_error`` after too many
        crashes (the process then exits non-zero, as the reference's Fatal does)."""
        srv = self._native_server
        if srv is None or self._stopping or self.fatal_error:
            return False
        why = srv.failure()
        if not why and srv.running:
            return False
        with self._lock:
            if self._native_server is not srv or self._stopping:
                return False
        if self._note_crash(why or "server stopped unexpectedly"):
            return False
        self.server_restarts += 1
        self.stop()
        self.start()
        return True

    def _supervise(self, server) -> None:
        """grpcio analogue of the Serve crash-restart loop (``plugin/plugin.go:107-129``):
        an unexpected termination restarts the server, >5 crashes within an hour is fatal.
        One thread per server: it acts for whichever plugin serves from it now (a
        successor that adopted the server is ``_front[0]``)."""
        name_os_thread("grpcio-sup")
        front = self._front
        while True:
            server.wait_for_termination()
            owner = front[0]
            with owner._lock:
                if owner._stopping or owner._server is not server:
                    return
            if owner._note_crash("terminated unexpectedly"):
                return
            with owner._lock:
                owner._serving = False
                try:
                    owner._start_grpcio_server_locked_restart()
                except Exception as e:  # pragma: no cover
                    log.error("restart failed: %s", e)
                return

    def _start_grpcio_server_locked_restart(self) -> None:
        try:
            os.remove(self.socket)
        except FileNotFoundError:
            pass
        self._start_grpcio_server()
        self._serving = True
        self._sock_ident = _socket_ident(self.socket)

    def list_and_watch_streams(self) -> int:
        """ListAndWatch streams open on this plugin's server now."""
        srv = self._native_server
        if srv is not None:
            return srv.list_and_watch_streams()
        return self._law[0] if self._serving else 0

    def list_and_watch_closed_at(self) -> float:
        """time.monotonic() when a ListAndWatch stream of this server last ended (0: none)."""
        srv = self._native_server
        if srv is not None:
            return srv.list_and_watch_closed_at()
        return self._law[1]

    def register(self) -> None:
        """Registration.Register with kubelet (``plugin/plugin.go:139-162``).  Sent by the
        compiled HTTP/2 client when the native module has one (no grpcio import, no
        channel teardown), else over a grpcio channel."""
        self.law_had, self.law_lost_since = False, None
        if not os.path.exists(self.kubelet_socket):  # fail fast instead of a 5 s dial timeout
            raise FileNotFoundError("kubelet socket %s does not exist" % self.kubelet_socket)
        pre_start = bool(self.cfg.health.canaryOnPreStart) if self.cfg is not None else False
        n = native.load()
        if hasattr(n, "H2Client"):
            req = v1beta1.encode_register_request(os.path.basename(self.socket), str(self.resource), pre_start)
            for attempt in (0, 1):
                c = n.H2Client(self.kubelet_socket, DIAL_TIMEOUT_S)
                try:
                    status, _, message = c.unary(v1beta1.METHOD_REGISTER, req)
                    break
                except RuntimeError as e:
                    # a GOAWAY that left the request unprocessed (kubelet's server going
                    # away under it): safe to send once more on a new connection
                    if attempt or "GOAWAY" not in str(e):
                        raise
                    log.info("Register with kubelet: %s; sending it again", e)
                finally:
                    c.close()
            if status != 0:
                raise RuntimeError("Register with kubelet failed: grpc-status %d %s" % (status, message))
            self.registered, self.registered_at = True, time.monotonic()
            return
        ch = dial(self.kubelet_socket, DIAL_TIMEOUT_S)
        try:
            req = v1beta1.RegisterRequest(version=v1beta1.VERSION, endpoint=os.path.basename(self.socket),
                                          resource_name=str(self.resource),
                                          options=v1beta1.plugin_options(pre_start_required=pre_start))
            call = ch.unary_unary(v1beta1.METHOD_REGISTER, request_serializer=v1beta1.RegisterRequest.SerializeToString,
                                  response_deserializer=v1beta1.Empty.FromString)
            call(req, timeout=DIAL_TIMEOUT_S)
            self.registered, self.registered_at = True, time.monotonic()
        finally:
            close_async(ch)

    # ------------------------------------------------------------------ health
    def notify(self) -> None:
        """Wakes ListAndWatch streams (health or stop)."""
        self.table.wake()  # grpcio ListAndWatch generators block in table.wait_change
        srv = self._native_server
        if srv is not None:
            srv.notify()

    def set_gpu_health(self, gpu: int, partition: int, healthy: bool, held=()) -> int:
        """Health lives in the native table only (the Python devices read it from there).
        ``held``: partitions a Healthy whole-GPU update leaves as they are (canary verdicts),
        in the same table update."""
        if healthy and partition < 0 and held:
            changed = self.table.set_gpu_health_except(gpu, sorted(held))
        else:
            changed = self.table.set_gpu_health(gpu, partition, healthy)
        if changed:
            self.notify()
        return changed

    def set_device_health(self, device_id: str, healthy: bool) -> bool:
        changed = self.table.set_health(device_id, healthy)
        if changed:
            self.notify()
        return changed

    def set_link_up(self, a: int, b: int, up: bool) -> None:
        self.table.set_link_up(a, b, up)

    def set_link_bandwidth(self, a: int, b: int, gbps: float) -> None:
        self.table.set_link_bandwidth(a, b, gbps)

    def set_link_pods(self, load) -> None:
        """n x n row-major counts of multi-GPU pods whose devices span each GPU pair."""
        self.table.set_link_pods(list(load))

    # ------------------------------------------------------------------ RPCs (grpcio)
    def _handler(self):
        """grpcio handlers.  They read the table through ``front``, the plugin currently
        serving this server: a reload that swaps in a successor's table redirects them."""
        import grpc
        n = native.load()
        front = self._front
        rpc_opt, rpc_law, rpc_pref, rpc_alloc, rpc_pre = (n.RPC_OPTIONS, n.RPC_LIST_AND_WATCH, n.RPC_PREFERRED,
                                                          n.RPC_ALLOCATE, n.RPC_PRE_START)
        perf = time.perf_counter

        def get_options(req: bytes, ctx) -> bytes:
            t0 = perf()
            table = front[0].table
            out = table.options()
            table.observe(rpc_opt, perf() - t0, False)
            return out

        def allocate(req: bytes, ctx) -> bytes:
            t0 = perf()
            table = front[0].table
            ok, out = table.allocate(req)
            table.observe(rpc_alloc, perf() - t0, not ok)
            if not ok:
                ctx.abort(grpc.StatusCode.UNKNOWN, out)
            return out

        def preferred(req: bytes, ctx) -> bytes:
            t0 = perf()
            table = front[0].table
            ok, out = table.preferred(req)
            table.observe(rpc_pref, perf() - t0, not ok)
            if not ok:
                ctx.abort(grpc.StatusCode.UNKNOWN, out)
            return out

        def pre_start(req: bytes, ctx) -> bytes:
            t0 = perf()
            plugin = front[0]
            table = plugin.table
            if not (plugin.cfg is not None and plugin.cfg.health.canaryOnPreStart):
                table.observe(rpc_pre, 0.0, False)
                return b""
            done = threading.Event()
            result = []

            def finished(ok: bool, err: str) -> None:
                result.append((ok, err))
                done.set()

            queued, err = table.submit_prestart(req, finished)
            if queued and not done.wait(30.0):  # kubelet's PreStartContainer deadline is 30 s
                result.append((False, "PreStartContainer check timed out"))
            ok, err = result[0] if result else (queued, err)
            table.observe(rpc_pre, perf() - t0, not ok)
            if not ok:
                ctx.abort(grpc.StatusCode.UNKNOWN, err)
            return b""

        law = self._law
        law_lock = threading.Lock()

        def list_and_watch(req: bytes, ctx):
            with law_lock:
                law[0] += 1
            try:
                yield from _list_and_watch(ctx)
            finally:
                with law_lock:
                    law[0] -= 1
                    law[1] = time.monotonic()

        def _list_and_watch(ctx):
            plugin = front[0]
            table = plugin.table
            version = table.version
            t0 = perf()
            payload = table.list_and_watch()
            table.observe(rpc_law, perf() - t0, False)
            yield payload
            while True:
                # native wait (GIL released): woken by any table change, including the
                # monitor thread's fail-fast Unhealthy path, by stop() -> table.wake(), or
                # by a successor's adopt() swapping its table in (it wakes the old one)
                while (front[0] is plugin and table.version == version and not plugin._stopping
                       and ctx.is_active()):
                    table.wait_change(version, 500)
                if front[0] is not plugin:  # table swapped: follow the successor
                    plugin = front[0]
                    table = plugin.table
                elif plugin._stopping or not ctx.is_active():
                    return
                version = table.version
                log.info("'%s' device list changed; sending update", plugin.resource)
                yield table.list_and_watch()

        u = grpc.unary_unary_rpc_method_handler
        return grpc.method_handlers_generic_handler(v1beta1.DEVICE_PLUGIN_SERVICE, {
            "GetDevicePluginOptions": u(get_options),
            "ListAndWatch": grpc.unary_stream_rpc_method_handler(list_and_watch),
            "GetPreferredAllocation": u(preferred),
            "Allocate": u(allocate),
            "PreStartContainer": u(pre_start),
        })
