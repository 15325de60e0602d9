"""In-process kubelet stand-in for tests, benchmarks and the GPU smoke run.

The reference has no kubelet stub.  This one:
  * serves ``v1beta1.Registration/Register`` on ``<dir>/kubelet.sock`` and records
    every ``RegisterRequest``;
  * dials registered plugin endpoints and exposes typed DevicePlugin calls;
  * keeps ListAndWatch streams open in background threads (like kubelet's device
    manager) and records every device-list update with its arrival time;
  * ``restart()`` simulates a kubelet restart: the socket is deleted and recreated,
    which is what the plugin manager watches for (``plugin/manager.go:80-84``).
"""
from __future__ import annotations

import concurrent.futures
import os
import queue
import threading
import time

import grpc

from ..api import v1beta1


class DevicePluginClient:
    """Typed client for one plugin endpoint (uses the kubelet-side message classes)."""

    def __init__(self, socket_path: str, timeout: float = 5.0) -> None:
        self.socket_path = socket_path
        self.channel = grpc.insecure_channel("unix://" + os.path.abspath(socket_path),
                                             options=[("grpc.enable_http_proxy", 0)])
        grpc.channel_ready_future(self.channel).result(timeout=timeout)
        self._calls = {}
        for path, (req_cls, resp_cls, stream) in v1beta1.METHODS.items():
            if not path.startswith("/" + v1beta1.DEVICE_PLUGIN_SERVICE + "/"):
                continue
            mk = self.channel.unary_stream if stream else self.channel.unary_unary
            self._calls[path.rsplit("/", 1)[1]] = mk(path, request_serializer=req_cls.SerializeToString,
                                                      response_deserializer=resp_cls.FromString)
        # raw-bytes variants for benchmarks (no Python protobuf on the client side)
        self.allocate_raw = self.channel.unary_unary(v1beta1.METHOD_ALLOCATE)
        self.preferred_raw = self.channel.unary_unary(v1beta1.METHOD_GET_PREFERRED)

    def close(self) -> None:
        self.channel.close()

    def get_options(self, timeout: float = 5.0):
        return self._calls["GetDevicePluginOptions"](v1beta1.Empty(), timeout=timeout)

    def allocate(self, *container_device_ids, timeout: float = 5.0):
        req = v1beta1.AllocateRequest(container_requests=[
            v1beta1.ContainerAllocateRequest(devices_ids=list(ids)) for ids in container_device_ids])
        return self._calls["Allocate"](req, timeout=timeout)

    def preferred(self, available, must_include=(), size: int = 1, timeout: float = 5.0):
        req = v1beta1.PreferredAllocationRequest(container_requests=[
            v1beta1.ContainerPreferredAllocationRequest(available_deviceIDs=list(available),
                                                        must_include_deviceIDs=list(must_include),
                                                        allocation_size=size)])
        return self._calls["GetPreferredAllocation"](req, timeout=timeout)

    def pre_start(self, ids, timeout: float = 5.0):
        return self._calls["PreStartContainer"](v1beta1.PreStartContainerRequest(devices_ids=list(ids)),
                                                timeout=timeout)

    def list_and_watch(self, timeout: float | None = None):
        return self._calls["ListAndWatch"](v1beta1.Empty(), timeout=timeout)


class _Watch:
    def __init__(self, client: DevicePluginClient) -> None:
        self.client = client
        self.updates: "queue.Queue[tuple[float, list]]" = queue.Queue()
        self.history: list[tuple[float, list]] = []
        self.stream = client.list_and_watch()
        self.thread = threading.Thread(target=self._run, daemon=True, name="kubelet-law")
        self.thread.start()

    def _run(self) -> None:
        try:
            for resp in self.stream:
                item = (time.monotonic(), [(d.ID, d.health, [n.ID for n in d.topology.nodes]) for d in resp.devices])
                self.history.append(item)
                self.updates.put(item)
        except grpc.RpcError:
            pass

    def next(self, timeout: float = 5.0):
        return self.updates.get(timeout=timeout)

    def last(self, timeout: float = 5.0, settle: float = 0.2) -> list:
        """The newest device list once the stream has been quiet for ``settle`` seconds
        (waits up to ``timeout`` for the first message)."""
        _, devs = self.updates.get(timeout=timeout)
        while True:
            try:
                _, devs = self.updates.get(timeout=settle)
            except queue.Empty:
                return devs

    def cancel(self) -> None:
        self.stream.cancel()


class KubeletStub:
    """``redial``: behave like kubelet's device manager on a Register for an endpoint it
    already watches - drop that connection and its ListAndWatch stream, dial the
    endpoint again and open a new stream (``reopened`` counts them)."""

    def __init__(self, plugin_dir: str, redial: bool = False) -> None:
        self.plugin_dir = plugin_dir
        self.redial = redial
        self.reopened = 0
        self.socket = os.path.join(plugin_dir, v1beta1.KUBELET_SOCKET_NAME)
        self.requests: list = []
        self.registered = threading.Condition()
        self._server = None
        self._clients: dict[str, DevicePluginClient] = {}
        self._watches: dict[str, _Watch] = {}

    def _handler(self):
        def register(req, ctx):
            with self.registered:
                self.requests.append(req)
                self.registered.notify_all()
            if self.redial and req.endpoint in self._watches:
                threading.Thread(target=self._redial, args=(req.endpoint,), daemon=True).start()
            return v1beta1.Empty()

        return grpc.method_handlers_generic_handler(v1beta1.REGISTRATION_SERVICE, {
            "Register": grpc.unary_unary_rpc_method_handler(
                register, request_deserializer=v1beta1.RegisterRequest.FromString,
                response_serializer=v1beta1.Empty.SerializeToString)})

    def _redial(self, endpoint: str) -> None:
        old_w, old_c = self._watches.pop(endpoint, None), self._clients.pop(endpoint, None)
        if old_w is not None:
            old_w.cancel()
        if old_c is not None:
            old_c.close()
        try:
            self._watches[endpoint] = _Watch(self.client(endpoint))
            self.reopened += 1
        except Exception:  # pragma: no cover - the plugin went away meanwhile
            pass

    def start(self) -> "KubeletStub":
        os.makedirs(self.plugin_dir, exist_ok=True)
        try:
            os.remove(self.socket)
        except FileNotFoundError:
            pass
        self._server = grpc.server(concurrent.futures.ThreadPoolExecutor(max_workers=4))
        self._server.add_generic_rpc_handlers((self._handler(),))
        self._server.add_insecure_port("unix://" + os.path.abspath(self.socket))
        self._server.start()
        return self

    def stop(self) -> None:
        for w in self._watches.values():
            w.cancel()
        self._watches.clear()
        for c in self._clients.values():
            c.close()
        self._clients.clear()
        if self._server is not None:
            self._server.stop(0).wait(2.0)
            self._server = None
        try:
            os.remove(self.socket)
        except FileNotFoundError:
            pass

    def restart(self) -> None:
        """Delete + recreate kubelet.sock (what a kubelet restart looks like on disk)."""
        self.stop()
        time.sleep(0.05)
        self.start()

    def wait_for_registrations(self, count: int, timeout: float = 10.0) -> list:
        deadline = time.monotonic() + timeout
        with self.registered:
            while len(self.requests) < count:
                left = deadline - time.monotonic()
                if left <= 0:
                    raise TimeoutError("expected %d registrations, got %d" % (count, len(self.requests)))
                self.registered.wait(left)
            return list(self.requests)

    def client(self, endpoint: str) -> DevicePluginClient:
        if endpoint not in self._clients:
            self._clients[endpoint] = DevicePluginClient(os.path.join(self.plugin_dir, endpoint))
        return self._clients[endpoint]

    def watch(self, endpoint: str, new: bool = False) -> _Watch:
        """The stream kubelet keeps on ``endpoint`` (``new``: open another, as kubelet
        does after a Register)."""
        if new or endpoint not in self._watches:
            self._watches[endpoint] = _Watch(self.client(endpoint))
        return self._watches[endpoint]

    def __enter__(self) -> "KubeletStub":
        return self.start()

    def __exit__(self, *exc) -> None:
        self.stop()


class PodResourcesStub:
    """In-process kubelet PodResources ``v1`` server (``List`` only) on a unix socket.
    ``set_pods([(namespace, pod, [(container, resource, [device ids])])])``."""

    def __init__(self, socket_path: str) -> None:
        from ..api import podresources_v1 as pr
        self._pr = pr
        self.socket_path = socket_path
        self._resp = pr.ListPodResourcesResponse()
        self._lock = threading.Lock()
        self.calls = 0
        self._server = None

    def set_pods(self, pods) -> None:
        pr = self._pr
        resp = pr.ListPodResourcesResponse()
        for ns, name, containers in pods:
            p = resp.pod_resources.add(name=name, namespace=ns)
            for cname, resource, ids in containers:
                c = p.containers.add(name=cname)
                c.devices.add(resource_name=resource, device_ids=list(ids))
        with self._lock:
            self._resp = resp

    def start(self) -> "PodResourcesStub":
        pr = self._pr

        def list_(req, ctx):
            with self._lock:
                self.calls += 1
                return self._resp

        handler = grpc.method_handlers_generic_handler(pr.SERVICE, {
            "List": grpc.unary_unary_rpc_method_handler(
                list_, request_deserializer=pr.ListPodResourcesRequest.FromString,
                response_serializer=pr.ListPodResourcesResponse.SerializeToString)})
        os.makedirs(os.path.dirname(self.socket_path), exist_ok=True)
        self._server = grpc.server(concurrent.futures.ThreadPoolExecutor(max_workers=2))
        self._server.add_generic_rpc_handlers((handler,))
        self._server.add_insecure_port("unix://" + self.socket_path)
        self._server.start()
        return self

    def stop(self) -> None:
        if self._server is not None:
            self._server.stop(grace=0.2).wait(2.0)
            self._server = None
        try:
            os.remove(self.socket_path)
        except FileNotFoundError:
            pass
