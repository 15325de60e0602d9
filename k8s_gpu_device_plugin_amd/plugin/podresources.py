"""Which pod holds which advertised device: a poller of the kubelet PodResources API.

Polls ``v1.PodResourcesLister/List`` every ``podResources.intervalS`` seconds. For
the plugin's own resources it keeps the map from ``(resource, device_id)`` to
``(namespace, pod, container)``. A change posts one event to the manager, which
republishes ``amdgpu_device_plugin_allocation_info``. With that family, per-GPU and
per-partition telemetry joins to workloads in PromQL:

    amdgpu_partition_gfx_busy_percent
      * on (device_id) group_left (namespace, pod, container)
      amdgpu_device_plugin_allocation_info

This is not in the reference. Its device plugin never learns what kubelet did with an
allocation.
"""
from __future__ import annotations

import threading
import time

import grpc

from ..api import podresources_v1 as pr
from ..utils.log import get_logger

log = get_logger("podresources")

Allocation = dict  # {(resource, device_id): (namespace, pod, container)}


def list_allocations(socket_path: str, resource_prefix: str, timeout: float = 5.0) -> Allocation:
    """One ``List`` call; keeps the devices of ``<resource_prefix>/`` resources."""
    ch = grpc.insecure_channel("unix://" + socket_path, options=[("grpc.enable_http_proxy", 0)])
    try:
        call = ch.unary_unary(pr.METHOD_LIST, request_serializer=pr.ListPodResourcesRequest.SerializeToString,
                              response_deserializer=pr.ListPodResourcesResponse.FromString)
        resp = call(pr.ListPodResourcesRequest(), timeout=timeout)
    finally:
        from .plugin import close_async
        close_async(ch)  # Channel.close() would block the poller ~200 ms per poll
    out: Allocation = {}
    prefix = resource_prefix.rstrip("/") + "/"
    for pod in resp.pod_resources:
        for c in pod.containers:
            for d in c.devices:
                if not d.resource_name.startswith(prefix):
                    continue
                for dev in d.device_ids:
                    out[(d.resource_name, dev)] = (pod.namespace, pod.name, c.name)
    return out


def checkpoint_allocations(path: str, resource_prefix: str) -> set:
    """``{(resource, device_id)}`` from kubelet's device-manager checkpoint
    (``<device-plugins dir>/kubelet_internal_checkpoint``): every device kubelet has
    handed to a pod it still tracks.  Read when PodResources is not polled (a plugin
    restarting on a busy node).  Understands both layouts kubelet has written
    (``DeviceIDs`` as a list, and as a NUMA-node -> list map); an unreadable file is
    an empty set."""
    import json
    try:
        with open(path, "r", encoding="utf-8") as f:
            raw = json.load(f)
    except (OSError, ValueError):
        return set()
    data = raw.get("Data") if isinstance(raw, dict) else None
    entries = data.get("PodDeviceEntries") if isinstance(data, dict) else None
    prefix = resource_prefix.rstrip("/") + "/"
    out = set()
    for e in entries if isinstance(entries, list) else []:
        if not isinstance(e, dict) or not str(e.get("ResourceName", "")).startswith(prefix):
            continue
        ids = e.get("DeviceIDs")
        if isinstance(ids, dict):
            ids = [d for v in ids.values() if isinstance(v, list) for d in v]
        for d in ids if isinstance(ids, list) else []:
            out.add((str(e["ResourceName"]), str(d)))
    return out


def _esc(v: str) -> str:
    return str(v).replace("\\", "\\\\").replace('"', '\\"').replace("\n", "\\n")


def render(allocs: Allocation, up: bool | None) -> list[str]:
    """Exposition lines for the manager's extra block."""
    lines = []
    if up is not None:
        lines += ["# HELP amdgpu_device_plugin_pod_resources_up 1 if the last kubelet PodResources List succeeded.",
                  "# TYPE amdgpu_device_plugin_pod_resources_up gauge",
                  "amdgpu_device_plugin_pod_resources_up %d" % int(up)]
    if allocs:
        lines += ["# HELP amdgpu_device_plugin_allocation_info Advertised device held by a container (value 1).",
                  "# TYPE amdgpu_device_plugin_allocation_info gauge"]
        for (res, dev), (ns, pod, ctr) in sorted(allocs.items()):
            lines.append('amdgpu_device_plugin_allocation_info{resource="%s",device_id="%s",namespace="%s",'
                         'pod="%s",container="%s"} 1' % (_esc(res), _esc(dev), _esc(ns), _esc(pod), _esc(ctr)))
    return lines


class PodResourcesWatcher:
    """Background poller.  ``on_change()`` runs on the poller thread; the manager
    passes a function that only enqueues an event."""

    def __init__(self, socket_path: str, interval_s: float, resource_prefix: str, on_change) -> None:
        self.socket_path = socket_path
        self.interval_s = max(0.05, float(interval_s))
        self.resource_prefix = resource_prefix
        self.on_change = on_change
        self.allocations: Allocation = {}
        self.up: bool | None = None
        self.polls = 0
        # CLOCK_MONOTONIC ns at which the List behind `allocations` was sent: every
        # Allocate answered before it is in the map (kubelet records the devices at
        # admission, before the containers start)
        self.covered_until_ns = 0
        self._stop = threading.Event()
        self._thread: threading.Thread | None = None
        self._lock = threading.Lock()

    def snapshot(self) -> tuple[Allocation, bool | None]:
        with self._lock:
            return dict(self.allocations), self.up

    # kubelet adds a container's devices to the map PodResources List reads only after
    # the plugin's Allocate answer came back (and its own bookkeeping ran): a List sent
    # within this window of an Allocate may not show it yet, so allocations that recent
    # are not counted as covered by that List
    COVER_GRACE_NS = 2_000_000_000

    def covered_until(self) -> int:
        """mono ns before which every allocation is in the last map: the last List's send
        time less the grace above (0 while no List has succeeded)."""
        with self._lock:
            return max(0, self.covered_until_ns - self.COVER_GRACE_NS) if self.covered_until_ns else 0

    def poll_once(self) -> bool:
        """Returns True when the allocation map or the up state changed."""
        t0 = time.monotonic_ns()
        try:
            allocs, up = list_allocations(self.socket_path, self.resource_prefix), True
        except Exception as e:  # kubelet restarting, socket not mounted, API disabled
            allocs, up = self.allocations, False
            if self.up is not False:
                log.warning("kubelet PodResources List failed on %s: %s", self.socket_path, e)
        with self._lock:
            self.polls += 1
            changed = allocs != self.allocations or up != self.up
            self.allocations, self.up = allocs, up
            if up:
                changed = changed or self.covered_until_ns == 0
                self.covered_until_ns = t0
        return changed

    def start(self) -> None:
        def loop():
            from .manager import background_thread
            background_thread()
            while not self._stop.is_set():
                if self.poll_once():
                    self.on_change()
                self._stop.wait(self.interval_s)

        self._thread = threading.Thread(target=loop, name="pod-resources", daemon=True)
        self._thread.start()

    def stop(self) -> None:
        self._stop.set()
        if self._thread is not None:
            self._thread.join(5.0)
            self._thread = None
