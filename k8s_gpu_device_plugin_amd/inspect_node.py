"""``python -m k8s_gpu_device_plugin_amd --inspect``: what the plugin would advertise on
this node, and where it would place multi-device pods, without serving anything.

An operator's question when a pod lands on the "wrong" GPUs, or a resource is missing
from the node's allocatable, is what the plugin saw.  This runs the same discovery,
strategy, device map and native allocator as the daemon (same config file and flags),
and prints one JSON document:

* ``gpus``: each physical GPU (index, UUID, BDF, product, gfx target, partition modes,
  NUMA node, partitions with their render nodes, driver / VBIOS versions) and one
  telemetry reading of it (power, hotspot temperature, ECC, retired pages, PCIe and
  xGMI link width / rate);
* ``resources``: each advertised resource name with its device IDs and health;
* ``xgmi``: every GPU pair's link (type, up, trained bandwidth, amdsmi weight, hops);
* ``placement``: per resource and request size, the devices GetPreferredAllocation
  would return with every device available (what kubelet gets for a fresh pod).

The reference has no equivalent (its allocator rebuilt the NVML view per call and
logged nothing).
"""
from __future__ import annotations

import json

LINK_TYPES = {0: "internal", 1: "pcie", 2: "xgmi", 3: "n/a", 4: "unknown"}


def _sample(backend, index: int) -> dict:
    """One telemetry reading of the GPU (what the health checks look at), -1 = unknown."""
    try:
        s = backend.sample(index)
    except Exception as e:  # a GPU that cannot be read is worth showing as such
        return {"error": str(e)}
    if s is None or not s.ok:
        return {"ok": False}
    return {"ok": True, "power_w": s.power_w, "temp_hotspot_c": s.temp_hotspot_c,
            "ecc_uncorrectable": s.ecc_uncorrectable, "retired_pages": s.retired_pages,
            "pcie_link_width": s.pcie_link_width, "pcie_link_speed_gtps": s.pcie_link_speed_gtps,
            "xgmi_link_width": s.xgmi_link_width, "xgmi_link_speed_gbps": s.xgmi_link_speed}


def inspect(cfg, sizes=None) -> dict:
    """The node as the daemon would advertise it under ``cfg`` (no sockets, no threads)."""
    import copy

    from .plugin.manager import PluginManager

    cfg = copy.deepcopy(cfg)  # a look, not a deployment: no CDI specs, node labels or canaries
    cfg.cdi, cfg.nodeFeatureFile = False, ""
    cfg.health.canaryOnStart = False
    m = PluginManager(cfg)
    try:
        m.load_plugins()
        gpus = []
        for g in m.gpus:
            gpus.append({
                "index": g.index, "uuid": g.uuid, "bdf": g.bdf, "product": g.market_name, "gfx": g.gfx_target,
                "compute_partition": g.compute_partition, "memory_partition": g.memory_partition,
                "numa_node": g.numa_node, "compute_units": g.num_compute_units, "vram_bytes": g.vram_total_bytes,
                "xgmi_links": g.num_xgmi_links, "oam_id": g.oam_id, "device_id": "%04x" % g.device_id,
                "driver_version": g.driver_version, "vbios_version": g.vbios_version,
                "partitions": [{"index": p.index, "id": p.id, "render_minor": p.render_minor, "hip_id": p.hip_id}
                               for p in g.partitions],
                "now": _sample(m.backend, g.index)})
        resources, placement = {}, {}
        for p in m.plugins:
            ids = list(p.table.ids())
            resources[str(p.resource)] = [{"id": d.id, "index": d.index, "health": d.health, "numa": d.numa_node}
                                          for d in p.devices()]
            want = sizes if sizes else [s for s in (2, 4, 8) if s <= len(ids)]
            placement[str(p.resource)] = {}
            for s in want:
                try:
                    placement[str(p.resource)][str(s)] = list(p.table.preferred_ids(ids, [], int(s)))
                except RuntimeError as e:
                    placement[str(p.resource)][str(s)] = {"error": str(e)}
        topo = m.topology
        xgmi = []
        if topo is not None:
            for a in range(topo.n):
                for b in range(a + 1, topo.n):
                    ln = topo.link(a, b)
                    xgmi.append({"gpus": [a, b], "type": LINK_TYPES.get(ln.type, str(ln.type)), "up": bool(ln.up),
                                 "bw_gbps": ln.bw_gbps, "weight": ln.weight, "hops": ln.hops})
        return {"backend": cfg.backend, "strategy": cfg.strategy, "gpus": gpus, "resources": resources,
                "xgmi": xgmi, "placement": placement}
    finally:
        m.exporter.stop()
        m.monitor.stop()


def main(cfg, sizes=None) -> int:
    print(json.dumps(inspect(cfg, sizes), indent=1))
    return 0
