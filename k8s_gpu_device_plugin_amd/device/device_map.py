"""Strategy -> ``{resource name: Devices}`` builder.

Reference ``device/device_map.go:24-125``: none/single use ``VisitDevices`` and match
the product name against the resource pattern (wildcard -> unanchored regexp), single
skips MIG-enabled GPUs, mixed visits MIG devices and matches the profile string; any
unmatched device aborts the whole build.

MI355X semantics:
  * none   - one device per physical GPU; Allocate exposes *all* its partitions'
             render nodes (a whole MI355X regardless of SPX/CPX mode).
  * single - every compute partition is one device (SPX GPU = 1, CPX GPU = 8).
  * mixed  - unpartitioned GPUs as in single under ``amd.com/gpu``-style resources,
             partitioned GPUs under ``amd.com/<cpx>_<nps>``.
Patterns are matched anchored (D15: ``1g.10gb`` must not match ``1g.10gb+me``) and an
unmatched device is skipped with a warning instead of failing every device (D3).
Optional time-slicing replicas expand each device into ``<id>::<n>``.
"""
from __future__ import annotations

import re
from collections import OrderedDict

from ..resource import STRATEGY_MIXED, STRATEGY_NONE, STRATEGY_SINGLE, Resource, ResourceName, profile_name
from ..utils.log import get_logger
from .devices import AnnotatedID, Device, Devices

log = get_logger("device")


def wildcard_to_regexp(pattern: str) -> str:
    """``*`` -> ``.*``, everything else literal (``device_map.go:114-125``), anchored."""
    return "^" + ".*".join(re.escape(p) for p in pattern.split("*")) + "$"


def matches(pattern: str, value: str) -> bool:
    return re.match(wildcard_to_regexp(pattern), value) is not None


def render_path(minor: int, dev_root: str = "/dev/dri") -> str:
    return "%s/renderD%d" % (dev_root, minor)


def card_path(minor: int, dev_root: str = "/dev/dri") -> str:
    return "%s/card%d" % (dev_root, minor)


def _paths(parts, mount_card: bool) -> list[str]:
    out = []
    for p in parts:
        if p.render_minor >= 0:
            out.append(render_path(p.render_minor))
        if mount_card and p.card_minor >= 0:
            out.append(card_path(p.card_minor))
    return out


def _numa(n: int) -> int | None:
    return n if n is not None and n >= 0 else None


def build_device_map(gpus, resources: list[Resource], strategy: str, mount_card: bool = False,
                     replicas: int = 1, rename_shared: bool = False) -> "OrderedDict[str, Devices]":
    dm: "OrderedDict[str, Devices]" = OrderedDict((str(r.name), Devices()) for r in resources)

    def pick(candidates, value) -> Resource | None:
        for r in candidates:
            if matches(r.pattern, value):
                return r
        return None

    if strategy not in (STRATEGY_NONE, STRATEGY_SINGLE, STRATEGY_MIXED):
        raise ValueError("invalid partition strategy: %r" % strategy)
    for g in gpus:
        nparts = len(g.partitions)
        profile = profile_name(g.compute_partition, g.memory_partition)
        if strategy == STRATEGY_NONE:
            r = pick(resources, g.market_name)
            if r is None:
                log.warning("GPU %d (%s) matches no resource pattern; skipped", g.index, g.market_name)
                continue
            dm[str(r.name)].add(Device(
                id=g.uuid, index=str(g.index), gpu=g.index, partition=-1, numa_node=_numa(g.numa_node),
                paths=_paths(g.partitions, mount_card), total_memory=g.vram_total_bytes,
                compute_capability=g.gfx_target, product=g.market_name, profile=profile))
            continue
        if strategy == STRATEGY_MIXED and nparts > 1:
            cands = [r for r in resources if r.pattern == profile] or \
                    [r for r in resources if matches(r.pattern, profile)]
            value = profile
        else:
            cands = [r for r in resources if not _is_profile_resource(r)] if strategy == STRATEGY_MIXED else resources
            value = g.market_name
        r = pick(cands, value)
        if r is None:
            log.warning("GPU %d (%s, %s) matches no resource pattern; skipped", g.index, g.market_name, profile)
            continue
        for p in g.partitions:
            dm[str(r.name)].add(Device(
                id=p.id, index=str(g.index) if nparts == 1 else "%d:%d" % (g.index, p.index), gpu=g.index,
                partition=-1 if nparts == 1 else p.index, numa_node=_numa(p.numa_node),
                paths=_paths([p], mount_card), total_memory=p.vram_bytes, compute_capability=g.gfx_target,
                product=g.market_name, profile=profile))
    if replicas > 1:
        out: "OrderedDict[str, Devices]" = OrderedDict()
        for name, devs in dm.items():
            rn = str(ResourceName(name).default_shared_rename()) if rename_shared else name
            expanded = Devices()
            for d in devs:
                for k in range(replicas):
                    expanded.add(Device(**{**d.__dict__, "id": str(AnnotatedID.new(d.id, k)),
                                           "replicas": replicas, "replica": k}))
            out[rn] = expanded
        dm = out
    return dm


def _is_profile_resource(r: Resource) -> bool:
    return re.fullmatch(r"[a-z]px_nps\d", r.pattern) is not None
