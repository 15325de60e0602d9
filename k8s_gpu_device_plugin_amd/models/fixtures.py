"""Hardware node models for the fixture backend (MI355X nodes without the hardware).

An MI355X node (OAM, 8 GPUs) is a full xGMI mesh: each GPU has 7 links, one direct
link to every peer.  Each GPU has 8 XCDs x 32 CUs and 288 GB HBM3E
(MI355X_MICROARCH.md); compute partitioning splits the XCDs: SPX 1, DPX 2, QPX 4,
CPX 8 partitions.

Partition model, pinned to what the box reports (``profiles/r4/amdsmi_probe.json``):
the current profile is SPX with memory caps NPS1|NPS2, and the memory-partition config
reports the same caps.  The driver's full profile list needs root (NO_PERM for the box's
user), so the fixture table lists the profiles 8 XCDs form (SPX/DPX/QPX/CPX) with those
caps.  A GPU may not declare a compute/memory mode outside its profile table:
``build_backend`` rejects it.  The BASELINE config names "CPX+NPS4", which this hardware
does not expose; ``8gpu_cpx_nps4`` is kept only as a declared hypothetical (it brings its
own profile table, marked ``hypothetical``), the measured config is ``8gpu_cpx_nps2``.

A node model is a plain dict (also loadable from JSON/YAML)::

    {"gpus": [{"compute_partition": "CPX", "memory_partition": "NPS2",
               "numa_node": 0, ...}, ...],
     "links": {"type": "xgmi", "down": [[0, 5]]},
     "events": [{"at": 2.0, "kind": "pre_reset", "gpu": 3}, ...],
     "hardware_events": true,   # false: no event notification (an unprivileged pod)
     "seed": 1}

Per GPU, ``ecc_uncorrectable`` sets the UE count the hardware reports from the start and
``fw_clock: false`` stops samples reporting the firmware clock; ``reset_query: true`` makes
them report the kernel's reset count (a plugin that can open the render node).
"""
from __future__ import annotations

import json
import os

import yaml

from .. import native

PARTITIONS = {"SPX": 1, "DPX": 2, "TPX": 3, "QPX": 4, "CPX": 8}
# recorded on the MI355X box (profiles/r4/amdsmi_probe.json): memory caps of the current
# profile and of the memory-partition config
MI355X_MEMORY_CAPS = ("NPS1", "NPS2")
# compute profiles of a gfx950 with 8 XCDs (partitions per GPU)
MI355X_PROFILES = (("SPX", 1), ("DPX", 2), ("QPX", 4), ("CPX", 8))
NPS_BITS = {"NPS1": 1, "NPS2": 2, "NPS4": 4, "NPS8": 8}
MI355X_HBM_BYTES = 288 * 10**9
MI355X_CUS = 256
MI355X_NAME = "AMD Instinct MI355X"
MI355X_DEVICE_ID = "0x75a3"  # PCI device id amdsmi reports on the MI355X box
FIXTURE_DRIVER_VERSION = "6.14.14"
FIXTURE_VBIOS_VERSION = "FIXTURE-VBIOS"

EVENT_KINDS = {
    "pre_reset": "EVT_PRE_RESET", "post_reset": "EVT_POST_RESET",
    "ecc_uncorrectable": "EVT_ECC_UNCORRECTABLE", "link_down": "EVT_LINK_DOWN",
    "link_up": "EVT_LINK_UP", "thermal": "EVT_THERMAL", "vm_fault": "EVT_VM_FAULT",
    "device_lost": "EVT_DEVICE_LOST", "device_recovered": "EVT_DEVICE_RECOVERED",
    # not an event: the GPU's firmware restarts (a reset as an unprivileged poller sees it)
    "firmware_reset": "EVT_FIXTURE_FIRMWARE_RESET",
}


def fixture_uuid(seed: int, gpu: int) -> str:
    return "%08x-0000-1000-80%02x-%012x" % (0x5a000000 + seed, gpu, 0x355000 + gpu)


def mi355x_node(num_gpus: int = 8, compute: str = "SPX", memory: str = "NPS1", gpus_per_numa: int = 4,
                nps_caps=("NPS1", "NPS2"), down_links=(), seed: int = 1, events=(), slow_links=(),
                hip_order=None) -> dict:
    """slow_links: [(a, b, gbps)] links that trained below the nominal 608 Gb/s.
    hip_order: GPUs (by BDF rank) in the order the HIP runtime numbers them (default: the
    same order); the runtime's numbering need not follow BDF order on every platform."""
    gpus = []
    for g in range(num_gpus):
        gpus.append({"compute_partition": compute, "memory_partition": memory,
                     "numa_node": g // max(1, gpus_per_numa), "nps_caps": list(nps_caps)})
    m = {"gpus": gpus, "links": {"type": "xgmi", "down": [list(p) for p in down_links],
                                 "slow": [list(p) for p in slow_links]},
         "events": list(events), "seed": seed}
    if hip_order is not None:
        m["hip_order"] = list(hip_order)
    return m


BUILTIN = {
    "1gpu_spx": lambda: mi355x_node(1),
    "2gpu_spx": lambda: mi355x_node(2),
    "4gpu_spx": lambda: mi355x_node(4),
    "8gpu_spx_mesh": lambda: mi355x_node(8),
    "8gpu_dpx_nps2": lambda: mi355x_node(8, "DPX", "NPS2"),
    "8gpu_qpx_nps2": lambda: mi355x_node(8, "QPX", "NPS2"),
    "8gpu_cpx_nps2": lambda: mi355x_node(8, "CPX", "NPS2"),
    # hypothetical: NPS4 is not exposed by MI355X (caps NPS1|NPS2 on the box); declared
    # with its own profile table so the 64-device CPX path can also run under "NPS4"
    "8gpu_cpx_nps4": lambda: dict(mi355x_node(8, "CPX", "NPS4", nps_caps=("NPS1", "NPS2", "NPS4")),
                                  hypothetical=True,
                                  profiles=[{"type": t, "partitions": k, "nps": ["NPS1", "NPS2", "NPS4"]}
                                            for t, k in MI355X_PROFILES]),
    "8gpu_spx_degraded": lambda: mi355x_node(8, down_links=[(0, 5), (2, 3)]),
    # one xGMI link trained at half rate (x8 instead of x16): up, but half the bandwidth
    "8gpu_spx_halfrate": lambda: mi355x_node(8, slow_links=[(0, 1, 304.0)]),
    # HIP ordinals permuted against BDF order (bench.py maps ranks by HIP ordinal)
    "2gpu_spx_hip_swapped": lambda: mi355x_node(2, hip_order=[1, 0]),
    "4gpu_spx_hip_permuted": lambda: mi355x_node(4, hip_order=[2, 0, 3, 1]),
}
XGMI_LINK_GBPS = 608.0  # MI355X: 16 lanes x 38 Gb/s per xGMI link (what amdsmi reports)


def load_model(spec) -> dict:
    """``spec``: builtin name, path to .json/.yaml, or a dict."""
    if isinstance(spec, dict):
        return spec
    if spec in BUILTIN:
        return BUILTIN[spec]()
    m = None
    if isinstance(spec, str) and os.path.isfile(spec):
        with open(spec, "r", encoding="utf-8") as f:
            m = json.load(f) if spec.endswith(".json") else yaml.safe_load(f)
    if m is None:
        # "<n>gpu_<mode>_<nps>" shorthand, e.g. 3gpu_qpx_nps2
        parts = str(spec).split("_")
        if len(parts) >= 2 and parts[0].endswith("gpu") and parts[0][:-3].isdigit():
            mode = parts[1].upper()
            nps = parts[2].upper() if len(parts) > 2 else "NPS1"
            if mode in PARTITIONS and nps in NPS_BITS:
                return mi355x_node(int(parts[0][:-3]), mode, nps)
        raise ValueError("unknown fixture %r (builtins: %s)" % (spec, ", ".join(sorted(BUILTIN))))
    return m


def _partitions(n, gpu_index: int, uuid: str, nparts: int, numa: int, vram: int, first_render: int,
                hip_base: int | None = None):
    parts = []
    hip_base = gpu_index * nparts if hip_base is None else hip_base
    for p in range(nparts):
        pi = n.PartitionInfo()
        pi.gpu = gpu_index
        pi.index = p
        pi.uuid = uuid if nparts == 1 else "%s-%d" % (uuid, p)
        pi.id = uuid if nparts == 1 else "%s-xcp%d" % (uuid, p)
        pi.render_minor = first_render + p
        pi.card_minor = first_render - 128 + p
        pi.hip_id = hip_base + p
        pi.hsa_id = hip_base + p
        pi.kfd_node = 1 + gpu_index * nparts + p
        pi.numa_node = numa
        pi.vram_bytes = vram // nparts
        parts.append(pi)
    return parts


def set_gpu_mode(backend, gpu_index: int, compute: str, memory: str = "NPS1", first_render: int = 200) -> None:
    """Simulates an operator re-partitioning one GPU (amd-smi set --compute-partition):
    the GPU's partitions (and their render nodes) are replaced.  ``gpu_index`` is the
    model's slot; the description is the model's own, not a discovery's (whose indices
    shift while a GPU is missing or left out)."""
    n = native.load()
    g = backend.slot_info(gpu_index)
    g.compute_partition, g.memory_partition = compute.upper(), memory.upper()
    if g.supported_profiles:  # the operator can only pick a mode the GPU supports
        check_mode(gpu_index, g.compute_partition, g.memory_partition, g.supported_profiles)
    g.partitions = _partitions(n, gpu_index, g.uuid, PARTITIONS[g.compute_partition], g.numa_node,
                               g.vram_total_bytes, first_render)
    g.partition_profile, g.profile_partitions = g.compute_partition, PARTITIONS[g.compute_partition]
    g.profile_index = list(PARTITIONS).index(g.compute_partition)
    backend.replace_gpu(gpu_index, g)


def profile_table(n, model: dict, g: dict, caps_mask: int):
    """The partition profiles a fixture GPU supports: the model's own ``profiles`` (a
    declared hypothetical part), else MI355X's with the GPU's memory caps."""
    out = []
    for i, p in enumerate(g.get("profiles") or model.get("profiles") or
                          [{"type": t, "partitions": k} for t, k in MI355X_PROFILES]):
        mask = caps_mask
        if "nps" in p:
            mask = 0
            for c in p["nps"]:
                mask |= NPS_BITS[str(c).upper()]
        out.append(n.PartitionProfile(str(p["type"]).upper(), int(p["partitions"]), mask, i, "fixture"))
    return out


def check_mode(gi: int, compute: str, memory: str, profiles) -> None:
    """A GPU cannot be in a compute/memory mode its profile table does not list."""
    for p in profiles:
        if p.type == compute and p.nps_caps & NPS_BITS.get(memory, 0):
            return
    raise ValueError("fixture GPU %d declares %s+%s, outside its supported profiles (%s); declare a profile "
                     "table (\"profiles\") to model a hypothetical part" % (
                         gi, compute, memory, ", ".join("%s[%s]" % (p.type, "|".join(
                             k for k, b in NPS_BITS.items() if p.nps_caps & b)) for p in profiles)))


def build_backend(spec):
    """Creates a native FixtureBackend populated from a node model."""
    n = native.load()
    model = load_model(spec)
    seed = int(model.get("seed", 1))
    be = n.FixtureBackend(seed)
    gpus = model.get("gpus", [])
    nparts_of = [int(g.get("num_partitions", PARTITIONS.get(str(g.get("compute_partition", "SPX")).upper(), 1)))
                 for g in gpus]
    order = list(model.get("hip_order") or range(len(gpus)))
    if sorted(order) != list(range(len(gpus))):
        raise ValueError("hip_order must be a permutation of the GPU indices: %r" % (order,))
    hip_base = {}
    nxt = 0
    for gi in order:  # the HIP runtime numbers partitions GPU after GPU in this order
        hip_base[gi] = nxt
        nxt += nparts_of[gi]
    render = 128
    for gi, g in enumerate(gpus):
        info = n.GpuInfo()
        info.uuid = g.get("uuid") or fixture_uuid(seed, gi)
        info.bdf = g.get("bdf") or "0000:%02x:00.0" % (0x05 + 0x10 * gi)
        info.market_name = g.get("name", MI355X_NAME)
        info.gfx_target = g.get("gfx_target", "gfx950")
        info.serial = g.get("serial", "FIXTURE%04d" % gi)
        info.numa_node = int(g.get("numa_node", 0))
        info.vram_total_bytes = int(g.get("vram_bytes", MI355X_HBM_BYTES))
        info.compute_partition = str(g.get("compute_partition", "SPX")).upper()
        info.memory_partition = str(g.get("memory_partition", "NPS1")).upper()
        caps = 0
        for c in g.get("nps_caps", list(MI355X_MEMORY_CAPS)):
            caps |= NPS_BITS[str(c).upper()]
        info.nps_caps = caps
        info.supported_profiles = profile_table(n, model, g, caps)
        info.profiles_status = "ok"
        check_mode(gi, info.compute_partition, info.memory_partition, info.supported_profiles)
        info.num_compute_units = int(g.get("num_cus", MI355X_CUS))
        info.device_id = int(str(g.get("device_id", MI355X_DEVICE_ID)), 0)
        info.oam_id = int(g.get("oam_id", gi))
        info.driver_version = str(g.get("driver_version", FIXTURE_DRIVER_VERSION))
        info.vbios_version = str(g.get("vbios_version", FIXTURE_VBIOS_VERSION))
        info.bad_page_threshold = int(g.get("bad_page_threshold", -1))  # -1: RAS threshold not readable
        nparts = int(g.get("num_partitions", PARTITIONS.get(info.compute_partition, 1)))
        # what amdsmi_get_gpu_accelerator_partition_profile reports for the mode
        info.partition_profile = info.compute_partition
        info.profile_partitions = int(g.get("profile_partitions", nparts))
        info.profile_index = list(PARTITIONS).index(info.compute_partition) if info.compute_partition in PARTITIONS else -1
        info.num_xgmi_links = max(0, len(gpus) - 1)
        info.partitions = _partitions(n, gi, info.uuid, nparts, info.numa_node, info.vram_total_bytes, render,
                                      hip_base[gi])
        render += nparts
        be.add_gpu(info)
        if int(g.get("ecc_uncorrectable", 0)):
            be.set_ecc_uncorrectable(gi, int(g["ecc_uncorrectable"]))
        if not g.get("fw_clock", True):
            be.set_fw_clock_reported(gi, False)
        if g.get("reset_query", False):  # the render node can be opened: kernel reset counts
            be.set_gpu_reset_query(gi, True)
    links = model.get("links", {}) or {}
    ltype = {"xgmi": n.LINK_XGMI, "pcie": n.LINK_PCIE}.get(str(links.get("type", "xgmi")).lower(), n.LINK_XGMI)
    down = {tuple(sorted(p)) for p in links.get("down", [])}
    slow = {tuple(sorted(p[:2])): float(p[2]) for p in links.get("slow", [])}
    for a in range(len(gpus)):
        for b in range(a + 1, len(gpus)):
            xgmi = ltype == n.LINK_XGMI
            be.set_link(a, b, n.Link(type=ltype, hops=1, weight=15 if xgmi else 40, up=(a, b) not in down, p2p=True,
                                     bw_gbps=slow.get((a, b), XGMI_LINK_GBPS) if xgmi else 0.0))
    be.set_events_enabled(bool(model.get("hardware_events", True)))
    for ev in model.get("events", []) or []:
        kind = getattr(n, EVENT_KINDS[str(ev["kind"]).lower()])
        be.schedule_event(float(ev.get("at", 0.0)),
                          n.HwEvent(kind, int(ev.get("gpu", -1)), int(ev.get("partition", -1)),
                                    int(ev.get("peer", -1)), str(ev.get("message", "scripted"))))
    be.discover()  # usable at once, like an amdsmi session that enumerated at init
    return be
