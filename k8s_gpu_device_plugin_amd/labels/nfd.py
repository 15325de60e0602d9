"""Node labels for schedulers (Node Feature Discovery "local" feature file).

Not in the reference (it advertises resources only).  Pods that need a particular
partition layout (a TP job wanting whole SPX GPUs, a CPX inference fleet) select nodes
by label; NFD's local source turns ``<key>=<value>`` lines from
``/etc/kubernetes/node-feature-discovery/features.d/<file>`` into node labels.  With
``nodeFeatureFile`` set, the manager (re)writes that file atomically whenever the
inventory is (re)loaded, so a partition-mode change is reflected in the labels.

Labels (prefix ``amd.com/``)::

    gpu.present=true                   gpu.count=8
    gpu.product=AMD_Instinct_MI355X    gpu.family=gfx950
    gpu.vram-gb=288                    gpu.compute-units=256
    gpu.compute-partition=CPX          gpu.memory-partition=NPS2   (when uniform)
    gpu.partitions=64                  gpu.xgmi-links=7
    gpu.device-id=75a3                 gpu.driver-version=6.14.14
    gpu.vbios-version=<IFWI version>   (each when the driver reports it)
    gpu.mixed-partitions=true          (when GPUs differ)
"""
from __future__ import annotations

import os
import re
import tempfile

PREFIX = "amd.com/"
_VALUE_BAD = re.compile(r"[^A-Za-z0-9._-]")


def _value(v) -> str:
    """Kubernetes label values: <= 63 chars of [A-Za-z0-9._-], alphanumeric ends."""
    s = _VALUE_BAD.sub("_", str(v))[:63].strip("._-")
    return s or "unknown"


def node_labels(gpus) -> dict:
    if not gpus:
        return {PREFIX + "gpu.present": "false"}
    g0 = gpus[0]
    labels = {
        PREFIX + "gpu.present": "true",
        PREFIX + "gpu.count": str(len(gpus)),
        PREFIX + "gpu.product": _value(g0.market_name),
        PREFIX + "gpu.family": _value(g0.gfx_target or "unknown"),
        PREFIX + "gpu.vram-gb": str(int(round(g0.vram_total_bytes / 1e9))),
        PREFIX + "gpu.partitions": str(sum(len(g.partitions) for g in gpus)),
    }
    if g0.num_compute_units:
        labels[PREFIX + "gpu.compute-units"] = str(g0.num_compute_units)
    if g0.num_xgmi_links:
        labels[PREFIX + "gpu.xgmi-links"] = str(g0.num_xgmi_links)
    # what AMD's node labeller publishes too: pods pinned to a driver / firmware level
    # (a validated stack) select nodes by these
    # (one label value per node: left out while the GPUs disagree, e.g. mid firmware update)
    for key, attr in (("gpu.device-id", "device_id"), ("gpu.driver-version", "driver_version"),
                      ("gpu.vbios-version", "vbios_version")):
        vals = {getattr(g, attr, "") for g in gpus}
        if len(vals) == 1 and next(iter(vals)):
            v = next(iter(vals))
            labels[PREFIX + key] = "%04x" % v if isinstance(v, int) else _value(v)
    modes = {(g.compute_partition, g.memory_partition) for g in gpus}
    if len(modes) == 1:
        cp, mp = next(iter(modes))
        labels[PREFIX + "gpu.compute-partition"] = _value(cp)
        labels[PREFIX + "gpu.memory-partition"] = _value(mp)
    else:
        labels[PREFIX + "gpu.mixed-partitions"] = "true"
    return labels


def write_feature_file(path: str, labels: dict) -> str:
    """Atomic replace so NFD never reads a torn file."""
    d = os.path.dirname(os.path.abspath(path))
    os.makedirs(d, exist_ok=True)
    fd, tmp = tempfile.mkstemp(prefix=".nfd-", dir=d)
    with os.fdopen(fd, "w") as f:
        for k in sorted(labels):
            f.write("%s=%s\n" % (k, labels[k]))
    os.chmod(tmp, 0o644)
    os.replace(tmp, path)
    return path
