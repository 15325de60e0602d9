"""Container Device Interface (CDI) spec for the advertised devices.

With ``cdi: true`` the Allocate response names devices as ``amd.com/gpu=<device id>``
(``ContainerAllocateResponse.cdi_devices``) instead of relying only on DeviceSpecs; a
CDI-enabled runtime (containerd >= 1.7, CRI-O) resolves those names through a spec file
in ``/var/run/cdi``.  The reference has no CDI support (its Allocate returns only an env
var, ``plugin/plugin.go:217-221``).

One spec per resource kind, e.g. ``/var/run/cdi/amd.com-gpu.json``::

    {"cdiVersion": "0.6.0", "kind": "amd.com/gpu",
     "containerEdits": {"deviceNodes": [{"path": "/dev/kfd"}]},
     "devices": [{"name": "<id>", "containerEdits": {"deviceNodes": [{"path": "/dev/dri/renderD128"}]}}]}

Per-device edits carry no env: with two devices in one container, two
``AMD_VISIBLE_DEVICES=<id>`` edits would conflict (last one wins).  The visible-devices
list comes from Allocate's env, which names every allocated device.
"""
from __future__ import annotations

import json
import os
import tempfile

CDI_VERSION = "0.6.0"


def _node(path: str) -> dict:
    return {"path": path, "permissions": "rw"}


def build_spec(kind: str, devices, kfd_path: str = "/dev/kfd") -> dict:
    out = []
    for d in devices:
        out.append({"name": d.get_uuid(), "containerEdits": {"deviceNodes": [_node(p) for p in d.paths]}})
    # replicas share one CDI device (the name is the base id)
    uniq, seen = [], set()
    for d in out:
        if d["name"] not in seen:
            seen.add(d["name"])
            uniq.append(d)
    return {"cdiVersion": CDI_VERSION, "kind": kind,
            "containerEdits": {"deviceNodes": [_node(kfd_path)] if kfd_path else []},
            "devices": uniq}


# The device plugin's own access to /dev/kfd (deploy/kfd-cdi-patch.yaml): the pod names
# PLUGIN_KFD_DEVICE in a cdi.k8s.io/ annotation and the runtime adds the node and its
# device-cgroup rule, no privileged container needed.
PLUGIN_KIND = "amd.com/device-plugin"
PLUGIN_KFD_DEVICE = PLUGIN_KIND + "=kfd"


def plugin_kfd_spec(kfd_path: str = "/dev/kfd", render_nodes=()) -> dict:
    """``render_nodes``: the GPUs' render nodes, added to the same device so the plugin can
    also read each GPU's kernel reset count (health.resetQuery; an amdgpu context on the
    node needs only the node in the container's device cgroup)."""
    nodes = [_node(kfd_path)] + [_node(p) for p in render_nodes]
    return {"cdiVersion": CDI_VERSION, "kind": PLUGIN_KIND,
            "devices": [{"name": "kfd", "containerEdits": {"deviceNodes": nodes}}]}


def amdgpu_render_nodes(dri_dir: str = "/dev/dri", sys_class: str = "/sys/class/drm") -> list:
    """The render nodes of AMD GPUs on this host (PCI vendor 0x1002), sorted."""
    out = []
    try:
        names = os.listdir(dri_dir)
    except OSError:
        return out
    for name in sorted(names, key=lambda x: (len(x), x)):
        if not name.startswith("renderD"):
            continue
        try:
            with open(os.path.join(sys_class, name, "device", "vendor")) as f:
                if f.read().strip().lower() != "0x1002":
                    continue
        except OSError:
            continue
        out.append(os.path.join(dri_dir, name))
    return out


def spec_path(spec_dir: str, kind: str) -> str:
    return os.path.join(spec_dir, kind.replace("/", "-") + ".json")


def write_spec(spec_dir: str, spec: dict) -> str:
    """Atomic write (temp file + rename) so a runtime never reads a torn spec."""
    os.makedirs(spec_dir, exist_ok=True)
    path = spec_path(spec_dir, spec["kind"])
    fd, tmp = tempfile.mkstemp(prefix=".cdi-", dir=spec_dir)
    with os.fdopen(fd, "w") as f:
        json.dump(spec, f, indent=1, sort_keys=True)
    os.chmod(tmp, 0o644)
    os.replace(tmp, path)
    return path
