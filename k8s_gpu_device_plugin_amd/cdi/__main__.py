"""``python -m k8s_gpu_device_plugin_amd.cdi plugin-kfd --spec-dir /var/run/cdi``

Writes the CDI spec that gives the device plugin's own container ``/dev/kfd`` without
``privileged: true`` (``deploy/kfd-cdi-patch.yaml`` runs it as an init container and
names the device in a ``cdi.k8s.io/`` pod annotation).  A hostPath mount of /dev/kfd is
not in the container's device cgroup; a CDI device node edit is, so amdsmi event
notification (GPU reset, thermal, VM fault) can be armed by an unprivileged pod.  The
AMD GPUs' render nodes go into the same device, for the kernel reset count
(``health.resetQuery``), unless ``--no-render-nodes``.
"""
from __future__ import annotations

import argparse
import sys

from .spec import amdgpu_render_nodes, plugin_kfd_spec, write_spec


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="python -m k8s_gpu_device_plugin_amd.cdi")
    sub = ap.add_subparsers(dest="cmd", required=True)
    p = sub.add_parser("plugin-kfd", help="CDI spec giving the device plugin's container /dev/kfd")
    p.add_argument("--spec-dir", default="/var/run/cdi")
    p.add_argument("--kfd", default="/dev/kfd")
    p.add_argument("--no-render-nodes", action="store_true",
                   help="leave out the GPUs' render nodes (then health.resetQuery has nothing to open)")
    p.add_argument("--dri-dir", default="/dev/dri")
    args = ap.parse_args(argv)
    renders = [] if args.no_render_nodes else amdgpu_render_nodes(args.dri_dir)
    path = write_spec(args.spec_dir, plugin_kfd_spec(args.kfd, renders))
    print("wrote", path)
    return 0


if __name__ == "__main__":
    sys.exit(main())
