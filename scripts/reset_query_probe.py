"""Read-only probe of the second unprivileged reset signal: the
amdgpu driver's own reset count, read through a context on each GPU's render node
(native/drm_reset.cpp, ``health.resetQuery``).

The firmware-clock signal (scripts/reset_signal_probe.py) only sees resets that reload
the power-management firmware.  This box supports engine/queue resets
(``compute_reset_mask`` / ``sdma_reset_mask``), and a mode-2 reset keeps the firmware
running; the kernel's reset counter moves for every reset the driver performs.  Records,
per GPU: the render node, whether this (non-root) user can open it, the reset count the
plugin's amdsmi backend reads over a few samples (0 while nothing resets; -1 = the node
could not be opened), the firmware clock alongside, and the reset masks the driver
exposes.  We cannot reset a GPU on the shared box: the record shows the query is
available and quiet without privileges.

    python scripts/reset_query_probe.py [--samples 5] [--out FILE]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _read(path: str):
    try:
        with open(path) as f:
            return f.read().strip()
    except OSError as e:
        return "error: %s" % e.strerror


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--samples", type=int, default=5)
    ap.add_argument("--interval", type=float, default=0.5)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    from k8s_gpu_device_plugin_amd import native
    n = native.load()
    be = n.make_amdsmi_backend()
    out = {"uid": os.getuid(), "kernel": os.uname().release,
           "boot_id": _read("/proc/sys/kernel/random/boot_id"), "gpus": []}
    try:
        gpus, _ = be.discover()
        rows = {g.index: [] for g in gpus}
        for _ in range(a.samples):
            for g in gpus:
                s = be.sample(g.index)
                rows[g.index].append({"reset_count": s.reset_count, "fw_clock_s": round(s.fw_clock_s, 3), "ok": s.ok}
                                     if s is not None else {"reset_count": -1, "fw_clock_s": None, "ok": False})
            time.sleep(a.interval)
        for g in gpus:
            minor = g.partitions[0].render_minor if g.partitions else -1
            node = "/dev/dri/renderD%d" % minor
            try:
                fd = os.open(node, os.O_RDWR | os.O_CLOEXEC)
                os.close(fd)
                opens = True
            except OSError as e:
                opens = "error: %s" % e.strerror
            base = "/sys/bus/pci/devices/%s" % g.bdf.lower()
            masks = {m: _read("%s/%s" % (base, m)) for m in ("compute_reset_mask", "sdma_reset_mask",
                                                              "jpeg_reset_mask", "vcn_reset_mask")
                     if os.path.exists("%s/%s" % (base, m))}
            counts = [r["reset_count"] for r in rows[g.index]]
            out["gpus"].append({"index": g.index, "bdf": g.bdf, "uuid": g.uuid, "render_node": node,
                                "render_node_opens": opens, "samples": rows[g.index],
                                "reset_query_available": all(c >= 0 for c in counts),
                                "resets_seen": max(counts) if counts and min(counts) >= 0 else None,
                                "reset_masks": masks})
    finally:
        be.shutdown()
    text = json.dumps(out, indent=1)
    print(text)
    if a.out:
        with open(a.out, "w") as f:
            f.write(text + "\n")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
