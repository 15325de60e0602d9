"""Read-only probe: which per-GPU values could tell an unprivileged pod that a GPU was
reset, without amdsmi event notification (which needs /dev/kfd)?

A GPU reset (mode-1 / whole-GPU) reloads the power-management firmware (PMFW).  The
PMFW stamps every gpu_metrics table with its own clock (``firmware_timestamp``, 10 ns
ticks since the firmware started) and counts its accumulation cycles
(``accumulation_counter``); both restart near zero when the firmware restarts.  This
probe records, for each GPU:

  * both counters across a few samples (they must be monotonic while nothing resets),
  * the firmware's implied uptime against the host's (/proc/uptime): firmware uptime
    shorter than the host's means the GPU's firmware restarted after the host booted,
  * the driver-stamped ``system_clock_counter`` and ``energy_accumulator`` for reference,
  * whether the same blob is readable straight from sysfs (``gpu_metrics``) by this user,
  * the host boot id (the persisted health state is keyed by it).

We cannot reset a GPU on the shared box (read-only, non-root); the record shows the
signal is present, monotonic and readable without privileges.  The plugin uses it in
native/health.cpp (firmware clock regression -> reset observed).
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import time


def _read(path: str):
    try:
        with open(path, "rb") as f:
            return f.read()
    except OSError as e:
        return e


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--samples", type=int, default=5)
    ap.add_argument("--interval", type=float, default=0.5)
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    import amdsmi

    out = {"uid": os.getuid(), "boot_id": _read("/proc/sys/kernel/random/boot_id").decode().strip(),
           "host_uptime_s": float(_read("/proc/uptime").split()[0]), "gpus": []}
    amdsmi.amdsmi_init(amdsmi.AmdSmiInitFlags.INIT_AMD_GPUS)
    try:
        handles = amdsmi.amdsmi_get_processor_handles()
        rows = {i: [] for i in range(len(handles))}
        for _ in range(args.samples):
            for i, h in enumerate(handles):
                t = time.monotonic()
                m = amdsmi.amdsmi_get_gpu_metrics_info(h)
                rows[i].append({"mono_s": round(t, 4),
                                **{k: m.get(k) for k in ("firmware_timestamp", "accumulation_counter",
                                                         "system_clock_counter", "energy_accumulator")}})
            time.sleep(args.interval)
        for i, h in enumerate(handles):
            bdf = amdsmi.amdsmi_get_gpu_device_bdf(h)
            r = rows[i]
            fw = [x["firmware_timestamp"] for x in r if isinstance(x["firmware_timestamp"], int)]
            acc = [x["accumulation_counter"] for x in r if isinstance(x["accumulation_counter"], int)]
            g = {"index": i, "bdf": bdf, "uuid": amdsmi.amdsmi_get_gpu_device_uuid(h), "samples": r,
                 "fw_monotonic": all(b > a for a, b in zip(fw, fw[1:])) if len(fw) > 1 else None,
                 "acc_monotonic": all(b >= a for a, b in zip(acc, acc[1:])) if len(acc) > 1 else None}
            if len(fw) > 1:
                dt = r[-1]["mono_s"] - r[0]["mono_s"]
                g["fw_ticks_per_s"] = (fw[-1] - fw[0]) / dt if dt > 0 else None
                g["fw_uptime_s_at_10ns"] = fw[-1] * 1e-8
                g["fw_uptime_lt_host"] = fw[-1] * 1e-8 < out["host_uptime_s"]
            # the same table straight from sysfs, if this user may read it
            dev = glob.glob("/sys/bus/pci/devices/%s/gpu_metrics" % bdf.lower())
            blob = _read(dev[0]) if dev else None
            g["sysfs_gpu_metrics"] = (None if blob is None else
                                      ("error: %s" % blob) if isinstance(blob, Exception) else "%d bytes" % len(blob))
            # anything in the device's sysfs directory that names a reset
            base = "/sys/bus/pci/devices/%s" % bdf.lower()
            g["sysfs_reset_files"] = sorted(os.path.relpath(p, base) for p in glob.glob(base + "/*reset*"))
            out["gpus"].append(g)
    finally:
        amdsmi.amdsmi_shut_down()
    text = json.dumps(out, indent=1, default=str)
    print(text)
    if args.out:
        with open(args.out, "w") as f:
            f.write(text + "\n")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
