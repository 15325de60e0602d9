"""What one telemetry pass costs, call by call, in CPU time (the idle daemon's largest
cost is its GPU's lane: ~1.7 ms of CPU per 1 s sample on MI355X, scripts/idle_wakeups.py).

Measures on the first GPU the amdsmi backend sees:
  * the backend's own per-call split (``sample_costs``: wall time per call) and the CPU
    time of a whole ``sample()``;
  * the sysfs files behind those calls read directly: open+read+close versus pread at
    offset 0 on a descriptor kept open (sysfs re-runs the attribute's show() for it),
    wall and CPU time per read.

    python scripts/sysfs_cost_probe.py [--reps 50] [--out FILE]
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def timed(fn, reps):
    fn()  # first touch
    w0, c0 = time.perf_counter_ns(), time.thread_time_ns()
    for _ in range(reps):
        fn()
    return round((time.perf_counter_ns() - w0) / reps / 1e3, 1), round((time.thread_time_ns() - c0) / reps / 1e3, 1)


def file_costs(path, reps):
    out = {}

    def reopen():
        with open(path, "rb", buffering=0) as f:
            f.read(1 << 16)
    try:
        out["open_read_close_us"] = timed(reopen, reps)
        fd = os.open(path, os.O_RDONLY)
        try:
            out["pread_us"] = timed(lambda: os.pread(fd, 1 << 16, 0), reps)
            out["bytes"] = len(os.pread(fd, 1 << 16, 0))
        finally:
            os.close(fd)
    except OSError as e:
        out["error"] = str(e)
    return out


def ras_tree(ras):
    """ras/ one level down: every small file's content (what the ECC counts read)."""
    out = {}
    for root, dirs, fnames in os.walk(ras):
        if root.count(os.sep) - ras.count(os.sep) > 1:
            continue
        for fn in fnames:
            p = os.path.join(root, fn)
            try:
                with open(p, "rb") as f:
                    data = f.read(512)
                out[os.path.relpath(p, ras)] = data.decode("ascii", "replace").strip()[:160]
            except OSError as e:
                out[os.path.relpath(p, ras)] = "error: %s" % e.strerror
    return out


def opens_during(dev, fn, reps):
    """Which sysfs files of the GPU a call opens (inotify IN_OPEN on the device directory,
    its ras/ tree and hwmon/: kernfs raises fsnotify events like any file system)."""
    import ctypes
    import select
    import struct
    libc = ctypes.CDLL(None, use_errno=True)
    fd = libc.inotify_init1(os.O_NONBLOCK)
    if fd < 0:
        return {"error": "inotify_init1 failed"}
    wds = {}
    dirs = [dev] + [r for r, _, _ in os.walk(os.path.join(dev, "ras"))] + glob.glob(os.path.join(dev, "hwmon", "hwmon*"))
    for d in dirs:
        wd = libc.inotify_add_watch(fd, d.encode(), 0x20)  # IN_OPEN
        if wd >= 0:
            wds[wd] = d
    counts = {}
    try:
        for _ in range(reps):
            fn()
        while select.select([fd], [], [], 0.05)[0]:
            buf = os.read(fd, 1 << 16)
            off = 0
            while off + 16 <= len(buf):
                wd, mask, cookie, ln = struct.unpack_from("iIII", buf, off)
                name = buf[off + 16:off + 16 + ln].rstrip(b"\0").decode()
                off += 16 + ln
                key = os.path.relpath(os.path.join(wds.get(wd, "?"), name), dev)
                counts[key] = counts.get(key, 0) + 1
    finally:
        os.close(fd)
    return {k: round(v / reps, 2) for k, v in sorted(counts.items())}


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    res = {}
    from k8s_gpu_device_plugin_amd import native
    n = native.load()
    if not n.amdsmi_available():
        raise SystemExit("amdsmi sees no AMD GPU")
    be = n.make_amdsmi_backend()
    gpus, _ = be.discover()
    g = gpus[0]
    res["gpu"] = {"bdf": g.bdf, "partitions": len(g.partitions)}
    be.sample(0)
    before = be.sample_costs()
    w0, c0 = time.perf_counter_ns(), time.process_time_ns()  # (process: wherever it runs)
    for _ in range(a.reps):
        be.sample(0)
    res["sample_us"] = {"wall": round((time.perf_counter_ns() - w0) / a.reps / 1e3, 1),
                        "cpu": round((time.process_time_ns() - c0) / a.reps / 1e3, 1)}
    after = be.sample_costs()
    be.set_reset_query(True)  # the daemon's default (health.resetQuery): one ioctl per sample
    be.sample(0)
    w0, c0 = time.perf_counter_ns(), time.process_time_ns()
    for _ in range(a.reps):
        be.sample(0)
    res["sample_with_reset_query_us"] = {"wall": round((time.perf_counter_ns() - w0) / a.reps / 1e3, 1),
                                         "cpu": round((time.process_time_ns() - c0) / a.reps / 1e3, 1)}
    # as the daemon runs it: one sample a second, caches cold in between
    cold = []
    c_before = be.sample_costs()
    for _ in range(8):
        time.sleep(1.0)
        w0, c0 = time.perf_counter_ns(), time.process_time_ns()
        be.sample(0)
        cold.append(((time.perf_counter_ns() - w0) / 1e3, (time.process_time_ns() - c0) / 1e3))
    c_after = be.sample_costs()
    res["sample_once_a_second_us"] = {"wall": round(sorted(x for x, _ in cold)[4], 1),
                                      "cpu": round(sorted(y for _, y in cold)[4], 1)}
    res["sample_once_a_second_split_wall_us"] = {k: round((c_after[k][0] - c_before[k][0]) / 8 * 1e6, 1)
                                                 for k in c_after if c_after[k][0] > 0}
    be.set_reset_query(False)
    res["sample_split_wall_us"] = {k: round((after[k][0] - before[k][0]) / a.reps * 1e6, 1) for k in after
                                   if not k.startswith(("xgmi_links_", "partition_busy_"))}
    dev = "/sys/bus/pci/devices/%s" % g.bdf.lower()
    files = [os.path.join(dev, x) for x in ("gpu_metrics", "mem_info_vram_used", "mem_info_vram_total",
                                           "ras/features", "ras/umc_err_count")]
    files += sorted(set(glob.glob(os.path.join(dev, "ras", "*_err_count")) + glob.glob(os.path.join(dev, "ras", "aca_*"))
                        + [os.path.join(dev, "ras", "event_state"), os.path.join(dev, "xgmi_error")]) - set(files))
    res["files"] = {os.path.relpath(f, dev): file_costs(f, a.reps) for f in files if os.path.exists(f)}
    try:
        res["ras_dir"] = sorted(os.listdir(os.path.join(dev, "ras")))
    except OSError as e:
        res["ras_dir"] = str(e)
    for f in glob.glob(os.path.join(dev, "ras", "*_err_count")):
        try:
            with open(f) as fh:
                res.setdefault("ras_values", {})[os.path.basename(f)] = fh.read().split()
        except OSError as e:
            res.setdefault("ras_values", {})[os.path.basename(f)] = str(e)
    res["ras_tree"] = ras_tree(os.path.join(dev, "ras"))
    res["opened_per_sample"] = opens_during(dev, lambda: be.sample(0), 5)
    be.shutdown()
    line = json.dumps(res)
    if a.out:
        with open(a.out, "w") as f:
            f.write(line + "\n")
    print(line, flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
