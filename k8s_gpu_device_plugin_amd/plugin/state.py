"""Health latches that outlive the plugin process.

The reference keeps no health state at all (its health channel has no producer,
``/root/reference/plugin/plugin.go:181-186``, defect D9), so a restart cannot lose any.
This plugin latches two verdicts that no later sample can re-derive:

  * an uncorrectable-ECC latch (``native/health.cpp``): the UE counter only tells that it
    grew, and a restarted process would take the grown count as its new baseline;
  * failed gfx950 canaries (PreStartContainer and recovery canaries, held by the manager).

Without persistence a DaemonSet rolling update, an OOM kill or a crash re-advertises such
a GPU Healthy although nothing reset it.  The state file keeps them, keyed by GPU identity
(UUID, else BDF) and by the host's boot id: a reboot resets every GPU, so a file from an
earlier boot is ignored.  Each latched GPU also records when its power-management
firmware started (``fw_boot_s``); a process that finds the firmware started later knows
the GPU was reset while no plugin watched and clears the latch on the first sample.

The file is JSON, written atomically (temporary file + rename) and only when its content
changes; a plugin that cannot write it keeps serving with in-memory latches.
"""
from __future__ import annotations

import json
import os
import time

from ..utils.log import get_logger

log = get_logger("state")

BOOT_ID_PATH = "/proc/sys/kernel/random/boot_id"
VERSION = 1


def read_boot_id(path: str | None = None) -> str:
    # AMDGPU_DP_BOOT_ID_FILE: tests stand in for a reboot with another file
    path = path or os.environ.get("AMDGPU_DP_BOOT_ID_FILE") or BOOT_ID_PATH
    try:
        with open(path, "r", encoding="ascii") as f:
            return f.read().strip()
    except OSError:
        return ""


def _i64(v) -> int:
    """int(v) that fits the native latch's int64 fields (ValueError otherwise)."""
    i = int(v)
    if not -(1 << 63) <= i < (1 << 63):
        raise ValueError("%r out of range" % v)
    return i


class HealthState:
    """Reader/writer of the state file.  ``snapshot`` dicts look like::

        {"ecc": {key: {"last_ue": int, "fw_boot_s": float | None, "reason": str, "since_ns": int}},
         "canary_failed": {key: [partition, ...]},   # -1 = the whole GPU
         "held": [key, ...]}                          # recovery canary pending or failed
    """

    def __init__(self, path: str, boot_id: str | None = None) -> None:
        self.path = path
        self.boot_id = boot_id if boot_id is not None else read_boot_id()
        self._written: dict | None = None
        self.write_errors = 0
        self.writes = 0

    def load(self) -> dict | None:
        """The snapshot the previous process of this boot left, or None."""
        try:
            with open(self.path, "r", encoding="utf-8") as f:
                raw = json.load(f)
        except FileNotFoundError:
            return None
        except (OSError, ValueError) as e:
            log.warning("ignoring unreadable health state file %s: %s", self.path, e)
            return None
        if not isinstance(raw, dict) or raw.get("version") != VERSION:
            log.warning("ignoring health state file %s: unknown format", self.path)
            return None
        if not self.boot_id or raw.get("boot_id") != self.boot_id:
            log.info("health state file %s is from another boot of this host: every GPU was reset since; "
                     "starting without its latches", self.path)
            return None
        snap = {"ecc": {}, "canary_failed": {}, "held": []}
        gpus = raw.get("gpus")
        for key, g in (gpus.items() if isinstance(gpus, dict) else ()):
            if not isinstance(g, dict):
                continue
            try:  # a damaged entry costs that GPU its latches, never the start-up
                ecc = g.get("ecc")
                if isinstance(ecc, dict):
                    fw = ecc.get("fw_boot_s")
                    e = {"last_ue": _i64(ecc.get("last_ue", -1)),
                         "fw_boot_s": None if fw is None else float(fw),
                         "reason": str(ecc.get("reason", "")),
                         "since_ns": _i64(ecc.get("since_ns", 0))}
                parts = g.get("canary_failed_partitions")
                parts = sorted({int(p) for p in parts}) if isinstance(parts, list) and parts else None
            except (TypeError, ValueError, OverflowError) as err:
                log.warning("ignoring the damaged health state of %s in %s: %s", key, self.path, err)
                continue
            if isinstance(ecc, dict):
                snap["ecc"][str(key)] = e
            if parts:
                snap["canary_failed"][str(key)] = parts
            if g.get("recovery_canary_held"):
                snap["held"].append(str(key))
        self._written = snap
        return snap

    def save(self, snap: dict) -> bool:
        """Writes ``snap`` unless it equals what is on disk.  Returns True on a write."""
        if snap == self._written:
            return False
        gpus: dict = {}
        for key, e in snap.get("ecc", {}).items():
            gpus.setdefault(key, {})["ecc"] = dict(e)
        for key, parts in snap.get("canary_failed", {}).items():
            gpus.setdefault(key, {})["canary_failed_partitions"] = sorted(parts)
        for key in snap.get("held", []):
            gpus.setdefault(key, {})["recovery_canary_held"] = True
        doc = {"version": VERSION, "boot_id": self.boot_id, "written_unix": round(time.time(), 3),
               "gpus": {k: gpus[k] for k in sorted(gpus)}}
        tmp = "%s.tmp.%d" % (self.path, os.getpid())
        try:
            os.makedirs(os.path.dirname(self.path) or ".", exist_ok=True)
            with open(tmp, "w", encoding="utf-8") as f:
                json.dump(doc, f, indent=1, sort_keys=True)
                f.flush()
                os.fsync(f.fileno())
            os.replace(tmp, self.path)
        except OSError as e:
            self.write_errors += 1
            if self.write_errors == 1:
                log.error("cannot persist health latches to %s: %s (they are kept in memory only)", self.path, e)
            try:
                os.remove(tmp)
            except OSError:
                pass
            return False
        self._written = {"ecc": {k: dict(v) for k, v in snap.get("ecc", {}).items()},
                         "canary_failed": {k: list(v) for k, v in snap.get("canary_failed", {}).items()},
                         "held": list(snap.get("held", []))}
        self.writes += 1
        return True
