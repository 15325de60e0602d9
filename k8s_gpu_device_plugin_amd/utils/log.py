"""Logging: per-level rotating JSON-lines files plus stderr.

Reference ``modules/log/log.go``: zap + lumberjack, four files
``<fileDir>/<app>-{error,warn,info,debug}.log`` where each level goes only to its own
file (``:131-184``), 100 MB / 60 backups / 30 days / gzip (``:17-22``), unix-millis
timestamps (``:190-192``).  Fixed here:
  * D12: ``fatal``/``critical`` records are written (to the error file) instead of
    being dropped by exact-level enablers; messages are %-formatted.
  * D13: console output is on by default (stderr), configurable.
"""
from __future__ import annotations

import gzip
import json
import logging
import logging.handlers
import os
import shutil
import sys
import time

LEVELS = {"DEBUG": logging.DEBUG, "INFO": logging.INFO, "WARN": logging.WARNING,
          "WARNING": logging.WARNING, "ERROR": logging.ERROR}

MAX_BYTES = 100 * 1024 * 1024   # log.go:18 MaxSize 100 (MB)
BACKUP_COUNT = 60               # log.go:19 MaxBackups
LOGGER_NAME = "amdgpu_dp"

_json_reserved = set(logging.LogRecord("", 0, "", 0, "", (), None).__dict__) | {"message", "asctime"}


def parse_level(level: str) -> int:
    """Case-insensitive DEBUG/INFO/WARN/ERROR (reference ``getZapLevel`` ``log.go:258-273``)."""
    try:
        return LEVELS[str(level).strip().upper()]
    except KeyError:
        raise ValueError("unknown log level %r (want debug|info|warn|error)" % (level,)) from None


class JsonFormatter(logging.Formatter):
    """zap JSON encoder analogue: ``{"level","ts"(ms),"caller","msg", fields...}``."""

    def format(self, record: logging.LogRecord) -> str:
        out = {
            "level": record.levelname.lower().replace("warning", "warn").replace("critical", "fatal"),
            "ts": int(record.created * 1000),
            "caller": "%s:%d" % (os.path.basename(record.pathname), record.lineno),
            "msg": record.getMessage(),
        }
        for k, v in record.__dict__.items():
            if k not in _json_reserved and not k.startswith("_"):
                try:
                    json.dumps(v)
                    out[k] = v
                except TypeError:
                    out[k] = repr(v)
        if record.exc_info:
            out["error"] = self.formatException(record.exc_info)
        return json.dumps(out, ensure_ascii=False)


class _LevelBand(logging.Filter):
    """Routes [lo, hi] levels into one file, like zap's per-level tee cores."""

    def __init__(self, lo: int, hi: int) -> None:
        super().__init__()
        self.lo, self.hi = lo, hi

    def filter(self, record: logging.LogRecord) -> bool:
        return self.lo <= record.levelno <= self.hi


MAX_AGE_DAYS = 30               # log.go:20 MaxAge


def _gzip_rotator(source: str, dest: str) -> None:
    with open(source, "rb") as fi, gzip.open(dest, "wb") as fo:
        shutil.copyfileobj(fi, fo)
    os.remove(source)


def _make_rotator(file_dir: str, app: str, max_age_days: float):
    def rotate(source: str, dest: str) -> None:
        _gzip_rotator(source, dest)
        prune_old_logs(file_dir, max_age_days, app)  # lumberjack prunes on every rotation too
    return rotate


def init_logger(level: str = "debug", file_dir: str | None = "./logs", app: str = "k8s-gpu-device-plugin",
                console: bool = True, max_bytes: int = MAX_BYTES, backups: int = BACKUP_COUNT,
                max_age_days: float = MAX_AGE_DAYS) -> logging.Logger:
    """Configures and returns the package logger (idempotent: replaces handlers).
    Rotated files older than ``max_age_days`` are deleted at start and after every
    rotation (lumberjack MaxAge; 0 keeps them)."""
    logger = logging.getLogger(LOGGER_NAME)
    logger.setLevel(parse_level(level))
    for h in list(logger.handlers):
        logger.removeHandler(h)
        h.close()
    logger.propagate = False
    fmt = JsonFormatter()
    if file_dir:
        os.makedirs(file_dir, exist_ok=True)
        prune_old_logs(file_dir, max_age_days, app)
        bands = [("debug", logging.DEBUG, logging.DEBUG), ("info", logging.INFO, logging.INFO),
                 ("warn", logging.WARNING, logging.WARNING), ("error", logging.ERROR, logging.CRITICAL)]
        for name, lo, hi in bands:
            h = logging.handlers.RotatingFileHandler(os.path.join(file_dir, "%s-%s.log" % (app, name)),
                                                     maxBytes=max_bytes, backupCount=backups, encoding="utf-8")
            h.rotator = _make_rotator(file_dir, app, max_age_days)
            h.namer = lambda n: n + ".gz"
            h.addFilter(_LevelBand(lo, hi))
            h.setFormatter(fmt)
            logger.addHandler(h)
    if console:
        h = logging.StreamHandler(sys.stderr)
        h.setFormatter(fmt)
        logger.addHandler(h)
    return logger


def get_logger(name: str | None = None) -> logging.Logger:
    base = logging.getLogger(LOGGER_NAME)
    return base.getChild(name) if name else base


def prune_old_logs(file_dir: str, max_age_days: float = MAX_AGE_DAYS, app: str = "") -> int:
    """lumberjack ``MaxAge`` (30 days, ``log.go:20``): deletes rotated (``.gz``) files of
    ``app`` older than that; the live log files are never touched.  0 disables."""
    if not max_age_days or max_age_days <= 0 or not os.path.isdir(file_dir):
        return 0
    cutoff = time.time() - max_age_days * 86400
    n = 0
    for f in os.listdir(file_dir):
        if not f.endswith(".gz") or (app and not f.startswith(app + "-")):
            continue
        p = os.path.join(file_dir, f)
        try:
            if os.path.getmtime(p) < cutoff:
                os.remove(p)
                n += 1
        except OSError:  # rotated away concurrently
            pass
    return n
