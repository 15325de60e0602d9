"""Process bootstrap / supervisor: ``python -m k8s_gpu_device_plugin_amd``.

Reference ``main.go:30-162``: ``--configFile`` flag, viper config, logger, plugin
manager, web server, ``oklog/run`` group of three actors (signal handler, manager,
web server gated on ``pluginReady``) and an optional pprof benchmark.

Kept: the flag (``--configFile``, lookup ``./<name>.yml``), SIGHUP/SIGINT/SIGQUIT/
SIGTERM -> graceful exit, "first actor to finish stops the others".  Fixed: the web
server is not gated on the plugins being ready (D20: /health must come up even when
no GPU is usable), profiles are flushed on every exit path (D19), and the process
exit code reports a fatal manager error.
"""
from __future__ import annotations

import argparse
import signal
import sys
import threading

from . import config as config_mod
from .utils.log import get_logger, init_logger
from .utils.util import CloseOnce
from .utils.version import APP_NAME, VERSION


def parse_args(argv=None) -> argparse.Namespace:
    ap = argparse.ArgumentParser(prog="k8s_gpu_device_plugin_amd",
                                 description="MI355X Kubernetes device plugin (amd.com/gpu)")
    ap.add_argument("--configFile", default="config", help="name of config file (without extension) or a path")
    ap.add_argument("--configDir", default=".", help="directory searched for <configFile>.yml")
    ap.add_argument("--backend", choices=["auto", "amdsmi", "fixture"], help="override config backend")
    ap.add_argument("--fixture", help="fixture node model (builtin name or file) for backend=fixture")
    ap.add_argument("--plugin-dir", dest="pluginDir", help="kubelet device-plugin directory")
    ap.add_argument("--web-listen-address", dest="webListenAddress", help="host:port of the HTTP ops server")
    ap.add_argument("--strategy", dest="migStrategy", choices=["none", "single", "mixed"])
    ap.add_argument("--log-level")
    ap.add_argument("--log-dir")
    ap.add_argument("--devices", help="GPUs to advertise: indices (e.g. 0-3), UUIDs or PCI BDFs")
    ap.add_argument("--version", action="store_true")
    ap.add_argument("--inspect", nargs="?", const="", metavar="SIZES",
                    help="print what would be advertised and where pods of SIZES devices (e.g. 2,4,8) would be "
                         "placed, as JSON, and exit (nothing is served)")
    return ap.parse_args(argv)


def _exit_with_parent() -> bool:
    """AMDGPU_DP_PARENT_PID (benchmarks and probes that spawn a daemon): SIGTERM this
    process when that parent exits, so a harness killed mid-run leaves no daemon behind.
    False if the parent is already gone."""
    import os
    want = os.environ.get("AMDGPU_DP_PARENT_PID")
    if not want:
        return True
    try:
        import ctypes
        ctypes.CDLL(None, use_errno=True).prctl(1, int(signal.SIGTERM), 0, 0, 0)  # PR_SET_PDEATHSIG
    except (OSError, AttributeError):
        pass
    return os.getppid() == int(want)


def main(argv=None) -> int:
    args = parse_args(argv)
    if not _exit_with_parent():
        return 1
    if args.version:
        print("%s %s" % (APP_NAME, VERSION))
        return 0
    try:
        cfg = config_mod.load(args.configFile, search_dirs=(args.configDir,))
    except config_mod.ConfigError as e:
        print("fatal config error: %s" % e, file=sys.stderr)
        return 2
    for k in ("backend", "fixture", "pluginDir", "webListenAddress", "migStrategy", "devices"):
        v = getattr(args, k)
        if v is not None:
            setattr(cfg, k, v)
    if args.log_level:
        cfg.log.level = args.log_level
    if args.log_dir is not None:
        cfg.log.fileDir = args.log_dir
    try:  # the command-line overrides are checked like the file's values
        config_mod.validate(cfg)
    except config_mod.ConfigError as e:
        print("fatal config error: %s" % e, file=sys.stderr)
        return 2
    if args.inspect is not None:
        from .inspect_node import main as inspect_main
        init_logger("error", None, APP_NAME, console=True)  # stdout carries the JSON only
        sizes = [int(x) for x in args.inspect.split(",") if x.strip()] if args.inspect else None
        return inspect_main(cfg, sizes)
    init_logger(cfg.log.level, cfg.log.fileDir or None, APP_NAME, console=cfg.log.console,
                max_age_days=cfg.log.maxAgeDays)
    log = get_logger()
    log.info("Starting %s %s", APP_NAME, VERSION)

    from .plugin.manager import PluginManager
    from .server.web import WebServer

    ready = CloseOnce()
    manager = PluginManager(cfg, ready)
    web = WebServer(cfg, manager)
    bench = None
    if cfg.benchmark:
        from .benchmark.profiling import Benchmark
        bench = Benchmark(cfg.benchmarkDir, render_metrics=manager.exporter.render)
        bench.run()

    done = threading.Event()
    reason = {"why": ""}

    def on_signal(signum, _frame):
        reason["why"] = reason["why"] or "messaged %s, exiting gracefully..." % signal.Signals(signum).name
        # not done.set() here: the handler runs on the main thread between any two
        # bytecodes, also while that thread holds done's lock inside done.wait() (e.g.
        # just woken by the parent watch's set), and the lock is not re-entrant
        threading.Thread(target=done.set, name="signal", daemon=True).start()

    for s in (signal.SIGHUP, signal.SIGINT, signal.SIGQUIT, signal.SIGTERM):
        signal.signal(s, on_signal)

    def run_manager():
        try:
            manager.start()
        except Exception as e:  # pragma: no cover
            log.exception("plugin manager crashed: %s", e)
            manager.fatal_error = str(e)
        finally:
            reason["why"] = reason["why"] or "plugin manager stopped"
            done.set()

    mt = threading.Thread(target=run_manager, name="plugin-manager", daemon=True)
    rc = 0
    import os
    parent = int(os.environ.get("AMDGPU_DP_PARENT_PID") or 0)
    poll_parent = bool(parent) and not _watch_parent(parent, reason, done)
    try:
        web.start()
        mt.start()
        # (signals interrupt the wait; the parent check is the only reason to poll, and
        # only where the kernel has no pidfd to wait on)
        while not done.wait(0.5 if poll_parent else 5.0):
            if poll_parent and os.getppid() != parent:  # the harness is gone (PDEATHSIG backstop)
                reason["why"] = "parent process %d exited, exiting gracefully..." % parent
                break
    except Exception as e:
        log.error("error starting web server: %s", e)
        rc = 1
    finally:
        log.info(reason["why"] or "shutting down")
        web.stop()
        manager.stop()
        mt.join(10)
        if bench is not None:
            bench.stop()
    if manager.fatal_error:
        rc = 1
    log.info("see you next time!")
    return rc


def _watch_parent(parent: int, reason: dict, done: threading.Event) -> bool:
    """A thread blocked on a pidfd of the harness process that started this daemon ends
    the daemon when that process exits: no periodic wake-up for it.  False where the
    kernel or Python has no pidfd (the caller polls getppid instead)."""
    import os
    import select
    try:
        fd = os.pidfd_open(parent)
    except (AttributeError, OSError):
        return False

    def wait():
        from .utils.util import name_os_thread
        name_os_thread("parent-watch")
        try:
            p = select.poll()  # (not select(): no FD_SETSIZE limit on the descriptor)
            p.register(fd, select.POLLIN)
            while not p.poll():
                pass
        finally:
            os.close(fd)
        reason["why"] = reason["why"] or "parent process %d exited, exiting gracefully..." % parent
        done.set()

    threading.Thread(target=wait, name="parent-watch", daemon=True).start()
    return True


if __name__ == "__main__":
    sys.exit(main())
