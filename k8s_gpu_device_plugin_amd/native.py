"""Loads the in-tree C++ core (``_native*.so``), building it first when it is missing
or older than ``native/*.cpp|h`` (g++ is part of the plugin's build image).

There is deliberately no pure-Python fallback for the core: if the extension cannot
be loaded the plugin fails loudly (a silently slower or partial plugin is worse than a
crash-looping DaemonSet pod that shows the error).

``AMDGPU_DP_NATIVE_SO=<path>`` loads another build of the same module instead, e.g. the
ASan+UBSan one from ``python -m k8s_gpu_device_plugin_amd._build --sanitize-ext address``
that ``tests/test_sanitized_suite.py`` runs the integration tests against.
"""
from __future__ import annotations

import importlib
import os
import threading

_lock = threading.Lock()
_mod = None
_bench = None


def _stale(so: str | None = None, dirs=None) -> bool:
    from . import _build
    so = so or _build.native_ext_path()
    if not os.path.exists(so):
        return True
    if not os.path.isdir(_build.NATIVE_DIR):
        return False  # installed without sources: use what ships
    t = os.path.getmtime(so)
    for d in dirs or (_build.NATIVE_DIR,):
        for f in os.listdir(d):
            if f.endswith((".cpp", ".h")) and os.path.getmtime(os.path.join(d, f)) > t:
                return True
    return False


def load():
    """Returns the ``_native`` module (building it if needed)."""
    global _mod
    if _mod is not None:
        return _mod
    with _lock:
        if _mod is not None:
            return _mod
        alt = os.environ.get("AMDGPU_DP_NATIVE_SO", "")
        if alt:
            _mod = _load_file(alt)
            return _mod
        if os.environ.get("AMDGPU_DP_NO_AUTOBUILD", "") not in ("1", "true") and _stale():
            from . import _build
            _build.build_native(verbose=False)
        try:
            _mod = importlib.import_module("k8s_gpu_device_plugin_amd._native")
        except ImportError as e:  # pragma: no cover - exercised only on broken installs
            raise RuntimeError("native core k8s_gpu_device_plugin_amd._native is not built/loadable: %s "
                               "(run: python -m k8s_gpu_device_plugin_amd._build)" % e) from e
        return _mod


def load_bench():
    """The harness extension ``_native_bench`` (load generators, latency probes): for
    bench.py, scripts/ and tests only - the plugin never imports it."""
    global _bench
    if _bench is not None:
        return _bench
    load()  # its types are _native's
    with _lock:
        if _bench is not None:
            return _bench
        from . import _build
        if os.environ.get("AMDGPU_DP_NO_AUTOBUILD", "") not in ("1", "true") and \
                _stale(_build.bench_ext_path(), (_build.NATIVE_DIR, _build.HARNESS_DIR)):
            _build.build_bench(verbose=False)
        try:
            _bench = importlib.import_module("k8s_gpu_device_plugin_amd._native_bench")
        except ImportError as e:  # pragma: no cover
            raise RuntimeError("bench extension k8s_gpu_device_plugin_amd._native_bench is not built/loadable: %s "
                               "(run: python -m k8s_gpu_device_plugin_amd._build)" % e) from e
        return _bench


def _load_file(path: str):
    import importlib.util
    import sys

    name = __package__ + "._native"
    spec = importlib.util.spec_from_file_location(name, path)
    if spec is None or not os.path.exists(path):
        raise RuntimeError("AMDGPU_DP_NATIVE_SO=%s: no such extension" % path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    sys.modules[name] = mod
    return mod
