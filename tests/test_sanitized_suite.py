"""The integration tests, re-run against a sanitizer-instrumented build of the native
core ("run the integration suite under them").

``test_native_selftest`` covers the C++ core on its own; this runs the Python-driven
paths through the same instrumented code: the kubelet stub against both gRPC servers,
the manager's lifecycle and health hand-over, the HTTP ops server and the exporter.
The extension is built once under ``build/ext-<sanitizer>/`` and loaded through
``AMDGPU_DP_NATIVE_SO`` by a child pytest that preloads the sanitizer runtime (python
itself is not instrumented).  A sanitizer report anywhere fails the run: the runtime
writes it to a log file, since it aborts the process before pytest can show output.
"""
import glob
import os
import subprocess
import sys

import pytest

from k8s_gpu_device_plugin_amd import _build

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SUITES = {
    "address": ["tests/test_grpc_native.py", "tests/test_plugin_e2e.py", "tests/test_manager.py",
                "tests/test_http.py", "tests/test_telemetry_health.py", "tests/test_prestart.py",
                "tests/test_allocator.py", "tests/test_v1beta1_wire.py", "tests/test_device_subset.py",
                "tests/test_checkpoint_resume.py", "tests/test_chaos.py", "tests/test_wedged_gpu.py",
                "tests/test_health_latches.py", "tests/test_canary_scope.py"],
    "thread": ["tests/test_grpc_native.py", "tests/test_plugin_e2e.py", "tests/test_manager.py",
               "tests/test_http.py", "tests/test_telemetry_health.py", "tests/test_prestart.py",
               "tests/test_chaos.py", "tests/test_wedged_gpu.py", "tests/test_health_latches.py",
               "tests/test_canary_scope.py"],
}


def run_sanitized(sanitize: str, tests, log_dir: str, extra_args=()) -> subprocess.CompletedProcess:
    ext = _build.build_native_sanitized(sanitize)
    preload = [_build.sanitizer_runtime(sanitize)]
    # libstdc++ must be mapped before the sanitizer resolves its __cxa_throw interceptor
    # (python does not link it, so a C++ exception would hit a null "real" function)
    preload.append(os.path.realpath(subprocess.run([_build._cxx(), "-print-file-name=libstdc++.so"],
                                                   stdout=subprocess.PIPE, text=True).stdout.strip()))
    rep = os.path.join(log_dir, "report")
    env = dict(os.environ)
    env.update({
        "LD_PRELOAD": ":".join(preload + ([env["LD_PRELOAD"]] if env.get("LD_PRELOAD") else [])),
        "AMDGPU_DP_NATIVE_SO": ext, "AMDGPU_DP_NO_AUTOBUILD": "1",
        "ASAN_OPTIONS": "detect_leaks=0:halt_on_error=1:log_path=" + rep,
        "UBSAN_OPTIONS": "halt_on_error=1:print_stacktrace=1:log_path=" + rep,
        # python, grpcio and libstdc++ are not instrumented: their synchronisation is
        # invisible, so accesses they make through interceptors are not checked; every
        # access from our instrumented code is
        "TSAN_OPTIONS": "halt_on_error=1:exitcode=66:ignore_noninstrumented_modules=1:log_path=" + rep,
    })
    cmd = [sys.executable, "-m", "pytest", "-q", "-m", "not gpu", "-p", "no:cacheprovider", "-x",
           "--timeout", "300"] + list(extra_args) + list(tests)
    return subprocess.run(cmd, cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                          timeout=1500)


@pytest.mark.slow
@pytest.mark.timeout(1800)  # an instrumented build plus the whole integration suite: past pytest.ini's 300 s
@pytest.mark.parametrize("sanitize", ["address", "thread"])
def test_integration_suite_under_sanitizer(sanitize, tmp_path):
    if os.environ.get("AMDGPU_DP_NATIVE_SO"):
        pytest.skip("already running against an alternative native build")
    p = run_sanitized(sanitize, SUITES[sanitize], str(tmp_path))
    reports = "".join(open(f).read() for f in sorted(glob.glob(str(tmp_path / "report*"))))
    assert not reports, reports[:6000]
    assert p.returncode == 0, p.stdout[-6000:]
    assert " passed" in p.stdout
    # the run really used the instrumented build
    syms = subprocess.run(["nm", "-D", "--undefined-only", _build.sanitized_ext_path(sanitize)],
                          stdout=subprocess.PIPE, text=True).stdout
    assert ("__tsan_func_entry" if sanitize == "thread" else "__asan_report_load8") in syms
