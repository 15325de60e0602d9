"""Builds and runs the standalone C++ self-test, plain and under ASan+UBSan and TSan
(the reference never ran a race detector and has real races)."""
import os
import subprocess
import sys

import pytest

from k8s_gpu_device_plugin_amd import _build


@pytest.mark.timeout(900)  # a fresh instrumented build of the core takes minutes on a small host
@pytest.mark.parametrize("sanitize", [None, "address", "thread"])
def test_native_selftest(sanitize):
    exe = _build.build_selftest(sanitize)
    env = {"TSAN_OPTIONS": "halt_on_error=1 exitcode=66", "ASAN_OPTIONS": "detect_leaks=1:halt_on_error=1",
           "UBSAN_OPTIONS": "halt_on_error=1:print_stacktrace=1", "PATH": "/usr/bin:/bin"}
    p = subprocess.run([exe], stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=600, env=env)
    assert p.returncode == 0, p.stdout[-4000:]
    assert "native selftest: ok" in p.stdout
    assert "ThreadSanitizer" not in p.stdout and "AddressSanitizer" not in p.stdout


def test_production_extension_carries_no_harness():
    """The plugin's own extension has no load generator in it: those
    live in the bench extension (tests/native/loadgen.cpp), which the plugin never loads."""
    from k8s_gpu_device_plugin_amd import native
    n = native.load()
    for name in ("http_load", "grpc_load", "uds_pingpong", "UdsPinger", "render_bench", "health_propagation",
                 "h2_bench_unary"):
        assert not hasattr(n, name), name
    syms = subprocess.run(["nm", "-DC", _build.native_ext_path()], stdout=subprocess.PIPE, text=True).stdout
    for sym in ("amdgpu_dp::http_load", "amdgpu_dp::grpc_load", "amdgpu_dp::uds_pingpong", "amdgpu_dp::h2_bench_unary",
                "amdgpu_dp::health_propagation"):
        assert sym not in syms, sym
    b = native.load_bench()
    assert callable(b.http_load) and hasattr(n.H2Client, "bench_unary")
    # and the daemon never imports it
    out = subprocess.run([sys.executable, "-c", "import sys; from k8s_gpu_device_plugin_amd.plugin import manager; "
                          "from k8s_gpu_device_plugin_amd import cli; "
                          "print('_native_bench' in ' '.join(sys.modules))"], stdout=subprocess.PIPE, text=True,
                         cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    assert out.stdout.strip() == "False"
