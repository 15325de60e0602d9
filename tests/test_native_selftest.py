"""Builds and runs the standalone C++ self-test, plain and under ASan+UBSan and TSan
(the reference never ran a race detector and has real races)."""
import subprocess

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
