"""libFuzzer + ASan + UBSan smoke runs of every peer-facing native parser
(tests/native/fuzz/*.cpp): kubelet protobuf decoding with the allocator contract, HPACK,
the HTTP/2 gRPC server and the HTTP/1.1 ops server.  The reference never fuzzed its
(Go) parsers; ours are hand-written C++, so each target runs a few seconds per test
run and longer on demand: ``python -m k8s_gpu_device_plugin_amd._build --fuzz``."""
import os

import pytest

from k8s_gpu_device_plugin_amd import _build

SECONDS = float(os.environ.get("FUZZ_SECONDS", "6"))


@pytest.mark.parametrize("target", _build.FUZZ_TARGETS)
def test_fuzz_target(target):
    try:
        _build.clangxx_path()
    except RuntimeError as e:
        pytest.skip(str(e))
    p = _build.run_fuzzer(target, SECONDS)
    assert p.returncode == 0, p.stdout[-6000:]
    assert "Done" in p.stdout or "stat::number_of_executed_units" in p.stdout
    execs = [int(ln.split()[-1]) for ln in p.stdout.splitlines() if ln.startswith("stat::number_of_executed_units")]
    assert execs and execs[0] > 1000, p.stdout[-2000:]
