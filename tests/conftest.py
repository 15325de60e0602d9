"""Shared fixtures.  GPU tests are marked ``@pytest.mark.gpu`` and run only on a real
MI355X (``pytest -m gpu``); everything else runs on CPU against the fixture backend."""
import os
import sys
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real AMD Instinct MI355X (gfx950)")
    config.addinivalue_line("markers", "slow: takes more than a few seconds")


@pytest.fixture(scope="session")
def n():
    from k8s_gpu_device_plugin_amd import native
    return native.load()


@pytest.fixture
def plugin_dir():
    # short path: unix socket paths are limited to 108 bytes
    d = tempfile.mkdtemp(prefix="dp-", dir="/tmp")
    yield d
    import shutil
    shutil.rmtree(d, ignore_errors=True)


@pytest.fixture
def make_cfg(plugin_dir):
    from k8s_gpu_device_plugin_amd import config as config_mod

    def _make(**over):
        raw = {"backend": "fixture", "fixture": "2gpu_spx", "pluginDir": plugin_dir, "log": {"fileDir": ""},
               "telemetry": {"intervalMs": 100}, "grpc": {"server": "python"}, "retrySeconds": 0.5}
        for k, v in over.items():
            if isinstance(v, dict) and isinstance(raw.get(k), dict):
                raw[k] = {**raw[k], **v}
            else:
                raw[k] = v
        return config_mod.validate(config_mod.from_dict(raw))
    return _make
