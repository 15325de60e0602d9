"""canary.run_isolated's reading of the child's output (CPU; the child itself runs in
tests/test_gpu.py)."""
import subprocess

from k8s_gpu_device_plugin_amd.ops import canary


def _fake(monkeypatch, stdout, rc, stderr=""):
    monkeypatch.setattr(subprocess, "run", lambda cmd, **kw: subprocess.CompletedProcess(cmd, rc, stdout, stderr))


def test_result_line_is_the_last_json_object(monkeypatch):
    _fake(monkeypatch, 'HIP banner\n{"ok": true, "device": 3}\n7\n', 0)
    assert canary.run_isolated(3) == {"ok": True, "device": 3}


def test_ok_line_from_a_crashed_child_is_not_a_pass(monkeypatch):
    _fake(monkeypatch, '{"ok": true, "device": 0}\n', -11, "Segmentation fault at teardown")
    r = canary.run_isolated(0)
    assert r["ok"] is False and "exited -11" in r["error"]


def test_no_result_line(monkeypatch):
    _fake(monkeypatch, "nothing useful\n", 1, "hipErrorNoDevice")
    r = canary.run_isolated(1)
    assert r["ok"] is False and "hipErrorNoDevice" in r["error"]


def test_timeout(monkeypatch):
    def boom(cmd, **kw):
        raise subprocess.TimeoutExpired(cmd, kw.get("timeout"))
    monkeypatch.setattr(subprocess, "run", boom)
    r = canary.run_isolated(2, timeout=0.5)
    assert r["ok"] is False and "timed out" in r["error"]
