"""Process-level tests: the daemon entry point (signals, config, profiling flag) and the
bench.py driver contract (single rank and 2 ranks over gloo)."""
import http.client
import json
import os
import signal
import socket
import subprocess
import sys
import time

import pytest

from k8s_gpu_device_plugin_amd.plugin.kubelet_stub import KubeletStub

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _env():
    env = dict(os.environ)
    env["PYTHONPATH"] = ROOT + os.pathsep + env.get("PYTHONPATH", "")
    return env


def test_version_and_bad_config(tmp_path):
    out = subprocess.run([sys.executable, "-m", "k8s_gpu_device_plugin_amd", "--version"], env=_env(),
                         stdout=subprocess.PIPE, text=True, timeout=60)
    assert out.returncode == 0 and out.stdout.strip() == "k8s-gpu-device-plugin 0.1.0"
    (tmp_path / "bad.yml").write_text("migStrategy: sometimes\n")
    out = subprocess.run([sys.executable, "-m", "k8s_gpu_device_plugin_amd", "--configFile", str(tmp_path / "bad.yml")],
                         env=_env(), stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=60)
    assert out.returncode == 2 and "invalid partition" in out.stderr
    # the same check on a command-line override: a clean exit 2, not a traceback
    out = subprocess.run([sys.executable, "-m", "k8s_gpu_device_plugin_amd", "--configFile", "",
                          "--web-listen-address", "9002"],  # the reference's default (D11)
                         env=_env(), stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=60)
    assert out.returncode == 2 and "host:port" in out.stderr and "Traceback" not in out.stderr


@pytest.mark.parametrize("sig", [signal.SIGTERM, signal.SIGINT, signal.SIGHUP, signal.SIGQUIT])
def test_daemon_serves_and_exits_gracefully(plugin_dir, tmp_path, sig):
    port = _port()
    bench_dir = tmp_path / "prof"
    cfg = tmp_path / "c.yml"
    cfg.write_text("webListenAddress: 127.0.0.1:%d\nbackend: fixture\nfixture: 2gpu_spx\npluginDir: %s\n"
                   "benchmark: %s\nbenchmarkDir: %s\nlog:\n  fileDir: %s\n  console: false\n"
                   % (port, plugin_dir, "true" if sig == signal.SIGTERM else "false", bench_dir, tmp_path / "logs"))
    with KubeletStub(plugin_dir) as k:
        p = subprocess.Popen([sys.executable, "-m", "k8s_gpu_device_plugin_amd", "--configFile", str(cfg)],
                             env=_env(), cwd=str(tmp_path), stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
        try:
            k.wait_for_registrations(1, timeout=60)
            c = http.client.HTTPConnection("127.0.0.1", port, timeout=5)
            c.request("GET", "/health")
            assert c.getresponse().read() == b'{"code":0,"data":"ok","msg":"success"}\n'
            c.request("GET", "/restart")
            r = c.getresponse()
            assert r.status == 200 and r.read()
            deadline = time.monotonic() + 30  # the reload swaps the table in, then registers again
            while time.monotonic() < deadline:
                c.request("GET", "/metrics")
                if 'amdgpu_device_plugin_events_total{event="table_swaps"} 1' in c.getresponse().read().decode():
                    break
                time.sleep(0.1)
            else:
                raise AssertionError("/restart did not reload")
            k.wait_for_registrations(2, timeout=10)  # the same socket, registered again
            assert len({r.endpoint for r in k.requests}) == 1
            time.sleep(0.2)
            p.send_signal(sig)
            rc = p.wait(30)
        finally:
            if p.poll() is None:
                p.kill()
    assert rc == 0, p.stdout.read().decode()[-3000:]
    logs = os.listdir(tmp_path / "logs")
    assert "k8s-gpu-device-plugin-info.log" in logs
    info = (tmp_path / "logs" / "k8s-gpu-device-plugin-info.log").read_text()
    assert "exiting gracefully" in info and "see you next time!" in info
    if sig == signal.SIGTERM:
        files = set(os.listdir(bench_dir))
        assert {"cpu.prof", "mem.prof", "threads.prof", "latency.prom", "native.prof"} <= files
        native_prof = (bench_dir / "native.prof").read_text()
        assert native_prof.startswith("# whole-process CPU samples")
        prom = (bench_dir / "latency.prom").read_text()
        assert "amdgpu_device_plugin_rpc_duration_seconds" in prom


def _run_bench(args, nproc=1, timeout=300):
    env = _env()
    env.pop("RANK", None)
    env.pop("WORLD_SIZE", None)
    if nproc == 1:
        cmd = [sys.executable, os.path.join(ROOT, "bench.py")] + args
    else:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(nproc),
               "--master-addr", "127.0.0.1", "--master-port", str(_port()), os.path.join(ROOT, "bench.py")] + args
    p = subprocess.run(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=timeout)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    return json.loads(lines[0])


def _check_contract(r, n, steps, warmup):
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config"):
        assert k in r, k
    assert r["metric"] == json.load(open(os.path.join(ROOT, "BASELINE.json")))["metric"]
    assert (r["n_gpus"], r["steps"], r["warmup"]) == (n, steps, warmup)
    assert r["value"] > 0 and r["higher_is_better"] is False and r["scaling"] == "weak"
    assert r["allocate_p50_us_grpcio_client"] > 0 and r["scrape_rps"] > 0
    assert set(r["config"]) >= {"model", "global_batch", "seq_len", "parallelism"}


def test_bench_single_rank():
    r = _run_bench(["--steps", "2", "--warmup", "1"])
    _check_contract(r, 1, 2, 1)


@pytest.mark.slow
def test_bench_two_ranks_gloo():
    r = _run_bench(["--gpus", "2", "--steps", "2", "--warmup", "1"], nproc=2)
    _check_contract(r, 2, 2, 1)
    assert r["config"]["global_batch"] == 2 * 256


@pytest.mark.slow
def test_bench_ranks_allocate_the_gpu_of_their_hip_ordinal():
    """on a node whose HIP numbering is not BDF order, rank r allocates
    the device whose HIP ordinal is its LOCAL_RANK (the GPU its canary and
    torch.cuda.set_device use), not the r-th device in BDF order."""
    from k8s_gpu_device_plugin_amd.models import fixtures
    gpus, _ = fixtures.build_backend("2gpu_spx_hip_swapped").discover()
    hip_of = {g.uuid: g.partitions[0].hip_id for g in gpus}
    assert [hip_of[g.uuid] for g in gpus] == [1, 0]  # BDF order != HIP order
    r = _run_bench(["--gpus", "2", "--steps", "1", "--warmup", "1", "--backend", "fixture",
                    "--fixture", "2gpu_spx_hip_swapped"], nproc=2)
    _check_contract(r, 2, 1, 1)
    devs = sorted(r["rank_devices"], key=lambda d: d["rank"])
    assert [d["mapped_by"] for d in devs] == ["hip_id", "hip_id"]
    for d in devs:
        assert d["hip_ids"] == [d["local_rank"]] and hip_of[d["device_id"]] == d["local_rank"], d
    assert devs[0]["device_id"] == gpus[1].uuid  # rank 0 = HIP 0 = the second GPU in BDF order
    assert r["dtype"] == "n/a"


def test_host_ordinals_follow_the_visible_devices_variables():
    """amdsmi's hip_id is the host's numbering; a launcher that sets HIP_VISIBLE_DEVICES
    (or CUDA_/ROCR_VISIBLE_DEVICES) renumbers what the ranks open.  bench.py advertises and
    allocates by the host ordinals of the ranks' GPUs."""
    sys.path.insert(0, ROOT)
    import bench
    assert bench.host_ordinals(2, {}) == [0, 1]
    assert bench.host_ordinals(2, {"HIP_VISIBLE_DEVICES": "4,5,6"}) == [4, 5]
    assert bench.host_ordinals(2, {"CUDA_VISIBLE_DEVICES": "7,3"}) == [7, 3]
    assert bench.host_ordinals(1, {"HIP_VISIBLE_DEVICES": "2", "CUDA_VISIBLE_DEVICES": "5"}) == [2]
    # ROCR renumbers first, HIP indexes into what ROCR left
    assert bench.host_ordinals(2, {"ROCR_VISIBLE_DEVICES": "2,4,6", "HIP_VISIBLE_DEVICES": "2,0"}) == [6, 2]
    assert bench.host_ordinals(1, {"HIP_VISIBLE_DEVICES": "GPU-abc"}) is None  # UUIDs: not mappable
    assert bench.host_ordinals(3, {"HIP_VISIBLE_DEVICES": "0,1"}) is None  # fewer GPUs than ranks


def test_bench_refuses_rank_gpu_mismatch():
    """--gpus must equal WORLD_SIZE (one kubelet-client rank per advertised GPU): a run
    that would report n_gpus it did not have fails before it starts a daemon."""
    env = _env()
    env.pop("RANK", None)
    env["WORLD_SIZE"] = "1"
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1"], env=env,
                       stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=120)
    assert p.returncode != 0
    assert "WORLD_SIZE=1 but --gpus 2" in p.stderr
    assert not [ln for ln in p.stdout.splitlines() if ln.startswith("{")]


def test_bench_reports_advertised_devices_and_tail():
    r = _run_bench(["--steps", "2", "--warmup", "1"])
    assert r["advertised_devices"] == 1 and r["world_size"] == 1
    t = r["allocate_tail"]
    # every slow call has exactly one cause; with the daemon's call trace each call is
    # matched to the server's record of it, so nothing is left unattributed
    assert t["calls"] == 2 * 256 and t["slow"] == sum(t["by_cause"].values())
    assert t["matched"] == t["calls"] and t["other"] == 0
    assert set(t["segment_p50_us"]) == {"inbound", "server", "outbound"}
    assert set(t["by_cause"]) <= {"inbound_worker_polling", "inbound_worker_asleep", "server_handling",
                                  "outbound_client_wakeup", "client_preempted"}
    assert r["allocate_p999_us"] >= r["allocate_p99_us"] >= r["allocate_p50_us"]
    assert 0 < r["preferred_allocator_8gpu_size4_p50_us"] < 1000
    assert r["uds_roundtrip_floor_spin_p99_us"] >= r["uds_roundtrip_floor_spin_p50_us"]


def test_inspect_prints_the_node_and_its_placements(tmp_path):
    """--inspect: one JSON document with the GPUs, resources, xGMI links and where pods
    of the asked sizes would go; nothing is served and nothing is written."""
    import json as _json
    import subprocess as _sp
    import sys as _sys
    feature = tmp_path / "features"
    cfg = tmp_path / "c.yml"
    cfg.write_text("nodeFeatureFile: %s\n" % feature)
    out = _sp.run([_sys.executable, "-m", "k8s_gpu_device_plugin_amd", "--configFile", str(cfg),
                   "--backend", "fixture", "--fixture", "8gpu_cpx_nps2", "--strategy", "single",
                   "--plugin-dir", str(tmp_path / "dp"), "--inspect", "8,16"],
                  cwd=ROOT, stdout=_sp.PIPE, stderr=_sp.PIPE, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    d = _json.loads(out.stdout)
    assert len(d["gpus"]) == 8 and all(len(g["partitions"]) == 8 for g in d["gpus"])
    assert all(g["now"]["ok"] and g["now"]["pcie_link_width"] == 16 for g in d["gpus"])
    assert len(d["resources"]["amd.com/gpu"]) == 64
    assert len(d["xgmi"]) == 28 and all(x["type"] == "xgmi" and x["up"] for x in d["xgmi"])
    eight = d["placement"]["amd.com/gpu"]["8"]
    assert len(eight) == 8 and len({i.rsplit("-xcp", 1)[0] for i in eight}) == 1  # one whole GPU
    assert len({i.rsplit("-xcp", 1)[0] for i in d["placement"]["amd.com/gpu"]["16"]}) == 2
    assert not feature.exists() and not (tmp_path / "dp").exists()


def test_bench_daemon_exits_with_a_harness_that_dies(tmp_path):
    """A benchmark or probe killed mid-run (timeout, OOM, an exception before its
    cleanup) must not leave its plugin daemon running: the daemon is told its parent's
    pid (AMDGPU_DP_PARENT_PID) and gets SIGTERM when that parent exits."""
    script = (
        "import os, sys\n"
        "sys.path.insert(0, %r)\n"
        "import bench\n"
        "proc, kubelet, port, reg, backend = bench.start_daemon(1, 'native', %r, backend='fixture')\n"
        "print(proc.pid, flush=True)\n"
        "os._exit(0)\n" % (ROOT, str(tmp_path)))
    out = subprocess.run([sys.executable, "-c", script], capture_output=True, text=True, timeout=90, cwd=ROOT)
    pid = int(out.stdout.strip().splitlines()[-1])
    deadline = time.monotonic() + 15
    while time.monotonic() < deadline:
        try:
            with open("/proc/%d/stat" % pid) as f:
                if f.read().rsplit(")", 1)[1].split()[0] in ("Z", "X"):
                    return  # exited; its new parent just has not reaped it yet
        except (FileNotFoundError, ProcessLookupError):
            return
        time.sleep(0.1)
    with open("/proc/%d/status" % pid) as f:
        status = [ln for ln in f.read().splitlines() if ln.startswith(("State", "PPid", "Threads", "Sig", "Shd"))]
    threads = []
    for tid in sorted(os.listdir("/proc/%d/task" % pid)):
        try:
            with open("/proc/%d/task/%s/comm" % (pid, tid)) as f:
                comm = f.read().strip()
            with open("/proc/%d/task/%s/wchan" % (pid, tid)) as f:
                wchan = f.read().strip()
            with open("/proc/%d/task/%s/status" % (pid, tid)) as f:
                sig = [ln.split()[1] for ln in f.read().splitlines() if ln.startswith(("SigPnd", "SigBlk"))]
            threads.append("%s %s %s pnd/blk=%s" % (tid, comm, wchan, "/".join(sig)))
        except OSError:
            pass
    os.kill(pid, signal.SIGKILL)
    with open(tmp_path / "daemon.log") as f:
        tail = f.read()[-3000:]
    raise AssertionError("daemon %d outlived its harness\n%s\n%s\n%s" % (pid, "\n".join(status), "\n".join(threads),
                                                                          tail))


def test_parent_watch_ends_the_daemon_when_its_harness_exits():
    """The pidfd watch (cli._watch_parent) sets the daemon's done event when the process it
    watches exits, with no periodic wake-up while it lives."""
    import threading
    from k8s_gpu_device_plugin_amd import cli
    child = subprocess.Popen([sys.executable, "-c", "import time; time.sleep(60)"])
    try:
        reason, done = {"why": ""}, threading.Event()
        if not cli._watch_parent(child.pid, reason, done):
            pytest.skip("no pidfd_open on this kernel")
        assert not done.wait(0.3)
        child.kill()
        child.wait(10)
        assert done.wait(5)
        assert "parent process %d exited" % child.pid in reason["why"]
    finally:
        if child.poll() is None:
            child.kill()
