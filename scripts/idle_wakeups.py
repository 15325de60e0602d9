"""What an idle plugin daemon costs the node: wake-ups per second
and CPU per thread, in the admission window right after kubelet RPCs and once the daemon
has been idle for longer than ``grpc.activeWindowMs``.

One daemon (bench config: amdsmi backend when it sees a GPU, else the fixture node), a
kubelet stub and one compiled kubelet-like connection.  Phases:

  * ``active``: 10 Allocates, then the next ``--window`` seconds (the admission window:
    idle wake-ups and keep-warm ticks run);
  * ``idle``: after ``--settle`` seconds without an RPC, ``--window`` seconds more.

Per phase: every thread's voluntary + involuntary context switches per second (from
/proc/<pid>/task/<tid>/status) and CPU time (.../schedstat, ns; utime + stime where the
kernel has no schedstat), grouped by thread name, and the daemon's totals.  Then the latency the idle phase costs: the first
Allocate after the idle phase against an Allocate 1 s later (both single calls, the
daemon's call trace splits them; inbound is the worker's wake-up).

    python scripts/idle_wakeups.py [--window 10] [--settle 12] [--out FILE] [--daemon-config JSON]
"""
from __future__ import annotations

import argparse
import collections
import json
import os
import shutil
import signal
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402

CLK_TCK = os.sysconf("SC_CLK_TCK")


def thread_stats(pid: int) -> dict:
    """tid -> (name, context switches, cpu seconds).  CPU time from schedstat (ns on the
    CPU, exact) where the kernel has it, else utime + stime (10 ms ticks)."""
    out = {}
    base = "/proc/%d/task" % pid
    for tid in os.listdir(base):
        try:
            with open("%s/%s/status" % (base, tid)) as f:
                st = f.read()
            with open("%s/%s/stat" % (base, tid)) as f:
                stat = f.read()
        except OSError:
            continue
        name = stat[stat.index("(") + 1:stat.rindex(")")]
        fields = stat[stat.rindex(")") + 2:].split()
        cpu = (int(fields[11]) + int(fields[12])) / CLK_TCK
        try:
            with open("%s/%s/schedstat" % (base, tid)) as f:
                cpu = int(f.read().split()[0]) * 1e-9
        except (OSError, ValueError, IndexError):
            pass
        cs = 0
        for line in st.splitlines():
            if line.startswith(("voluntary_ctxt_switches", "nonvoluntary_ctxt_switches")):
                cs += int(line.split()[1])
        out[tid] = (name, cs, cpu)
    return out


def phase(pid: int, seconds: float) -> dict:
    a = thread_stats(pid)
    t0 = time.monotonic()
    time.sleep(seconds)
    b = thread_stats(pid)
    dt = time.monotonic() - t0
    by = collections.defaultdict(lambda: [0, 0.0, 0])
    for tid, (name, cs, cpu) in b.items():
        if tid not in a:
            continue
        grp = name.rstrip("0123456789-")
        by[grp][0] += cs - a[tid][1]
        by[grp][1] += cpu - a[tid][2]
        by[grp][2] += 1
    threads = {k: {"threads": v[2], "wakeups_per_s": round(v[0] / dt, 1), "cpu_pct": round(100 * v[1] / dt, 3)}
               for k, v in sorted(by.items())}
    return {"seconds": round(dt, 2), "wakeups_per_s": round(sum(v[0] for v in by.values()) / dt, 1),
            "cpu_pct_of_a_core": round(100 * sum(v[1] for v in by.values()) / dt, 3), "threads": threads}


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--window", type=float, default=10.0)
    ap.add_argument("--settle", type=float, default=12.0)
    ap.add_argument("--backend", default="auto")
    ap.add_argument("--daemon-config", default="")
    ap.add_argument("--out", default="")
    a = ap.parse_args()

    from k8s_gpu_device_plugin_amd import native
    from k8s_gpu_device_plugin_amd.api import v1beta1
    n = native.load()
    nb = native.load_bench()
    workdir = tempfile.mkdtemp(prefix="amdgpu-dp-idle-")
    overrides = json.loads(a.daemon_config) if a.daemon_config else None
    proc, kubelet, port, reg, backend = bench.start_daemon(1, "native", workdir, backend=a.backend,
                                                           overrides=overrides)
    res = {"backend": backend, "daemon_config": overrides or {}}
    try:
        sock = os.path.join(workdir, "device-plugins", reg.endpoint)
        h2 = n.H2Client(sock)
        law = kubelet.watch(reg.endpoint)  # kubelet's stream is open throughout, like on a node
        _, devs = law.next(timeout=10)
        req = v1beta1.AllocateRequest(container_requests=[v1beta1.ContainerAllocateRequest(
            devices_ids=[devs[0][0]])]).SerializeToString()
        time.sleep(2.0)  # start-up work (discovery, first samples) out of the way
        h2.bench_unary(v1beta1.METHOD_ALLOCATE, req, 10)
        res["active"] = phase(proc.pid, a.window)
        print("active: %s wake-ups/s, %s %% of a core" % (res["active"]["wakeups_per_s"],
                                                         res["active"]["cpu_pct_of_a_core"]), file=sys.stderr, flush=True)
        time.sleep(max(0.0, a.settle - a.window))
        res["idle"] = phase(proc.pid, a.window)
        print("idle: %s wake-ups/s, %s %% of a core" % (res["idle"]["wakeups_per_s"],
                                                       res["idle"]["cpu_pct_of_a_core"]), file=sys.stderr, flush=True)
        # what the quiet costs the next call: first Allocate after the idle phase, then one 1 s later
        first = h2.bench_unary_ts(v1beta1.METHOD_ALLOCATE, req, 1)
        time.sleep(1.0)
        second = h2.bench_unary_ts(v1beta1.METHOD_ALLOCATE, req, 1)
        trace = bench.read_call_trace(os.path.join(workdir, "calltrace-%s.bin" % reg.resource_name.split("/")[-1]))
        calls = {}
        for label, (starts, lats) in (("first_after_idle", first[:2]), ("one_second_later", second[:2])):
            e = bench.match_calls(starts, lats, trace, n.RPC_ALLOCATE)[0]
            seg = bench.segments(int(starts[0]), lats[0], e) if e is not None else None
            calls[label] = {"us": round(lats[0] * 1e6, 2),
                            "segments_us": [round(x / 1e3, 2) for x in seg] if seg else None,
                            "worker_polling": int(e["spinning"]) if e is not None else None}
        res["calls"] = calls
        h2.close()
    finally:
        try:
            os.killpg(proc.pid, signal.SIGTERM)
            proc.wait(15)
        except Exception:
            pass
        kubelet.stop()
        shutil.rmtree(workdir, ignore_errors=True)
    line = json.dumps(res)
    if a.out:
        with open(a.out, "w") as f:
            f.write(line + "\n")
    print(line, flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
