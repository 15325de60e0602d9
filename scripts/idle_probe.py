"""Allocate latency as a function of how long the plugin sat idle before the call
(VERDICT r3 item 6).

Kubelet calls the plugin a few times per pod admission, seconds or minutes apart, so the
call it makes almost never finds a warm server.  For each idle gap this measures, on one
daemon (bench config, amdsmi backend when present), three kinds of call, each after the
same gap, interleaved call by call (the kind order rotates every iteration) so slow drift
of the machine hits all three alike:

  * ``allocate``  - Allocate after the gap (compiled HTTP/2 client, kubelet-like);
  * ``preferred`` - GetPreferredAllocation after the gap: the first call of a kubelet pod
    admission, the one that pays for the idle gap;
  * ``floor``     - the bare unix-socket exchange of Allocate's sizes after the gap, to a
    server thread that sleeps in epoll_wait(100 ms) like the plugin's workers do
    (``native.UdsPinger``; no HTTP/2, protobuf or table work).

Reported per gap: p50/p90 of each kind, and the median of the paired differences
allocate - floor and preferred - floor (iteration i's calls are a pair) with a bootstrap
95 % confidence interval.  Evidence for where an excess comes from, per call: minor and
major page faults and scheduler counters (run time, run-queue wait, time slices) of the
daemon's gRPC worker threads (``dpgrpc-*`` in /proc/<pid>/task) and of the calling
thread, read before and after the call; and the daemon's own record of the call
(grpc.callTraceFile, see bench.match_calls), which splits it into inbound (client send ->
the worker's epoll_wait returning with it; the worker's wake-up), server (-> response
sent) and outbound (-> the client has it; the client's wake-up), with whether the worker
was asleep.  ``attribution`` compares each segment's median at the longest gap with the
shortest (bootstrap 95 % intervals): the parts of the idle excess, summing to it.

    python scripts/idle_probe.py [--gaps 0.001,0.01,0.1,1] [--calls 300] [--out FILE]
    python scripts/idle_probe.py --gaps 1 --calls 100 --ab-keep-warm 0,10   # A/B, interleaved

Prints a progress line every 30 s, one JSON line per gap, then the whole result.
"""
from __future__ import annotations

import argparse
import json
import os
import random
import resource
import shutil
import signal
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402

KINDS = ("allocate", "preferred", "floor")
SEGMENTS = ("inbound", "server_recv_parse", "server_handle_send", "outbound")


def segments4(start, lat, e):
    """bench.segments with the server part split at dispatch."""
    inbound, _, outbound = bench.segments(start, lat, e)
    return (inbound, int(e["t_dispatch"]) - int(e["t_ready"]), int(e["t_sent"]) - int(e["t_dispatch"]), outbound)


def pct(xs, q):
    xs = sorted(xs)
    return xs[min(len(xs) - 1, int(q * len(xs)))] if xs else None


def median(xs):
    return pct(xs, 0.5)


def bootstrap_ci(diffs, n=2000, seed=7):
    """95 % percentile-bootstrap interval of the median of paired differences."""
    rng = random.Random(seed)
    k = len(diffs)
    meds = sorted(median([diffs[rng.randrange(k)] for _ in range(k)]) for _ in range(n))
    return meds[int(0.025 * n)], meds[int(0.975 * n)]


def process_cpu_s(pid: int) -> float:
    """utime + stime of the whole process, seconds."""
    with open("/proc/%d/stat" % pid) as f:
        fields = f.read().rsplit(")", 1)[1].split()
    return (int(fields[11]) + int(fields[12])) / os.sysconf("SC_CLK_TCK")


def median_shift(a, b, n=2000, seed=11):
    """median(a) - median(b) and its 95 % percentile-bootstrap interval (a and b are
    independent samples, resampled separately)."""
    rng = random.Random(seed)
    ds = sorted(median([a[rng.randrange(len(a))] for _ in a]) - median([b[rng.randrange(len(b))] for _ in b])
                for _ in range(n))
    return median(a) - median(b), (ds[int(0.025 * n)], ds[int(0.975 * n)])


def worker_tids(pid: int, prefix: str = "dpgrpc-"):
    out = []
    for tid in os.listdir("/proc/%d/task" % pid):
        try:
            with open("/proc/%d/task/%s/comm" % (pid, tid)) as f:
                if f.read().strip().startswith(prefix):
                    out.append(int(tid))
        except OSError:
            pass
    return out


def thread_counters(pid: int, tids):
    """Sum over `tids` of (minflt, majflt, run_ns, wait_ns, slices)."""
    tot = [0, 0, 0, 0, 0]
    for tid in tids:
        try:
            with open("/proc/%d/task/%d/stat" % (pid, tid)) as f:
                fields = f.read().rsplit(")", 1)[1].split()
            with open("/proc/%d/task/%d/schedstat" % (pid, tid)) as f:
                run, wait, slices = (int(x) for x in f.read().split())
        except OSError:
            continue
        tot[0] += int(fields[7])   # minflt (field 10)
        tot[1] += int(fields[9])   # majflt (field 12)
        tot[2] += run
        tot[3] += wait
        tot[4] += slices
    return tot


def server_seconds(conn, rpc: str) -> float:
    """Sum of the daemon's own time for `rpc` so far (amdgpu_device_plugin_rpc_duration_
    seconds: request dispatched -> answer encoded, no transport)."""
    conn.request("GET", "/metrics")
    body = conn.getresponse().read().decode()
    tot = 0.0
    for line in body.splitlines():
        if line.startswith("amdgpu_device_plugin_rpc_duration_seconds_sum") and 'rpc="%s"' % rpc in line:
            tot += float(line.rsplit(" ", 1)[1])
    return tot


def self_faults():
    r = resource.getrusage(resource.RUSAGE_THREAD)
    return r.ru_minflt, r.ru_majflt


class Daemon:
    """One plugin daemon (bench config) with a kubelet-like compiled HTTP/2 client."""

    def __init__(self, n, a, keep_warm_ms, overrides=None):
        from k8s_gpu_device_plugin_amd.api import v1beta1
        from k8s_gpu_device_plugin_amd.plugin.kubelet_stub import DevicePluginClient
        self.keep_warm_ms = keep_warm_ms
        self.workdir = tempfile.mkdtemp(prefix="idleprobe-", dir="/tmp")
        over = {"grpc": {"keepWarmMs": keep_warm_ms}} if keep_warm_ms is not None else None
        if overrides:
            over = overrides
        self.proc, self.kubelet, self.port, reg, self.backend = bench.start_daemon(
            1, "native", self.workdir, busy_poll_us=a.busy_poll_us, admission_poll_us=a.admission_poll_us,
            backend=a.backend, overrides=over)
        sock = os.path.join(self.workdir, "device-plugins", reg.endpoint)
        c = DevicePluginClient(sock)
        law = c.list_and_watch()
        ids = [d.ID for d in next(iter(law)).devices]
        law.cancel()
        self.alloc = v1beta1.AllocateRequest(container_requests=[
            v1beta1.ContainerAllocateRequest(devices_ids=ids[:1])]).SerializeToString()
        self.pref = v1beta1.PreferredAllocationRequest(container_requests=[
            v1beta1.ContainerPreferredAllocationRequest(available_deviceIDs=ids, must_include_deviceIDs=ids[:1],
                                                        allocation_size=1)]).SerializeToString()
        self.resp_len = len(c.allocate_raw(self.alloc))
        c.close()
        self.h2 = n.H2Client(sock)
        self.h2.bench_unary(v1beta1.METHOD_ALLOCATE, self.alloc, 2000)  # warm the connection and the code
        self.tids = worker_tids(self.proc.pid)
        self.cpu0 = (process_cpu_s(self.proc.pid), time.monotonic())
        import http.client
        self.mconn = http.client.HTTPConnection("127.0.0.1", self.port, timeout=10)
        self.base = {}
        self.trace_path = os.path.join(self.workdir, "calltrace-%s.bin" % reg.resource_name.split("/")[-1])
        self.starts = {"allocate": [], "preferred": []}  # client start (mono ns) of every timed call

        def timed(kind, method, req):
            starts, lat = self.h2.bench_unary_ts(method, req, 1)[:2]
            self.starts[kind].append(starts[0])
            return lat[0]
        self.allocate = lambda: timed("allocate", v1beta1.METHOD_ALLOCATE, self.alloc)
        self.preferred = lambda: timed("preferred", v1beta1.METHOD_GET_PREFERRED, self.pref)

    def close(self):
        try:
            self.h2.close()
        except Exception:
            pass
        try:
            os.killpg(self.proc.pid, signal.SIGTERM)
        except ProcessLookupError:
            pass
        try:
            self.proc.wait(15)
        except subprocess.TimeoutExpired:
            os.killpg(self.proc.pid, signal.SIGKILL)
        self.kubelet.stop()
        shutil.rmtree(self.workdir, ignore_errors=True)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gaps", default="0.001,0.01,0.1,1")
    ap.add_argument("--calls", type=int, default=300, help="calls per kind per gap")
    ap.add_argument("--backend", default="auto")
    ap.add_argument("--admission-poll-us", type=int, default=None, help="override grpc.admissionPollUs")
    ap.add_argument("--busy-poll-us", type=int, default=None, help="override grpc.busyPollUs / http.busyPollUs")
    ap.add_argument("--keep-warm-ms", type=int, default=None, help="override grpc.keepWarmMs")
    ap.add_argument("--ab-keep-warm", default="",
                    help="A,B[,C..]: one daemon per grpc.keepWarmMs value, their Allocate and "
                         "GetPreferredAllocation calls interleaved with the floor's (kinds allocate@A, ...); "
                         "paired differences of A to each other value")
    ap.add_argument("--ab-overrides", default="",
                    help='JSON {"name": {config overrides}, ...}: one daemon per entry (arms in that '
                         'order, the first compared with each other), like --ab-keep-warm')
    ap.add_argument("--replicas", type=int, default=1,
                    help="with --ab-keep-warm: daemons per value (their placement on the host's CPUs "
                         "differs; several per value keep one daemon's placement from passing for the "
                         "setting's effect)")
    ap.add_argument("--rpcs", default="allocate,preferred", help="RPC kinds to time (allocate, preferred)")
    ap.add_argument("--server-time", action="store_true",
                    help="also read the daemon's own time per call from its RPC histogram (a /metrics "
                         "scrape after each timed call)")
    ap.add_argument("--out", default="")
    a = ap.parse_args()

    from k8s_gpu_device_plugin_amd import native

    n = native.load()
    native.load_bench()  # the harness extension: load generators, H2Client.bench_unary
    ab = [int(x) for x in a.ab_keep_warm.split(",")] if a.ab_keep_warm else None
    arms = None  # (name, overrides) per arm
    if a.ab_overrides:
        arms = list(json.loads(a.ab_overrides).items())
    elif ab:
        arms = [(str(kw), {"grpc": {"keepWarmMs": kw}}) for kw in ab]
    daemons = {}
    t_progress = time.monotonic()
    res = {"calls_per_kind_per_gap": a.calls, "floor_server_epoll_timeout_ms": 100, "rows": []}
    try:
        if arms:
            for r in range(a.replicas):
                for name, over in arms:
                    daemons["@%s" % name + ("#%d" % r if a.replicas > 1 else "")] = Daemon(n, a, None, over)
        else:
            daemons[""] = Daemon(n, a, a.keep_warm_ms)
        first = next(iter(daemons.values()))
        res["backend"] = first.backend
        res["keep_warm_ms"] = ab if ab else a.keep_warm_ms
        res["arms"] = dict(arms) if arms else None
        sizes = (9 + 80 + 9 + 5 + len(first.alloc), 9 + 20 + 9 + 5 + first.resp_len + 9 + 16)
        pinger = native.load_bench().UdsPinger(*sizes, server_timeout_ms=100)
        for _ in range(200):
            pinger.once()
        # kinds: <rpc><daemon tag>, and the floor
        call, owner = {"floor": pinger.once}, {}
        want = a.rpcs.split(",")
        for tag, d in daemons.items():
            if "allocate" in want:
                call["allocate" + tag], owner["allocate" + tag] = d.allocate, d
            if "preferred" in want:
                call["preferred" + tag], owner["preferred" + tag] = d.preferred, d
        kinds = tuple(k for k in call if k != "floor") + ("floor",)
        rpcs = [k for k in kinds if k != "floor"]
        res["kinds"] = list(kinds)
        res["daemon_grpc_workers"] = len(first.tids)
        rpc_name = {"allocate": "Allocate", "preferred": "GetPreferredAllocation"}
        segs_by_gap, lat_by_gap = {}, {}  # rpc kind -> gap -> per-call segments / latencies
        for gap in [float(x) for x in a.gaps.split(",")]:
            lat = {k: [] for k in kinds}
            srv = {k: [] for k in rpcs}  # the daemon's own time per call
            for d in daemons.values():
                d.base = {}
                d.starts = {"allocate": [], "preferred": []}
            ev = {k: {"daemon_minflt": 0, "daemon_majflt": 0, "daemon_run_us": 0.0, "daemon_wait_us": 0.0,
                      "daemon_slices": 0, "client_minflt": 0} for k in kinds}
            for i in range(a.calls):
                r = i % len(kinds)
                order = kinds[r:] + kinds[:r]
                for kind in order:
                    time.sleep(gap)
                    # the counters are read around every kind, the floor's too, so each
                    # call follows the same client-side work
                    d = owner.get(kind, first)
                    d0 = thread_counters(d.proc.pid, d.tids)
                    s0 = self_faults()
                    lat[kind].append(call[kind]())
                    s1 = self_faults()
                    d1 = thread_counters(d.proc.pid, d.tids)
                    if kind != "floor":
                        e = ev[kind]
                        e["daemon_minflt"] += d1[0] - d0[0]
                        e["daemon_majflt"] += d1[1] - d0[1]
                        e["daemon_run_us"] += (d1[2] - d0[2]) / 1e3
                        e["daemon_wait_us"] += (d1[3] - d0[3]) / 1e3
                        e["daemon_slices"] += d1[4] - d0[4]
                    ev[kind]["client_minflt"] += s1[0] - s0[0]
                    if kind != "floor" and a.server_time:  # read after the timed call
                        base = d.base.get(kind)
                        cur = server_seconds(d.mconn, rpc_name[kind.split("@")[0].split("#")[0]])
                        if base is not None:
                            srv[kind].append(cur - base)
                        d.base[kind] = cur
                if time.monotonic() - t_progress > 30:
                    t_progress = time.monotonic()
                    print(json.dumps({"progress": {"gap_s": gap, "iteration": i + 1, "of": a.calls}}), flush=True)
            us = lambda v: round(v * 1e6, 2)  # noqa: E731
            row = {"gap_s": gap, "calls": a.calls}
            for k in kinds:
                row[k] = {"p50_us": us(median(lat[k])), "p90_us": us(pct(lat[k], 0.9))}
            for k in rpcs:
                diffs = [x - y for x, y in zip(lat[k], lat["floor"])]
                lo, hi = bootstrap_ci(diffs)
                row[k]["minus_floor_median_us"] = us(median(diffs))
                row[k]["minus_floor_ci95_us"] = [us(lo), us(hi)]
                row[k]["per_call"] = {kk: round(v / a.calls, 3) for kk, v in ev[k].items()}
                if srv[k]:  # the daemon's own part of the call (dispatch -> encoded answer)
                    row[k]["server_p50_us"] = us(median(srv[k]))
                    row[k]["server_p90_us"] = us(pct(srv[k], 0.9))
            if arms:  # paired difference of the first arm to each other one, iteration by
                # iteration (each arm's latency averaged over its replicas)
                def arm(rpc, name):
                    ks = [k for k in kinds if k.split("#")[0] == "%s@%s" % (rpc, name)]
                    return [sum(v) / len(v) for v in zip(*(lat[k] for k in ks))]
                first_arm = arms[0][0]
                for other, _ in arms[1:]:
                    for rpc in [r for r in ("allocate", "preferred") if r in want]:
                        x, y = arm(rpc, first_arm), arm(rpc, other)
                        diffs = [p - q for p, q in zip(x, y)]
                        lo, hi = bootstrap_ci(diffs)
                        row["%s_@%s_minus_@%s" % (rpc, first_arm, other)] = {
                            "median_us": us(median(diffs)), "ci95_us": [us(lo), us(hi)]}
            row["floor"]["per_call"] = {"client_minflt": round(ev["floor"]["client_minflt"] / a.calls, 3)}
            # the daemon's record of each timed call: segments and whether the worker slept
            for k in rpcs:
                d = owner[k]
                base = k.split("@")[0].split("#")[0]
                rpc = n.RPC_ALLOCATE if base == "allocate" else n.RPC_PREFERRED
                recs = bench.match_calls(d.starts[base], lat[k], bench.read_call_trace(d.trace_path), rpc)
                seg = [segments4(st, x, e) for st, x, e in zip(d.starts[base], lat[k], recs) if e is not None]
                if seg:
                    got = [e for e in recs if e is not None]
                    row[k]["matched"] = len(seg)
                    row[k]["segments_p50_us"] = {name: round(median([s_[i] for s_ in seg]) / 1e3, 2)
                                                 for i, name in enumerate(SEGMENTS)}
                    row[k]["worker_asleep_fraction"] = round(sum(1 for e in got if not e["spinning"]) / len(got), 3)
                    # the worker woke on another CPU than its previous work (request or tick) ran on
                    row[k]["worker_cpu_changed_fraction"] = round(
                        sum(1 for e in got if e["prev_cpu"] != 0xFFFF and e["prev_cpu"] != e["cpu"]) / len(got), 3)
                    row[k]["worker_idle_p50_ms"] = round(median([int(e["idle_ns"]) for e in got]) / 1e6, 3)
                    segs_by_gap.setdefault(k, {})[gap] = seg
                    lat_by_gap.setdefault(k, {})[gap] = [x for x, e in zip(lat[k], recs) if e is not None]
            res["rows"].append(row)
            print(json.dumps(row), flush=True)
        del pinger
        # what each daemon cost while the probe ran (mostly idle: keep-warm ticks, telemetry)
        res["daemon_cpu_percent"] = {}
        for tag, d in daemons.items():
            c0, t0 = d.cpu0
            res["daemon_cpu_percent"][tag or "daemon"] = round(
                100.0 * (process_cpu_s(d.proc.pid) - c0) / max(1e-9, time.monotonic() - t0), 3)
        # where the idle excess goes: each segment's median at the longest gap minus at the
        # shortest, with a bootstrap 95 % interval (independent samples resampled apart)
        res["attribution"] = {}
        for k, by_gap in segs_by_gap.items():
            if len(by_gap) < 2:
                continue
            lo_gap, hi_gap = min(by_gap), max(by_gap)
            cold, warm = by_gap[hi_gap], by_gap[lo_gap]
            att = {"from_gap_s": lo_gap, "to_gap_s": hi_gap}
            for i, name in enumerate(SEGMENTS):
                d, ci = median_shift([x[i] for x in cold], [x[i] for x in warm])
                att[name + "_us"] = {"median": round(d / 1e3, 2), "ci95": [round(ci[0] / 1e3, 2), round(ci[1] / 1e3, 2)]}
            d, ci = median_shift(lat_by_gap[k][hi_gap], lat_by_gap[k][lo_gap])
            att["total_us"] = {"median": round(d * 1e6, 2), "ci95": [round(ci[0] * 1e6, 2), round(ci[1] * 1e6, 2)]}
            att["sum_of_segments_us"] = round(sum(att[n_ + "_us"]["median"] for n_ in SEGMENTS), 2)
            res["attribution"][k] = att
        print(json.dumps({"attribution": res["attribution"]}), flush=True)
    finally:
        for d in daemons.values():
            d.close()
    if a.out:
        os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)
    print(json.dumps(res), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
