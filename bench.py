"""Headline benchmark: Allocate() p50 latency + /metrics scrape RPS with N MI355X advertised.

Metric and configs come from BASELINE.json.  One rank per GPU (``torch.distributed.run
--nproc-per-node N``); rank 0 launches the plugin daemon as a child process *before*
anything touches the GPU, advertising the N GPUs that HIP numbers 0..N-1 (``devices:
hip:0-<N-1>``; amdsmi backend on MI355X, an N-GPU fixture node model elsewhere) and an in-process kubelet stub for it
to register with.  Every rank then acts as one kubelet-side client for "its" GPU:

  step = ALLOCS Allocate RPCs through a compiled HTTP/2 gRPC client (kubelet-like)
       + ALLOCS Allocate RPCs through a persistent grpcio client (BASELINE.md method)
       + PREFS GetPreferredAllocation RPCs over the whole advertised set, compiled
         client and grpcio client (each timed)
       + SCRAPE_S seconds of closed-loop GET /metrics on SCRAPE_CONNS keep-alive
         connections from the compiled load generator (tests/native/loadgen.cpp)

W warm-up steps, then K timed steps bracketed by barrier + torch.cuda.synchronize().
With N > 1 the ranks also barrier between a step's RPC phase and its scrape phase.
Work per rank is fixed as N grows (weak scaling).  ``value`` = Allocate p50 in
microseconds over every compiled-client Allocate of every rank in the timed window (lower
is better; kubelet is a compiled grpc-go client, and a Python client's own ~80 us per
call would hide the plugin); the grpcio-client p50/p99 are reported alongside;
``scrape_rps`` = all ranks' completed scrapes / the slowest rank's scrape window (the
ranks scrape concurrently, so this is the daemon's aggregate throughput).  Before timing,
each rank validates its GPU and its allocation: the gfx950 canary (HBM pattern + MFMA
exactness/throughput) passes on the rank's device, in a child process that exits before
the rank loads torch or joins the RCCL group, and the returned render node exists.  The
run fails unless WORLD_SIZE == --gpus == the number of devices the daemon advertised
(one kubelet-client rank per advertised GPU).  Rank r allocates the device whose host HIP
ordinals (``hip_ids`` of ``amdgpu_partition_info``, from amdsmi's enumeration info) hold
its LOCAL_RANK (mapped through ROCR_/HIP_VISIBLE_DEVICES to the host's numbering when
they are set), so the canary, ``torch.cuda.set_device(local_rank)`` and the allocation
name the same GPU even where the HIP runtime's numbering differs from BDF order.

Speed-of-light references, measured untimed in the same run: ``uds_roundtrip_floor_p50_us``
(the same unix-socket exchange between two threads, no protocol work, sleeping server
thread) and ``uds_roundtrip_floor_spin_p50_us`` (server thread polling, which is what the
daemon's ``grpc.busyPollUs`` window gives back-to-back kubelet RPCs).  Also untimed:
``allocate_cold_p50_us``, Allocate calls 1 ms apart, each of which finds the server thread
asleep (kubelet's pod admissions are sparse; its speed of light is
``uds_roundtrip_floor_cold_p50_us``, the bare exchange with the same 1 ms idle gap), and
``allocate_admission_p50_us``, the Allocate of a kubelet-like admission (GetPreferredAllocation,
200 us of client-side work, Allocate) after 2 ms idle (``grpc.admissionPollUs``).

The reference publishes no numbers, so ``vs_baseline`` is null.
"""
from __future__ import annotations

import argparse
import collections
import http.client
import json
import os
import shutil
import signal
import socket
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

ALLOCS, PREFS = 256, 32
SCRAPE_S, SCRAPE_CONNS = 0.05, 2
METRIC = "Allocate() p50 latency + /metrics scrape RPS at 1/2/4/8 MI355X advertised"


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _pct(xs, q):
    if not xs:
        return None
    xs = sorted(xs)
    return xs[min(len(xs) - 1, int(q * len(xs)))]


def _wait_http(port: int, timeout: float) -> None:
    deadline = time.time() + timeout
    while time.time() < deadline:
        try:
            c = http.client.HTTPConnection("127.0.0.1", port, timeout=1)
            c.request("GET", "/health")
            if c.getresponse().status == 200:
                c.close()
                return
        except OSError:
            pass
        time.sleep(0.1)
    raise TimeoutError("plugin web server did not come up on port %d" % port)


TRACE_DTYPE = [("t_ready", "<i8"), ("t_dispatch", "<i8"), ("t_sent", "<i8"), ("conn", "<u8"), ("idle_ns", "<i8"),
               ("seq", "<u4"), ("method", "u1"), ("spinning", "u1"), ("cpu", "<u2"), ("prev_cpu", "<u2"),
               ("handle_ns", "<u2"), ("recv_ns", "<u4")]  # native/grpc_h2.h CallTraceEntry (56 bytes)


def read_call_trace(path: str):
    """The daemon's per-call trace ring (grpc.callTraceFile), as a numpy record array of
    the records written so far (None when absent or malformed)."""
    import numpy as np
    try:
        raw = open(path, "rb").read()
    except OSError:
        return None
    if len(raw) < 64 or int.from_bytes(raw[:8], "little") != 0x5452434c4c414344:
        return None
    cap = int.from_bytes(raw[12:16], "little")
    recs = np.frombuffer(raw, dtype=np.dtype(TRACE_DTYPE), count=cap, offset=64)
    return recs[recs["seq"] > 0]


def match_calls(starts, lats, trace, rpc: int) -> list:
    """The server's record (grpc.callTraceFile) of each client call (start mono ns,
    latency s), or None: a record of that RPC dispatched within the call, on the client's
    connection - the one most calls with a single candidate record were answered on."""
    import collections

    import numpy as np
    out = [None] * len(starts)
    if trace is None or not len(trace):
        return out
    a = trace[(trace["method"] == rpc) & (trace["t_sent"] > 0)]
    a = a[np.argsort(a["t_dispatch"], kind="stable")]
    td = a["t_dispatch"]
    ranges = [(int(np.searchsorted(td, s, "left")), int(np.searchsorted(td, s + int(x * 1e9), "right")))
              for s, x in zip(starts, lats)]
    votes = collections.Counter(int(a["conn"][i0]) for i0, i1 in ranges if i1 - i0 == 1)
    if not votes:
        return out
    mine = votes.most_common(1)[0][0]
    for k, (i0, i1) in enumerate(ranges):
        for j in range(i0, i1):
            if int(a["conn"][j]) == mine:
                out[k] = a[j]
                break
    return out


def segments(start: int, lat: float, e) -> tuple:
    """(inbound, server, outbound) ns of one call matched to its server record: client
    start -> the worker's epoll_wait returning with the request -> response sent -> the
    client has the answer."""
    return (int(e["t_ready"]) - start, int(e["t_sent"]) - int(e["t_ready"]), start + int(lat * 1e9) - int(e["t_sent"]))


def _tail_stats(batches, trace=None, rpc_allocate: int = 3) -> dict:
    """Attribution of this rank's slow Allocates (> 2x the rank's p50), call by call.

    Client-side evidence for every call: the first call of a batch (it follows the
    previous step's scrape phase, so it meets a server worker whose busy-poll window has
    closed), a call that ran on another CPU than the call before it (the client thread
    migrated), and the client thread's involuntary context switches during the call
    (preempted).  With the daemon's call trace (grpc.callTraceFile) each call is matched
    to the server's record of it and split into inbound (client send -> the worker's
    epoll_wait returning with it), server (-> response sent) and outbound (-> the client
    has the answer); a slow call is put on the segment with the largest excess over that
    segment's median, inbound split by whether the worker was polling or asleep.  What
    has no evidence at all is "other"."""
    import collections

    import numpy as np
    lat = [x for b in batches for x in b[1]]
    if not lat:
        return {"calls": 0}
    thr = 2 * _pct(lat, 0.5)
    calls = []  # (start ns, latency s, client cpu, preempted, first, migrated)
    for b in batches:
        starts, lats, cpus = b[0], b[1], b[2]
        pre = b[3] if len(b) > 3 else [0] * len(lats)
        for i, x in enumerate(lats):
            calls.append((int(starts[i]), x, cpus[i], pre[i], i == 0, i > 0 and cpus[i] != cpus[i - 1]))
    out = {"calls": len(calls), "slow": 0, "first_of_batch": 0, "cpu_migrated": 0, "client_preempted": 0,
           "threshold_us": round(thr * 1e6, 2)}
    matched = match_calls([c[0] for c in calls], [c[1] for c in calls], trace, rpc_allocate)
    seg_med = None
    if trace is not None and len(trace):
        segs = [segments(c[0], c[1], e) for c, e in zip(calls, matched) if e is not None]
        if segs:
            seg_med = [float(np.median([sg[i] for sg in segs])) for i in range(3)]
            out["matched"] = len(segs)
            out["segment_p50_us"] = {"inbound": round(seg_med[0] / 1e3, 2), "server": round(seg_med[1] / 1e3, 2),
                                     "outbound": round(seg_med[2] / 1e3, 2)}
            # the server segment split at dispatch: recv + HTTP/2 + HPACK before it, the
            # table, the response framing and send() (which wakes the client) after it
            rp = [int(e["t_dispatch"]) - int(e["t_ready"]) for e in matched if e is not None]
            hs = [int(e["t_sent"]) - int(e["t_dispatch"]) for e in matched if e is not None]
            rv = [int(e["recv_ns"]) for e in matched if e is not None]
            hd = [int(e["handle_ns"]) for e in matched if e is not None]
            tails = [int(t) for b in batches if len(b) > 4 for t in b[4]]
            if tails:  # outbound = the client's wake-up and recv (kernel) + its own parsing after it
                out["outbound_split_p50_us"] = {"client_parse": round(float(np.median(tails)) / 1e3, 2)}
            out["server_split_p50_us"] = {"recv_parse": round(float(np.median(rp)) / 1e3, 2),
                                          "recv": round(float(np.median(rv)) / 1e3, 2),
                                          "parse": round(float(np.median([a - b for a, b in zip(rp, rv)])) / 1e3, 2),
                                          "handle_send": round(float(np.median(hs)) / 1e3, 2),
                                          "handle": round(float(np.median(hd)) / 1e3, 2),
                                          "send": round(float(np.median([a - b for a, b in zip(hs, hd)])) / 1e3, 2)}
    causes = collections.Counter()
    excess = collections.defaultdict(list)
    slowest = []  # (latency s, cause, [inbound, server, outbound] us, worker was polling)
    same_cpu = 0
    for c, e in zip(calls, matched):
        s, x, cpu, pre, first, migrated = c
        if x <= thr:
            continue
        out["slow"] += 1
        out["first_of_batch"] += int(first)
        out["cpu_migrated"] += int(migrated)
        out["client_preempted"] += int(pre > 0)
        if e is None or seg_med is None:
            cause = "client_preempted" if pre > 0 else ("first_of_batch" if first else
                                                        "cpu_migrated" if migrated else "other")
        else:
            if int(e["cpu"]) == cpu:
                same_cpu += 1
            seg = segments(s, x, e)
            ex = [seg[i] - seg_med[i] for i in range(3)]
            k = int(np.argmax(ex))
            cause = (("inbound_worker_polling" if e["spinning"] else "inbound_worker_asleep"), "server_handling",
                     "outbound_client_wakeup")[k]
            if pre > 0 and k != 1:
                cause = "client_preempted"
            excess[cause].append(ex[k])
            slowest.append((x, cause, [round(v / 1e3, 2) for v in seg], int(e["spinning"])))
        if e is None or seg_med is None:
            slowest.append((x, cause, None, None))
        causes[cause] += 1
    out["by_cause"] = dict(sorted(causes.items()))
    out["cause_mean_excess_us"] = {k: round(sum(v) / len(v) / 1e3, 2) for k, v in sorted(excess.items())}
    out["same_cpu_as_worker"] = same_cpu
    # the calls p99.9 is made of, each with its cause and segments
    out["slowest"] = [{"us": round(x * 1e6, 2), "cause": c, "segments_us": sg, "worker_polling": sp}
                      for x, c, sg, sp in sorted(slowest, key=lambda r: -r[0])[:8]]
    return out


def _merge_tail(parts) -> dict:
    import collections
    out = {"calls": 0, "slow": 0, "first_of_batch": 0, "cpu_migrated": 0, "client_preempted": 0, "matched": 0,
           "same_cpu_as_worker": 0}
    causes = collections.Counter()
    for p in parts:
        for k in out:
            out[k] += p.get(k, 0)
        causes.update(p.get("by_cause", {}))
    out["by_cause"] = dict(sorted(causes.items()))
    out["other"] = causes.get("other", 0)  # slow calls with no evidence at all
    out["slow_fraction"] = round(out["slow"] / max(1, out["calls"]), 4)
    if parts and parts[0].get("segment_p50_us"):
        out["segment_p50_us"] = parts[0]["segment_p50_us"]
        out["cause_mean_excess_us"] = parts[0].get("cause_mean_excess_us")
        out["server_split_p50_us"] = parts[0].get("server_split_p50_us")
        out["outbound_split_p50_us"] = parts[0].get("outbound_split_p50_us")
    out["slowest"] = sorted((x for p in parts for x in p.get("slowest", [])), key=lambda r: -r["us"])[:8]
    return out


def _read(path: str, default=None):
    try:
        with open(path) as f:
            return f.read().strip()
    except OSError:
        return default


def _cpu_list(spec):
    """'0-3,8,10-11' -> [0, 1, 2, 3, 8, 10, 11] (None for an unreadable list)."""
    if spec is None:
        return None
    out = []
    for part in spec.split(","):
        part = part.strip()
        if not part:
            continue
        a, _, b = part.partition("-")
        out.extend(range(int(a), int(b or a) + 1))
    return out


def cpu_topology(cpus) -> dict:
    """For each CPU: (package, core id, SMT siblings, L3 siblings, NUMA node), from sysfs."""
    out = {}
    base = "/sys/devices/system/cpu/cpu%d"
    for c in cpus:
        d = base % c
        l3 = None
        for idx in range(8):
            if _read("%s/cache/index%d/level" % (d, idx)) == "3":
                l3 = _cpu_list(_read("%s/cache/index%d/shared_cpu_list" % (d, idx)))
                break
        node = None
        try:
            node = next(int(x[4:]) for x in os.listdir(d) if x.startswith("node") and x[4:].isdigit())
        except (OSError, StopIteration):
            pass
        out[c] = {"package": _read(d + "/topology/physical_package_id"), "core": _read(d + "/topology/core_id"),
                  "smt": _cpu_list(_read(d + "/topology/thread_siblings_list")), "l3": l3, "numa": node}
    return out


def cpu_relation(a: int, b: int, topo: dict) -> str:
    """Where two CPUs sit relative to each other: same_cpu, smt_sibling, same_l3,
    same_package (another L3 of the socket), other_package, or unknown."""
    if a == b:
        return "same_cpu"
    ta, tb = topo.get(a), topo.get(b)
    if not ta or not tb:
        return "unknown"
    if ta["smt"] and b in ta["smt"]:
        return "smt_sibling"
    if ta["l3"] and b in ta["l3"]:
        return "same_l3"
    if ta["package"] is not None and ta["package"] == tb["package"]:
        return "same_package"
    return "other_package"


def host_fingerprint(cpus=()) -> dict:
    """What a latency number depends on besides the code: CPU model and measured clock,
    frequency driver and governor, SMT, idle states, CPU quota and set, speculative-execution
    mitigations (every syscall pays them) and the load, for the CPUs named in `cpus`
    (the client's and the daemon workers')."""
    cpuinfo = _read("/proc/cpuinfo", "") or ""
    model = next((ln.split(":", 1)[1].strip() for ln in cpuinfo.splitlines() if ln.startswith("model name")), None)
    sysc = "/sys/devices/system/cpu"
    fp = {"cpu_model": model, "logical_cpus": os.cpu_count(), "affinity_cpus": len(os.sched_getaffinity(0)),
          "kernel": os.uname().release, "smt_active": _read(sysc + "/smt/active"),
          "cpufreq_driver": _read(sysc + "/cpu0/cpufreq/scaling_driver"),
          "cpufreq_governor": _read(sysc + "/cpu0/cpufreq/scaling_governor"),
          "amd_pstate": _read(sysc + "/amd_pstate/status"), "boost": _read(sysc + "/cpufreq/boost"),
          "cpuidle_driver": _read(sysc + "/cpuidle/current_driver"),
          "cpuidle_governor": _read(sysc + "/cpuidle/current_governor_ro") or _read(sysc + "/cpuidle/current_governor"),
          "cgroup_cpu_max": _read("/sys/fs/cgroup/cpu.max"),
          "cgroup_cpuset": _read("/sys/fs/cgroup/cpuset.cpus.effective"),
          "loadavg": _read("/proc/loadavg")}
    vul = {}
    try:
        for name in sorted(os.listdir(sysc + "/vulnerabilities")):
            v = _read(sysc + "/vulnerabilities/" + name)
            if v and not v.startswith("Not affected"):
                vul[name] = v
    except OSError:
        pass
    fp["mitigations"] = vul
    per = {}
    topo = cpu_topology(sorted(set(c for c in cpus if c is not None and c >= 0)))
    for c, t in topo.items():
        d = "%s/cpu%d" % (sysc, c)
        states = []
        for k in range(16):
            name = _read("%s/cpuidle/state%d/name" % (d, k))
            if name is None:
                break
            states.append({"name": name, "latency_us": _read("%s/cpuidle/state%d/latency" % (d, k)),
                           "disabled": _read("%s/cpuidle/state%d/disable" % (d, k)),
                           "usage": _read("%s/cpuidle/state%d/usage" % (d, k))})
        per[str(c)] = {**{k: v for k, v in t.items() if k not in ("smt", "l3")},
                       "smt": t["smt"], "l3_size": len(t["l3"]) if t["l3"] else None,
                       "cur_khz": _read(d + "/cpufreq/scaling_cur_freq"), "max_khz": _read(d + "/cpufreq/cpuinfo_max_freq"),
                       "idle_states": states}
    fp["cpus"] = per
    return fp


def placement_floor(nb, client_cpu: int, sizes, n: int = 3000) -> dict:
    """The bare spin exchange (uds_roundtrip_floor_spin) between the client's CPU and one
    CPU of each relation to it that this process may use: p50 us per relation.  Says what
    a worker on another core, L3 or socket costs on this host, independent of the plugin."""
    allowed = sorted(os.sched_getaffinity(0))
    topo = cpu_topology(allowed)
    picks = {}
    for c in allowed:
        rel = cpu_relation(client_cpu, c, topo)
        if rel not in ("same_cpu", "unknown") and rel not in picks:
            picks[rel] = c
    out = {}
    for rel, c in sorted(picks.items()):
        try:
            lat = nb.uds_pingpong(n, 300, *sizes, server_spin=True, client_cpu=client_cpu, server_cpu=c)
        except RuntimeError as e:
            out[rel] = {"server_cpu": c, "error": str(e)}
            continue
        out[rel] = {"server_cpu": c, "p50_us": round(_pct(lat, 0.5) * 1e6, 2)}
    return out


def paired_floor(h2, nb, method: str, req: bytes, sizes, rounds: int = 16, batch: int = 256) -> dict:
    """Allocate and the bare spin exchange (uds_roundtrip_floor_spin) in alternating
    batches, untimed: per round the ratio of the two p50s.  On a shared host the floor
    measured once, after the timed loop, meets other moments of the host than the
    Allocates did; paired rounds compare like with like."""
    import statistics
    ratios, alloc_p50, floor_p50 = [], [], []
    for r in range(rounds):
        order = (0, 1) if r % 2 == 0 else (1, 0)
        got = {}
        for k in order:
            if k == 0:
                got[0] = _pct(h2.bench_unary(method, req, batch), 0.5)
            else:
                got[1] = _pct(nb.uds_pingpong(batch, 32, *sizes, server_spin=True), 0.5)
        alloc_p50.append(got[0])
        floor_p50.append(got[1])
        ratios.append(got[0] / got[1])
    ratios.sort()
    # distribution-free ~95 % interval of the median: order statistics n/2 -+ 0.98 sqrt(n)
    k = max(0, int(rounds / 2 - 0.98 * rounds ** 0.5))
    lo, hi = ratios[max(0, k - 1)], ratios[min(rounds - 1, rounds - k)]
    return {"rounds": rounds, "batch": batch, "allocate_p50_us": round(statistics.median(alloc_p50) * 1e6, 2),
            "floor_spin_p50_us": round(statistics.median(floor_p50) * 1e6, 2),
            "ratio_median": round(statistics.median(ratios), 3), "ratio_ci95": [round(lo, 3), round(hi, 3)]}


def _proc_stat_busy() -> dict:
    """cpu -> (busy jiffies, total jiffies) from /proc/stat."""
    out = {}
    with open("/proc/stat") as f:
        for line in f:
            if not line.startswith("cpu") or line.startswith("cpu "):
                continue
            parts = line.split()
            vals = [int(x) for x in parts[1:]]
            idle = vals[3] + (vals[4] if len(vals) > 4 else 0)
            out[int(parts[0][3:])] = (sum(vals) - idle, sum(vals))
    return out


def _busy_study(batches, trace, busy_log, rpc_allocate: int) -> list:
    """Per timed batch: its p50, the client's and the worker's CPU, and how busy each of
    those and their SMT siblings were during the batch (fraction of jiffies)."""
    if not busy_log or trace is None:
        return []
    topo = cpu_topology(sorted(os.sched_getaffinity(0)))
    rows = []
    for b, (s0, s1) in zip(batches, busy_log):
        m = match_calls([int(x) for x in b[0]], list(b[1]), trace, rpc_allocate)
        workers = collections.Counter(int(e["cpu"]) for e in m if e is not None)
        clients = collections.Counter(b[2])
        if not workers or not clients:
            continue
        c, w = clients.most_common(1)[0][0], workers.most_common(1)[0][0]

        def frac(cpu):
            if cpu not in s0 or cpu not in s1 or s1[cpu][1] == s0[cpu][1]:
                return None
            return round((s1[cpu][0] - s0[cpu][0]) / (s1[cpu][1] - s0[cpu][1]), 2)

        def sib(cpu):
            t = topo.get(cpu)
            return [x for x in (t["smt"] if t and t["smt"] else []) if x != cpu]
        rows.append({"p50_us": round(_pct(list(b[1]), 0.5) * 1e6, 2), "client": c, "worker": w,
                     "relation": cpu_relation(c, w, topo), "client_busy": frac(c), "worker_busy": frac(w),
                     "client_sibling_busy": [frac(x) for x in sib(c)], "worker_sibling_busy": [frac(x) for x in sib(w)]})
    return rows


def _placement_stats(batches, trace, topo_cpus: dict, rpc_allocate: int) -> dict:
    """Allocate latency by where the daemon's worker ran relative to the client (the
    worker's CPU is in its call-trace record, the client's in bench_unary_ts)."""
    import collections
    if trace is None or not len(trace):
        return {}
    starts = [int(s) for b in batches for s in b[0]]
    lats = [x for b in batches for x in b[1]]
    cpus = [c for b in batches for c in b[2]]
    matched = match_calls(starts, lats, trace, rpc_allocate)
    topo = cpu_topology(sorted(set(cpus) | {int(e["cpu"]) for e in matched if e is not None}))
    topo_cpus.update(topo)
    by = collections.defaultdict(list)
    pairs = collections.defaultdict(list)
    for x, c, e in zip(lats, cpus, matched):
        if e is not None:
            by[cpu_relation(c, int(e["cpu"]), topo)].append(x)
            pairs[(c, int(e["cpu"]))].append(x)
    out = {rel: {"calls": len(v), "p50_us": round(_pct(v, 0.5) * 1e6, 2)} for rel, v in sorted(by.items())}
    # the (client CPU, worker CPU) pairs the calls ran on, busiest first, and each batch's p50
    out["pairs"] = [{"client": c, "worker": w, "relation": cpu_relation(c, w, topo), "calls": len(v),
                     "p50_us": round(_pct(v, 0.5) * 1e6, 2)}
                    for (c, w), v in sorted(pairs.items(), key=lambda kv: -len(kv[1]))[:6]]
    out["batch_p50_us"] = [round(_pct(list(b[1]), 0.5) * 1e6, 2) for b in batches]
    return out


def _server_mean(text: str, rpc: str):
    """Mean of the daemon's amdgpu_device_plugin_rpc_duration_seconds for one RPC: the
    time from a request's dispatch to its encoded answer, without the transport."""
    tot = cnt = 0.0
    for line in text.splitlines():
        if 'rpc="%s"' % rpc not in line:
            continue
        if line.startswith("amdgpu_device_plugin_rpc_duration_seconds_sum"):
            tot += float(line.rsplit(" ", 1)[1])
        elif line.startswith("amdgpu_device_plugin_rpc_duration_seconds_count"):
            cnt += float(line.rsplit(" ", 1)[1])
    return tot / cnt if cnt else None


def _scrape_server_mean(text: str):
    """Mean of the daemon's echo_http_request_duration_seconds for GET /metrics: from a
    parsed request to its answer handed to the kernel (render + sendmsg)."""
    tot = cnt = 0.0
    for line in text.splitlines():
        if 'handler="/metrics"' not in line or 'method="GET"' not in line:
            continue
        if line.startswith("echo_http_request_duration_seconds_sum"):
            tot += float(line.rsplit(" ", 1)[1])
        elif line.startswith("echo_http_request_duration_seconds_count"):
            cnt += float(line.rsplit(" ", 1)[1])
    return tot / cnt if cnt else None


def _allocator_probe(n) -> float:
    """The xGMI allocator's own cost for a size-4 request over an 8-GPU mesh (two NUMA
    nodes), timed natively.  On a 1-GPU box the kubelet GetPreferredAllocation above
    can only return its one device, so this is what says what the policy costs."""
    topo = n.Topology(8)
    for a in range(8):
        for b in range(a + 1, 8):
            topo.set_link(a, b, n.Link(type=n.LINK_XGMI, hops=1, up=True))
    devs = [n.AllocDevice(g, -1, g // 4, "gpu%d" % g) for g in range(8)]
    lat = n.bench_aligned_alloc(topo, devs, list(range(8)), [1], 4, 2000)
    return round(_pct(lat[200:], 0.5) * 1e6, 2)


def device_for_rank(metrics_text: str, ids, resource: str, local_rank: int, rank: int):
    """The advertised device whose host HIP ordinals include ``local_rank`` (from the
    daemon's ``amdgpu_partition_info{device_id, resource, hip_ids}``); ``(device, hip_ids,
    how)``.  Falls back to enumeration order (``ids[rank]``) only when the daemon reports
    no HIP ordinals."""
    from prometheus_client.parser import text_string_to_metric_families
    hips = {}
    for fam in text_string_to_metric_families(metrics_text):
        if fam.name != "amdgpu_partition_info":
            continue
        for smp in fam.samples:
            if smp.labels.get("resource") == resource and smp.labels.get("hip_ids"):
                hips[smp.labels["device_id"]] = [int(x) for x in smp.labels["hip_ids"].split(",")]
    mine = [d for d in ids if local_rank in hips.get(d, [])]
    if len(mine) == 1:
        return mine[0], hips[mine[0]], "hip_id"
    if hips:
        raise RuntimeError("no single advertised device holds HIP ordinal %d: %s" % (local_rank, hips))
    return ids[rank], [], "enumeration order"


def host_ordinals(count: int, env=None):
    """The host's HIP ordinal of each of this process's GPU ordinals 0..count-1.  amdsmi
    reports a partition's ``hip_id`` in the host's numbering, while ROCR_VISIBLE_DEVICES
    and then HIP_VISIBLE_DEVICES (or CUDA_VISIBLE_DEVICES) renumber what a process - torch,
    the canary - sees.  ``None`` when a list is not plain ordinals (UUIDs): then the two
    numberings are taken to agree."""
    env = os.environ if env is None else env
    phys = list(range(4096))
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES" if "HIP_VISIBLE_DEVICES" in env else "CUDA_VISIBLE_DEVICES"):
        spec = env.get(var)
        if spec is None or spec.strip() == "":
            continue
        try:
            sel = [int(x) for x in spec.split(",") if x.strip()]
        except ValueError:
            return None
        if any(i < 0 or i >= len(phys) for i in sel):
            return None
        phys = [phys[i] for i in sel]
    return phys[:count] if len(phys) >= count else None


def resolve_backend(n, requested: str = "auto") -> str:
    """amdsmi when asked for, or when auto and amdsmi sees a GPU; else the fixture node
    model (CPU runs, and multi-rank rehearsals on a box with fewer GPUs than ranks)."""
    if requested == "auto":
        return "amdsmi" if n.amdsmi_available() else "fixture"
    return requested


def start_daemon(n_gpus: int, grpc_server: str, workdir: str, profile_dir: str = "", busy_poll_us=None,
                 admission_poll_us=None, overrides=None, backend: str = "auto", fixture: str = "", hips=None):
    """Rank 0: kubelet stub + plugin daemon subprocess.  Must run before GPU init.
    ``overrides``: config sections merged over the bench's own (probes, A/B runs)."""
    import yaml

    from k8s_gpu_device_plugin_amd import native
    from k8s_gpu_device_plugin_amd.plugin.kubelet_stub import KubeletStub

    n = native.load()
    backend = resolve_backend(n, backend)
    plugin_dir = os.path.join(workdir, "device-plugins")
    os.makedirs(plugin_dir, exist_ok=True)
    kubelet = KubeletStub(plugin_dir).start()
    port = _free_port()
    cfg_path = os.path.join(workdir, "bench-config.yml")
    # one server worker per client connection: every rank holds two kubelet-side
    # connections (compiled h2 + grpcio) and SCRAPE_CONNS scrapers
    cfg = {"webListenAddress": "127.0.0.1:%d" % port, "migStrategy": "none", "backend": backend,
           "fixture": fixture or "%dgpu_spx" % n_gpus, "devices": ",".join("hip:%d" % h for h in (hips or range(n_gpus))), "pluginDir": plugin_dir,
           "log": {"level": "info", "fileDir": ""},
           "http": {"accessLog": False, "threads": max(4, SCRAPE_CONNS * n_gpus)},
           "telemetry": {"intervalMs": 1000},
           "grpc": {"server": grpc_server, "threads": max(4, 2 * n_gpus),
                    # per-call server records: the tail attribution reads them (allocate_tail)
                    "callTraceFile": os.path.join(workdir, "calltrace-{resource}.bin"), "callTraceEntries": 1 << 18}}
    if busy_poll_us is not None:
        cfg["http"]["busyPollUs"] = cfg["grpc"]["busyPollUs"] = busy_poll_us
    if admission_poll_us is not None:
        cfg["grpc"]["admissionPollUs"] = admission_poll_us
    if profile_dir:  # benchmark: true -> cpu/mem/threads/native profiles when the daemon exits
        cfg["benchmark"] = True
        cfg["benchmarkDir"] = os.path.abspath(profile_dir)
    for k, v in (overrides or {}).items():
        if isinstance(v, dict) and isinstance(cfg.get(k), dict):
            cfg[k] = {**cfg[k], **v}
        else:
            cfg[k] = v
    with open(cfg_path, "w") as f:
        yaml.safe_dump(cfg, f)
    env = dict(os.environ)
    env["PYTHONPATH"] = ROOT + os.pathsep + env.get("PYTHONPATH", "")
    env["AMDGPU_DP_PARENT_PID"] = str(os.getpid())  # the daemon exits with this process
    log = open(os.path.join(workdir, "daemon.log"), "w")
    proc = subprocess.Popen([sys.executable, "-m", "k8s_gpu_device_plugin_amd", "--configFile", cfg_path],
                            cwd=workdir, env=env, stdout=log, stderr=subprocess.STDOUT, start_new_session=True)
    regs = kubelet.wait_for_registrations(1, timeout=60)
    _wait_http(port, 30)
    return proc, kubelet, port, regs[0], backend


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--grpc-server", choices=["native", "python"], default="native")
    ap.add_argument("--no-canary", action="store_true")
    ap.add_argument("--busy-poll-us", type=int, default=None,
                    help="override grpc.busyPollUs of the daemon (default: the config default)")
    ap.add_argument("--admission-poll-us", type=int, default=None,
                    help="override grpc.admissionPollUs of the daemon (default: the config default)")
    ap.add_argument("--profile-dir", default="", help="run the daemon with benchmark: true, profiles here")
    ap.add_argument("--backend", choices=["auto", "amdsmi", "fixture"], default="auto",
                    help="daemon backend (auto: amdsmi when it sees a GPU); the canary runs only on amdsmi")
    ap.add_argument("--fixture", default="", help="fixture node model of a fixture daemon (default: <N>gpu_spx)")
    ap.add_argument("--daemon-config", default="",
                    help='JSON config sections merged over the daemon\'s (A/B runs), e.g. {"grpc": {"keepWarmMs": 0}}')
    ap.add_argument("--diag-cpu-busy", action="store_true",
                    help="diagnostics: read /proc/stat around every compiled-client Allocate batch and report how "
                         "busy the client's and the worker's CPUs and their SMT siblings were (placement study)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    n_gpus = args.gpus
    if world != n_gpus:
        # one kubelet-client rank per advertised GPU (weak scaling): anything else would
        # report n_gpus for a run that did not have that many ranks or devices
        raise SystemExit("bench.py: WORLD_SIZE=%d but --gpus %d; launch one rank per GPU "
                         "(torch.distributed.run --nproc-per-node %d)" % (world, n_gpus, n_gpus))

    from k8s_gpu_device_plugin_amd import native
    n = native.load()
    nb = native.load_bench()  # load generators and latency probes (not part of the plugin)
    if args.grpc_server == "native" and not hasattr(n, "GrpcServer"):
        args.grpc_server = "python"

    # one directory per job: ranks of one torchrun job share it (same MASTER_PORT), two
    # single-process runs on one host (concurrent test workers) must not
    master_port = os.environ.get("MASTER_PORT") or "pid%d" % os.getpid()
    workdir = os.path.join(tempfile.gettempdir(), "amdgpu-dp-bench-%s-%d" % (master_port, os.getuid()))
    proc = kubelet = None
    info = None
    # the host HIP ordinals of the ranks' GPUs (local rank r opens its ordinal r, which the
    # *_VISIBLE_DEVICES variables may have renumbered); a fixture node numbers its own
    real = resolve_backend(n, args.backend) == "amdsmi"
    hips = (host_ordinals(n_gpus) if real else None) or list(range(n_gpus))
    if rank == 0:  # daemon first: nothing has touched the GPU in this process yet
        shutil.rmtree(workdir, ignore_errors=True)
        os.makedirs(workdir)
        proc, kubelet, port, reg, backend = start_daemon(n_gpus, args.grpc_server, workdir, args.profile_dir,
                                                         args.busy_poll_us, args.admission_poll_us,
                                                         backend=args.backend, fixture=args.fixture, hips=hips,
                                                         overrides=json.loads(args.daemon_config) if args.daemon_config
                                                         else None)
        info = {"port": port, "endpoint": reg.endpoint, "resource": reg.resource_name, "backend": backend,
                "plugin_dir": os.path.join(workdir, "device-plugins")}

    # Validate this rank's GPU with the gfx950 canary (HBM pattern + MFMA exactness and
    # rate) in a child process, before this process loads torch or initialises RCCL: each
    # rank then holds exactly one HIP runtime (torch's) when the communicator comes up.
    canary_res = None
    if not args.no_canary and resolve_backend(n, args.backend) == "amdsmi":
        from k8s_gpu_device_plugin_amd.ops import canary
        canary_res = canary.run_isolated(local_rank, hbm_bytes=1 << 30, timeout=300.0, passes=3)
        if not canary_res.get("ok"):
            raise RuntimeError("canary failed on rank %d (GPU %d): %s" % (rank, local_rank, canary_res))

    import torch
    import torch.distributed as dist

    use_cuda = torch.cuda.is_available()
    if world > 1:
        if use_cuda:
            torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl" if use_cuda else "gloo",
                                device_id=torch.device("cuda", local_rank) if use_cuda else None)
        obj = [info]
        dist.broadcast_object_list(obj, src=0)
        info = obj[0]
    elif use_cuda:
        torch.cuda.set_device(local_rank)

    def barrier():
        if world > 1:
            dist.barrier()
        if use_cuda:
            torch.cuda.synchronize()

    from k8s_gpu_device_plugin_amd.api import v1beta1
    from k8s_gpu_device_plugin_amd.plugin.kubelet_stub import DevicePluginClient

    client = DevicePluginClient(os.path.join(info["plugin_dir"], info["endpoint"]))
    law = client.list_and_watch()
    first = next(iter(law))
    law.cancel()
    ids = [d.ID for d in first.devices]
    if len(ids) != n_gpus:
        raise RuntimeError("the plugin advertised %d device(s) of %s, --gpus is %d" % (len(ids), info["resource"],
                                                                                     n_gpus))
    conn = http.client.HTTPConnection("127.0.0.1", info["port"], timeout=10)
    conn.request("GET", "/metrics")
    body = conn.getresponse().read()
    if b"amdgpu_info{" not in body:
        raise RuntimeError("/metrics lacks the GPU inventory")
    # the device of this rank's GPU (HIP ordinal local_rank, in the host's numbering), not
    # the rank-th in BDF order
    my_id, my_hips, mapped_by = device_for_rank(body.decode(), ids, info["resource"],
                                                hips[local_rank] if local_rank < len(hips) else local_rank, rank)
    alloc_req = v1beta1.AllocateRequest(container_requests=[
        v1beta1.ContainerAllocateRequest(devices_ids=[my_id])]).SerializeToString()
    pref_req = v1beta1.PreferredAllocationRequest(container_requests=[
        v1beta1.ContainerPreferredAllocationRequest(available_deviceIDs=ids, must_include_deviceIDs=[my_id],
                                                    allocation_size=min(2, len(ids)))]).SerializeToString()
    alloc_raw, pref_raw = client.allocate_raw, client.preferred_raw
    h2 = n.H2Client(os.path.join(info["plugin_dir"], info["endpoint"]))  # compiled, kubelet-like client

    # ---- validate the allocation on the real device (untimed) ----
    resp = v1beta1.AllocateResponse.FromString(alloc_raw(alloc_req))
    specs = [s.host_path for s in resp.container_responses[0].devices]
    if info["backend"] == "amdsmi":
        missing = [p for p in specs if not os.path.exists(p)]
        if missing:
            raise RuntimeError("allocated device nodes missing: %s" % missing)

    perf = time.perf_counter

    def phase_sync():
        # Ranks move through a step's phases together: the kubelet RPC phase is measured
        # under N concurrent kubelet-like clients, not under N-1 other ranks' max-rate
        # scrapers, and every rank's scrape window overlaps (aggregate daemon throughput).
        if world > 1:
            dist.barrier()

    def step(rec):
        a, p, s, an, pn, tl = rec
        phase_sync()
        busy0 = _proc_stat_busy() if args.diag_cpu_busy else None
        starts, lat, cpus, pre, tail = h2.bench_unary_ts(v1beta1.METHOD_ALLOCATE, alloc_req, ALLOCS)
        if busy0 is not None:
            busy_log.append((busy0, _proc_stat_busy()))
        an.extend(lat)
        tl.append((starts, lat, cpus, pre, tail))
        pn.extend(h2.bench_unary(v1beta1.METHOD_GET_PREFERRED, pref_req, PREFS))
        for _ in range(ALLOCS):
            t0 = perf()
            alloc_raw(alloc_req)
            a.append(perf() - t0)
        for _ in range(PREFS):
            t0 = perf()
            pref_raw(pref_req)
            p.append(perf() - t0)
        phase_sync()
        r = nb.http_load("127.0.0.1", info["port"], "/metrics", SCRAPE_CONNS, SCRAPE_S, 0.0)
        if r["errors"]:
            raise RuntimeError("%d /metrics scrape errors" % r["errors"])
        s.extend(r["latencies_s"])
        return r["elapsed_s"], r["bytes"] // max(1, r["ok"])

    busy_log = []  # --diag-cpu-busy: (/proc/stat before, after) per timed batch
    junk = ([], [], [], [], [], [])
    for _ in range(args.warmup):
        step(junk)
    busy_log.clear()
    barrier()
    rec = ([], [], [], [], [], [])
    scrape_time, body_len = 0.0, len(body)
    t_start = perf()
    for _ in range(args.steps):
        st, body_len = step(rec)
        scrape_time += st
    barrier()
    elapsed = perf() - t_start
    # the daemon's record of every call so far (untimed): the tail attribution matches them
    trace = read_call_trace(os.path.join(workdir, "calltrace-%s.bin" % info["resource"].split("/")[-1]))
    mine = {"elapsed": elapsed, "scrape_time": scrape_time, "alloc": rec[0], "pref": rec[1], "scrape": rec[2],
            "alloc_native": rec[3], "pref_native": rec[4], "alloc_tail": _tail_stats(rec[5], trace, n.RPC_ALLOCATE),
            "canary": canary_res, "body": body_len,
            "device": {"rank": rank, "local_rank": local_rank, "device_id": my_id, "hip_ids": my_hips,
                       "mapped_by": mapped_by}}
    # where the client and the daemon's worker ran, per call, and what the host is (untimed)
    topo_cpus = {}
    mine["placement"] = _placement_stats(rec[5], trace, topo_cpus, n.RPC_ALLOCATE)
    if args.diag_cpu_busy:
        mine["placement"]["batch_cpu_busy"] = _busy_study(rec[5], trace, busy_log, n.RPC_ALLOCATE)
    client_cpus = collections.Counter(c for b in rec[5] for c in b[2])
    client_cpu = client_cpus.most_common(1)[0][0] if client_cpus else os.sched_getcpu()
    worker_cpus = collections.Counter(int(c) for c in trace["cpu"]) if trace is not None and len(trace) else {}
    mine["client_cpus"] = dict(client_cpus.most_common(4))
    mine["worker_cpus"] = dict(collections.Counter(worker_cpus).most_common(4))
    # Untimed speed-of-light reference: the same send/epoll_wait/recv/send/recv exchange
    # between two threads with no HTTP/2, HPACK or protobuf work (sizes ~ this Allocate's).
    alloc_resp_len = len(alloc_raw(alloc_req))
    sizes = (9 + 80 + 9 + 5 + len(alloc_req), 9 + 20 + 9 + 5 + alloc_resp_len + 9 + 16)
    floor = nb.uds_pingpong(10000, 500, *sizes)
    mine["uds_floor_p50"] = _pct(floor, 0.5)
    # ... and with a server thread that polls instead of sleeping (the busy-poll window);
    # its p99 is this machine's tail for a bare back-to-back exchange (timer ticks,
    # interrupts and other tenants land on either thread's CPU), the floor Allocate's p99
    # is compared against
    spin = nb.uds_pingpong(10000, 500, *sizes, server_spin=True)
    mine["uds_floor_spin_p50"] = _pct(spin, 0.5)
    mine["uds_floor_spin_p99"] = _pct(spin, 0.99)
    mine["uds_floor_spin_p999"] = _pct(spin, 0.999)
    # ... and with the server consuming each request only after its answer (MSG_PEEK, the
    # daemon's grpc.peekReads): the bare exchange without the client's spurious wake-up
    mine["uds_floor_spin_peek_p50"] = _pct(nb.uds_pingpong(10000, 500, *sizes, server_spin=True, peek=True), 0.5)
    # ... and in the timed loop's own rhythm (batches of ALLOCS back-to-back exchanges, a
    # scrape phase apart) against a server with the plugin worker's polling policy: this
    # host's tail for that pattern, which Allocate's p99 / p99.9 are compared against
    bf = nb.uds_pingpong_batched(args.steps, ALLOCS, int(SCRAPE_S * 1e6), *sizes,
                                 server_poll_us=args.busy_poll_us if args.busy_poll_us is not None else 50)
    mine["uds_floor_batched"] = (_pct(bf, 0.5), _pct(bf, 0.99), _pct(bf, 0.999), max(bf))
    mine["uds_floor_batched_batch_p50"] = [round(_pct(bf[i:i + ALLOCS], 0.5) * 1e6, 2) for i in range(0, len(bf), ALLOCS)]
    # Allocate against the spin floor paired in time: batches of each alternate, so a busy
    # moment on the shared host lands on both (the floor above runs after the timed loop)
    mine["paired"] = paired_floor(h2, nb, v1beta1.METHOD_ALLOCATE, alloc_req, sizes)
    # kubelet-like sparse calls: 1 ms apart, every one meets a sleeping server thread
    mine["alloc_cold"] = h2.bench_unary(v1beta1.METHOD_ALLOCATE, alloc_req, 400, 1000)
    # ... and the bare exchange with the same 1 ms idle gap (cold caches, idle CPU states)
    mine["uds_floor_cold_p50"] = _pct(nb.uds_pingpong(400, 20, *sizes, gap_us=1000), 0.5)
    # a pod admission as kubelet runs it: GetPreferredAllocation, ~200 us of kubelet
    # bookkeeping, then Allocate of the same container (2 ms idle before each admission)
    adm = []
    for _ in range(200):
        time.sleep(0.002)
        h2.bench_unary(v1beta1.METHOD_GET_PREFERRED, pref_req, 1)
        t_go = perf() + 200e-6
        while perf() < t_go:
            pass
        adm.extend(h2.bench_unary(v1beta1.METHOD_ALLOCATE, alloc_req, 1))
    mine["alloc_admission"] = adm
    # /metrics: one loopback TCP exchange of a scrape's size, polling server
    mine["tcp_scrape_floor_p50"] = _pct(nb.uds_pingpong(3000, 300, 90, body_len + 400, server_spin=True, tcp=True),
                                        0.5)
    mine["placement_floor"] = placement_floor(nb, client_cpu, sizes)
    if rank == 0:
        mine["host"] = host_fingerprint(list(mine["client_cpus"]) + list(mine["worker_cpus"]))
        mine["host"]["core_ghz"] = round(nb.core_ghz(), 3)
    if rank == 0:  # the daemon's own time per Allocate (decode, lookup, encode), from its histogram
        conn.request("GET", "/metrics")
        text = conn.getresponse().read().decode()
        mine["server_allocate_mean_s"] = _server_mean(text, "Allocate")
        mine["server_preferred_mean_s"] = _server_mean(text, "GetPreferredAllocation")
        mine["server_scrape_mean_s"] = _scrape_server_mean(text)
    if world > 1:
        gathered = [None] * world
        dist.all_gather_object(gathered, mine)
    else:
        gathered = [mine]
    rc = 0
    if rank == 0:
        allocs = [x for g in gathered for x in g["alloc"]]
        allocs_native = [x for g in gathered for x in g["alloc_native"]]
        prefs = [x for g in gathered for x in g["pref"]]
        prefs_native = [x for g in gathered for x in g["pref_native"]]
        scrapes = [x for g in gathered for x in g["scrape"]]
        t_max = max(g["elapsed"] for g in gathered)
        scrape_t = max(g["scrape_time"] for g in gathered)
        p50 = _pct(allocs_native, 0.5) * 1e6
        p50_grpcio = _pct(allocs, 0.5) * 1e6
        can = [g["canary"] for g in gathered if g["canary"]]
        out = {
            "metric": METRIC, "value": round(p50, 2), "unit": "us (Allocate p50, compiled h2 client; lower is better)",
            "n_gpus": n_gpus, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(t_max / args.steps * 1e3, 3), "higher_is_better": False, "scaling": "weak",
            # a control-plane workload: no tensor arithmetic on the timed path (the gfx950
            # canary's bf16/MX-fp8/fp4 checks run untimed, see "canary")
            "vs_baseline": None, "dtype": "n/a",
            "data": "synthetic kubelet allocation workload (%d Allocate + %d GetPreferredAllocation per client "
                    "per rank per step, %d ms of /metrics scraping on %d connections per rank per step) against "
                    "%s-discovered devices" % (ALLOCS, PREFS, SCRAPE_S * 1e3, SCRAPE_CONNS, info["backend"]),
            "config": {"model": "MI355X device plugin, %s, strategy=none (SPX/NPS1 whole GPUs)" % info["resource"],
                       "global_batch": ALLOCS * world, "seq_len": 0,
                       "parallelism": "%d kubelet-client rank(s), 1 plugin daemon" % world,
                       "backend": info["backend"], "grpc_server": args.grpc_server},
            "allocate_p50_us": round(p50, 2), "allocate_p99_us": round(_pct(allocs_native, 0.99) * 1e6, 2),
            "allocate_p999_us": round(_pct(allocs_native, 0.999) * 1e6, 2),
            "allocate_max_us": round(max(allocs_native) * 1e6, 2),
            "allocate_tail": _merge_tail([g["alloc_tail"] for g in gathered]),
            "uds_roundtrip_floor_spin_p99_us": round(gathered[0]["uds_floor_spin_p99"] * 1e6, 2),
            "uds_roundtrip_floor_spin_p999_us": round(gathered[0]["uds_floor_spin_p999"] * 1e6, 2),
            # the bare exchange timed in the same batches as Allocate (p50, p99, p99.9, max)
            "uds_roundtrip_floor_batched_us": [round(x * 1e6, 2) for x in gathered[0]["uds_floor_batched"]],
            # Allocate and the spin floor in alternating batches after the timed loop (rank 0)
            "allocate_vs_spin_floor_paired": gathered[0].get("paired"),
            # per-batch p50 of the bare exchange timed in the loop's rhythm (rank 0): a host
            # whose batches fall into a slow mode shows it here too
            "uds_floor_batched_batch_p50_us": gathered[0].get("uds_floor_batched_batch_p50"),
            "preferred_allocator_8gpu_size4_p50_us": _allocator_probe(n),
            "allocate_server_mean_us": (round(gathered[0]["server_allocate_mean_s"] * 1e6, 3)
                                        if gathered[0].get("server_allocate_mean_s") else None),
            "advertised_devices": len(ids), "world_size": world,
            "rank_devices": [g["device"] for g in gathered],
            "dist_backend": (dist.get_backend() if world > 1 else None),
            "uds_roundtrip_floor_p50_us": round(gathered[0]["uds_floor_p50"] * 1e6, 2),
            "uds_roundtrip_floor_spin_p50_us": round(gathered[0]["uds_floor_spin_p50"] * 1e6, 2),
            "uds_roundtrip_floor_spin_peek_p50_us": round(gathered[0]["uds_floor_spin_peek_p50"] * 1e6, 2),
            "uds_roundtrip_floor_cold_p50_us": round(gathered[0]["uds_floor_cold_p50"] * 1e6, 2),
            "allocate_cold_p50_us": round(_pct([x for g in gathered for x in g["alloc_cold"]], 0.5) * 1e6, 2),
            "allocate_admission_p50_us": round(_pct([x for g in gathered for x in g["alloc_admission"]], 0.5) * 1e6, 2),
            "tcp_scrape_floor_p50_us": round(gathered[0]["tcp_scrape_floor_p50"] * 1e6, 2),
            "allocate_p50_us_grpcio_client": round(p50_grpcio, 2),
            "allocate_p99_us_grpcio_client": round(_pct(allocs, 0.99) * 1e6, 2),
            "preferred_p50_us": round(_pct(prefs_native, 0.5) * 1e6, 2),
            "preferred_p99_us": round(_pct(prefs_native, 0.99) * 1e6, 2),
            "preferred_server_mean_us": (round(gathered[0]["server_preferred_mean_s"] * 1e6, 3)
                                         if gathered[0].get("server_preferred_mean_s") else None),
            "preferred_p50_us_grpcio_client": round(_pct(prefs, 0.5) * 1e6, 2),
            "scrape_p50_us": round(_pct(scrapes, 0.5) * 1e6, 2),
            "scrape_rps": round(len(scrapes) / scrape_t, 1) if scrape_t > 0 else None,
            "scrape_p99_us": round(_pct(scrapes, 0.99) * 1e6, 2),
            # the daemon's own time per /metrics answer (render + the sendmsg that hands it over)
            "scrape_server_mean_us": (round(gathered[0]["server_scrape_mean_s"] * 1e6, 3)
                                      if gathered[0].get("server_scrape_mean_s") else None),
            "scrapes": len(scrapes),
            # where each Allocate's client and daemon worker ran relative to each other, the
            # bare exchange between the client's CPU and one CPU of each relation, and the host
            "placement": {"allocate_by_relation": gathered[0].get("placement"),
                          "client_cpus": gathered[0].get("client_cpus"), "worker_cpus": gathered[0].get("worker_cpus"),
                          "floor_spin_by_relation": gathered[0].get("placement_floor")},
            "host": gathered[0].get("host"),
            "allocate_calls": len(allocs) + len(allocs_native),
            "metrics_bytes": gathered[0]["body"],
            "canary": ({"arch": can[0]["arch"], "hbm_read_gbps": round(min(c["read_gbps"] for c in can), 1),
                        "hbm_write_gbps": round(min(c["write_gbps"] for c in can), 1),
                        "mfma_bf16_tflops": round(min(c["mfma_tflops"] for c in can), 1),
                        "lds_gemm_bf16_tflops": round(min(c["gemm_tflops"] for c in can), 1),
                        "mfma_mxfp8_tflops": round(min(c["fp8_tflops"] for c in can), 1),
                        "mfma_mxfp4_tflops": round(min(c["fp4_tflops"] for c in can), 1),
                        "lds_march_kb": min(c["lds_bytes"] for c in can) // 1024} if can else None),
        }
        print(json.dumps(out), flush=True)
    client.close()
    h2.close()
    conn.close()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    if rank == 0:
        if proc is not None:
            try:
                os.killpg(proc.pid, signal.SIGTERM)
            except ProcessLookupError:
                pass
            try:
                proc.wait(15)
            except subprocess.TimeoutExpired:
                os.killpg(proc.pid, signal.SIGKILL)
        if kubelet is not None:
            kubelet.stop()
        shutil.rmtree(workdir, ignore_errors=True)
    return rc


if __name__ == "__main__":
    sys.exit(main())
