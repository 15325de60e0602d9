"""Allocate with the daemon's gRPC workers pinned next to the client, per grpc.pollGapNs.

On a shared host the scheduler sometimes runs the gRPC worker on the SMT sibling of the
client's CPU, and those batches take ~4.5 us instead of ~2.6 (bench.py `placement`): the
worker's busy-poll loop and the client share one core.  This probe pins the client thread
to one CPU and the daemon's gRPC workers either to its SMT sibling or to another core of
the same L3, or starts them on the sibling and then lets them go anywhere (what a busy
host's scheduler does; grpc.coreEscape is then free to move them), for one daemon per
pollGapNs value (or per --arms entry), and alternates daemons and placements
batch by batch (rounds), so every value meets the same moments of the host.  The bare
spin exchange between the same CPU pairs is the floor.

    python scripts/smt_probe.py [--gaps 0,200,500] [--rounds 8] [--batch 512] [--out FILE]
    python scripts/smt_probe.py --arms '{"base": {}, "peek": {"grpc": {"peekReads": true}}}'
"""
from __future__ import annotations

import argparse
import json
import os
import shutil
import signal
import statistics
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def pick_cpus():
    """(client, its SMT sibling, another core of its L3), all in this process's cpuset."""
    allowed = sorted(os.sched_getaffinity(0))
    topo = bench.cpu_topology(allowed)
    for c in allowed:
        sib = [s for s in (topo[c]["smt"] or []) if s != c and s in allowed]
        if not sib:
            continue
        other = [o for o in allowed if bench.cpu_relation(c, o, topo) == "same_l3"]
        if other:
            return c, sib[0], other[0]
    return None


def worker_tids(pid):
    out = []
    for tid in os.listdir("/proc/%d/task" % pid):
        try:
            with open("/proc/%d/task/%s/comm" % (pid, tid)) as f:
                if f.read().startswith("dpgrpc"):
                    out.append(int(tid))
        except OSError:
            pass
    return out


def _last_cpu(pid, tid):
    try:
        with open("/proc/%d/task/%d/stat" % (pid, tid)) as f:
            return int(f.read().rsplit(")", 1)[1].split()[36])  # field 39: processor
    except (OSError, ValueError, IndexError):
        return -1


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gaps", default="0,200,500")
    ap.add_argument("--arms", default="", help="JSON {name: daemon config overrides}; replaces --gaps")
    ap.add_argument("--rounds", type=int, default=8)
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    cpus = pick_cpus()
    res = {"host": bench.host_fingerprint()}
    if cpus is None:
        res["error"] = "no CPU with an SMT sibling and another core of its L3 in this cpuset"
        print(json.dumps(res))
        return 0
    client, sib, other = cpus
    res["cpus"] = {"client": client, "smt_sibling": sib, "same_l3": other}
    from k8s_gpu_device_plugin_amd import native
    from k8s_gpu_device_plugin_amd.api import v1beta1
    n = native.load()
    nb = native.load_bench()
    if a.arms:
        arms = json.loads(a.arms)
    else:
        arms = {"pollGapNs=%d" % int(g): {"grpc": {"pollGapNs": int(g)}} for g in a.gaps.split(",")}
    gaps = list(arms)
    daemons = []
    try:
        for g in gaps:
            wd = tempfile.mkdtemp(prefix="amdgpu-dp-smt-")
            proc, kubelet, _port, reg, backend = bench.start_daemon(1, "native", wd, overrides=arms[g])
            h2 = n.H2Client(os.path.join(wd, "device-plugins", reg.endpoint))
            law = kubelet.watch(reg.endpoint)
            _, devs = law.next(timeout=10)
            req = v1beta1.AllocateRequest(container_requests=[v1beta1.ContainerAllocateRequest(
                devices_ids=[devs[0][0]])]).SerializeToString()
            daemons.append({"gap": g, "proc": proc, "kubelet": kubelet, "wd": wd, "h2": h2, "req": req,
                            "workers": worker_tids(proc.pid)})
            res["backend"] = backend
        os.sched_setaffinity(0, {client})  # this thread is the client
        for d in daemons:
            d["h2"].bench_unary(v1beta1.METHOD_ALLOCATE, d["req"], 2000)  # warm
        wheres = ("smt_sibling", "same_l3", "sibling_start")
        got = {(d["gap"], w): [] for d in daemons for w in wheres}
        ended = {(d["gap"], "sibling_start"): [] for d in daemons}
        for r in range(a.rounds):
            order = daemons if r % 2 == 0 else list(reversed(daemons))
            for d in order:
                full = os.sched_getaffinity(d["proc"].pid)
                # pinned to the client's sibling / to another core; or started on the sibling
                # and then free to go anywhere (what the scheduler does on a busy host)
                places = (("smt_sibling", sib, None), ("same_l3", other, None), ("sibling_start", sib, full))
                for where, cpu, then in (places if r % 2 == 0 else tuple(reversed(places))):
                    for tid in d["workers"]:
                        try:
                            os.sched_setaffinity(tid, {cpu})
                        except OSError:
                            pass
                    # (a sibling start waits out the escape's 100 ms gap that a pinned batch's
                    # failed attempt may have started)
                    time.sleep(0.15 if then is not None else 0.005)
                    if then is not None:
                        for tid in d["workers"]:
                            try:
                                os.sched_setaffinity(tid, then)
                            except OSError:
                                pass
                    lat = d["h2"].bench_unary(v1beta1.METHOD_ALLOCATE, d["req"], a.batch)
                    got[(d["gap"], where)].append(round(statistics.median(lat) * 1e6, 3))
                    if then is not None:
                        ended[(d["gap"], where)].append(sorted({_last_cpu(d["proc"].pid, t) for t in d["workers"]}))
        sizes = (9 + 80 + 9 + 5 + len(daemons[0]["req"]), 9 + 20 + 9 + 5 + 60 + 9 + 16)
        floors, floors_peek = {}, {}
        for where, cpu in (("smt_sibling", sib), ("same_l3", other)):
            lat = nb.uds_pingpong(4000, 300, *sizes, server_spin=True, client_cpu=client, server_cpu=cpu)
            floors[where] = round(statistics.median(lat) * 1e6, 3)
            lat = nb.uds_pingpong(4000, 300, *sizes, server_spin=True, client_cpu=client, server_cpu=cpu, peek=True)
            floors_peek[where] = round(statistics.median(lat) * 1e6, 3)
        res["floor_spin_p50_us"] = floors
        res["floor_spin_peek_p50_us"] = floors_peek
        res["allocate"] = {}
        for g in gaps:
            row = {}
            for where in wheres:
                xs = got[(g, where)]
                row[where] = {"p50_of_batches_us": round(statistics.median(xs), 3), "batches_us": xs}
            row["sibling_start"]["worker_cpus_after"] = ended[(g, "sibling_start")]
            res["allocate"][g] = row
    finally:
        for d in daemons:
            try:
                d["h2"].close()
                os.killpg(d["proc"].pid, signal.SIGTERM)
                d["proc"].wait(15)
            except Exception:
                pass
            d["kubelet"].stop()
            shutil.rmtree(d["wd"], ignore_errors=True)
    line = json.dumps(res)
    if a.out:
        with open(a.out, "w") as f:
            f.write(line + "\n")
    print(line, flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
