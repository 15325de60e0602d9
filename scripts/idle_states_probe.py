"""Does a ping-pong client's CPU enter cpuidle once per call?  (It does not: the check
tried first for grpc.coreEscape's "is the client on my SMT sibling" question.)

Pins the bare unix-socket exchange (the plugin's syscall pattern, tests/native/loadgen.cpp)
between CPU 0 and its SMT sibling (128 on the MI355X hosts), then CPU 0 and CPU 1, and
prints how often each CPU entered each cpuidle state during 10000 calls.

    python scripts/idle_states_probe.py
"""
import os, sys, json, glob
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
from k8s_gpu_device_plugin_amd import native
nb = native.load_bench()
def states(cpu):
    out = {}
    for d in sorted(glob.glob("/sys/devices/system/cpu/cpu%d/cpuidle/state*" % cpu)):
        try:
            out[open(d + "/name").read().strip()] = int(open(d + "/usage").read())
        except OSError as e:
            out[d] = str(e)
    return out
res = {}
for srv in (128, 1):
    a0, a1 = states(0), states(srv)
    lat = nb.uds_pingpong(10000, 300, 200, 300, server_spin=True, client_cpu=0, server_cpu=srv)
    b0, b1 = states(0), states(srv)
    res[srv] = {"client_cpu0_delta": {k: b0[k] - a0[k] for k in b0 if isinstance(b0[k], int)},
                "server_delta": {k: b1[k] - a1[k] for k in b1 if isinstance(b1[k], int)},
                "p50_us": sorted(lat)[len(lat) // 2] * 1e6}
print(json.dumps(res))
