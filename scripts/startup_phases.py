"""Per-phase start-up timing of the amdsmi path (import, native load, amdsmi init, discover, first sample).

Run from the repo root on a GPU box: PYTHONPATH=$PWD python scripts/startup_phases.py
"""
import time, sys, os, tempfile
t0 = time.perf_counter()
def lap(msg):
    print("%7.1f ms  %s" % ((time.perf_counter() - t0) * 1e3, msg))
import k8s_gpu_device_plugin_amd.cli
lap("import cli")
from k8s_gpu_device_plugin_amd import native
n = native.load()
lap("native.load")
be = n.make_amdsmi_backend() if n.amdsmi_available(keep=True) else None
lap("amdsmi_available + make backend (%s)" % (be is not None))
if be is not None:
    gpus, topo = be.discover()
    lap("discover (%d gpus)" % len(gpus))
    be.sample(0)
    lap("first sample")
