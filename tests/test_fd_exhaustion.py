"""Out of file descriptors: both native servers shed the connections they cannot hold
instead of spinning.  A connection left in the listen backlog keeps the level-triggered
listener readable, so a worker that just retries accept4 on EMFILE returns from every
epoll_wait at once and burns a core for as long as the flood lasts (here: ~1 s of CPU
per second).  With a reserve descriptor the server accepts and closes the excess, stays
idle, and serves again as soon as descriptors free up."""
import json
import os
import socket
import subprocess
import sys
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import json, os, resource, sys
sys.path.insert(0, %(root)r)
from k8s_gpu_device_plugin_amd import native
n = native.load()
kind, sock_dir = sys.argv[1], sys.argv[2]
if kind == "http":
    cfg = n.HttpConfig()
    cfg.host, cfg.port, cfg.threads, cfg.access_log = "127.0.0.1", 0, 2, False
    srv = n.HttpServer(cfg, n.Exporter())
    addr = srv.start()
else:
    tc = n.TableConfig()
    table = n.DeviceTable(tc, [n.TableDevice("dev-0", 0, 0, 0, -1, ["/dev/dri/renderD128"], True)], n.Topology(1))
    addr = os.path.join(sock_dir, "amd-gpu.sock")
    srv = n.GrpcServer(addr, 2)
    srv.set_table(table)
    srv.start()
soft, hard = resource.getrlimit(resource.RLIMIT_NOFILE)
resource.setrlimit(resource.RLIMIT_NOFILE, (len(os.listdir("/proc/self/fd")) + 6, hard))
print(json.dumps({"addr": addr}), flush=True)
for line in sys.stdin:
    if line.strip() == "stats":
        t = os.times()
        print(json.dumps({"cpu": t.user + t.system, "shed": srv.shed_connections}), flush=True)
    else:
        break
srv.stop()
"""


def _connect(kind, addr):
    if kind == "http":
        s = socket.create_connection(("127.0.0.1", addr), timeout=2)
    else:
        s = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
        s.settimeout(2)
        s.connect(addr)
    return s


@pytest.mark.parametrize("kind", ["http", "grpc"])
def test_server_sheds_instead_of_spinning_when_out_of_fds(kind, tmp_path):
    p = subprocess.Popen([sys.executable, "-c", CHILD % {"root": ROOT}, kind, str(tmp_path)], stdin=subprocess.PIPE,
                         stdout=subprocess.PIPE, text=True)
    try:
        addr = json.loads(p.stdout.readline())["addr"]

        def stats():
            p.stdin.write("stats\n")
            p.stdin.flush()
            return json.loads(p.stdout.readline())

        held = [_connect(kind, addr) for _ in range(40)]  # far more than the server can hold
        time.sleep(0.3)
        before = stats()
        time.sleep(1.0)
        after = stats()
        assert after["cpu"] - before["cpu"] < 0.3, (before, after)  # idle, not spinning on accept
        assert after["shed"] > 0, after
        for s in held:
            s.close()
        time.sleep(0.3)
        # descriptors are back: a new client is served again
        c = _connect(kind, addr)
        if kind == "http":
            c.sendall(b"GET /health HTTP/1.1\r\nHost: x\r\n\r\n")
            assert c.recv(4096).startswith(b"HTTP/1.1 200 OK")
        else:
            data = c.recv(64)  # the server preface (SETTINGS) arrives unprompted
            assert len(data) >= 9 and data[3] == 4, data
        c.close()
    finally:
        try:
            p.stdin.write("quit\n")
            p.stdin.flush()
        except OSError:
            pass
        p.wait(10)
