"""Native HTTP/2 gRPC server protocol behaviour (flow control, errors, streams),
exercised with the native H2Client, raw sockets and grpcio."""
import os
import socket
import struct
import threading
import time

import grpc
import pytest

from k8s_gpu_device_plugin_amd import native
from k8s_gpu_device_plugin_amd.api import v1beta1

PREFACE = b"PRI * HTTP/2.0\r\n\r\nSM\r\n\r\n"


@pytest.fixture
def server(n, plugin_dir):
    tc = n.TableConfig()
    devs = [n.TableDevice("dev-%03d" % i, i // 8, i % 8, i // 32, -1, ["/dev/dri/renderD%d" % (128 + i)], True)
            for i in range(64)]
    table = n.DeviceTable(tc, devs, n.Topology(8))
    path = os.path.join(plugin_dir, "amd-gpu.sock")
    srv = n.GrpcServer(path, 2)
    srv.set_table(table)
    srv.start()
    yield srv, table, path
    srv.stop()


def test_unary_and_status_codes(n, server):
    srv, table, path = server
    c = n.H2Client(path)
    req = v1beta1.AllocateRequest(container_requests=[v1beta1.ContainerAllocateRequest(
        devices_ids=["dev-001"])]).SerializeToString()
    st, body, msg = c.unary(v1beta1.METHOD_ALLOCATE, req)
    assert st == 0 and v1beta1.AllocateResponse.FromString(body).container_responses[0].envs["AMD_VISIBLE_DEVICES"] \
        == "dev-001"
    st, _, msg = c.unary("/v1beta1.DevicePlugin/Bogus", b"")
    assert st == 12 and "unknown method" in msg
    st, _, msg = c.unary("/other.Service/Allocate", b"")
    assert st == 12
    st, _, msg = c.unary(v1beta1.METHOD_ALLOCATE, v1beta1.AllocateRequest(container_requests=[
        v1beta1.ContainerAllocateRequest(devices_ids=["zzz"])]).SerializeToString())
    assert st == 2 and "unknown device: zzz" in msg
    st, body, _ = c.unary(v1beta1.METHOD_GET_OPTIONS, b"")
    assert st == 0 and v1beta1.DevicePluginOptions.FromString(body).get_preferred_allocation_available
    st, body, _ = c.unary(v1beta1.METHOD_PRE_START, b"")
    assert st == 0 and body == b""
    assert srv.requests >= 6 and srv.connections == 1
    c.close()


def test_large_request_exercises_flow_control(n, server):
    """A GetPreferredAllocation with ~200 KB of ids spans many DATA frames and both windows."""
    srv, table, path = server
    ids = ["dev-%03d" % (i % 64) for i in range(12000)]
    req = v1beta1.PreferredAllocationRequest(container_requests=[v1beta1.ContainerPreferredAllocationRequest(
        available_deviceIDs=ids, allocation_size=4)]).SerializeToString()
    assert len(req) > 100_000
    c = n.H2Client(path)
    for _ in range(12):  # > 1 MiB total: needs connection-level WINDOW_UPDATEs from the server
        st, body, msg = c.unary(v1beta1.METHOD_GET_PREFERRED, req)
        assert st == 0, msg
        assert len(v1beta1.PreferredAllocationResponse.FromString(body).container_responses[0].deviceIDs) == 4
    c.close()


def test_large_response_respects_peer_window(n, plugin_dir):
    """64 KiB default client window: a ListAndWatch over 2000 devices (>64 KiB) must be
    split and continued only after WINDOW_UPDATE (grpcio client handles that)."""
    tc = n.TableConfig()
    devs = [n.TableDevice("a-very-long-device-identifier-%05d" % i, 0, -1, 0, -1, [], True) for i in range(2000)]
    table = n.DeviceTable(tc, devs, n.Topology(1))
    path = os.path.join(plugin_dir, "big.sock")
    srv = n.GrpcServer(path, 1)
    srv.set_table(table)
    srv.start()
    try:
        assert len(table.list_and_watch()) > 65535
        ch = grpc.insecure_channel("unix://" + path)
        law = ch.unary_stream(v1beta1.METHOD_LIST_AND_WATCH, request_serializer=v1beta1.Empty.SerializeToString,
                              response_deserializer=v1beta1.ListAndWatchResponse.FromString)
        it = law(v1beta1.Empty())
        first = next(it)
        assert len(first.devices) == 2000
        table.set_health(devs[5].id, False)
        srv.notify()
        second = next(it)
        assert second.devices[5].health == "Unhealthy"
        it.cancel()
        ch.close()
    finally:
        srv.stop()


def test_list_and_watch_push_without_notify(n, server):
    """Version polling pushes updates even if nobody calls notify()."""
    srv, table, path = server
    ch = grpc.insecure_channel("unix://" + path)
    law = ch.unary_stream(v1beta1.METHOD_LIST_AND_WATCH, request_serializer=v1beta1.Empty.SerializeToString,
                          response_deserializer=v1beta1.ListAndWatchResponse.FromString)
    it = law(v1beta1.Empty())
    assert len(next(it).devices) == 64
    t0 = time.monotonic()
    table.set_gpu_health(2, -1, False)
    upd = next(it)
    assert sum(d.health == "Unhealthy" for d in upd.devices) == 8 and time.monotonic() - t0 < 1.0
    it.cancel()
    ch.close()


def test_server_stop_ends_streams_cleanly(n, server):
    srv, table, path = server
    ch = grpc.insecure_channel("unix://" + path)
    law = ch.unary_stream(v1beta1.METHOD_LIST_AND_WATCH, request_serializer=v1beta1.Empty.SerializeToString,
                          response_deserializer=v1beta1.ListAndWatchResponse.FromString)
    it = law(v1beta1.Empty())
    next(it)
    srv.stop()
    with pytest.raises(StopIteration):
        next(it)  # OK trailers, like the reference's ListAndWatch returning nil on stop
    ch.close()
    assert not os.path.exists(path)
    srv.stop()  # idempotent


def _frame(ftype, flags, sid, payload=b""):
    return struct.pack(">I", len(payload))[1:] + bytes([ftype, flags]) + struct.pack(">I", sid) + payload


def _read_frames(s, until_type=None, timeout=2.0):
    s.settimeout(timeout)
    buf, frames = b"", []
    deadline = time.monotonic() + timeout
    while time.monotonic() < deadline:
        try:
            chunk = s.recv(65536)
        except socket.timeout:
            break
        if not chunk:
            break
        buf += chunk
        while len(buf) >= 9:
            ln = int.from_bytes(buf[:3], "big")
            if len(buf) < 9 + ln:
                break
            frames.append((buf[3], buf[4], int.from_bytes(buf[5:9], "big") & 0x7FFFFFFF, buf[9:9 + ln]))
            buf = buf[9 + ln:]
        if until_type is not None and any(f[0] == until_type for f in frames):
            break
    return frames


def test_raw_protocol_ping_settings_and_bad_preface(server):
    srv, table, path = server
    s = socket.socket(socket.AF_UNIX)
    s.connect(path)
    s.sendall(PREFACE + _frame(4, 0, 0) + _frame(6, 0, 0, b"12345678"))
    frames = _read_frames(s, until_type=6)
    types = [(f[0], f[1]) for f in frames]
    assert (4, 0) in types and (4, 1) in types  # server SETTINGS + ACK of ours
    assert any(f[0] == 6 and f[1] == 1 and f[3] == b"12345678" for f in frames)  # PING ACK echoes payload
    s.close()
    s = socket.socket(socket.AF_UNIX)
    s.connect(path)
    s.sendall(b"GET / HTTP/1.1\r\nHost: x\r\n\r\n")
    frames = _read_frames(s, until_type=7)
    assert any(f[0] == 7 and struct.unpack(">I", f[3][4:8])[0] == 1 for f in frames)  # GOAWAY PROTOCOL_ERROR
    s.close()


def test_oversized_frame_is_rejected(server):
    srv, table, path = server
    s = socket.socket(socket.AF_UNIX)
    s.connect(path)
    s.sendall(PREFACE + b"\x00\x80\x00" + bytes([0, 0]) + b"\x00\x00\x00\x01" + b"x" * 100)
    frames = _read_frames(s, until_type=7)
    assert any(f[0] == 7 and struct.unpack(">I", f[3][4:8])[0] == 6 for f in frames)  # FRAME_SIZE_ERROR
    s.close()


def test_stop_right_after_start(n, plugin_dir):
    """stop() held the server lock while joining the workers, and a worker that had not
    run yet took that lock first thing: stop() right after start() deadlocked (seen as a
    rare hang of a fixture teardown on a loaded machine)."""
    tc = n.TableConfig()
    table = n.DeviceTable(tc, [n.TableDevice("dev-000", 0)], n.Topology(1))
    path = os.path.join(plugin_dir, "amd-gpu.sock")
    for _ in range(100):
        srv = n.GrpcServer(path, 8)
        srv.set_table(table)
        srv.start()
        srv.stop()
        assert not srv.running


def test_many_connections_and_threads(n, server):
    srv, table, path = server
    req = v1beta1.AllocateRequest(container_requests=[v1beta1.ContainerAllocateRequest(
        devices_ids=["dev-010"])]).SerializeToString()
    errs = []

    def run():
        try:
            lat = native.load_bench().h2_bench_unary(path, v1beta1.METHOD_ALLOCATE, req, 500)
            assert len(lat) == 500
        except Exception as e:  # pragma: no cover
            errs.append(e)
    ts = [threading.Thread(target=run) for _ in range(8)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errs and srv.requests >= 4000


def test_first_stream_message_helper(n, server):
    srv, table, path = server
    c = n.H2Client(path)
    body = c.first_stream_message(v1beta1.METHOD_LIST_AND_WATCH, b"")
    assert len(v1beta1.ListAndWatchResponse.FromString(body).devices) == 64
    st, _, _ = c.unary(v1beta1.METHOD_GET_OPTIONS, b"")  # connection still usable after RST_STREAM
    assert st == 0


def _grpc_call_frames(sid, path, msg, end_stream=True):
    hb = bytes([0x83, 0x86]) + bytes([0x44, len(path)]) + path.encode() + bytes([0x5f, 16]) + b"application/grpc"
    body = b"\x00" + struct.pack(">I", len(msg)) + msg
    return _frame(1, 0x4, sid, hb) + _frame(0, 0x1 if end_stream else 0, sid, body)


def _goaway_code(frames):
    codes = [struct.unpack(">I", f[3][4:8])[0] for f in frames if f[0] == 7]
    return codes[0] if codes else None


def test_data_after_end_stream_is_stream_closed(server):
    """Found by fuzz_grpc: a second END_STREAM on a dispatched stream used to dispatch the
    request again (duplicate response HEADERS).  It is now RST_STREAM(STREAM_CLOSED)."""
    srv, table, path = server
    s = socket.socket(socket.AF_UNIX)
    s.connect(path)
    law = _grpc_call_frames(1, v1beta1.METHOD_LIST_AND_WATCH, b"")
    s.sendall(PREFACE + _frame(4, 0, 0) + law + _frame(0, 0x1, 1, b"\x00\x00\x00\x00\x00"))
    frames = _read_frames(s, until_type=3)
    assert [f for f in frames if f[0] == 3 and f[2] == 1 and struct.unpack(">I", f[3])[0] == 5]
    assert sum(1 for f in frames if f[0] == 1 and f[2] == 1) == 1  # response HEADERS sent once
    s.close()


@pytest.mark.parametrize("bad,code", [
    (_frame(8, 0, 0, struct.pack(">I", 0x7FFFFFFF)), 3),  # connection window overflow -> FLOW_CONTROL
    (_frame(8, 0, 0, struct.pack(">I", 0)), 1),           # zero increment -> PROTOCOL_ERROR
    (_frame(1, 0x5, 0, b"\x83"), 1),                      # HEADERS on stream 0
    (_frame(0, 0x1, 0, b"x"), 1),                         # DATA on stream 0
])
def test_connection_errors(server, bad, code):
    srv, table, path = server
    s = socket.socket(socket.AF_UNIX)
    s.connect(path)
    s.sendall(PREFACE + _frame(4, 0, 0) + bad)
    assert _goaway_code(_read_frames(s, until_type=7)) == code
    s.close()


def test_preferred_size_contract(n, server):
    """Found by fuzz_pbwire: allocation_size below |must_include| returned a larger set.
    Now: size <= 0 -> empty answer, size < |must| -> error; must ids are de-duplicated."""
    srv, table, path = server
    c = n.H2Client(path)

    def pref(avail, must, size):
        return c.unary(v1beta1.METHOD_GET_PREFERRED, v1beta1.PreferredAllocationRequest(container_requests=[
            v1beta1.ContainerPreferredAllocationRequest(available_deviceIDs=avail, must_include_deviceIDs=must,
                                                        allocation_size=size)]).SerializeToString())
    st, body, _ = pref(["dev-000", "dev-001"], [], 0)
    assert st == 0 and list(v1beta1.PreferredAllocationResponse.FromString(body).container_responses[0].deviceIDs) \
        == []
    st, _, msg = pref(["dev-000", "dev-001", "dev-002"], ["dev-000", "dev-001"], 1)
    assert st == 2 and "smaller than must_include" in msg
    st, body, _ = pref(["dev-000", "dev-001", "dev-009"], ["dev-001", "dev-001"], 2)
    ids = list(v1beta1.PreferredAllocationResponse.FromString(body).container_responses[0].deviceIDs)
    assert st == 0 and len(ids) == 2 and len(set(ids)) == 2 and "dev-001" in ids
    c.close()


def test_native_watch_client_follows_list_and_watch(n, server):
    """The compiled client can hold a ListAndWatch stream like kubelet does; a table
    change reaches it through the table -> server listener (no notify() call)."""
    srv, table, path = server
    c = n.H2Client(path)
    c.open_stream(v1beta1.METHOD_LIST_AND_WATCH, b"")
    first = v1beta1.ListAndWatchResponse.FromString(c.next_stream_message(5.0))
    assert len(first.devices) == 64 and all(d.health == "Healthy" for d in first.devices)
    for k in range(40):  # more than one receive window of pushes overall
        table.set_gpu_health((k // 2) % 8, -1, k % 2 == 1)
        upd = v1beta1.ListAndWatchResponse.FromString(c.next_stream_message(5.0))
        assert sum(d.health == "Unhealthy" for d in upd.devices) == (0 if k % 2 else 8)
    srv.stop()
    assert c.next_stream_message(5.0) is None  # OK trailers end the stream
    c.close()


def test_busy_poll_window_answers_and_idles_without_spinning(n, plugin_dir):
    """grpc.busyPollUs: after a request the worker polls instead of sleeping, so calls in
    a burst skip the wake-up; an idle server must not burn CPU (the window closes)."""
    tc = n.TableConfig()
    devs = [n.TableDevice("dev-%d" % i, i, 0, 0, -1, ["/dev/dri/renderD%d" % (128 + i)], True) for i in range(4)]
    table = n.DeviceTable(tc, devs, n.Topology(4))
    path = os.path.join(plugin_dir, "amd-gpu.sock")
    srv = n.GrpcServer(path, 2, busy_poll_us=20000)
    srv.set_table(table)
    srv.start()
    try:
        c = n.H2Client(path)
        req = v1beta1.AllocateRequest(container_requests=[v1beta1.ContainerAllocateRequest(
            devices_ids=["dev-2"])]).SerializeToString()
        for _ in range(200):
            st, body, _ = c.unary(v1beta1.METHOD_ALLOCATE, req)
            assert st == 0
        assert v1beta1.AllocateResponse.FromString(body).container_responses[0].envs["AMD_VISIBLE_DEVICES"] == "dev-2"
        time.sleep(0.1)  # the 20 ms window has closed
        cpu0, wall0 = time.process_time(), time.perf_counter()
        time.sleep(0.5)
        cpu = time.process_time() - cpu0
        assert cpu < 0.1 * (time.perf_counter() - wall0), "idle server used %.3f s of CPU" % cpu
        # a request re-opens the window; the next call is still answered normally
        st, _, _ = c.unary(v1beta1.METHOD_ALLOCATE, req)
        assert st == 0
        c.close()
    finally:
        srv.stop()


@pytest.mark.parametrize("full", [True, False])
def test_keep_warm_ticks_are_invisible_to_kubelet_and_metrics(n, plugin_dir, full):
    """grpc.keepWarmMs: a worker that owns a connection and has been idle that long
    replays a canned header decode + Allocate/GetPreferredAllocation against its table,
    so the first call after a long gap finds warm caches (profiles/r4/idle_probe_*).  The
    tick is not an RPC: no request, histogram observation or answer leaves the server,
    and a worker without connections does not tick."""
    tc = n.TableConfig()
    devs = [n.TableDevice("dev-%d" % i, i, 0, 0, -1, ["/dev/dri/renderD%d" % (128 + i)], True) for i in range(4)]
    table = n.DeviceTable(tc, devs, n.Topology(4))
    path = os.path.join(plugin_dir, "amd-gpu.sock")
    # the production polling windows: a tick must open neither (a GetPreferredAllocation
    # on the internal connection is not an admission)
    srv = n.GrpcServer(path, 2, busy_poll_us=50, admission_poll_us=1000)
    srv.set_keep_warm_ms(10)
    srv.set_keep_warm_full(full)  # full: canned requests through an in-memory connection
    srv.set_table(table)
    srv.start()
    try:
        time.sleep(0.2)
        assert srv.warm_ticks == 0, "ticked with no connection"
        c = n.H2Client(path)
        req = v1beta1.AllocateRequest(container_requests=[v1beta1.ContainerAllocateRequest(
            devices_ids=["dev-1"])]).SerializeToString()
        st, _, _ = c.unary(v1beta1.METHOD_ALLOCATE, req)
        assert st == 0
        requests = srv.requests
        time.sleep(0.3)
        assert srv.warm_ticks >= 5
        assert srv.requests == requests
        text = table.render_metrics()
        assert 'rpc="Allocate"' in text and 'rpc="GetPreferredAllocation"' not in text
        count = [ln for ln in text.splitlines()
                 if ln.startswith("amdgpu_device_plugin_rpc_duration_seconds_count") and 'rpc="Allocate"' in ln]
        assert count and count[0].endswith(" 1"), count
        st, body, _ = c.unary(v1beta1.METHOD_ALLOCATE, req)  # the next real call is answered as usual
        assert st == 0 and v1beta1.AllocateResponse.FromString(body).container_responses[0].envs[
            "AMD_VISIBLE_DEVICES"] == "dev-1"
        # thousands of ticks: the private connection's stream ids, flow-control window and
        # HPACK table keep working, and an idle server with a 1 ms tick stays cheap
        srv.set_keep_warm_ms(1)
        ticks = srv.warm_ticks
        cpu0, wall0 = time.process_time(), time.perf_counter()
        time.sleep(1.5)
        cpu = time.process_time() - cpu0
        assert srv.warm_ticks - ticks > 300, srv.warm_ticks - ticks
        assert srv.admission_windows == 0
        assert cpu < 0.25 * (time.perf_counter() - wall0), "1 ms ticks used %.3f s of CPU" % cpu
        assert srv.requests == requests + 1
        assert 'rpc="GetPreferredAllocation"' not in table.render_metrics()
        st, body, _ = c.unary(v1beta1.METHOD_ALLOCATE, req)
        assert st == 0
        srv.set_keep_warm_ms(10)
        c.close()
        srv.set_keep_warm_ms(0)
        ticks = srv.warm_ticks
        c = n.H2Client(path)
        time.sleep(0.2)
        assert srv.warm_ticks == ticks, "ticked with keep-warm off"
        c.close()
    finally:
        srv.stop()


def test_call_trace_records_every_call_in_per_worker_slices(n, plugin_dir, tmp_path):
    """grpc.callTraceFile: one record per unary call (ListAndWatch and keep-warm ticks are
    not traced), each worker in its own slice of the ring (no shared counter), the ring
    pre-written, and t_ready <= t_dispatch <= t_sent."""
    import numpy as np
    import bench
    tc = n.TableConfig()
    devs = [n.TableDevice("dev-%d" % i, i, 0, 0, -1, ["/dev/dri/renderD%d" % (128 + i)], True) for i in range(2)]
    table = n.DeviceTable(tc, devs, n.Topology(2))
    path = os.path.join(plugin_dir, "amd-gpu.sock")
    trace = str(tmp_path / "trace.bin")
    srv = n.GrpcServer(path, 2, busy_poll_us=0, admission_poll_us=0)
    srv.set_call_trace(trace, 64)
    srv.set_keep_warm_ms(1)
    srv.set_table(table)
    srv.start()
    try:
        req = v1beta1.AllocateRequest(container_requests=[v1beta1.ContainerAllocateRequest(
            devices_ids=["dev-1"])]).SerializeToString()
        clients = [n.H2Client(path) for _ in range(2)]  # one connection per worker
        for c in clients:
            for _ in range(10):
                assert c.unary(v1beta1.METHOD_ALLOCATE, req)[0] == 0
        time.sleep(0.05)  # keep-warm ticks: never traced
        recs = bench.read_call_trace(trace)
        assert len(recs) == 20
        assert (recs["method"] == n.RPC_ALLOCATE).all()
        assert ((recs["t_ready"] <= recs["t_dispatch"]) & (recs["t_dispatch"] <= recs["t_sent"])).all()
        workers = recs["conn"] >> np.uint64(48)
        assert sorted(set(workers.tolist())) == [0, 1]
        raw = np.fromfile(trace, dtype=np.dtype(bench.TRACE_DTYPE), count=64, offset=64)
        for wi in (0, 1):  # worker i writes records [32 i, 32 i + 10)
            mine = raw[32 * wi:32 * (wi + 1)]
            assert list(mine["seq"][:10]) == list(range(1, 11)) and (mine["seq"][10:] == 0).all()
        for c in clients:
            c.close()
    finally:
        srv.stop()


def _switches(tids):
    """voluntary context switches of each thread in `tids` (a sleeping worker's wake-ups)."""
    out = {}
    for tid in tids:
        try:
            with open("/proc/self/task/%s/status" % tid) as f:
                for ln in f:
                    if ln.startswith("voluntary_ctxt_switches:"):
                        out[tid] = int(ln.split()[1])
        except OSError:
            pass
    return out


def _grpc_workers(exclude):
    tids = []
    for tid in set(os.listdir("/proc/self/task")) - exclude:
        try:
            with open("/proc/self/task/%s/comm" % tid) as f:
                if f.read().startswith("dpgrpc"):
                    tids.append(tid)
        except OSError:
            pass
    return tids


def test_idle_wake_wakes_only_the_worker_holding_a_connection(n, plugin_dir):
    """grpc.idleWakeMs: the worker that holds kubelet's connection wakes every idle
    millisecond (its core stays out of deep idle states) without running the request path
    (no keep-warm tick, no request); workers without a connection keep their 100 ms sleep."""
    tc = n.TableConfig()
    devs = [n.TableDevice("dev-%d" % i, i, 0, 0, -1, ["/dev/dri/renderD%d" % (128 + i)], True) for i in range(2)]
    table = n.DeviceTable(tc, devs, n.Topology(2))
    path = os.path.join(plugin_dir, "amd-gpu.sock")
    before = set(os.listdir("/proc/self/task"))
    srv = n.GrpcServer(path, 2, busy_poll_us=0, admission_poll_us=0)
    srv.set_keep_warm_ms(0)
    srv.set_idle_wake_ms(1)
    srv.set_table(table)
    srv.start()
    try:
        deadline = time.monotonic() + 5
        while len(_grpc_workers(before)) < 2 and time.monotonic() < deadline:
            time.sleep(0.01)
        workers = _grpc_workers(before)
        assert len(workers) == 2
        s0 = _switches(workers)
        time.sleep(0.3)
        s1 = _switches(workers)
        assert max(s1[t] - s0[t] for t in workers) <= 12, "woke without a connection: %s %s" % (s0, s1)
        c = n.H2Client(path)
        req = v1beta1.AllocateRequest(container_requests=[v1beta1.ContainerAllocateRequest(
            devices_ids=["dev-1"])]).SerializeToString()
        assert c.unary(v1beta1.METHOD_ALLOCATE, req)[0] == 0
        requests = srv.requests
        time.sleep(0.05)
        s0 = _switches(workers)
        time.sleep(0.4)
        s1 = _switches(workers)
        d = sorted(s1[t] - s0[t] for t in workers)
        assert d[-1] >= 100 and d[0] <= 12, d  # the holder ~400 wake-ups, the other ~4
        assert srv.warm_ticks == 0 and srv.requests == requests
        srv.set_idle_wake_ms(0)
        time.sleep(0.15)
        s0 = _switches(workers)
        time.sleep(0.3)
        s1 = _switches(workers)
        assert max(s1[t] - s0[t] for t in workers) <= 12
        assert c.unary(v1beta1.METHOD_ALLOCATE, req)[0] == 0
        c.close()
    finally:
        srv.stop()


def test_connections_spread_over_workers(n, plugin_dir):
    """Concurrent kubelet-side clients (bench ranks, kubelet + a debugging client) are
    owned by different worker threads, not queued behind one that accepted them all."""
    tc = n.TableConfig()
    devs = [n.TableDevice("dev-%d" % i, i, 0, 0, -1, ["/dev/dri/renderD%d" % (128 + i)], True) for i in range(4)]
    table = n.DeviceTable(tc, devs, n.Topology(4))
    path = os.path.join(plugin_dir, "amd-gpu.sock")
    srv = n.GrpcServer(path, 4, busy_poll_us=50)
    srv.set_table(table)
    srv.start()
    try:
        req = v1beta1.AllocateRequest(container_requests=[v1beta1.ContainerAllocateRequest(
            devices_ids=["dev-1"])]).SerializeToString()
        clients = [n.H2Client(path) for _ in range(4)]
        for c in clients:  # every handed-over connection is adopted and answers
            assert c.unary(v1beta1.METHOD_ALLOCATE, req)[0] == 0
        assert sorted(srv.worker_connections) == [1, 1, 1, 1]
        errors = []

        def hammer(c):
            try:
                for _ in range(300):
                    assert c.unary(v1beta1.METHOD_ALLOCATE, req)[0] == 0
            except Exception as e:  # pragma: no cover - reported below
                errors.append(e)
        ts = [threading.Thread(target=hammer, args=(c,)) for c in clients]
        for t in ts:
            t.start()
        for t in ts:
            t.join(60)
        assert not errors and srv.requests >= 1204
        for c in clients:
            c.close()
        deadline = time.time() + 5
        while sum(srv.worker_connections) and time.time() < deadline:
            time.sleep(0.02)
        assert srv.worker_connections == [0, 0, 0, 0] and srv.connections == 0
    finally:
        srv.stop()


def test_admission_window_polls_after_preferred_only(n, plugin_dir):
    """grpc.admissionPollUs: a GetPreferredAllocation keeps its worker polling (the same
    container's Allocate comes next); any other RPC leaves it asleep when busyPollUs is 0."""
    tc = n.TableConfig()
    devs = [n.TableDevice("dev-%d" % i, i, 0, 0, -1, ["/dev/dri/renderD%d" % (128 + i)], True) for i in range(4)]
    table = n.DeviceTable(tc, devs, n.Topology(4))
    path = os.path.join(plugin_dir, "amd-gpu.sock")
    srv = n.GrpcServer(path, 1, busy_poll_us=0, admission_poll_us=100000)
    srv.set_table(table)
    srv.start()
    try:
        c = n.H2Client(path)
        alloc = v1beta1.AllocateRequest(container_requests=[v1beta1.ContainerAllocateRequest(
            devices_ids=["dev-2"])]).SerializeToString()
        pref = v1beta1.PreferredAllocationRequest(container_requests=[v1beta1.ContainerPreferredAllocationRequest(
            available_deviceIDs=["dev-0", "dev-1", "dev-2", "dev-3"], allocation_size=2)]).SerializeToString()

        def cpu_after(method, req):
            assert c.unary(method, req)[0] == 0
            cpu0 = time.process_time()
            time.sleep(0.06)
            return time.process_time() - cpu0
        assert cpu_after(v1beta1.METHOD_ALLOCATE, alloc) < 0.02  # asleep
        assert srv.admission_windows == 0
        yielded = srv.poll_windows_yielded
        cpu = cpu_after(v1beta1.METHOD_GET_PREFERRED, pref)
        assert srv.admission_windows == 1
        # polling for the Allocate, unless another thread wanted the worker's CPU (on a
        # host where everything shares one CPU the window gives way at once)
        assert cpu > 0.03 or srv.poll_windows_yielded > yielded, (cpu, srv.poll_windows_yielded)
        time.sleep(0.1)  # the 100 ms window closes
        cpu0 = time.process_time()
        time.sleep(0.1)
        assert time.process_time() - cpu0 < 0.02
        c.close()
    finally:
        srv.stop()


def test_polling_window_gives_way_to_a_client_on_its_cpu(n, plugin_dir):
    """Found on a shared host: kubelet's thread is woken next to the worker that answered
    its GetPreferredAllocation and is busy on that CPU before it sends the Allocate; a
    worker polling through its admission window kept that CPU, so the Allocate waited for
    the window's end (~0.8 ms of a 1 ms window).  With client and server on one CPU the
    Allocate must now come back long before a 20 ms window would have ended."""
    cpus = os.sched_getaffinity(0)
    one = {min(cpus)}
    tc = n.TableConfig()
    devs = [n.TableDevice("dev-%d" % i, i, 0, 0, -1, ["/dev/dri/renderD%d" % (128 + i)], True) for i in range(4)]
    table = n.DeviceTable(tc, devs, n.Topology(4))
    path = os.path.join(plugin_dir, "amd-gpu.sock")
    os.sched_setaffinity(0, one)  # this thread, and the worker threads it starts
    try:
        srv = n.GrpcServer(path, 1, busy_poll_us=50, admission_poll_us=20000)
        srv.set_table(table)
        srv.start()
        try:
            native.load_bench()  # H2Client.bench_unary
            c = n.H2Client(path)
            alloc = v1beta1.AllocateRequest(container_requests=[v1beta1.ContainerAllocateRequest(
                devices_ids=["dev-2"])]).SerializeToString()
            pref = v1beta1.PreferredAllocationRequest(container_requests=[v1beta1.ContainerPreferredAllocationRequest(
                available_deviceIDs=["dev-0", "dev-1", "dev-2", "dev-3"], allocation_size=2)]).SerializeToString()
            lat = []
            for _ in range(10):
                time.sleep(0.03)  # the previous window has ended
                assert c.bench_unary(v1beta1.METHOD_GET_PREFERRED, pref, 1)
                t_go = time.perf_counter() + 300e-6  # kubelet's own work between the two calls
                while time.perf_counter() < t_go:
                    pass
                lat.extend(c.bench_unary(v1beta1.METHOD_ALLOCATE, alloc, 1))
            c.close()
            assert sorted(lat)[len(lat) // 2] < 2e-3, lat  # not the 20 ms window, nor a scheduler slice
            assert srv.admission_windows == 10  # the windows were opened, and gave way
        finally:
            srv.stop()
    finally:
        os.sched_setaffinity(0, cpus)


def test_connection_churn_across_workers(n, plugin_dir):
    """1600 short kubelet-side connections from 8 threads (connect, one Allocate, close):
    every call answers, and afterwards no worker still counts a connection."""
    tc = n.TableConfig()
    devs = [n.TableDevice("dev-%d" % i, i, 0, 0, -1, ["/dev/dri/renderD%d" % (128 + i)], True) for i in range(4)]
    table = n.DeviceTable(tc, devs, n.Topology(4))
    path = os.path.join(plugin_dir, "amd-gpu.sock")
    srv = n.GrpcServer(path, 4, busy_poll_us=50)
    srv.set_table(table)
    srv.start()
    try:
        req = v1beta1.AllocateRequest(container_requests=[v1beta1.ContainerAllocateRequest(
            devices_ids=["dev-3"])]).SerializeToString()
        errors = []

        def churn():
            for _ in range(200):
                try:
                    c = n.H2Client(path)
                    if c.unary(v1beta1.METHOD_ALLOCATE, req)[0] != 0:
                        errors.append("status")
                    c.close()
                except Exception as e:  # pragma: no cover - reported below
                    errors.append(repr(e))
        ts = [threading.Thread(target=churn) for _ in range(8)]
        for t in ts:
            t.start()
        for t in ts:
            t.join(120)
        assert not errors, errors[:3]
        deadline = time.time() + 5
        while (srv.connections or sum(srv.worker_connections)) and time.time() < deadline:
            time.sleep(0.02)
        assert srv.connections == 0 and srv.worker_connections == [0, 0, 0, 0]
        assert srv.requests >= 1600
    finally:
        srv.stop()


def test_hostile_clients_do_not_disturb_allocate(n, server):
    """While a kubelet-like client runs Allocates, other local clients misbehave on the
    same socket: random bytes, a valid call cut off mid-frame, a preface and then silence,
    a flood of PINGs that is never read, streams opened and reset, and connections closed
    at every point.  Every Allocate must succeed, and the server must report no fault."""
    import random
    srv, table, path = server
    req = v1beta1.AllocateRequest(container_requests=[v1beta1.ContainerAllocateRequest(
        devices_ids=["dev-007"])]).SerializeToString()
    stop = threading.Event()
    errs = []
    done = [0]
    idle = []

    def good():
        c = n.H2Client(path)
        try:
            while not stop.is_set():
                st, body, msg = c.unary(v1beta1.METHOD_ALLOCATE, req)
                if st != 0:
                    errs.append(msg)
                done[0] += 1
        except Exception as e:  # pragma: no cover - reported below
            errs.append(repr(e))
        finally:
            c.close()

    call = _grpc_call_frames(1, v1beta1.METHOD_ALLOCATE, req)

    def hostile(seed):
        rng = random.Random(seed)
        while not stop.is_set():
            s = socket.socket(socket.AF_UNIX)
            try:
                s.settimeout(0.5)
                s.connect(path)
                kind = rng.randrange(6)
                if kind == 0:
                    s.sendall(bytes(rng.randrange(256) for _ in range(rng.randrange(1, 200))))
                elif kind == 1:
                    blob = PREFACE + _frame(4, 0, 0) + call
                    s.sendall(blob[:rng.randrange(1, len(blob))])
                elif kind == 2:
                    s.sendall(PREFACE)
                    idle.append(s)  # holds the connection open, says nothing more
                    s = None
                    if len(idle) > 16:
                        idle.pop(0).close()
                elif kind == 3:
                    s.sendall(PREFACE + _frame(4, 0, 0) + b"".join(_frame(6, 0, 0, b"%08d" % i) for i in range(400)))
                elif kind == 4:
                    sid = 1 + 2 * rng.randrange(100)
                    s.sendall(PREFACE + _frame(4, 0, 0) + _grpc_call_frames(sid, v1beta1.METHOD_ALLOCATE, req, False)
                              + _frame(3, 0, sid, struct.pack(">I", 8)))  # RST_STREAM(CANCEL)
                else:
                    s.sendall(PREFACE + _frame(4, 0, 0) + call)
                    s.recv(rng.choice([1, 9, 4096]))
            except OSError:
                pass
            finally:
                if s is not None:
                    s.close()

    ts = [threading.Thread(target=good)] + [threading.Thread(target=hostile, args=(i,)) for i in range(4)]
    for t in ts:
        t.start()
    time.sleep(3.0)
    stop.set()
    for t in ts:
        t.join(10)
    for s in idle:
        s.close()
    assert not errs, errs[:3]
    assert done[0] > 100
    assert srv.failure() == "" and srv.running
    c = n.H2Client(path)
    assert c.unary(v1beta1.METHOD_ALLOCATE, req)[0] == 0
    c.close()


def test_idle_wake_and_keep_warm_run_only_in_the_admission_window(n, plugin_dir):
    """grpc.activeWindowMs.  Right after a kubelet RPC the worker that
    holds the connection wakes every idle millisecond and runs keep-warm ticks; once the
    window has passed without an RPC every worker sleeps (about one wake-up a second, no
    tick), and the next RPC opens the window again."""
    tc = n.TableConfig()
    devs = [n.TableDevice("dev-%d" % i, i, 0, 0, -1, ["/dev/dri/renderD%d" % (128 + i)], True) for i in range(2)]
    table = n.DeviceTable(tc, devs, n.Topology(2))
    path = os.path.join(plugin_dir, "amd-gpu.sock")
    before = set(os.listdir("/proc/self/task"))
    srv = n.GrpcServer(path, 2, busy_poll_us=0, admission_poll_us=0)
    srv.set_keep_warm_ms(10)
    srv.set_idle_wake_ms(1)
    srv.set_active_window_ms(400)
    srv.set_table(table)
    srv.start()
    try:
        deadline = time.monotonic() + 5
        while len(_grpc_workers(before)) < 2 and time.monotonic() < deadline:
            time.sleep(0.01)
        workers = _grpc_workers(before)
        c = n.H2Client(path)
        req = v1beta1.AllocateRequest(container_requests=[v1beta1.ContainerAllocateRequest(
            devices_ids=["dev-1"])]).SerializeToString()
        assert c.unary(v1beta1.METHOD_ALLOCATE, req)[0] == 0
        s0, t0 = _switches(workers), srv.warm_ticks
        time.sleep(0.25)  # inside the window
        s1, t1 = _switches(workers), srv.warm_ticks
        assert max(s1[t] - s0[t] for t in workers) >= 60 and t1 > t0, (s0, s1)
        time.sleep(0.4)  # the window closes
        s0, t0, i0 = _switches(workers), srv.warm_ticks, srv.idle_wakeups
        time.sleep(1.0)
        s1, t1, i1 = _switches(workers), srv.warm_ticks, srv.idle_wakeups
        assert max(s1[t] - s0[t] for t in workers) <= 4, (s0, s1)  # ~1 per worker per second
        assert t1 == t0 and i1 - i0 <= 6
        assert c.unary(v1beta1.METHOD_ALLOCATE, req)[0] == 0  # a sleeping worker answers
        s0 = _switches(workers)
        time.sleep(0.2)
        s1 = _switches(workers)
        assert max(s1[t] - s0[t] for t in workers) >= 50  # the window is open again
        c.close()
    finally:
        srv.stop()


def test_idle_daemon_threads_sleep(n, plugin_dir, make_cfg):
    """An idle daemon's own threads (HTTP workers, sampler, watchdog, event thread,
    directory watch, health pump) wake about once a second at most, and still stop at once."""
    from k8s_gpu_device_plugin_amd.models import fixtures
    from k8s_gpu_device_plugin_amd.plugin.manager import PluginManager
    from k8s_gpu_device_plugin_amd.server.web import WebServer
    model = fixtures.mi355x_node(2)
    model["hardware_events"] = False
    before = set(os.listdir("/proc/self/task"))
    cfg = make_cfg(webListenAddress="127.0.0.1:0", http={"accessLog": True}, telemetry={"intervalMs": 1000})
    m = PluginManager(cfg, backend=fixtures.build_backend(model))
    t = m.start_background()
    w = WebServer(cfg, m)
    w.start()
    try:
        time.sleep(1.5)
        mine = [x for x in os.listdir("/proc/self/task") if x not in before]

        def switches():
            out = {}
            for tid in mine:
                try:
                    with open("/proc/self/task/%s/comm" % tid) as f:
                        name = f.read().strip()
                    with open("/proc/self/task/%s/status" % tid) as f:
                        st = f.read()
                except OSError:
                    continue
                out[tid] = (name, sum(int(ln.split()[1]) for ln in st.splitlines()
                                      if ln.startswith(("voluntary_ctxt", "nonvoluntary_ctxt"))))
            return out
        a = switches()
        time.sleep(2.0)
        b = switches()
        rates = {a[k][0] + "/" + k: (b[k][1] - a[k][1]) / 2.0 for k in a if k in b}
        native_threads = {k: v for k, v in rates.items() if k.startswith(("dphttp", "dpsampler", "dpwatchdog",
                                                                          "dpaccesslog", "dpgrpc"))}
        # (round 5: the watchdog woke 40 times a second, the sampler 20, the HTTP workers 5)
        assert native_threads and max(native_threads.values()) <= 8.0, rates
        t0 = time.monotonic()
    finally:
        w.stop()
        m.stop()
        t.join(10)
    assert time.monotonic() - t0 < 3.0


def test_peek_reads_serve_every_request_once(n, plugin_dir):
    """grpc.peekReads (opt-in): requests read with MSG_PEEK and consumed after the answer -
    back-to-back unary calls, a request spanning many frames and reads, and a stream all
    see exactly one answer per request and nothing replayed."""
    tc = n.TableConfig()
    devs = [n.TableDevice("dev-%03d" % i, i // 8, i % 8, 0, -1, ["/dev/dri/renderD%d" % (128 + i)], True)
            for i in range(64)]
    table = n.DeviceTable(tc, devs, n.Topology(8))
    path = os.path.join(plugin_dir, "amd-gpu.sock")
    srv = n.GrpcServer(path, 2)
    srv.set_peek_reads(True)
    srv.set_table(table)
    srv.start()
    try:
        c = n.H2Client(path)
        for i in range(300):
            req = v1beta1.AllocateRequest(container_requests=[v1beta1.ContainerAllocateRequest(
                devices_ids=["dev-%03d" % (i % 64)])]).SerializeToString()
            st, body, msg = c.unary(v1beta1.METHOD_ALLOCATE, req)
            assert st == 0, msg
            envs = v1beta1.AllocateResponse.FromString(body).container_responses[0].envs
            assert envs["AMD_VISIBLE_DEVICES"] == "dev-%03d" % (i % 64)
        ids = ["dev-%03d" % (i % 64) for i in range(12000)]  # ~200 KB: many frames, several reads
        big = v1beta1.PreferredAllocationRequest(container_requests=[v1beta1.ContainerPreferredAllocationRequest(
            available_deviceIDs=ids, allocation_size=4)]).SerializeToString()
        for _ in range(4):
            st, body, msg = c.unary(v1beta1.METHOD_GET_PREFERRED, big)
            assert st == 0, msg
        assert srv.requests == 304
        c.open_stream(v1beta1.METHOD_LIST_AND_WATCH, b"")
        first = c.next_stream_message(5.0)
        assert len(v1beta1.ListAndWatchResponse.FromString(first).devices) == 64
        table.set_gpu_health(1, -1, False)
        srv.notify()
        upd = v1beta1.ListAndWatchResponse.FromString(c.next_stream_message(5.0))
        assert sum(d.health == "Unhealthy" for d in upd.devices) == 8
        c.close()
    finally:
        srv.stop()


def _fake_h2_server(path, frames_after_request):
    """One-connection HTTP/2 server: reads the client's preface, SETTINGS and request,
    then writes ``frames_after_request`` (raw frames) and closes."""
    lsock = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
    lsock.bind(path)
    lsock.listen(1)

    def run():
        conn, _ = lsock.accept()
        got = b""
        conn.settimeout(5)
        while b"\x00\x00\x05\x00\x01\x00\x00\x00\x01" not in got:  # the request's END_STREAM DATA
            chunk = conn.recv(65536)
            if not chunk:
                break
            got += chunk
        conn.sendall(frames_after_request)
        time.sleep(0.2)
        conn.close()
        lsock.close()
    t = threading.Thread(target=run, daemon=True)
    t.start()
    return t


def _frame(ftype, flags, sid, payload=b""):
    return struct.pack(">I", len(payload))[1:] + bytes([ftype, flags]) + struct.pack(">I", sid) + payload


def _lit(name, value):  # HPACK literal without indexing, new name
    return b"\x00" + bytes([len(name)]) + name + bytes([len(value)]) + value


@pytest.mark.parametrize("last_sid", [0x7FFFFFFF, 0])
def test_client_honours_goaway_last_stream_id(n, tmp_path, last_sid):
    """A GOAWAY that still covers the request (a gRPC server shutting down gracefully
    sends last = 2^31-1 and then answers what it took) does not fail the call; one below
    the request's stream says it was not processed, so the caller may send it again
    (plugin.register does, once)."""
    path = str(tmp_path / "h2.sock")
    goaway = _frame(7, 0, 0, struct.pack(">II", last_sid, 0))
    answer = (_frame(1, 0x4, 1, b"\x88" + _lit(b"content-type", b"application/grpc"))
              + _frame(0, 0, 1, b"\x00\x00\x00\x00\x00")
              + _frame(1, 0x5, 1, _lit(b"grpc-status", b"0")))
    t = _fake_h2_server(path, _frame(4, 0, 0) + goaway + (answer if last_sid else b""))
    c = n.H2Client(path)
    try:
        if last_sid:
            status, payload, _ = c.unary(v1beta1.METHOD_ALLOCATE, b"")
            assert status == 0 and payload == b""
            with pytest.raises(RuntimeError, match="GOAWAY"):  # no new stream on it
                c.unary(v1beta1.METHOD_ALLOCATE, b"")
        else:
            with pytest.raises(RuntimeError, match="not processed"):
                c.unary(v1beta1.METHOD_ALLOCATE, b"")
    finally:
        c.close()
        t.join(5)


def test_contention_detector_moves_only_on_a_sustained_slowdown(n):
    """grpc.coreEscape's decision: 32-call windows against the worker's own best window;
    two windows in a row 35 % over it ask for a move, at most once per 10 ms; a slow
    host is learnt (the best drifts up 0.4 % a window)."""
    d = n.ContentionDetector()
    t = 0
    moves = []

    def feed(svc_ns, windows):
        nonlocal t
        for _ in range(32 * windows):
            t += 3000
            if d.note(svc_ns, t):
                moves.append(t)
    feed(1360, 5)
    assert d.best_ns == 1360 and not moves
    feed(1700, 2)  # 25 % over: noise, not contention
    assert not moves
    feed(1970, 1)  # one slow window: not yet
    assert not moves
    feed(1970, 1)  # the second in a row
    assert len(moves) == 1
    feed(1970, 4)  # still slow, but within 10 ms of the move
    assert len(moves) == 1
    t += 20_000_000
    feed(1970, 2)
    assert len(moves) == 2
    # a host that got slower for good: the best drifts up until nothing is "over" it
    e = n.ContentionDetector()
    for _ in range(32):
        e.note(1000, 1)
    for _ in range(32 * 80):
        e.note(1300, 1)
    assert 1300 * 100 <= e.best_ns * 135 and e.best_ns <= 1300


def test_parse_cpu_list(n):
    assert n.parse_cpu_list("0-3,8,10-11\n") == [0, 1, 2, 3, 8, 10, 11]
    assert n.parse_cpu_list("5") == [5]
    assert n.parse_cpu_list("") == []


def test_core_escape_is_off_by_default_and_counts(n, plugin_dir):
    srv = n.GrpcServer(os.path.join(plugin_dir, "esc.sock"), 2)
    assert srv.core_escapes == 0
    srv.set_core_escape(True)
    srv.set_core_escape(False)


def test_peer_on_sibling_reads_the_peer_threads_cpus(n, tmp_path):
    """The escape's check: SO_PEERCRED names the client process, whose threads' last CPUs
    (/proc/<pid>/task/*/stat field 39) are compared with the SMT siblings of a CPU.  On a
    host without SMT there is never a sibling."""
    import socket as socket_mod
    a, b = socket_mod.socketpair(socket_mod.AF_UNIX, socket_mod.SOCK_STREAM)
    try:
        cpu = os.sched_getaffinity(0).pop()
        sib_path = "/sys/devices/system/cpu/cpu%d/topology/thread_siblings_list" % cpu
        sibs = n.parse_cpu_list(open(sib_path).read()) if os.path.exists(sib_path) else [cpu]
        got = n.peer_on_sibling(b.fileno(), cpu)
        if len(sibs) < 2:
            assert got is False
        assert n.peer_on_sibling(-1, cpu) is False
    finally:
        a.close()
        b.close()
