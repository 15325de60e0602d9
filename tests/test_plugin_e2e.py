"""DevicePlugin endpoint end-to-end against the in-process kubelet stub, for both gRPC
servers (native C++ HTTP/2 and grpcio).  BASELINE config 1: mock backend, 2 fake GPUs."""
import os
import time

import grpc
import pytest

from k8s_gpu_device_plugin_amd.api import v1beta1
from k8s_gpu_device_plugin_amd.device import build_device_map
from k8s_gpu_device_plugin_amd.models import fixtures
from k8s_gpu_device_plugin_amd.plugin.kubelet_stub import KubeletStub
from k8s_gpu_device_plugin_amd.plugin.plugin import AmdDevicePlugin, socket_name
from k8s_gpu_device_plugin_amd.resource import new_resources


@pytest.fixture(params=["native", "python"])
def server_kind(request):
    return request.param


def _plugin(plugin_dir, kind, spec="2gpu_spx", strategy="none", **kw):
    g, topo = fixtures.build_backend(spec).discover()
    dm = build_device_map(g, new_resources(g, strategy), strategy, **kw)
    name, devs = next(iter(dm.items()))
    return AmdDevicePlugin(name, devs, topo, plugin_dir=plugin_dir, server_kind=kind), g


def test_socket_name():
    assert socket_name("amd.com/gpu") == "amd-gpu.sock"
    assert socket_name("amd.com/cpx_nps2") == "amd-cpx_nps2.sock"


def test_register_and_serve(plugin_dir, server_kind):
    with KubeletStub(plugin_dir) as k:
        p, g = _plugin(plugin_dir, server_kind)
        p.start()
        try:
            reg = k.wait_for_registrations(1)[0]
            assert (reg.version, reg.endpoint, reg.resource_name) == ("v1beta1", "amd-gpu.sock", "amd.com/gpu")
            assert reg.options.get_preferred_allocation_available and not reg.options.pre_start_required
            c = k.client(reg.endpoint)
            assert c.get_options().get_preferred_allocation_available
            assert c.pre_start([g[0].uuid]) == v1beta1.PreStartContainerResponse()
            _, devs = k.watch(reg.endpoint).next()
            assert [d[0] for d in devs] == [g[0].uuid, g[1].uuid]
            assert all(h == "Healthy" for _, h, _ in devs) and devs[0][2] == [0]
            r = c.allocate([g[1].uuid], [g[0].uuid, g[1].uuid])
            c0, c1 = r.container_responses
            assert dict(c0.envs) == {"AMD_VISIBLE_DEVICES": g[1].uuid}
            assert [s.host_path for s in c0.devices] == ["/dev/kfd", "/dev/dri/renderD129"]
            assert [s.host_path for s in c1.devices] == ["/dev/kfd", "/dev/dri/renderD128", "/dev/dri/renderD129"]
            pref = c.preferred([g[0].uuid, g[1].uuid], [g[1].uuid], 1)
            assert list(pref.container_responses[0].deviceIDs) == [g[1].uuid]
        finally:
            p.stop()
    assert not os.path.exists(p.socket)


def test_allocate_errors(plugin_dir, server_kind):
    with KubeletStub(plugin_dir) as k:
        p, g = _plugin(plugin_dir, server_kind)
        p.start()
        try:
            c = k.client("amd-gpu.sock")
            with pytest.raises(grpc.RpcError) as e:
                c.allocate(["not-a-device"])
            assert e.value.code() == grpc.StatusCode.UNKNOWN
            assert "invalid allocation request for 'amd.com/gpu'" in e.value.details()
            p.set_gpu_health(0, -1, False)
            with pytest.raises(grpc.RpcError) as e:
                c.allocate([g[0].uuid])
            assert "Unhealthy" in e.value.details()
            with pytest.raises(grpc.RpcError):
                c.preferred([g[0].uuid], [], 5)
        finally:
            p.stop()


def test_health_updates_both_ways(plugin_dir, server_kind):
    with KubeletStub(plugin_dir) as k:
        p, g = _plugin(plugin_dir, server_kind, "8gpu_cpx_nps2", "single")
        p.start()
        try:
            w = k.watch("amd-gpu.sock")
            t0, devs = w.next()
            assert len(devs) == 64
            t_set = time.monotonic()
            assert p.set_gpu_health(3, -1, False) == 8
            t1, devs = w.next()
            bad = [i for i, h, _ in devs if h == "Unhealthy"]
            assert len(bad) == 8 and all(i.startswith(g[3].uuid) for i in bad)
            assert t1 - t_set < 1.0
            assert p.set_gpu_health(3, 2, True) == 1  # one partition recovers
            _, devs = w.next()
            assert sum(h == "Unhealthy" for _, h, _ in devs) == 7
            assert p.set_device_health(g[3].partitions[0].id, True)
            _, devs = w.next()
            assert sum(h == "Unhealthy" for _, h, _ in devs) == 6
            assert not p.set_device_health("nope", True)
        finally:
            p.stop()


def test_stop_is_idempotent_and_restartable(plugin_dir, server_kind):
    with KubeletStub(plugin_dir) as k:
        p, _ = _plugin(plugin_dir, server_kind)
        p.stop()  # before start
        p.start()
        w = k.watch("amd-gpu.sock")
        w.next()
        p.stop()
        p.stop()
        assert not p.serving
        p.start()  # same object can serve again (D6/D10)
        k.wait_for_registrations(2)
        assert k.client("amd-gpu.sock") is not None
        p.stop()


def test_register_fails_without_kubelet(plugin_dir, server_kind):
    p, _ = _plugin(plugin_dir, server_kind)
    with pytest.raises(Exception):
        p.start()
    assert not p.serving and not os.path.exists(p.socket)


def test_concurrent_clients(plugin_dir, server_kind):
    import threading
    with KubeletStub(plugin_dir) as k:
        p, g = _plugin(plugin_dir, server_kind, "8gpu_spx_mesh")
        p.start()
        errors = []

        def worker(i):
            from k8s_gpu_device_plugin_amd.plugin.kubelet_stub import DevicePluginClient
            c = DevicePluginClient(p.socket)
            try:
                for _ in range(50):
                    r = c.allocate([g[i].uuid])
                    if dict(r.container_responses[0].envs)["AMD_VISIBLE_DEVICES"] != g[i].uuid:
                        errors.append(i)
            except Exception as e:  # pragma: no cover
                errors.append(e)
            finally:
                c.close()
        ts = [threading.Thread(target=worker, args=(i,)) for i in range(8)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        p.stop()
        assert not errors


def test_native_table_change_reaches_watchers_without_notify(plugin_dir, server_kind):
    """The monitor thread's fail-fast path changes the table directly (no Python
    notify): both servers must push it at once (native: table listener; grpcio: the
    generator blocks in table.wait_change), and the Python device view follows."""
    with KubeletStub(plugin_dir) as k:
        p, g = _plugin(plugin_dir, server_kind, "2gpu_spx", "none")
        p.start()
        try:
            w = k.watch("amd-gpu.sock")
            w.next()
            t0 = time.monotonic()
            assert p.table.set_gpu_health(1, -1, False) == 1  # bypasses AmdDevicePlugin
            t1, devs = w.next()
            assert [h for _, h, _ in devs] == ["Healthy", "Unhealthy"] and t1 - t0 < 0.25
            assert p.set_gpu_health(1, -1, False) == 0  # manager catching up: no change, no push
            assert p.devices()[devs[1][0]].health == v1beta1.UNHEALTHY
        finally:
            p.stop()


@pytest.mark.parametrize("server", ["native"])
def test_stop_leaves_a_newer_instances_socket_alone(make_cfg, plugin_dir, server):
    """Rolling update: the next plugin pod binds amd-gpu.sock while this one is still
    stopping.  This one's stop must not delete the newer socket (kubelet would lose the
    new plugin until its socket watcher re-served it).  The native server (the default);
    grpcio's core unlinks its unix socket path on shutdown whatever is there, so with
    grpc.server: python the newer instance's socket watcher re-serves instead."""
    import socket as _socket
    from k8s_gpu_device_plugin_amd.plugin.kubelet_stub import KubeletStub
    from k8s_gpu_device_plugin_amd.plugin.manager import PluginManager
    with KubeletStub(plugin_dir):
        m = PluginManager(make_cfg(grpc={"server": server}))
        m.load_plugins()
        m.start_plugins()
        p = m.plugins[0]
        assert p.serving and os.path.exists(p.socket)
        os.remove(p.socket)  # the newer instance: remove the stale file, bind its own
        newer = _socket.socket(_socket.AF_UNIX, _socket.SOCK_STREAM)
        newer.bind(p.socket)
        newer.listen(1)
        try:
            ident = os.stat(p.socket).st_ino
            m.stop_plugins()
            assert os.path.exists(p.socket) and os.stat(p.socket).st_ino == ident
        finally:
            newer.close()
            os.remove(p.socket)
        m.exporter.stop()
        m.monitor.stop()
    # and its own socket is removed as before
    with KubeletStub(plugin_dir):
        m = PluginManager(make_cfg(grpc={"server": server}))
        m.load_plugins()
        m.start_plugins()
        sock = m.plugins[0].socket
        m.stop_plugins()
        assert not os.path.exists(sock)
        m.exporter.stop()
        m.monitor.stop()


def test_crash_accounting_matches_the_reference_serve_loop(plugin_dir, monkeypatch):
    """``plugin/plugin.go:107-129``: each crash within an hour of the previous one adds
    one; the 6th such crash is fatal; a crash more than an hour after the previous one
    starts the count again from 0."""
    from k8s_gpu_device_plugin_amd.plugin import plugin as plugin_mod
    now = [1000.0]
    monkeypatch.setattr(plugin_mod.time, "monotonic", lambda: now[0])
    p, _ = _plugin(plugin_dir, "native")
    for i in range(5):
        now[0] += 60
        assert not p._note_crash("test"), i
    now[0] += plugin_mod.SERVE_CRASH_WINDOW_S + 1  # quiet for over an hour: count resets
    assert not p._note_crash("test") and p._crashes == 0
    for i in range(5):
        now[0] += 60
        assert not p._note_crash("test"), i
    now[0] += 60
    assert p._note_crash("test")  # 6th crash within the hour
    assert p.fatal_error and "repeatedly crashed" in p.fatal_error
