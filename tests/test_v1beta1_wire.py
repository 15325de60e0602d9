"""Golden wire tests for the kubelet v1beta1 contract and for the
native protobuf encoders in DeviceTable (they must parse identically to the
runtime-descriptor messages kubelet-side code would use)."""
import pytest

from k8s_gpu_device_plugin_amd.api import v1beta1 as v


def test_register_request_golden():
    # field 1 (version) = "v1beta1"  ->  0a 07 76 31 62 65 74 61 31
    assert v.RegisterRequest(version="v1beta1").SerializeToString().hex() == "0a0776316265746131"
    full = v.RegisterRequest(version="v1beta1", endpoint="amd-gpu.sock", resource_name="amd.com/gpu",
                             options=v.plugin_options())
    b = full.SerializeToString()
    assert b == bytes.fromhex("0a0776316265746131") + b"\x12\x0camd-gpu.sock" + b"\x1a\x0bamd.com/gpu" + \
        bytes.fromhex("22021001")  # options{get_preferred_allocation_available(2)=true}


def test_options_golden():
    assert v.plugin_options().SerializeToString() == b"\x10\x01"
    assert v.DevicePluginOptions(pre_start_required=True).SerializeToString() == b"\x08\x01"


def test_device_golden_with_numa_zero():
    d = v.Device(ID="g0", health="Healthy")
    d.topology.nodes.add(ID=0)  # NUMA 0: proto3 omits the zero scalar, node stays as empty message
    assert d.SerializeToString() == b"\x0a\x02g0" + b"\x12\x07Healthy" + b"\x1a\x02\x0a\x00"
    d2 = v.Device(ID="g1", health="Unhealthy")
    d2.topology.nodes.add(ID=1)
    assert d2.SerializeToString() == b"\x0a\x02g1\x12\x09Unhealthy\x1a\x04\x0a\x02\x08\x01"


def test_allocate_response_map_and_specs():
    r = v.ContainerAllocateResponse(envs={"A": "b"}, devices=[
        v.DeviceSpec(container_path="/dev/kfd", host_path="/dev/kfd", permissions="rw")])
    assert r.SerializeToString().hex() == "0a060a01411201621a180a082f6465762f6b666412082f6465762f6b66641a027277"


def test_method_paths():
    assert v.METHOD_REGISTER == "/v1beta1.Registration/Register"
    assert v.METHOD_ALLOCATE == "/v1beta1.DevicePlugin/Allocate"
    assert v.METHOD_LIST_AND_WATCH == "/v1beta1.DevicePlugin/ListAndWatch"
    assert set(v.METHODS) == {
        "/v1beta1.Registration/Register", "/v1beta1.DevicePlugin/GetDevicePluginOptions",
        "/v1beta1.DevicePlugin/ListAndWatch", "/v1beta1.DevicePlugin/GetPreferredAllocation",
        "/v1beta1.DevicePlugin/Allocate", "/v1beta1.DevicePlugin/PreStartContainer"}
    assert v.METHODS[v.METHOD_LIST_AND_WATCH][2] is True


def test_constants():
    assert v.VERSION == "v1beta1"
    assert v.DEVICE_PLUGIN_PATH == "/var/lib/kubelet/device-plugins/"
    assert v.KUBELET_SOCKET == "/var/lib/kubelet/device-plugins/kubelet.sock"
    assert (v.HEALTHY, v.UNHEALTHY) == ("Healthy", "Unhealthy")


def _table(n, devs, cfg_over=None):
    tc = n.TableConfig()
    for k, val in (cfg_over or {}).items():
        setattr(tc, k, val)
    topo = n.Topology(max([d[1] for d in devs]) + 1)
    tds = [n.TableDevice(i, g, p, numa, -1, paths, True) for (i, g, p, numa, paths) in devs]
    return n.DeviceTable(tc, tds, topo)


DEVS = [("gpu-a", 0, -1, 0, ["/dev/dri/renderD128"]), ("gpu-b", 1, -1, 1, ["/dev/dri/renderD129"]),
        ("gpu-c", 2, -1, -1, ["/dev/dri/renderD130", "/dev/dri/card2"])]


def test_native_list_and_watch_matches_python_encoding(n):
    t = _table(n, DEVS)
    expect = v.ListAndWatchResponse()
    for i, _, _, numa, _ in DEVS:
        d = expect.devices.add(ID=i, health="Healthy")
        if numa >= 0:
            d.topology.nodes.add(ID=numa)
    assert t.list_and_watch() == expect.SerializeToString()
    assert t.set_health("gpu-b", False)
    expect.devices[1].health = "Unhealthy"
    assert t.list_and_watch() == expect.SerializeToString()


def test_native_allocate_encoding(n):
    t = _table(n, DEVS, {"extra_envs": [("X", "1")]})
    req = v.AllocateRequest(container_requests=[v.ContainerAllocateRequest(devices_ids=["gpu-a", "gpu-c"]),
                                                v.ContainerAllocateRequest(devices_ids=["gpu-b"])])
    ok, out = t.allocate(req.SerializeToString())
    assert ok
    resp = v.AllocateResponse.FromString(out)
    c0, c1 = resp.container_responses
    assert dict(c0.envs) == {"AMD_VISIBLE_DEVICES": "gpu-a,gpu-c", "X": "1"}
    assert [(s.container_path, s.host_path, s.permissions) for s in c0.devices] == [
        ("/dev/kfd", "/dev/kfd", "rw"), ("/dev/dri/renderD128", "/dev/dri/renderD128", "rw"),
        ("/dev/dri/renderD130", "/dev/dri/renderD130", "rw"), ("/dev/dri/card2", "/dev/dri/card2", "rw")]
    assert dict(c1.envs)["AMD_VISIBLE_DEVICES"] == "gpu-b"
    assert len(c1.mounts) == 0 and len(c1.annotations) == 0 and len(c1.cdi_devices) == 0


def test_native_allocate_cdi_and_no_kfd(n):
    t = _table(n, DEVS, {"cdi": True, "cdi_prefix": "amd.com/gpu=", "mount_kfd": False, "visible_env": ""})
    ok, out = t.allocate(v.AllocateRequest(container_requests=[
        v.ContainerAllocateRequest(devices_ids=["gpu-b"])]).SerializeToString())
    c = v.AllocateResponse.FromString(out).container_responses[0]
    assert [d.name for d in c.cdi_devices] == ["amd.com/gpu=gpu-b"]
    assert [s.host_path for s in c.devices] == ["/dev/dri/renderD129"]
    assert len(c.envs) == 0


def test_native_allocate_errors(n):
    t = _table(n, DEVS)
    ok, msg = t.allocate(v.AllocateRequest(container_requests=[
        v.ContainerAllocateRequest(devices_ids=["nope"])]).SerializeToString())
    assert not ok and "unknown device: nope" in msg and "amd.com/gpu" in msg
    t.set_health("gpu-a", False)
    ok, msg = t.allocate(v.AllocateRequest(container_requests=[
        v.ContainerAllocateRequest(devices_ids=["gpu-a"])]).SerializeToString())
    assert not ok and "Unhealthy" in msg
    ok, msg = t.allocate(b"\x0a\xff")  # truncated length-delimited field
    assert not ok and "malformed" in msg


def test_native_decoder_skips_unknown_fields(n):
    t = _table(n, DEVS)
    # container request with an unknown varint field 7 and fixed32 field 8 before the id
    inner = b"\x38\x05" + b"\x45\x01\x02\x03\x04" + b"\x0a\x05gpu-a"
    ok, out = t.allocate(b"\x0a" + bytes([len(inner)]) + inner)
    assert ok, out
    assert dict(v.AllocateResponse.FromString(out).container_responses[0].envs)["AMD_VISIBLE_DEVICES"] == "gpu-a"


def test_native_preferred_encoding(n):
    t = _table(n, DEVS)
    req = v.PreferredAllocationRequest(container_requests=[v.ContainerPreferredAllocationRequest(
        available_deviceIDs=["gpu-a", "gpu-b", "gpu-c"], must_include_deviceIDs=["gpu-c"], allocation_size=2)])
    ok, out = t.preferred(req.SerializeToString())
    assert ok
    ids = list(v.PreferredAllocationResponse.FromString(out).container_responses[0].deviceIDs)
    assert len(ids) == 2 and ids[0] == "gpu-c"
    ok, msg = t.preferred(v.PreferredAllocationRequest(container_requests=[v.ContainerPreferredAllocationRequest(
        available_deviceIDs=["gpu-a"], allocation_size=3)]).SerializeToString())
    assert not ok and "not enough available devices" in msg


@pytest.mark.parametrize("size", [0, 1, 2, 3])
def test_options_bytes(n, size):
    t = _table(n, DEVS)
    assert v.DevicePluginOptions.FromString(t.options()).get_preferred_allocation_available


@pytest.mark.parametrize("pre_start", [False, True])
@pytest.mark.parametrize("endpoint,resource", [("amd-gpu.sock", "amd.com/gpu"), ("a" * 300, "amd.com/cpx_nps4"),
                                               ("", ""), ("e" * 16384, "amd.com/gpu"),
                                               ("e" * 20000, "r" * 40000)])
def test_protobuf_free_register_request_matches_runtime(pre_start, endpoint, resource):
    """The native Register path encodes RegisterRequest by hand; it must be byte-identical
    to the protobuf runtime's serialisation."""
    want = v.RegisterRequest(version=v.VERSION, endpoint=endpoint, resource_name=resource,
                             options=v.plugin_options(pre_start)).SerializeToString()
    assert v.encode_register_request(endpoint, resource, pre_start) == want


def test_daemon_imports_stay_light():
    """Start-up path: the CLI and manager import neither grpcio, protobuf nor PyYAML (the
    native servers, the compiled Register client and lazy v1beta1 classes need none)."""
    import subprocess
    import sys
    code = ("import sys, k8s_gpu_device_plugin_amd.cli, k8s_gpu_device_plugin_amd.plugin.manager;"
            "print(sorted(m for m in ('grpc', 'google.protobuf', 'yaml') if m in sys.modules))")
    out = subprocess.run([sys.executable, "-c", code], stdout=subprocess.PIPE, text=True, check=True)
    assert out.stdout.strip() == "[]"


def test_lazy_classes_built_once_under_concurrent_first_use():
    """the first message-class access from several threads at once must build
    one descriptor pool; every thread gets the same class objects."""
    import subprocess
    import sys
    code = """
import threading
from k8s_gpu_device_plugin_amd.api import v1beta1 as v
start = threading.Barrier(16)
seen = []
def go():
    start.wait()
    seen.append((v.Device, v.ListAndWatchResponse, v.METHODS[v.METHOD_ALLOCATE][0]))
ts = [threading.Thread(target=go) for _ in range(16)]
[t.start() for t in ts]
[t.join() for t in ts]
assert len(set(seen)) == 1, len(set(seen))
r = v.ListAndWatchResponse(devices=[v.Device(ID="x", health=v.HEALTHY)])
assert v.ListAndWatchResponse.FromString(r.SerializeToString()).devices[0].ID == "x"
print("ok")
"""
    out = subprocess.run([sys.executable, "-c", code], stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    assert out.stdout.strip().endswith("ok"), out.stdout
