"""kubelet Device Plugin API ``v1beta1`` built at import time.

The reference links the generated Go package
``k8s.io/kubelet/pkg/apis/deviceplugin/v1beta1`` (``go.mod:20``; used at
``plugin/plugin.go:24``).  This image has no ``protoc``/``grpc_tools`` so the
file descriptor is assembled here from ``descriptor_pb2`` and fed to the
protobuf runtime; the resulting message classes are wire-identical to the
generated ones (field numbers/types below mirror the published ``api.proto``,
SURVEY.md Appendix A; golden byte tests live in ``tests/test_v1beta1_wire.py``).

Exports:
  * one message class per proto message (``RegisterRequest``, ``Device`` ...)
  * constants ``VERSION``, ``DEVICE_PLUGIN_PATH``, ``KUBELET_SOCKET``,
    ``HEALTHY``, ``UNHEALTHY`` (reference: ``plugin/plugin.go:47,141,149``,
    ``device/devices.go:74``)
  * fully-qualified method paths used by both the grpcio server and the native
    HTTP/2 server (``native/grpc_h2.cpp``).
"""
from __future__ import annotations

import os
import threading

# The protobuf runtime (~30 ms to import and build) is loaded on first use of a message
# class: the native daemon path needs only the constants and method paths below, so
# start-up does not pay for it (PEP 562 module __getattr__).

VERSION = "v1beta1"
DEVICE_PLUGIN_PATH = "/var/lib/kubelet/device-plugins/"
KUBELET_SOCKET_NAME = "kubelet.sock"
KUBELET_SOCKET = os.path.join(DEVICE_PLUGIN_PATH, KUBELET_SOCKET_NAME)
HEALTHY = "Healthy"
UNHEALTHY = "Unhealthy"

PACKAGE = "v1beta1"
REGISTRATION_SERVICE = PACKAGE + ".Registration"
DEVICE_PLUGIN_SERVICE = PACKAGE + ".DevicePlugin"

METHOD_REGISTER = "/%s/Register" % REGISTRATION_SERVICE
METHOD_GET_OPTIONS = "/%s/GetDevicePluginOptions" % DEVICE_PLUGIN_SERVICE
METHOD_LIST_AND_WATCH = "/%s/ListAndWatch" % DEVICE_PLUGIN_SERVICE
METHOD_GET_PREFERRED = "/%s/GetPreferredAllocation" % DEVICE_PLUGIN_SERVICE
METHOD_ALLOCATE = "/%s/Allocate" % DEVICE_PLUGIN_SERVICE
METHOD_PRE_START = "/%s/PreStartContainer" % DEVICE_PLUGIN_SERVICE

# FieldDescriptorProto enum values (descriptor.proto: TYPE_STRING = 9, TYPE_BOOL = 8,
# TYPE_INT32 = 5, TYPE_INT64 = 3, TYPE_MESSAGE = 11; LABEL_OPTIONAL = 1, LABEL_REPEATED = 3)
_STR, _BOOL, _I32, _I64, _MSG = 9, 8, 5, 3, 11
_OPT, _REP = 1, 3

# (message name, [(field name, number, type, label, type_name or None)])
_MESSAGES = [
    ("DevicePluginOptions", [("pre_start_required", 1, _BOOL, _OPT, None),
                             ("get_preferred_allocation_available", 2, _BOOL, _OPT, None)]),
    ("RegisterRequest", [("version", 1, _STR, _OPT, None),
                         ("endpoint", 2, _STR, _OPT, None),
                         ("resource_name", 3, _STR, _OPT, None),
                         ("options", 4, _MSG, _OPT, "DevicePluginOptions")]),
    ("Empty", []),
    ("ListAndWatchResponse", [("devices", 1, _MSG, _REP, "Device")]),
    ("TopologyInfo", [("nodes", 1, _MSG, _REP, "NUMANode")]),
    ("NUMANode", [("ID", 1, _I64, _OPT, None)]),
    ("Device", [("ID", 1, _STR, _OPT, None),
                ("health", 2, _STR, _OPT, None),
                ("topology", 3, _MSG, _OPT, "TopologyInfo")]),
    ("PreStartContainerRequest", [("devices_ids", 1, _STR, _REP, None)]),
    ("PreStartContainerResponse", []),
    ("PreferredAllocationRequest", [("container_requests", 1, _MSG, _REP,
                                     "ContainerPreferredAllocationRequest")]),
    ("ContainerPreferredAllocationRequest", [("available_deviceIDs", 1, _STR, _REP, None),
                                             ("must_include_deviceIDs", 2, _STR, _REP, None),
                                             ("allocation_size", 3, _I32, _OPT, None)]),
    ("PreferredAllocationResponse", [("container_responses", 1, _MSG, _REP,
                                      "ContainerPreferredAllocationResponse")]),
    ("ContainerPreferredAllocationResponse", [("deviceIDs", 1, _STR, _REP, None)]),
    ("AllocateRequest", [("container_requests", 1, _MSG, _REP, "ContainerAllocateRequest")]),
    ("ContainerAllocateRequest", [("devices_ids", 1, _STR, _REP, None)]),
    ("CDIDevice", [("name", 1, _STR, _OPT, None)]),
    ("AllocateResponse", [("container_responses", 1, _MSG, _REP, "ContainerAllocateResponse")]),
    # map<string,string> fields are repeated nested *Entry messages (added below)
    ("ContainerAllocateResponse", [("envs", 1, _MSG, _REP, "ContainerAllocateResponse.EnvsEntry"),
                                   ("mounts", 2, _MSG, _REP, "Mount"),
                                   ("devices", 3, _MSG, _REP, "DeviceSpec"),
                                   ("annotations", 4, _MSG, _REP,
                                    "ContainerAllocateResponse.AnnotationsEntry"),
                                   ("cdi_devices", 5, _MSG, _REP, "CDIDevice")]),
    ("Mount", [("container_path", 1, _STR, _OPT, None),
               ("host_path", 2, _STR, _OPT, None),
               ("read_only", 3, _BOOL, _OPT, None)]),
    ("DeviceSpec", [("container_path", 1, _STR, _OPT, None),
                    ("host_path", 2, _STR, _OPT, None),
                    ("permissions", 3, _STR, _OPT, None)]),
]

_MAP_FIELDS = {"ContainerAllocateResponse": ["EnvsEntry", "AnnotationsEntry"]}

# (service, method, input, output, server_streaming)
_SERVICES = [
    ("Registration", [("Register", "RegisterRequest", "Empty", False)]),
    ("DevicePlugin", [
        ("GetDevicePluginOptions", "Empty", "DevicePluginOptions", False),
        ("ListAndWatch", "Empty", "ListAndWatchResponse", True),
        ("GetPreferredAllocation", "PreferredAllocationRequest",
         "PreferredAllocationResponse", False),
        ("Allocate", "AllocateRequest", "AllocateResponse", False),
        ("PreStartContainer", "PreStartContainerRequest", "PreStartContainerResponse", False),
    ]),
]


def _build_file():
    from google.protobuf import descriptor_pb2
    fdp = descriptor_pb2.FileDescriptorProto()
    fdp.name = "k8s_gpu_device_plugin_amd/deviceplugin/v1beta1/api.proto"
    fdp.package = PACKAGE
    fdp.syntax = "proto3"
    fdp.options.go_package = "v1beta1"
    for name, fields in _MESSAGES:
        m = fdp.message_type.add()
        m.name = name
        for entry in _MAP_FIELDS.get(name, []):
            e = m.nested_type.add()
            e.name = entry
            e.options.map_entry = True
            for fname, num in (("key", 1), ("value", 2)):
                f = e.field.add()
                f.name, f.number, f.type, f.label = fname, num, _STR, _OPT
        for fname, num, ftype, label, tname in fields:
            f = m.field.add()
            f.name, f.number, f.type, f.label = fname, num, ftype, label
            if tname:
                f.type_name = ".%s.%s" % (PACKAGE, tname)
    for sname, methods in _SERVICES:
        s = fdp.service.add()
        s.name = sname
        for mname, inp, out, stream in methods:
            md = s.method.add()
            md.name = mname
            md.input_type = ".%s.%s" % (PACKAGE, inp)
            md.output_type = ".%s.%s" % (PACKAGE, out)
            md.server_streaming = stream
    return fdp


_CLASS_NAMES = [name for name, _ in _MESSAGES]
_LAZY = set(_CLASS_NAMES) | {"FILE_DESCRIPTOR_PROTO", "FILE_DESCRIPTOR", "METHODS"}
_loaded = False
_load_lock = threading.Lock()


def _load() -> None:
    """Builds the descriptor pool and message classes into this module (idempotent).
    The first access may come from several threads at once (grpcio handler threads, the
    kubelet stub): one builds, the others wait, so every caller sees classes from one
    pool.  Globals are published before ``_loaded`` is set."""
    global _loaded
    if _loaded:
        return
    with _load_lock:
        if not _loaded:
            _load_locked()


def _load_locked() -> None:
    global _loaded
    from google.protobuf import descriptor_pool, message_factory
    g = globals()
    fdp = _build_file()
    pool = descriptor_pool.DescriptorPool()
    fd = pool.Add(fdp)

    def cls(name: str):
        return message_factory.GetMessageClass(pool.FindMessageTypeByName(PACKAGE + "." + name))

    for name in _CLASS_NAMES:
        g[name] = cls(name)
    # method path -> (request class, response class, server_streaming)
    g["METHODS"] = {"/%s.%s/%s" % (PACKAGE, sname, mname): (g[inp], g[out], stream)
                    for sname, methods in _SERVICES for mname, inp, out, stream in methods}
    g["FILE_DESCRIPTOR_PROTO"], g["FILE_DESCRIPTOR"] = fdp, fd
    _loaded = True


def __getattr__(name: str):
    if name in _LAZY:
        _load()
        return globals()[name]
    raise AttributeError("module %r has no attribute %r" % (__name__, name))


def plugin_options(pre_start_required: bool = False) -> "DevicePluginOptions":
    """Options the plugin advertises (``plugin/plugin.go:165-170``)."""
    _load()
    return globals()["DevicePluginOptions"](pre_start_required=pre_start_required,
                                            get_preferred_allocation_available=True)


def _varint(n: int) -> bytes:
    out = bytearray()
    while n >= 0x80:
        out.append((n & 0x7F) | 0x80)
        n >>= 7
    out.append(n)
    return bytes(out)


def _ld(field: int, payload: bytes) -> bytes:  # length-delimited field, any length
    return _varint((field << 3) | 2) + _varint(len(payload)) + payload


def encode_register_request(endpoint: str, resource_name: str, pre_start_required: bool = False,
                            version: str = VERSION) -> bytes:
    """``RegisterRequest`` wire bytes without the protobuf runtime, byte-identical to
    ``RegisterRequest(...).SerializeToString()`` (proto3: fields in number order, empty
    strings and false bools omitted; ``tests/test_v1beta1_wire.py`` checks it)."""
    opts = (b"\x08\x01" if pre_start_required else b"") + b"\x10\x01"
    out = b""
    for num, val in ((1, version), (2, endpoint), (3, resource_name)):
        if val:
            out += _ld(num, val.encode())
    return out + _ld(4, opts)
