"""kubelet PodResources API ``v1`` (``k8s.io/kubelet/pkg/apis/podresources/v1``),
built at import time like ``v1beta1.py`` (no protoc in this image).

The reference does not use it.  Here it answers "which pod holds which device": the
plugin polls ``List`` on the kubelet's ``pod-resources/kubelet.sock`` and exports
``amdgpu_device_plugin_allocation_info{resource,device_id,namespace,pod,container}``
so GPU telemetry joins to workloads in PromQL.

Only the fields the plugin reads are declared; proto3 parsing skips the rest (cpu ids,
memory, dynamic resources), so newer kubelets stay compatible.
"""
from __future__ import annotations

from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

PACKAGE = "v1"
SERVICE = PACKAGE + ".PodResourcesLister"
METHOD_LIST = "/%s/List" % SERVICE
METHOD_GET_ALLOCATABLE = "/%s/GetAllocatableResources" % SERVICE
DEFAULT_SOCKET = "/var/lib/kubelet/pod-resources/kubelet.sock"

_F = descriptor_pb2.FieldDescriptorProto
_STR, _I64, _MSG = _F.TYPE_STRING, _F.TYPE_INT64, _F.TYPE_MESSAGE
_OPT, _REP = _F.LABEL_OPTIONAL, _F.LABEL_REPEATED

_MESSAGES = [
    ("ListPodResourcesRequest", []),
    ("ListPodResourcesResponse", [("pod_resources", 1, _MSG, _REP, "PodResources")]),
    ("PodResources", [("name", 1, _STR, _OPT, None),
                      ("namespace", 2, _STR, _OPT, None),
                      ("containers", 3, _MSG, _REP, "ContainerResources")]),
    ("ContainerResources", [("name", 1, _STR, _OPT, None),
                            ("devices", 2, _MSG, _REP, "ContainerDevices"),
                            ("cpu_ids", 3, _I64, _REP, None)]),
    ("ContainerDevices", [("resource_name", 1, _STR, _OPT, None),
                          ("device_ids", 2, _STR, _REP, None),
                          ("topology", 3, _MSG, _OPT, "TopologyInfo")]),
    ("TopologyInfo", [("nodes", 1, _MSG, _REP, "NUMANode")]),
    ("NUMANode", [("ID", 1, _I64, _OPT, None)]),
    ("AllocatableResourcesRequest", []),
    ("AllocatableResourcesResponse", [("devices", 1, _MSG, _REP, "ContainerDevices"),
                                      ("cpu_ids", 2, _I64, _REP, None)]),
]

_SERVICES = [("PodResourcesLister", [
    ("List", "ListPodResourcesRequest", "ListPodResourcesResponse"),
    ("GetAllocatableResources", "AllocatableResourcesRequest", "AllocatableResourcesResponse"),
])]


def _build_file() -> descriptor_pb2.FileDescriptorProto:
    fdp = descriptor_pb2.FileDescriptorProto()
    fdp.name = "k8s_gpu_device_plugin_amd/podresources/v1/api.proto"
    fdp.package = PACKAGE
    fdp.syntax = "proto3"
    for name, fields in _MESSAGES:
        m = fdp.message_type.add()
        m.name = name
        for fname, num, ftype, label, tname in fields:
            f = m.field.add()
            f.name, f.number, f.type, f.label = fname, num, ftype, label
            if tname:
                f.type_name = ".%s.%s" % (PACKAGE, tname)
    for sname, methods in _SERVICES:
        s = fdp.service.add()
        s.name = sname
        for mname, inp, out in methods:
            md = s.method.add()
            md.name, md.input_type, md.output_type = mname, ".%s.%s" % (PACKAGE, inp), ".%s.%s" % (PACKAGE, out)
    return fdp


FILE_DESCRIPTOR_PROTO = _build_file()
_POOL = descriptor_pool.DescriptorPool()
_POOL.Add(FILE_DESCRIPTOR_PROTO)


def _cls(name: str):
    return message_factory.GetMessageClass(_POOL.FindMessageTypeByName(PACKAGE + "." + name))


ListPodResourcesRequest = _cls("ListPodResourcesRequest")
ListPodResourcesResponse = _cls("ListPodResourcesResponse")
PodResources = _cls("PodResources")
ContainerResources = _cls("ContainerResources")
ContainerDevices = _cls("ContainerDevices")
TopologyInfo = _cls("TopologyInfo")
NUMANode = _cls("NUMANode")
AllocatableResourcesRequest = _cls("AllocatableResourcesRequest")
AllocatableResourcesResponse = _cls("AllocatableResourcesResponse")
