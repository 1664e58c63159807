"""kubelet device-plugin API ``v1beta1`` message classes, built from a hand-written descriptor.

There is no ``protoc`` / ``grpc_tools`` in this image, so
the ``k8s.io/kubelet/pkg/apis/deviceplugin/v1beta1/api.proto`` schema is
declared here as a ``FileDescriptorProto`` and turned into message classes at
import time.  Field numbers and types match the upstream proto (the wire
format is all that matters to kubelet); names follow its snake_case.
"""
from __future__ import annotations

from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

PKG = "v1beta1"
VERSION = "v1beta1"
KUBELET_SOCKET = "kubelet.sock"
DEVICE_PLUGIN_PATH = "/var/lib/kubelet/device-plugins/"
HEALTHY = "Healthy"
UNHEALTHY = "Unhealthy"

F = descriptor_pb2.FieldDescriptorProto
_STR, _BOOL, _I64, _I32, _MSG = F.TYPE_STRING, F.TYPE_BOOL, F.TYPE_INT64, F.TYPE_INT32, F.TYPE_MESSAGE
_OPT, _REP = F.LABEL_OPTIONAL, F.LABEL_REPEATED

# message -> [(name, number, type, label, type_name)]
_MESSAGES = {
    "DevicePluginOptions": [("pre_start_required", 1, _BOOL, _OPT, None),
                            ("get_preferred_allocation_available", 2, _BOOL, _OPT, None)],
    "RegisterRequest": [("version", 1, _STR, _OPT, None), ("endpoint", 2, _STR, _OPT, None),
                        ("resource_name", 3, _STR, _OPT, None), ("options", 4, _MSG, _OPT, "DevicePluginOptions")],
    "Empty": [],
    "ListAndWatchResponse": [("devices", 1, _MSG, _REP, "Device")],
    "TopologyInfo": [("nodes", 1, _MSG, _REP, "NUMANode")],
    "NUMANode": [("ID", 1, _I64, _OPT, None)],
    "Device": [("ID", 1, _STR, _OPT, None), ("health", 2, _STR, _OPT, None),
               ("topology", 3, _MSG, _OPT, "TopologyInfo")],
    "PreStartContainerRequest": [("devices_ids", 1, _STR, _REP, None)],
    "PreStartContainerResponse": [],
    "PreferredAllocationRequest": [("container_requests", 1, _MSG, _REP, "ContainerPreferredAllocationRequest")],
    "ContainerPreferredAllocationRequest": [("available_deviceIDs", 1, _STR, _REP, None),
                                            ("must_include_deviceIDs", 2, _STR, _REP, None),
                                            ("allocation_size", 3, _I32, _OPT, None)],
    "PreferredAllocationResponse": [("container_responses", 1, _MSG, _REP, "ContainerPreferredAllocationResponse")],
    "ContainerPreferredAllocationResponse": [("deviceIDs", 1, _STR, _REP, None)],
    "AllocateRequest": [("container_requests", 1, _MSG, _REP, "ContainerAllocateRequest")],
    "ContainerAllocateRequest": [("devices_ids", 1, _STR, _REP, None)],
    "AllocateResponse": [("container_responses", 1, _MSG, _REP, "ContainerAllocateResponse")],
    "ContainerAllocateResponse": [("envs", 1, _MSG, _REP, "ContainerAllocateResponse.EnvsEntry"),
                                  ("mounts", 2, _MSG, _REP, "Mount"),
                                  ("devices", 3, _MSG, _REP, "DeviceSpec"),
                                  ("annotations", 4, _MSG, _REP, "ContainerAllocateResponse.AnnotationsEntry"),
                                  ("cdi_devices", 5, _MSG, _REP, "CDIDevice")],
    "Mount": [("container_path", 1, _STR, _OPT, None), ("host_path", 2, _STR, _OPT, None),
              ("read_only", 3, _BOOL, _OPT, None)],
    "DeviceSpec": [("container_path", 1, _STR, _OPT, None), ("host_path", 2, _STR, _OPT, None),
                   ("permissions", 3, _STR, _OPT, None)],
    "CDIDevice": [("name", 1, _STR, _OPT, None)],
}
_MAPS = {"ContainerAllocateResponse": ["EnvsEntry", "AnnotationsEntry"]}

SERVICES = {
    "Registration": {"Register": ("RegisterRequest", "Empty", False)},
    "DevicePlugin": {
        "GetDevicePluginOptions": ("Empty", "DevicePluginOptions", False),
        "ListAndWatch": ("Empty", "ListAndWatchResponse", True),
        "GetPreferredAllocation": ("PreferredAllocationRequest", "PreferredAllocationResponse", False),
        "Allocate": ("AllocateRequest", "AllocateResponse", False),
        "PreStartContainer": ("PreStartContainerRequest", "PreStartContainerResponse", False),
    },
}


def _build():
    fd = descriptor_pb2.FileDescriptorProto(name="gsx/deviceplugin/v1beta1/api.proto", package=PKG, syntax="proto3")
    for mname, fields in _MESSAGES.items():
        m = fd.message_type.add(name=mname)
        for entry in _MAPS.get(mname, []):
            e = m.nested_type.add(name=entry)
            e.options.map_entry = True
            e.field.add(name="key", number=1, type=_STR, label=_OPT)
            e.field.add(name="value", number=2, type=_STR, label=_OPT)
        for name, num, typ, label, tname in fields:
            f = m.field.add(name=name, number=num, type=typ, label=label)
            if tname:
                f.type_name = f".{PKG}.{tname}"
    for sname, methods in SERVICES.items():
        s = fd.service.add(name=sname)
        for meth, (inp, out, stream) in methods.items():
            s.method.add(name=meth, input_type=f".{PKG}.{inp}", output_type=f".{PKG}.{out}", server_streaming=stream)
    pool = descriptor_pool.DescriptorPool()
    fdesc = pool.Add(fd)
    classes = {}
    for mname in _MESSAGES:
        classes[mname] = message_factory.GetMessageClass(pool.FindMessageTypeByName(f"{PKG}.{mname}"))
    return pool, fdesc, classes


POOL, FILE, _CLASSES = _build()
globals().update(_CLASSES)

DevicePluginOptions = _CLASSES["DevicePluginOptions"]
RegisterRequest = _CLASSES["RegisterRequest"]
Empty = _CLASSES["Empty"]
ListAndWatchResponse = _CLASSES["ListAndWatchResponse"]
Device = _CLASSES["Device"]
TopologyInfo = _CLASSES["TopologyInfo"]
NUMANode = _CLASSES["NUMANode"]
AllocateRequest = _CLASSES["AllocateRequest"]
AllocateResponse = _CLASSES["AllocateResponse"]
ContainerAllocateRequest = _CLASSES["ContainerAllocateRequest"]
ContainerAllocateResponse = _CLASSES["ContainerAllocateResponse"]
PreferredAllocationRequest = _CLASSES["PreferredAllocationRequest"]
PreferredAllocationResponse = _CLASSES["PreferredAllocationResponse"]
ContainerPreferredAllocationRequest = _CLASSES["ContainerPreferredAllocationRequest"]
ContainerPreferredAllocationResponse = _CLASSES["ContainerPreferredAllocationResponse"]
PreStartContainerRequest = _CLASSES["PreStartContainerRequest"]
PreStartContainerResponse = _CLASSES["PreStartContainerResponse"]
DeviceSpec = _CLASSES["DeviceSpec"]
Mount = _CLASSES["Mount"]


def method_path(service: str, method: str) -> str:
    return f"/{PKG}.{service}/{method}"


def io_types(service: str, method: str):
    inp, out, stream = SERVICES[service][method]
    return _CLASSES[inp], _CLASSES[out], stream
