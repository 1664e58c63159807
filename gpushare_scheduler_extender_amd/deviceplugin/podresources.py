"""kubelet PodResources API ``v1`` (``/var/lib/kubelet/pod-resources/kubelet.sock``): which container holds which
device IDs, as kubelet's device manager recorded them.

The Allocate contract matches a container to a pod by size and earliest ``ASSUME_TIME`` only
(``docs/designs/designs.md:93-103``): kubelet never says which pod it is admitting.  When kubelet admits a
batch of equal-size pods in another order than they were bound (its own restart, a re-list, pods it first
meets together: it sorts a batch by creationTimestamp), a container can start with the allocation the plugin
built for another pod.  kubelet's record of device IDs per container is the ground truth the plugin
reconciles against (:mod:`.reconcile`).  The device plugin API tells the plugin which IDs each Allocate
served; this API tells it which pod those IDs went to.

As in :mod:`.api`, there is no ``protoc`` here: the ``k8s.io/kubelet/pkg/apis/podresources/v1/api.proto``
schema is declared as a ``FileDescriptorProto``; field numbers and types match upstream (only the wire
format matters to kubelet).  :class:`PodResourcesServer` is the kubelet side, used by the kubelet stand-in.
"""
from __future__ import annotations

import os

import grpc
from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

PKG = "v1"
DEFAULT_SOCKET = "/var/lib/kubelet/pod-resources/kubelet.sock"

F = descriptor_pb2.FieldDescriptorProto
_STR, _I64, _U64, _MSG = F.TYPE_STRING, F.TYPE_INT64, F.TYPE_UINT64, F.TYPE_MESSAGE
_OPT, _REP = F.LABEL_OPTIONAL, F.LABEL_REPEATED

_MESSAGES = {
    "AllocatableResourcesRequest": [],
    "AllocatableResourcesResponse": [("devices", 1, _MSG, _REP, "ContainerDevices"), ("cpu_ids", 2, _I64, _REP, None),
                                     ("memory", 3, _MSG, _REP, "ContainerMemory")],
    "ListPodResourcesRequest": [],
    "ListPodResourcesResponse": [("pod_resources", 1, _MSG, _REP, "PodResources")],
    "PodResources": [("name", 1, _STR, _OPT, None), ("namespace", 2, _STR, _OPT, None),
                     ("containers", 3, _MSG, _REP, "ContainerResources")],
    "ContainerResources": [("name", 1, _STR, _OPT, None), ("devices", 2, _MSG, _REP, "ContainerDevices"),
                           ("cpu_ids", 3, _I64, _REP, None), ("memory", 4, _MSG, _REP, "ContainerMemory"),
                           ("dynamic_resources", 5, _MSG, _REP, "DynamicResource")],
    "ContainerMemory": [("memory_type", 1, _STR, _OPT, None), ("size", 2, _U64, _OPT, None),
                        ("topology", 3, _MSG, _OPT, "TopologyInfo")],
    "ContainerDevices": [("resource_name", 1, _STR, _OPT, None), ("device_ids", 2, _STR, _REP, None),
                         ("topology", 3, _MSG, _OPT, "TopologyInfo")],
    "TopologyInfo": [("nodes", 1, _MSG, _REP, "NUMANode")],
    "NUMANode": [("ID", 1, _I64, _OPT, None)],
    "DynamicResource": [("class_name", 1, _STR, _OPT, None), ("claim_name", 2, _STR, _OPT, None),
                        ("claim_namespace", 3, _STR, _OPT, None),
                        ("claim_resources", 4, _MSG, _REP, "ClaimResource")],
    "ClaimResource": [("cdi_devices", 1, _MSG, _REP, "CDIDevice")],
    "CDIDevice": [("name", 1, _STR, _OPT, None)],
    "GetPodResourcesRequest": [("pod_name", 1, _STR, _OPT, None), ("pod_namespace", 2, _STR, _OPT, None)],
    "GetPodResourcesResponse": [("pod_resources", 1, _MSG, _OPT, "PodResources")],
}
SERVICE = "PodResourcesLister"
METHODS = {
    "List": ("ListPodResourcesRequest", "ListPodResourcesResponse"),
    "GetAllocatableResources": ("AllocatableResourcesRequest", "AllocatableResourcesResponse"),
    "Get": ("GetPodResourcesRequest", "GetPodResourcesResponse"),
}


def _build():
    fd = descriptor_pb2.FileDescriptorProto(name="gsx/podresources/v1/api.proto", package=PKG, syntax="proto3")
    for mname, fields in _MESSAGES.items():
        m = fd.message_type.add(name=mname)
        for name, num, typ, label, tname in fields:
            f = m.field.add(name=name, number=num, type=typ, label=label)
            if tname:
                f.type_name = f".{PKG}.{tname}"
    s = fd.service.add(name=SERVICE)
    for meth, (inp, out) in METHODS.items():
        s.method.add(name=meth, input_type=f".{PKG}.{inp}", output_type=f".{PKG}.{out}")
    pool = descriptor_pool.DescriptorPool()
    pool.Add(fd)
    return {m: message_factory.GetMessageClass(pool.FindMessageTypeByName(f"{PKG}.{m}")) for m in _MESSAGES}


_CLASSES = _build()
ListPodResourcesRequest = _CLASSES["ListPodResourcesRequest"]
ListPodResourcesResponse = _CLASSES["ListPodResourcesResponse"]
GetPodResourcesRequest = _CLASSES["GetPodResourcesRequest"]
GetPodResourcesResponse = _CLASSES["GetPodResourcesResponse"]
AllocatableResourcesRequest = _CLASSES["AllocatableResourcesRequest"]
AllocatableResourcesResponse = _CLASSES["AllocatableResourcesResponse"]
PodResources = _CLASSES["PodResources"]


def method_path(method: str) -> str:
    return f"/{PKG}.{SERVICE}/{method}"


class PodResourcesClient:
    """What the device plugin asks kubelet: ``List`` (every pod's containers and their device IDs)."""

    def __init__(self, socket_path: str = DEFAULT_SOCKET):
        self.socket_path = socket_path
        self._ch: grpc.aio.Channel | None = None

    def available(self) -> bool:
        return os.path.exists(self.socket_path)

    def _channel(self) -> grpc.aio.Channel:
        if self._ch is None:
            self._ch = grpc.aio.insecure_channel(f"unix://{self.socket_path}")
        return self._ch

    async def list(self, timeout: float = 5.0):
        call = self._channel().unary_unary(method_path("List"), request_serializer=ListPodResourcesRequest.SerializeToString,
                                           response_deserializer=ListPodResourcesResponse.FromString)
        return await call(ListPodResourcesRequest(), timeout=timeout)

    async def get(self, name: str, namespace: str, timeout: float = 5.0):
        call = self._channel().unary_unary(method_path("Get"), request_serializer=GetPodResourcesRequest.SerializeToString,
                                           response_deserializer=GetPodResourcesResponse.FromString)
        return await call(GetPodResourcesRequest(pod_name=name, pod_namespace=namespace), timeout=timeout)

    async def device_ids(self, resource: str, timeout: float = 2.0) -> dict[tuple[str, str], list[tuple[str, ...]]]:
        """{(namespace, name): [sorted device IDs of ``resource`` per container]} — kubelet's assignments."""
        try:
            resp = await self.list(timeout)
        except grpc.aio.AioRpcError:
            await self.close()  # kubelet restarted (new socket) or not up yet: reconnect on the next call
            raise
        out: dict[tuple[str, str], list[tuple[str, ...]]] = {}
        for pr in resp.pod_resources:
            per = []
            for c in pr.containers:
                ids = [i for d in c.devices if d.resource_name == resource for i in d.device_ids]
                if ids:
                    per.append(tuple(sorted(ids)))
            if per:
                out[(pr.namespace, pr.name)] = per
        return out

    async def close(self):
        if self._ch is not None:
            await self._ch.close()
            self._ch = None


class PodResourcesServer:
    """kubelet's side of the API for the kubelet stand-in: ``source()`` returns
    ``[(namespace, name, [(container, resource, [ids])])]`` of the pods kubelet currently holds devices for."""

    def __init__(self, socket_path: str, source):
        self.socket_path = socket_path
        self.source = source
        self._server: grpc.aio.Server | None = None
        self.calls = 0

    def _fill(self, pr, ns: str, name: str, containers) -> None:
        pr.namespace, pr.name = ns, name
        for cname, resource, ids in containers:
            c = pr.containers.add(name=cname)
            c.devices.add(resource_name=resource, device_ids=list(ids))

    async def List(self, request, context):
        self.calls += 1
        resp = ListPodResourcesResponse()
        for ns, name, containers in self.source():
            self._fill(resp.pod_resources.add(), ns, name, containers)
        return resp

    async def Get(self, request, context):
        self.calls += 1
        for ns, name, containers in self.source():
            if ns == request.pod_namespace and name == request.pod_name:
                resp = GetPodResourcesResponse()
                self._fill(resp.pod_resources, ns, name, containers)
                return resp
        await context.abort(grpc.StatusCode.NOT_FOUND, f"pod {request.pod_namespace}/{request.pod_name} not found")

    async def GetAllocatableResources(self, request, context):
        return AllocatableResourcesResponse()

    async def start(self):
        os.makedirs(os.path.dirname(self.socket_path) or ".", exist_ok=True)
        try:
            os.unlink(self.socket_path)
        except FileNotFoundError:
            pass
        handlers = {}
        for meth, (inp, out) in METHODS.items():
            handlers[meth] = grpc.unary_unary_rpc_method_handler(
                getattr(self, meth), request_deserializer=_CLASSES[inp].FromString,
                response_serializer=_CLASSES[out].SerializeToString)
        self._server = grpc.aio.server()
        self._server.add_generic_rpc_handlers((grpc.method_handlers_generic_handler(f"{PKG}.{SERVICE}", handlers),))
        self._server.add_insecure_port(f"unix://{self.socket_path}")
        await self._server.start()

    async def stop(self):
        if self._server is not None:
            await self._server.stop(0.2)
            self._server = None
        try:
            os.unlink(self.socket_path)
        except FileNotFoundError:
            pass
