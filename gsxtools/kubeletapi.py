"""The kubelet side of the device-plugin API, for the harness and the tests (not shipped in the package):
:class:`PluginClient` calls a plugin as kubelet's device manager does, :class:`FakeKubelet` serves kubelet's
Registration service on ``<dir>/kubelet.sock`` and records what registers."""
from __future__ import annotations

import asyncio
import os

import grpc

from gpushare_scheduler_extender_amd.deviceplugin import api


class PluginClient:
    """What kubelet does with a plugin (the Python kubelet stand-in and the tests)."""

    def __init__(self, socket_path: str):
        self.channel = grpc.aio.insecure_channel(f"unix://{socket_path}")

    def _call(self, meth: str):
        ic, oc, stream = api.io_types("DevicePlugin", meth)
        path = api.method_path("DevicePlugin", meth)
        if stream:
            return self.channel.unary_stream(path, request_serializer=ic.SerializeToString,
                                             response_deserializer=oc.FromString)
        return self.channel.unary_unary(path, request_serializer=ic.SerializeToString,
                                        response_deserializer=oc.FromString)

    async def options(self):
        return await self._call("GetDevicePluginOptions")(api.Empty())

    def list_and_watch(self):
        return self._call("ListAndWatch")(api.Empty())

    async def preferred(self, available: list[str], size: int, must: list[str] | None = None):
        req = api.PreferredAllocationRequest()
        req.container_requests.add(available_deviceIDs=available, must_include_deviceIDs=must or [],
                                   allocation_size=size)
        return await self._call("GetPreferredAllocation")(req)

    async def allocate(self, ids_per_container: list[list[str]]):
        req = api.AllocateRequest()
        for ids in ids_per_container:
            req.container_requests.add(devices_ids=ids)
        return await self._call("Allocate")(req)

    async def close(self):
        await self.channel.close()


class FakeKubelet:
    """Registration server on ``<dir>/kubelet.sock`` that records plugin registrations."""

    def __init__(self, socket_dir: str):
        self.socket_dir = socket_dir
        self.registrations: list = []
        self.registered = asyncio.Event()
        self._server: grpc.aio.Server | None = None

    async def Register(self, request, context):
        self.registrations.append(request)
        self.registered.set()
        return api.Empty()

    async def start(self):
        os.makedirs(self.socket_dir, exist_ok=True)
        path = os.path.join(self.socket_dir, api.KUBELET_SOCKET)
        try:
            os.unlink(path)
        except FileNotFoundError:
            pass
        ic, oc, _ = api.io_types("Registration", "Register")
        h = grpc.method_handlers_generic_handler(f"{api.PKG}.Registration", {
            "Register": grpc.unary_unary_rpc_method_handler(self.Register, request_deserializer=ic.FromString,
                                                            response_serializer=oc.SerializeToString)})
        self._server = grpc.aio.server()
        self._server.add_generic_rpc_handlers((h,))
        self._server.add_insecure_port(f"unix://{path}")
        await self._server.start()

    async def stop(self):
        if self._server is not None:
            await self._server.stop(0.2)
