"""Node agent: kubelet + device-plugin + container-runtime stand-in for one node (or some of its GPUs).

Where there is no kubelet (tests, the simulator, ``bench.py``), this drives
the same Allocate logic the gRPC device plugin serves to kubelet
(:mod:`.allocator`), then "starts" the pod through a runtime
(:mod:`.runtime`) and reports it Running — the tail of the reference's
sequence diagram (``docs/designs/sequence.jpg``): bound pod -> Allocate ->
``ASSIGNED=true`` -> container env -> pod runs on the chosen GPU.

It watches only pods bound to its node (``fieldSelector=spec.nodeName``) and,
with ``devices`` set, only those whose ``*_IDX`` annotation names one of its
GPUs, so one agent per GPU (one per rank in ``bench.py``) can share a node.
A pod that completes or is deleted is stopped and its slice (and CU
partition) released.
"""
from __future__ import annotations

import asyncio
import logging
import time

from ..k8s.client import ApiError, KubeClient
from ..k8s.informer import Handler, Informer, obj_key
from ..models import pod as podutil
from ..models.profile import NamingProfile
from .allocator import CU_COUNT_ANNOTATION, CUPartitioner, assigned_patch, build_response
from .devices import UNITS, Device
from .runtime import AdmissionError, admit_local

log = logging.getLogger("gsx.agent")


class NodeAgent:
    def __init__(self, client: KubeClient, node: str, devices: list[Device], profile: NamingProfile, runtime, *,
                 unit: str = "GiB", verify_each: bool = True, mount_mode: str = "isolated", report_status: bool = True,
                 workers: int = 8):
        self.client = client
        self.node = node
        self.devices = {d.index: d for d in devices}
        self.profile = profile
        self.runtime = runtime
        self.unit_bytes = UNITS[unit]
        self.verify_each = verify_each
        # a host-process launcher cannot hide device nodes: it needs host GPU indices in *_VISIBLE_DEVICES
        self.mount_mode = getattr(runtime, "mount_mode", mount_mode)
        self.report_status = report_status
        self.cus = {d.index: CUPartitioner(d.cu_count, d.xcc_count) for d in devices}
        self.pods = Informer(client, "pods", field_selector=f"spec.nodeName={node}")
        self.running: dict[str, str] = {}  # uid -> pod key
        self.inflight: set[str] = set()
        self.allocations: dict[str, dict] = {}  # uid -> container env of the last Allocate
        self.admitted = 0
        self.failed = 0
        self.bad_stamps = 0
        self.latency: list[float] = []  # bound-observed -> Running
        self._bg: set[asyncio.Task] = set()
        self._releasing: set[asyncio.Task] = set()
        self._assign_retries: dict[str, int] = {}
        self.queue: asyncio.Queue = asyncio.Queue()
        self.queued: set[str] = set()
        self.seen: dict[str, float] = {}
        # Allocate candidates (pending, ASSIGNED=false, one of our GPUs): uid -> (assume_time, key, units);
        # kept incrementally so an Allocate is O(candidates) instead of a scan + sort of every pod on the node
        self._cands: dict[str, tuple[int, str, int]] = {}
        self.workers = workers
        self.pods.add_handler(Handler(self._on_pod, lambda o, n, r: self._on_pod(n, r), self._on_delete))

    def _mine(self, pod: dict) -> bool:
        return podutil.gpu_id_from_annotation(pod, self.profile) in self.devices

    def _on_pod(self, pod: dict, raw):
        uid = podutil.meta(pod).get("uid", "")
        if podutil.is_complete(pod):
            self._cands.pop(uid, None)
            self._stop(uid)
            return
        if not podutil.is_gpushare_pod(pod, self.profile) or not self._mine(pod):
            self._cands.pop(uid, None)
            return
        ann = podutil.annotations(pod)
        if ann.get(self.profile.annotation_assigned) == "false" and podutil.phase(pod) in ("Pending", ""):
            self._cands[uid] = (podutil.assume_time(pod, self.profile), obj_key(pod),
                                podutil.gpu_mem_request(pod, self.profile))
        else:
            self._cands.pop(uid, None)
        if (ann.get(self.profile.annotation_assigned) == "false" and uid not in self.inflight
                and uid not in self.running and uid not in self.queued):
            self.queued.add(uid)
            self.seen.setdefault(uid, time.perf_counter())
            self.queue.put_nowait(obj_key(pod))

    def _on_delete(self, pod: dict, raw):
        uid = podutil.meta(pod).get("uid", "")
        self._cands.pop(uid, None)
        self._stop(uid)

    def _stop(self, uid: str):
        if uid in self.running:
            self.running.pop(uid, None)
            self._release(uid)
            for p in self.cus.values():
                p.release(uid)

    def _release(self, uid: str):
        rel = getattr(self.runtime, "release", None)
        if rel is None:
            self.runtime.stop(uid)
            return
        t = asyncio.get_running_loop().create_task(rel(uid))
        self._bg.add(t)
        self._releasing.add(t)
        t.add_done_callback(self._bg.discard)
        t.add_done_callback(self._releasing.discard)

    async def _admit_runtime(self, uid: str, dev: int, nbytes: int, cus) -> int:
        # a container runtime tears down before it starts: releases already decided (e.g. the previous
        # wave, whose device the extender has just freed) reach the runtime before this slice is carved
        if self._releasing:
            await asyncio.gather(*list(self._releasing), return_exceptions=True)
        adm = getattr(self.runtime, "admit", None)
        if adm is not None:
            if getattr(self.runtime, "wants_envs", False):  # a launcher: give it the Allocate container env
                return await adm(uid, dev, nbytes, cus, self.verify_each, envs=self.allocations.get(uid))
            return await adm(uid, dev, nbytes, cus, self.verify_each)
        return admit_local(self.runtime, uid, dev, nbytes, cus, self.verify_each)

    async def _worker(self):
        while True:
            key = await self.queue.get()
            pod = self.pods.get(key)
            if pod is None:
                continue
            self.queued.discard(podutil.meta(pod).get("uid", ""))
            await self._admit(key)

    async def _admit(self, key: str):
        """One kubelet Allocate for the container(s) of the pod behind ``key``."""
        pod = self.pods.get(key)
        uid = podutil.meta(pod).get("uid", "") if pod else ""
        try:
            if pod is None or uid in self.running or uid in self.inflight:
                return
            units = podutil.gpu_mem_request(pod, self.profile)
            # kubelet's Allocate(N ids): pick the pod exactly as the device plugin does —
            # earliest ASSUME_TIME among unassigned pods of that size (not yet claimed here)
            best = None
            for cu, (at, ck, cu_units) in self._cands.items():
                if cu_units == units and cu not in self.inflight and cu not in self.running:
                    if best is None or (at, ck) < best[0]:
                        best = ((at, ck), cu)
            chosen = self.pods.get(best[0][1]) if best is not None else None
            if chosen is None:
                return
            cuid = podutil.meta(chosen).get("uid", "")
            if cuid != uid:
                # an earlier same-size pod wins this Allocate; ours is served by the next one
                self.queued.add(uid)
                self.queue.put_nowait(key)
                key, pod, uid = obj_key(chosen), chosen, cuid
            self.inflight.add(uid)
            t0 = self.seen.get(uid, time.perf_counter())
            dev_idx = podutil.gpu_id_from_annotation(pod, self.profile)
            device = self.devices[dev_idx]
            cus = None
            want_cus = podutil.annotations(pod).get(CU_COUNT_ANNOTATION)
            if want_cus:
                cus = self.cus[dev_idx].allocate(uid, int(want_cus))
            alloc = build_response(pod, device, units, self.profile, mount_mode=self.mount_mode, cus=cus)
            try:
                await self.client.patch("pods", podutil.meta(pod)["name"], assigned_patch(pod, self.profile,
                                        alloc.annotations), podutil.meta(pod)["namespace"])
            except (ApiError, OSError) as e:
                # 409: stale copy, retry from the informer's latest version; 5xx / transport: retry with
                # capped backoff (as kubelet does); other 4xx: give up
                if isinstance(e, ApiError) and not (e.conflict or e.status >= 500):
                    raise
                if cus:
                    self.cus[dev_idx].release(uid)
                if uid not in self.queued:
                    n = self._assign_retries[uid] = self._assign_retries.get(uid, 0) + 1
                    self.queued.add(uid)
                    asyncio.get_running_loop().call_later(min(0.2, 0.001 * 2 ** min(n, 8)), self.queue.put_nowait,
                                                          key)
                return
            self.allocations[uid] = alloc.envs
            try:
                bad = await self._admit_runtime(uid, dev_idx, units * self.unit_bytes, cus)
                if bad:
                    self.bad_stamps += bad
                    raise AdmissionError(f"{bad} bad HBM stamps after admitting {key}")
            except AdmissionError as e:
                self.failed += 1
                log.error("admission of %s on GPU %d failed: %s", key, dev_idx, e)
                self._release(uid) if getattr(self.runtime, "release", None) else self.runtime.stop(uid)
                if self.report_status:
                    await self._patch_status(pod, {"phase": "Failed", "reason": "UnexpectedAdmissionError",
                                                   "message": str(e)})
                return
            self.running[uid] = key
            self.admitted += 1
            self._assign_retries.pop(uid, None)
            if self.report_status:
                await self._patch_status(pod, {"phase": "Running"})
            self.latency.append(time.perf_counter() - t0)
            self.seen.pop(uid, None)
        except Exception as e:  # noqa: BLE001
            log.exception("admit %s: %r", key, e)
        finally:
            self.inflight.discard(uid)

    async def _patch_status(self, pod: dict, status: dict):
        """kubelet's status manager: retried on 409 / 5xx / transport errors with capped backoff; 404 ends it."""
        md = podutil.meta(pod)
        for attempt in range(50):
            try:
                await self.client.patch("pods", md["name"], {"status": status}, md["namespace"], sub="status")
                return
            except ApiError as e:
                if e.not_found or not (e.conflict or e.status >= 500):
                    return
            except OSError:
                pass
            await asyncio.sleep(min(0.1, 0.0005 * 2 ** min(attempt, 8)))

    async def start(self):
        await self.pods.start()
        await self.pods.wait_synced(30)
        for i in range(self.workers):
            t = asyncio.get_running_loop().create_task(self._worker(), name=f"agent-{self.node}-{i}")
            self._bg.add(t)

    async def stop(self):
        for t in list(self._bg):
            t.cancel()
        await self.pods.stop()


async def node_devices_and_endpoints(client: KubeClient, node: str, timeout: float = 60.0):
    """Wait for the node's device inventory + runtime endpoints annotations; return (devices, endpoints)."""
    import json  # noqa: PLC0415

    from ..models.profile import NODE_DEVICE_INFO_ANNOTATION, NODE_RUNTIME_ENDPOINTS_ANNOTATION  # noqa: PLC0415

    deadline = time.monotonic() + timeout
    while True:
        try:
            n = await client.get("nodes", node)
            ann = podutil.annotations(n)
            inv = json.loads(ann.get(NODE_DEVICE_INFO_ANNOTATION, "[]"))
            eps = {int(k): v for k, v in json.loads(ann.get(NODE_RUNTIME_ENDPOINTS_ANNOTATION, "{}")).items()}
            if inv and all(d["index"] in eps for d in inv):
                devs = [Device(index=d["index"], bdf=d.get("bdf", ""), uuid=d.get("uuid", ""),
                               total_bytes=int(d.get("total_bytes", d.get("units", 0) * UNITS["GiB"])),
                               cu_count=int(d.get("cu", 256)), render_minor=int(d.get("render", -1)),
                               card_minor=int(d.get("card", -1)), partition=d.get("partition", "SPX"))
                        for d in inv]
                return devs, eps
        except ApiError:
            pass
        if time.monotonic() > deadline:
            raise TimeoutError(f"node {node} never published devices + runtime endpoints")
        await asyncio.sleep(0.05)


def main(argv=None) -> int:
    """``python -m gpushare_scheduler_extender_amd.deviceplugin.agent``: one node agent driving remote GPU runtimes."""
    import argparse  # noqa: PLC0415
    import os  # noqa: PLC0415
    import signal  # noqa: PLC0415

    from ..k8s.client import KubeConfig  # noqa: PLC0415
    from ..models.profile import get_profile  # noqa: PLC0415
    from .runtime import RemoteRuntime  # noqa: PLC0415

    ap = argparse.ArgumentParser()
    ap.add_argument("--node", required=True)
    ap.add_argument("--apiserver", default=os.environ.get("GSX_APISERVER"))
    ap.add_argument("--kubeconfig", default=os.environ.get("KUBECONFIG"))
    ap.add_argument("--profile", default="shared-gpu")
    ap.add_argument("--unit", default="GiB")
    ap.add_argument("--workers", type=int, default=32)
    ap.add_argument("--no-verify", action="store_true")
    ap.add_argument("--port-file", default="")
    a = ap.parse_args(argv)
    logging.basicConfig(level=logging.WARNING)

    async def run():
        client = KubeClient(KubeConfig.auto(a.kubeconfig, a.apiserver))
        if a.port_file:  # no listening port; signal readiness for the process harness
            with open(a.port_file + ".tmp", "w") as f:
                f.write("1")
            os.replace(a.port_file + ".tmp", a.port_file)
        devs, eps = await node_devices_and_endpoints(client, a.node, timeout=600)
        rt = RemoteRuntime(eps)
        agent = NodeAgent(client, a.node, devs, get_profile(a.profile), rt, unit=a.unit,
                          verify_each=not a.no_verify, workers=a.workers)
        await agent.start()
        from ..utils.gctune import tune  # noqa: PLC0415

        tune()
        stop = asyncio.Event()
        loop = asyncio.get_running_loop()
        for s in (signal.SIGINT, signal.SIGTERM):
            loop.add_signal_handler(s, stop.set)
        await stop.wait()
        await agent.stop()
        await rt.close()
        await client.close()

    asyncio.run(run())
    return 0


if __name__ == "__main__":
    import sys  # noqa: PLC0415

    sys.exit(main())
