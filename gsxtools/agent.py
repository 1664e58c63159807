"""Node agent: the kubelet + container-runtime stand-in for one node (or some of its GPUs).

Where there is no kubelet (tests, the simulator, ``bench.py``), this plays
kubelet against the *shipped* device plugin — the tail of the reference's
sequence diagram (``docs/designs/sequence.jpg``): pod bound to the node ->
kubelet admission -> device plugin ``Allocate`` -> ``ASSIGNED=true`` ->
container env -> the pod runs on the chosen GPU.

* Which pod an Allocate belongs to is decided by the plugin alone
  (:meth:`GpuSharePlugin.allocate_container` over :mod:`.state`); the agent
  has no matching logic of its own.  ``plugin_socket`` set: the agent is a
  gRPC client of a running plugin, exactly as kubelet's device manager is
  (ListAndWatch for the IDs, GetPreferredAllocation to pick IDs, Allocate);
  otherwise it calls an in-process :class:`GpuSharePlugin` that shares its
  pod informer.
* Admission is serial, in the order pods are seen (kubelet's
  ``HandlePodAdditions``); starting containers and reporting status run on
  ``workers`` tasks (kubelet's per-pod workers).
* If the plugin matched a different pod than the one being admitted (two
  pending pods of one size), the allocation goes to the pod the plugin
  committed — the ``gpushare.amd.com/pod`` container annotation names it —
  and the admitted pod waits for the next Allocate.  ``stats["swapped_equivalent"]`` counts swaps between
  pods with the same allocation (same GPU and partition request, which the extender binds unordered);
  ``stats["mismatch"]`` counts the others, where a real kubelet would have started a container on another
  pod's GPU (the plugin's landing-order matching, or the extender's ASSUME_TIME ordering of binds for an
  ASSUME_TIME-matching plugin, keeps this at 0).
* ``faithful=True`` plays kubelet as it is, not as the protocol would like it: the container of the pod
  being admitted starts with whatever allocation the plugin returned (no re-routing), pods are admitted one
  at a time in watch order (kubelet's apiserver config source pushes every watch event and its pod config
  merges it into an ADD of just the new pod, so ``HandlePodAdditions`` sees one pod per batch in steady state),
  or, with ``batch_window`` > 0, the pods met within the window as one batch sorted by creationTimestamp (what
  kubelet does with the pods of its initial LIST after a restart: the case reconciliation exists for), and
  kubelet's record
  of device IDs per container is served on the PodResources API (:mod:`.podresources`), which the plugin
  reconciles against (:mod:`.reconcile`).  ``/v1/allocations/<uid>`` is then the container's real env.
* A pod that completes or is deleted is stopped and its slice released; the
  plugin's own informer releases its CU partition.  A graceful deletion is ended
  the way kubelet ends it: the pod's containers stop (``stop_delay`` seconds, at
  most its grace period), its slice is released and kubelet's PodResources record
  drops it, the terminal phase is reported, and the object is deleted with grace 0
  under a UID precondition -- the apiserver never removes it on its own.

With ``devices`` set to a subset of the node's GPUs, only pods whose
``*_IDX`` annotation names one of them are admitted, so one agent per GPU
(one per rank in ``bench.py --agent rank``) can share a node.
"""
from __future__ import annotations

import asyncio
import logging
import time

from gpushare_scheduler_extender_amd.k8s.client import ApiError, KubeClient
from gpushare_scheduler_extender_amd.k8s.informer import Handler, Informer, obj_key
from gpushare_scheduler_extender_amd.models import pod as podutil
from gpushare_scheduler_extender_amd.models.profile import NamingProfile
from gpushare_scheduler_extender_amd.deviceplugin.allocator import CU_COUNT_ANNOTATION, AllocateError
from gpushare_scheduler_extender_amd.deviceplugin.devices import UNITS, Device
from gpushare_scheduler_extender_amd.deviceplugin.plugin import POD_ANNOTATION, GpuSharePlugin
from gsxtools.kubeletapi import PluginClient
from gpushare_scheduler_extender_amd.deviceplugin.runtime import AdmissionError, admit_local

log = logging.getLogger("gsx.agent")


class _Alloc:
    """What kubelet keeps from one container's Allocate response."""

    def __init__(self, uid: str, key: str, dev: int, envs: dict, cus: list[int] | None, ids: list[str]):
        self.uid, self.key, self.dev, self.envs, self.cus, self.ids = uid, key, dev, envs, cus, ids


class NodeAgent:
    def __init__(self, client: KubeClient, node: str, devices: list[Device], profile: NamingProfile, runtime, *,
                 unit: str = "GiB", verify_each: bool = True, mount_mode: str = "isolated", report_status: bool = True,
                 workers: int = 8, plugin: GpuSharePlugin | None = None, plugin_socket: str | None = None,
                 faithful: bool = False, batch_window: float = 0.0, podresources_socket: str | None = None,
                 stop_delay: float = 0.0):
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
        self.pods = Informer(client, "pods", field_selector=f"spec.nodeName={node}")
        self.pclient = PluginClient(plugin_socket) if plugin_socket else None
        self._preferred: bool | None = None  # the plugin's GetPreferredAllocation option, read on first use
        self._own_plugin = plugin is None and plugin_socket is None
        if self._own_plugin:
            plugin = GpuSharePlugin(client, node, devices, profile, unit=unit, mount_mode=self.mount_mode,
                                    informer=self.pods)
        self.plugin = plugin
        self.running: dict[str, str] = {}  # uid -> pod key
        self.allocations: dict[str, dict] = {}  # uid -> container env of the last Allocate
        self.admitted = 0
        self.failed = 0
        self.bad_stamps = 0
        self.latency: list[float] = []  # bound-observed -> Running
        self.stats = {"allocate_calls": 0, "allocate_errors": 0, "mismatch": 0, "swapped_equivalent": 0,
                      "gone_during_allocate": 0,
                      "allocate_ms_max": 0.0}
        # kubelet-side time per admission step (seconds, summed): the pod's wait for admission, the two gRPC
        # calls as kubelet sees them, the wait for a pod worker, the runtime start, the Running status patch
        self.timing = {"n": 0, "admit_queue": 0.0, "grpc_preferred": 0.0, "grpc_allocate": 0.0, "start_queue": 0.0,
                       "runtime": 0.0, "status_patch": 0.0}
        self._bg: set[asyncio.Task] = set()
        self._releasing: set[asyncio.Task] = set()
        self.stop_delay = stop_delay
        self._terminating: set[str] = set()  # uids whose graceful deletion this kubelet is ending
        self.finalized = 0
        self.admit_q: asyncio.Queue = asyncio.Queue()
        # a pod whose Allocate went to another pod is admitted next, ahead of later arrivals: it was bound before
        # them, and at the back of the queue it would push every later Allocate one pod off (a cascade a real
        # kubelet, which never re-queues, does not have)
        self.admit_first: list[str] = []
        self.start_q: asyncio.Queue = asyncio.Queue()
        self.queued: set[str] = set()
        self.claimed: set[str] = set()  # uids whose allocation is done (starting or running)
        self.seen: dict[str, float] = {}
        self.workers = workers
        self.faithful = faithful
        self.batch_window = batch_window
        self._held_starts: list | None = None
        self._last_of_batch = False
        self._enqueued: dict[str, float] = {}
        # kubelet's device-ID accounting (gRPC mode): all plugin IDs, and the ones each pod holds
        self.all_ids: list[str] = []
        self.used_ids: dict[str, list[str]] = {}
        self.id_keys: dict[str, str] = {}  # uid -> ns/name of the pod holding used_ids[uid]
        self.stopping: dict[str, tuple[str, list]] = {}  # uid -> (ns/name, IDs) of a container still stopping
        self.plugin_stats_url: str | None = None  # the plugin's /debug/state when it runs as its own process
        self.prserver = None
        if podresources_socket:
            from gpushare_scheduler_extender_amd.deviceplugin.podresources import PodResourcesServer  # noqa: PLC0415

            self.prserver = PodResourcesServer(podresources_socket, self._pod_resources)
        self.pods.add_handler(Handler(self._on_pod, lambda o, n, r: self._on_pod(n, r), self._on_delete))

    # ------------------------------------------------------------ pod watch (kubelet's pod config source)
    def _mine(self, pod: dict) -> bool:
        return podutil.gpu_id_from_annotation(pod, self.profile) in self.devices

    def _on_pod(self, pod: dict, raw):
        uid = podutil.meta(pod).get("uid", "")
        if podutil.meta(pod).get("deletionTimestamp") and not podutil.is_terminal(pod):
            if podutil.gpu_id_from_annotation(pod, self.profile) < 0 or self._mine(pod):
                self._terminate(pod)
            return
        if podutil.is_complete(pod):
            self._stop(uid)
            return
        if not podutil.is_gpushare_pod(pod, self.profile) or not self._mine(pod):
            return
        if (podutil.annotations(pod).get(self.profile.annotation_assigned) == "false" and uid not in self.claimed
                and uid not in self.queued and podutil.phase(pod) in ("Pending", "")):
            self.queued.add(uid)
            self.seen.setdefault(uid, time.perf_counter())
            self.admit_q.put_nowait(obj_key(pod))

    def _alive(self, uid: str, key: str) -> bool:
        pod = self.pods.get(key)
        return (pod is not None and podutil.meta(pod).get("uid") == uid and not podutil.is_complete(pod))

    def _on_delete(self, pod: dict, raw):
        self._stop(podutil.meta(pod).get("uid", ""))

    def _pod_resources(self):
        """kubelet's podresources view: every pod holding device IDs, one container each -- a stopped pod's until
        its runtime slice is released (the container has stopped): this kubelet's report is the truth about what
        runs (the plugin's GSX_PLUGIN_FORCE_DELETE=report)."""
        out = []
        for uid, ids in list(self.used_ids.items()) + [(u, ids) for u, (_, ids) in self.stopping.items()]:
            key = self.id_keys.get(uid, "") or self.stopping.get(uid, ("", None))[0]
            ns, _, name = key.partition("/")
            out.append((ns, name, [("main", self.profile.resource, ids)]))
        return out

    def _stop(self, uid: str):
        self.claimed.discard(uid)
        ids = self.used_ids.pop(uid, None)
        key = self.id_keys.pop(uid, None)
        if self.running.pop(uid, None) is not None:
            if ids:
                self.stopping[uid] = (key or "", ids)  # listed, and its IDs taken, until the release completes
            self._release(uid)

    def _terminate(self, pod: dict):
        uid = podutil.meta(pod).get("uid", "")
        if not uid or uid in self._terminating:
            return
        self._terminating.add(uid)
        t = asyncio.get_running_loop().create_task(self._finalize(pod))
        self._bg.add(t)
        t.add_done_callback(self._bg.discard)

    async def _finalize(self, pod: dict):
        """kubelet's end of a graceful deletion: SIGTERM the containers and give them ``stop_delay`` (at most the
        grace period) to exit, release what they held, report the terminal phase, then delete the object with grace
        0 and a UID precondition."""
        md = podutil.meta(pod)
        uid = md["uid"]
        ran = uid in self.running or uid in self.claimed
        try:
            if ran and self.stop_delay > 0:
                grace = md.get("deletionGracePeriodSeconds")
                await asyncio.sleep(min(self.stop_delay, float(grace)) if grace is not None else self.stop_delay)
            self._stop(uid)
            if self._releasing:
                await asyncio.gather(*list(self._releasing), return_exceptions=True)
            if ran and self.report_status:
                await self._patch_status(pod, {"phase": "Succeeded"})
            for attempt in range(50):
                try:
                    await self.client.delete("pods", md["name"], md["namespace"], grace_seconds=0, uid=uid)
                    break
                except ApiError as e:
                    # 404: gone already; 409: the UID precondition failed (a new pod took the name)
                    if e.not_found or e.conflict or (400 <= e.status < 500 and e.status != 429):
                        break
                except OSError:
                    pass
                await asyncio.sleep(min(0.1, 0.0005 * 2 ** min(attempt, 8)))
            self.finalized += 1
        finally:
            self._terminating.discard(uid)

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
        t.add_done_callback(lambda _t, uid=uid: self.stopping.pop(uid, None))

    # ------------------------------------------------------------ device plugin calls (kubelet's device manager)
    def _free_ids(self) -> list[str]:
        return sorted(set(self.all_ids) - {i for ids in self.used_ids.values() for i in ids}
                      - {i for _, ids in self.stopping.values() for i in ids})

    async def _allocate_grpc(self, uid: str, units: int) -> _Alloc:
        free = self._free_ids()
        # containers of deleted pods still stopping hold the IDs this pod needs: the admission waits for their
        # release (as the node agent does: nodeagent.cc, stopping_), bounded
        deadline = time.monotonic() + 30.0
        while len(free) < units and self.stopping and time.monotonic() < deadline:
            self.stats["waited_for_stopping"] = self.stats.get("waited_for_stopping", 0) + 1
            if self._releasing:
                await asyncio.wait(list(self._releasing), timeout=0.05)
            await asyncio.sleep(0.001)  # (the release's done callbacks drop its stopping entry)
            free = self._free_ids()
        if len(free) < units:
            raise AllocateError(f"kubelet: {units} {self.profile.resource} requested, {len(free)} IDs free")
        t0 = time.perf_counter()
        if self._preferred is None:  # as kubelet: ask GetPreferredAllocation only if the plugin advertises it
            self._preferred = bool((await self.pclient.options()).get_preferred_allocation_available)
        if self._preferred:
            pref = await self.pclient.preferred(free, units)
            ids = list(pref.container_responses[0].deviceIDs)
        else:
            ids = free[:units]  # kubelet's own pick without a preference
        t1 = time.perf_counter()
        r = (await self.pclient.allocate([ids])).container_responses[0]
        self.timing["grpc_preferred"] += t1 - t0
        self.timing["grpc_allocate"] += time.perf_counter() - t1
        who = r.annotations.get(POD_ANNOTATION, "")
        envs = dict(r.envs)
        cus = None
        if envs.get("GSX_CU_MASK"):
            from gpushare_scheduler_extender_amd.deviceplugin.state import parse_cu_mask  # noqa: PLC0415

            cus = parse_cu_mask(envs["GSX_CU_MASK"])
        key, _, cuid = who.rpartition("/")
        return _Alloc(cuid or uid, key, int(envs.get(self.profile.annotation_idx, "-1")), envs, cus, ids)

    async def _allocate_inproc(self, units: int) -> _Alloc:
        rec, alloc = await self.plugin.allocate_container(units)
        cus = None
        if alloc.envs.get("GSX_CU_MASK"):
            from gpushare_scheduler_extender_amd.deviceplugin.state import parse_cu_mask  # noqa: PLC0415

            cus = parse_cu_mask(alloc.envs["GSX_CU_MASK"])
        return _Alloc(rec.uid, rec.key, rec.dev, alloc.envs, cus, [])

    async def _allocate(self, uid: str, units: int) -> _Alloc:
        t0 = time.perf_counter()
        self.stats["allocate_calls"] += 1
        try:
            if self.pclient is not None:
                return await self._allocate_grpc(uid, units)
            return await self._allocate_inproc(units)
        finally:
            self.stats["allocate_ms_max"] = max(self.stats["allocate_ms_max"], 1e3 * (time.perf_counter() - t0))

    # ------------------------------------------------------------ admission (serial, like kubelet)
    async def _next_batch(self) -> list[str]:
        """kubelet's HandlePodAdditions: the pods it meets together, sorted by creationTimestamp."""
        keys = [await self.admit_q.get()]
        await asyncio.sleep(self.batch_window)
        while not self.admit_q.empty():
            keys.append(self.admit_q.get_nowait())

        def created(k):
            p = self.pods.get(k) or {}
            return (podutil.meta(p).get("creationTimestamp", ""), k)
        return sorted(keys, key=created)

    def _flush_starts(self):
        held, self._held_starts = self._held_starts, None
        for item in held or []:
            self.start_q.put_nowait(item)

    async def _admission_worker(self):
        batch: list[str] = []
        while True:
            if self.admit_first:
                key = self.admit_first.pop(0)
            elif self.batch_window > 0:
                if not batch:
                    self._flush_starts()
                    batch = await self._next_batch()
                    # kubelet admits the whole batch (every Allocate) in one pass of HandlePodAdditions; its pod
                    # workers start containers later (image pulls, runtime calls): starts wait for the batch
                    self._held_starts = []
                key = batch.pop(0)
                if not batch:
                    self._last_of_batch = True
            else:
                key = await self.admit_q.get()
            pod = self.pods.get(key)
            if pod is None:
                continue
            uid = podutil.meta(pod).get("uid", "")
            self.queued.discard(uid)
            if uid in self.claimed or podutil.is_complete(pod):
                continue
            try:
                await self._admit(key, pod, uid)
            except Exception as e:  # noqa: BLE001
                log.exception("admit %s: %r", key, e)
            finally:
                if self._last_of_batch:
                    self._last_of_batch = False
                    self._flush_starts()

    async def _admit(self, key: str, pod: dict, uid: str):
        self.timing["admit_queue"] += time.perf_counter() - self.seen.get(uid, time.perf_counter())
        conts = [podutil.container_limit(c, self.profile.resource) for c in (pod.get("spec") or {}).get("containers") or []]
        allocs: list[_Alloc] = []
        try:
            for units in (u for u in conts if u > 0):
                allocs.append(await self._allocate(uid, units))
        except (AllocateError, ApiError, OSError, Exception) as e:  # noqa: BLE001 - grpc errors included
            self.stats["allocate_errors"] += 1
            # a pod another Allocate already served, or one that went away meanwhile, needs nothing
            cur = self.pods.get(key)
            if cur is None or podutil.is_complete(cur) or podutil.meta(cur).get("uid") in self.claimed:
                return
            self.failed += 1
            log.error("Allocate for %s failed: %s", key, e)
            if self.report_status:
                await self._patch_status(cur, {"phase": "Failed", "reason": "UnexpectedAdmissionError",
                                               "message": f"Allocate failed: {e}"})
            return
        got = allocs[0]
        if self.faithful and got.uid != uid and self._alive(uid, key):
            pass  # kubelet starts the pod it admitted with whatever it got, whether or not its builder still exists
        elif not self._alive(got.uid, got.key or key):
            # the pod went away (deleted / completed) while its Allocate was in flight: kubelet's pod worker
            # drops it; its device IDs and runtime slice are never taken (the plugin's informer frees its CUs)
            self.stats["gone_during_allocate"] += 1
            if got.uid != uid and self._alive(uid, key):
                self.queued.add(uid)
                self.admit_first.append(key)
            return
        if got.uid != uid and self.faithful:
            # a real kubelet: our container starts with this allocation, whichever pod it was built for
            want_cus = podutil.annotations(pod).get(CU_COUNT_ANNOTATION, "") or "0"
            same = (got.dev == podutil.gpu_id_from_annotation(pod, self.profile) and
                    str(len(got.cus or [])) == str(int(want_cus) if want_cus.isdigit() else want_cus))
            self.stats["swapped_equivalent" if same else "mismatch"] += 1
            if not same:
                log.warning("kubelet starts %s (annotated GPU %s) with the allocation built for %s: GPU %s",
                            key, podutil.gpu_id_from_annotation(pod, self.profile), got.key, got.dev)
            got = _Alloc(uid, key, got.dev, got.envs, got.cus, got.ids)
            allocs[0] = got
        elif got.uid != uid:
            # the plugin committed an earlier pod of this size: that pod starts with this allocation, ours
            # is served by the next Allocate.  Harmless when both pods carry the same allocation (same GPU, same
            # partition request: the extender leaves such binds unordered); a real kubelet would have started
            # our container with the other pod's GPU otherwise ("mismatch")
            want_cus = podutil.annotations(pod).get(CU_COUNT_ANNOTATION, "") or "0"
            same = (got.dev == podutil.gpu_id_from_annotation(pod, self.profile) and
                    str(len(got.cus or [])) == str(int(want_cus) if want_cus.isdigit() else want_cus))
            self.stats["swapped_equivalent" if same else "mismatch"] += 1
            if not same:
                log.warning("Allocate for %s (GPU %s) was matched to %s: GPU %s, %d CUs", key,
                            podutil.gpu_id_from_annotation(pod, self.profile), got.key, got.dev, len(got.cus or []))
            self.queued.add(uid)
            self.admit_first.append(key)
            key = got.key or key
        self.claimed.add(got.uid)
        if allocs[0].ids:
            self.used_ids[got.uid] = [i for a in allocs for i in a.ids]
            self.id_keys[got.uid] = got.key or key
        self.allocations[got.uid] = got.envs
        self._enqueued[got.uid] = time.perf_counter()
        if self._held_starts is not None:
            self._held_starts.append((got.uid, key, allocs))
        else:
            self.start_q.put_nowait((got.uid, key, allocs))

    # ------------------------------------------------------------ container start (per-pod workers)
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

    async def _start_worker(self):
        while True:
            uid, key, allocs = await self.start_q.get()
            try:
                await self._start(uid, key, allocs)
            except Exception as e:  # noqa: BLE001
                log.exception("start %s: %r", key, e)

    async def _start(self, uid: str, key: str, allocs: list[_Alloc]):
        if uid not in self.claimed or not self._alive(uid, key):
            self._stop(uid)
            return  # deleted while waiting to start
        pod = self.pods.get(key)
        t0 = self.seen.pop(uid, time.perf_counter())
        ts = time.perf_counter()
        self.timing["start_queue"] += ts - self._enqueued.pop(uid, ts)
        dev = allocs[0].dev
        units = sum(int(a.envs.get(self.profile.env_container, "0") or 0) for a in allocs)
        try:
            bad = await self._admit_runtime(uid, dev, units * self.unit_bytes, allocs[0].cus)
            self.timing["runtime"] += time.perf_counter() - ts
            if bad:
                self.bad_stamps += bad
                raise AdmissionError(f"{bad} bad HBM stamps after admitting {key}")
        except AdmissionError as e:
            self.failed += 1
            log.error("admission of %s on GPU %d failed: %s", key, dev, e)
            self._release(uid) if getattr(self.runtime, "release", None) else self.runtime.stop(uid)
            if self.report_status and pod is not None:
                await self._patch_status(pod, {"phase": "Failed", "reason": "UnexpectedAdmissionError",
                                               "message": str(e)})
            return
        if uid not in self.claimed or not self._alive(uid, key):  # deleted while starting: tear it down
            self.claimed.discard(uid)
            ids = self.used_ids.pop(uid, None)
            ikey = self.id_keys.pop(uid, None)
            if ids:
                self.stopping[uid] = (ikey or key, ids)
            self._release(uid)
            return
        self.running[uid] = key
        self.admitted += 1
        tp = time.perf_counter()
        if self.report_status and pod is not None:
            await self._patch_status(pod, {"phase": "Running"})
        self.timing["status_patch"] += time.perf_counter() - tp
        self.timing["n"] += 1
        self.latency.append(time.perf_counter() - t0)

    async def _patch_status(self, pod: dict, status: dict):
        """kubelet's status manager: retried on 409 / 5xx / transport errors with capped backoff; 404 ends it."""
        md = podutil.meta(pod)
        for attempt in range(50):
            try:
                await self.client.patch("pods", md["name"], {"status": status}, md["namespace"], sub="status")
                return
            except ApiError as e:
                if e.not_found or not e.transient:
                    return
            except OSError:
                pass
            await asyncio.sleep(min(0.1, 0.0005 * 2 ** min(attempt, 8)))

    # ------------------------------------------------------------ lifecycle
    async def start(self):
        loop = asyncio.get_running_loop()
        if self.prserver is not None:
            await self.prserver.start()
        if self.pclient is not None:
            stream = self.pclient.list_and_watch()
            first = await asyncio.wait_for(stream.read(), 30)
            self.all_ids = [d.ID for d in first.devices if d.health == "Healthy"]
            stream.cancel()
        await self.pods.start()
        await self.pods.wait_synced(30)
        if self._own_plugin:
            await self.plugin.start(register=False, publish=False, serve=False)
        self._bg.add(loop.create_task(self._admission_worker(), name=f"kubelet-admit-{self.node}"))
        for i in range(self.workers):
            self._bg.add(loop.create_task(self._start_worker(), name=f"kubelet-pod-{self.node}-{i}"))

    async def stop(self):
        for t in list(self._bg):
            t.cancel()
        if self._own_plugin:
            await self.plugin.stop()
        if self.pclient is not None:
            await self.pclient.close()
        if self.prserver is not None:
            await self.prserver.stop()
        await self.pods.stop()


async def _spawn_plugin(a, sock_dir: str, devs: list[Device], prsock: str | None, box: dict):
    """Start the shipped device plugin as its own process, the way the DaemonSet runs it, and wait for it to
    register with kubelet (this stand-in's Registration service).  Returns (child, endpoint socket, stats URL)."""
    import dataclasses  # noqa: PLC0415
    import json  # noqa: PLC0415
    import os  # noqa: PLC0415
    import sys  # noqa: PLC0415

    from gsxtools.kubeletapi import FakeKubelet  # noqa: PLC0415

    kubelet = FakeKubelet(sock_dir)
    await kubelet.start()
    box["kubelet"] = kubelet
    spec = os.path.join(sock_dir, "devices.json")  # the node's inventory, as the plugin's (fake) backend sees it
    with open(spec, "w") as f:
        json.dump([dataclasses.asdict(d) for d in devs], f)
    port_file = os.path.join(sock_dir, "plugin-debug.port")
    cmd = [sys.executable, "-m", "gpushare_scheduler_extender_amd.deviceplugin", "--node", a.node,
           "--profile", a.profile, "--unit", a.unit, "--backend", "fake", "--socket-dir", sock_dir, "--no-publish",
           "--podresources-socket", "" if (a.no_reconcile or not prsock) else prsock, "--reconcile-interval", "0.5",
           "--isolation", "enforce" if a.isolation_dir else "advisory", "--debug-port", "0",
           "--debug-port-file", port_file, "--log-level", "warning"]
    if a.isolation_dir:
        cmd += ["--isolation-dir", a.isolation_dir]
    if not os.environ.get("GSX_EXTENDER_URL"):
        cmd.append("--no-extender")  # a harness run without an extender: reconciliation detects, cannot repair
    if a.apiserver:
        cmd += ["--apiserver", a.apiserver]
    if a.kubeconfig:
        cmd += ["--kubeconfig", a.kubeconfig]
    env = dict(os.environ, GSX_FAKE_DEVICES=spec)
    child = await asyncio.create_subprocess_exec(*cmd, env=env)
    box["plugin_child"] = child
    try:
        await asyncio.wait_for(kubelet.registered.wait(), 120)
    except asyncio.TimeoutError:
        raise RuntimeError("the device plugin never registered with kubelet") from None
    reg = kubelet.registrations[-1]
    deadline = time.monotonic() + 30
    while not os.path.exists(port_file):
        if time.monotonic() > deadline:
            raise RuntimeError("the device plugin published no debug port")
        await asyncio.sleep(0.02)
    with open(port_file) as f:
        url = f"http://127.0.0.1:{int(f.read().strip())}"
    return child, os.path.join(sock_dir, reg.endpoint), url


async def node_devices_and_endpoints(client: KubeClient, node: str, timeout: float = 60.0):
    """Wait for the node's device inventory + runtime endpoints annotations; return (devices, endpoints)."""
    import json  # noqa: PLC0415

    from gpushare_scheduler_extender_amd.models.profile import NODE_DEVICE_INFO_ANNOTATION, NODE_RUNTIME_ENDPOINTS_ANNOTATION  # noqa: PLC0415

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
                               share_bytes=int(d.get("share_bytes", 0)),
                               cu_count=int(d.get("cu", 256)), xcc_count=int(d.get("xcc", 8)),
                               render_minor=int(d.get("render", -1)),
                               card_minor=int(d.get("card", -1)), partition=d.get("partition", "SPX"))
                        for d in inv]
                return devs, eps
        except ApiError:
            pass
        if time.monotonic() > deadline:
            raise TimeoutError(f"node {node} never published devices + runtime endpoints")
        await asyncio.sleep(0.05)


async def serve_stats(box: dict, host: str = "127.0.0.1", port: int = 0):
    """``GET /v1/stats`` and ``GET /v1/allocations/<uid>`` (the native node agent serves the same) for the
    agent in ``box["agent"]`` (503 until it is there: the port is published before the node exists)."""
    import json  # noqa: PLC0415

    from aiohttp import web  # noqa: PLC0415

    async def stats(_):
        agent = box.get("agent")
        if agent is None:
            return web.Response(status=503, text="{}", content_type="application/json")
        lat = sorted(agent.latency)
        body = {"admitted": agent.admitted, "failed": agent.failed, "bad_stamps": agent.bad_stamps,
                "running": len(agent.running), "admit_p50_ms": round(1e3 * lat[len(lat) // 2], 3) if lat else 0.0,
                "admit_max_ms": round(1e3 * lat[-1], 3) if lat else 0.0, **agent.stats, "native": False,
                "finalized": agent.finalized,
                "plugin": ("process" if getattr(agent, "plugin_stats_url", None) else "grpc")
                if agent.pclient is not None else "inproc",
                "plugin_debug": getattr(agent, "plugin_stats_url", None)}
        n = max(1, agent.timing["n"])
        body["breakdown_ms"] = {k: round(1e3 * v / n, 4) for k, v in agent.timing.items() if k != "n"}
        pstats = pt = prec = None
        if agent.plugin is not None:
            pstats, pt = dict(agent.plugin.stats), getattr(agent.plugin, "timing", None)
            rc = getattr(agent.plugin, "reconciler", None)
            prec = dict(rc.stats) if rc is not None else None
        elif getattr(agent, "plugin_stats_url", None):  # the plugin's own process: its /debug/state
            try:
                from gpushare_scheduler_extender_amd.k8s.fasthttp import Client as HttpClient  # noqa: PLC0415

                hc = HttpClient(agent.plugin_stats_url)
                try:
                    st = json.loads((await hc.request("GET", "/debug/state")).body)
                finally:
                    await hc.close()
                pstats, pt, prec = st.get("stats"), st.get("timing"), st.get("reconcile")
            except (OSError, ValueError) as e:
                body["plugin_error"] = repr(e)
        if pstats is not None:
            body["plugin_stats"] = pstats
            if pt:
                na, npf = max(1, pt["n"]), max(1, pt["preferred_n"])
                body["plugin_breakdown_ms"] = {
                    "preferred_handler": round(1e3 * pt["preferred"] / npf, 4),
                    "allocate_handler": round(1e3 * pt["handler"] / na, 4),
                    "match": round(1e3 * pt["match"] / na, 4), "assign_patch": round(1e3 * pt["assign_patch"] / na, 4),
                    "isolate": round(1e3 * pt["isolate"] / na, 4)}
                bd = body["breakdown_ms"]
                # gRPC + serialisation as kubelet pays it = client-side call time minus the handler's own time
                body["plugin_breakdown_ms"]["grpc_overhead_preferred"] = round(
                    bd["grpc_preferred"] - body["plugin_breakdown_ms"]["preferred_handler"], 4)
                body["plugin_breakdown_ms"]["grpc_overhead_allocate"] = round(
                    bd["grpc_allocate"] - body["plugin_breakdown_ms"]["allocate_handler"], 4)
            if prec is not None:
                body["reconcile"] = prec
        body["faithful"] = agent.faithful
        return web.Response(text=json.dumps(body), content_type="application/json")

    async def allocation(request):
        agent = box.get("agent")
        env = agent.allocations.get(request.match_info["uid"]) if agent is not None else None
        if env is None:
            return web.Response(status=404, text="{}", content_type="application/json")
        return web.Response(text=json.dumps({"envs": env}), content_type="application/json")

    app = web.Application()
    app.router.add_get("/v1/stats", stats)
    app.router.add_get("/v1/allocations/{uid}", allocation)
    runner = web.AppRunner(app, access_log=None)
    await runner.setup()
    site = web.TCPSite(runner, host, port)
    await site.start()
    return runner, site._server.sockets[0].getsockname()[1]


def main(argv=None) -> int:
    """``python -m gsxtools.agent``: kubelet stand-in for one node.

    ``--plugin grpc`` (default): the shipped :class:`GpuSharePlugin` is served on a unix socket in this process
    (devices from the node's inventory annotation) and driven over gRPC like kubelet drives it;
    ``--plugin process``: the plugin runs as deployed -- its own process (``python -m
    gpushare_scheduler_extender_amd.deviceplugin``) that registers with this stand-in's Registration service on
    ``<socket-dir>/kubelet.sock`` and is then called on the endpoint it registered;
    ``--plugin inproc``: the same plugin called directly.
    """
    import argparse  # noqa: PLC0415
    import os  # noqa: PLC0415
    import signal  # noqa: PLC0415
    import tempfile  # noqa: PLC0415

    from gpushare_scheduler_extender_amd.k8s.client import KubeConfig  # noqa: PLC0415
    from gpushare_scheduler_extender_amd.models.profile import get_profile  # noqa: PLC0415
    from gpushare_scheduler_extender_amd.deviceplugin.runtime import RemoteRuntime  # noqa: PLC0415

    ap = argparse.ArgumentParser()
    ap.add_argument("--node", required=True)
    ap.add_argument("--apiserver", default=os.environ.get("GSX_APISERVER"))
    ap.add_argument("--kubeconfig", default=os.environ.get("KUBECONFIG"))
    ap.add_argument("--profile", default="shared-gpu")
    ap.add_argument("--unit", default="GiB")
    ap.add_argument("--workers", type=int, default=32)
    ap.add_argument("--plugin", default="grpc", choices=["grpc", "process", "inproc"],
                    help="grpc: the plugin served from this process; process: the shipped plugin as its own process "
                         "(python -m ...deviceplugin), found through kubelet's Registration service; inproc: called")
    ap.add_argument("--socket-dir", default="")
    ap.add_argument("--no-verify", action="store_true")
    ap.add_argument("--faithful", action="store_true",
                    help="kubelet as it is: no re-routing of a mismatched Allocate, creationTimestamp-sorted batches, "
                         "PodResources API served for the plugin's reconciliation")
    ap.add_argument("--batch-window", type=float, default=-1.0,
                    help="seconds kubelet collects pods into one creationTimestamp-sorted admission batch (default 0: "
                         "one pod per watch event, kubelet's steady state; > 0 models the multi-pod batch of "
                         "kubelet's initial LIST after a restart)")
    ap.add_argument("--no-reconcile", action="store_true", help="the plugin does not reconcile with PodResources")
    ap.add_argument("--isolation-dir", default="",
                    help="enforced isolation: the plugin writes each pod's config + HBM ledger here (and answers the "
                         "container mounts); '' = advisory env only")
    ap.add_argument("--stop-delay", type=float, default=0.0,
                    help="seconds a container takes to stop after SIGTERM on a graceful deletion (capped by the pod's "
                         "grace period); kubelet deletes the object once it has")
    ap.add_argument("--port-file", default="")
    a = ap.parse_args(argv)
    logging.basicConfig(level=logging.WARNING)

    async def run():
        client = KubeClient(KubeConfig.auto(a.kubeconfig, a.apiserver))
        box: dict = {}
        runner, port = await serve_stats(box)
        if a.port_file:  # published before the node exists: the harness starts us first
            with open(a.port_file + ".tmp", "w") as f:
                f.write(str(port))
            os.replace(a.port_file + ".tmp", a.port_file)
        devs, eps = await node_devices_and_endpoints(client, a.node, timeout=600)
        rt = RemoteRuntime(eps)
        profile = get_profile(a.profile)
        plugin = None
        sock_dir = a.socket_dir or tempfile.mkdtemp(prefix="gsx-dp-")
        prsock = os.path.join(sock_dir, "pod-resources", "kubelet.sock") if a.faithful else None
        window = max(0.0, a.batch_window)
        if a.plugin == "grpc":
            iso = None
            if a.isolation_dir:
                from gpushare_scheduler_extender_amd.deviceplugin.isolation import IsolationManager  # noqa: PLC0415

                iso = IsolationManager(a.isolation_dir)
            plugin = GpuSharePlugin(KubeClient(KubeConfig.auto(a.kubeconfig, a.apiserver)), a.node, devs, profile,
                                    unit=a.unit, socket_dir=sock_dir,
                                    podresources_socket=None if a.no_reconcile else prsock,
                                    reconcile_interval=0.5, isolation=iso)
            await plugin.start(register=False, publish=False)
            agent = NodeAgent(client, a.node, devs, profile, rt, unit=a.unit, verify_each=not a.no_verify,
                              workers=a.workers, plugin_socket=plugin.socket_path, faithful=a.faithful,
                              batch_window=window, podresources_socket=prsock, stop_delay=a.stop_delay)
        elif a.plugin == "process":
            child, endpoint, stats_url = await _spawn_plugin(a, sock_dir, devs, prsock, box)
            agent = NodeAgent(client, a.node, devs, profile, rt, unit=a.unit, verify_each=not a.no_verify,
                              workers=a.workers, plugin_socket=endpoint, faithful=a.faithful,
                              batch_window=window, podresources_socket=prsock, stop_delay=a.stop_delay)
            agent.plugin_stats_url = stats_url
        else:
            agent = NodeAgent(client, a.node, devs, profile, rt, unit=a.unit, verify_each=not a.no_verify,
                              workers=a.workers, stop_delay=a.stop_delay)
        await agent.start()
        if plugin is not None:
            agent.plugin = plugin  # for /v1/stats
        box["agent"] = agent
        from gpushare_scheduler_extender_amd.utils.gctune import tune  # noqa: PLC0415

        tune()
        stop = asyncio.Event()
        loop = asyncio.get_running_loop()
        for s in (signal.SIGINT, signal.SIGTERM):
            loop.add_signal_handler(s, stop.set)
        await stop.wait()
        await agent.stop()
        if box.get("plugin_child") is not None:
            box["plugin_child"].terminate()
            try:
                await asyncio.wait_for(box["plugin_child"].wait(), 10)
            except asyncio.TimeoutError:
                box["plugin_child"].kill()
            await box["kubelet"].stop()
        if plugin is not None:
            await plugin.stop()
            await plugin.client.close()
        await runner.cleanup()
        await rt.close()
        await client.close()

    asyncio.run(run())
    return 0


if __name__ == "__main__":
    import sys  # noqa: PLC0415

    sys.exit(main())
