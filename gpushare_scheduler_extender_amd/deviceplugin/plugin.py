"""GPU-share device plugin for kubelet (``v1beta1`` gRPC over a unix socket).

The companion the reference depends on but does not ship (SURVEY.md §2.8;
``docs/designs/designs.md:57-61,93-103``; ``docs/install.md:58-67``),
re-built for MI355X:

* **inventory** from amdsmi (``_mxdev``) or HIP, not NVML; per-device HBM in
  GiB units (MiB would be ~2.4 M fake IDs for 8 x 288 GB);
* **ListAndWatch** advertises ``<resource>`` as one fake device ID per unit
  per GPU, with NUMA topology, and re-sends with ``Unhealthy`` IDs when a
  GPU's uncorrectable-ECC count rises or amdsmi reports a reset / VM fault;
* the plugin also publishes ``<count>`` (GPU count) in node capacity and the
  per-device totals annotation the extender's ledger prefers over
  ``capacity / count`` (``pkg/cache/nodeinfo.go:34``);
* **GetPreferredAllocation** steers kubelet's fake-ID choice onto the GPU the
  extender picked, so kubelet's own per-ID accounting matches the annotation;
* **Allocate** matches the container to a pod through :mod:`.state` (earliest
  ``ASSUME_TIME`` pod of that size), commits ``ASSIGNED=true`` under a
  resourceVersion precondition and answers env + ``/dev/kfd`` + render node +
  optional CU partition (:mod:`.allocator`);
* every Allocate is **recorded** with kubelet's device IDs and **reconciled** against kubelet's own record of
  which pod holds them (PodResources ``List``, :mod:`.reconcile`): when kubelet gave a container the
  allocation built for another pod of the same size, the two pods' annotations are exchanged so the durable
  record names what each container really got (records are checkpointed next to the plugin socket);
* **enforced isolation** (optional, :mod:`.isolation`): Allocate also mounts the per-pod config, the shared
  HBM ledger and ``libgsx_isolate.so`` (via ``/etc/ld.so.preload``), which confine every HIP/HSA process of
  the container to its CU partition and HBM share;
* a **pod informer** on ``spec.nodeName=<node>`` keeps that state current: CU
  partitions and multi-container progress are released when a pod completes
  or is deleted, and rebuilt from the ``gpushare.amd.com/cu-mask`` /
  ``ASSIGNED`` annotations when the plugin starts, before it serves;
* re-registers when kubelet restarts (its socket is re-created);
* optional debug port: ``/healthz``, ``/metrics``, ``/debug/state``.
"""
from __future__ import annotations

import asyncio
import logging
import os
import time

import grpc

from ..k8s.client import ApiError, KubeClient
from ..models import pod as podutil
from ..models.profile import (NODE_ALLOCATE_ORDER_ANNOTATION, NODE_DEVICE_INFO_ANNOTATION, NODE_DEVICE_MEMORY_ANNOTATION,
                              NODE_PHYSICAL_PUBLICATION_ANNOTATION,
                              POD_CU_MASK_ANNOTATION, NamingProfile)
from . import api
from ..k8s.informer import Handler, Informer
from .allocator import AllocateError, ContainerAllocation, assigned_patch, build_response
from .devices import UNITS, Device
from .isolation import IsolationManager
from .podresources import PodResourcesClient
from .state import AllocationState, AllocRecord, PodRec

log = logging.getLogger("gsx.deviceplugin")

ID_SEP = "-_-"


def device_tag(dev: Device, width: int = 5) -> str:
    """A short, stable name for a device in its fake IDs: base32 of a hash of its UUID (else BDF, else index).

    kubelet sends every free ID of the node in each GetPreferredAllocation (8 x 287 on an MI355X node), so the ID
    length is paid per admission: ``<uuid>-_-<k>`` made that ~100 KB a pod on real GPUs, ``<tag>-_-<k>`` ~25 KB.
    Stable across restarts and re-enumeration (kubelet checkpoints the IDs its pods hold)."""
    import base64
    import hashlib

    key = (dev.uuid or dev.bdf or f"gpu{dev.index}").encode()
    return base64.b32encode(hashlib.blake2b(key, digest_size=8).digest()).decode().lower()[:width]


def fake_ids(dev: Device, units: int, tag: str | None = None) -> list[str]:
    base = tag or device_tag(dev)
    # unit numbers zero-padded to one width, so a GPU's IDs sort as they are numbered (an Allocate's IDs arrive
    # in that order and are recorded without a sort)
    w = len(str(max(units - 1, 0)))
    return [f"{base}{ID_SEP}{k:0{w}d}" for k in range(units)]


def device_tags(devices) -> dict[int, str]:
    """index -> tag for a node's devices, widened until no two collide."""
    devices = list(devices)
    for width in range(5, 14):
        tags = {d.index: device_tag(d, width) for d in devices}
        if len(set(tags.values())) == len(tags):
            return tags
    return {d.index: f"{device_tag(d, 13)}{d.index}" for d in devices}


ALLOCATE_ATTEMPTS = 8  # per container request: transient apiserver failures retried with capped backoff
INFORMER_WAIT_S = 0.02  # how long an Allocate waits for the pod event before LISTing
PHYSICAL_TTL_S = 60.0  # the extender drops a physical-use publication this plugin stopped refreshing
PHYSICAL_REFRESH_S = 15.0
# how often the plugin reads the extender's epoch (GET .../epoch, a few bytes): a restarted extender or a new leader
# knows nothing of the unaccounted use the old one was told, and holds binds to this node until it is republished
EPOCH_POLL_S = float(os.environ.get("GSX_PLUGIN_EPOCH_POLL_S", "1.0"))
SA_TOKEN_FILE = "/var/run/secrets/kubernetes.io/serviceaccount/token"
# how long an Allocate waits for a physically full GPU to drain a stopping container (env: tests scale it down)
GUARD_WAIT_S = float(os.environ.get("GSX_PLUGIN_GUARD_WAIT_S", "5.0"))
# ... and how long when the room it needs is held by deleted pods' containers kubelet still lists: they are stopping,
# and a failed Allocate fails the pod for good, so the admission waits for them instead -- bounded, since kubelet's
# admission of every other pod of the node waits behind this call (30 s, the default termination grace, let the
# kubelet-restart chaos rows time out with admissions queued: 1 of 1900 seeds)
GUARD_GONE_WAIT_S = float(os.environ.get("GSX_PLUGIN_GUARD_GONE_WAIT_S", "10.0"))
# how long an Allocate that found no candidate waits for an exchange that is about to make one (allocate_container):
# the whole call stays within the node agent stand-in's 10 s gRPC deadline (past it the pod fails all the same)
MISS_EXCHANGE_WAIT_S = float(os.environ.get("GSX_PLUGIN_MISS_EXCHANGE_WAIT_S", "5.0"))
# A pod deleted outright (a force delete) vanishes from kubelet's PodResources at once while its containers get their
# termination grace.  "grace" (default, for kubelet): what they hold stays counted -- and published to the extender --
# until spec.terminationGracePeriodSeconds + 2 s have passed (AllocState::deleted).  "report": kubelet's report is
# taken as the truth, for a kubelet that lists a container until it has stopped (the node agent stand-in): it stays
# counted, and published, while listed, and goes when it is not
FORCE_DELETE = os.environ.get("GSX_PLUGIN_FORCE_DELETE", "grace")
POD_ANNOTATION = "gpushare.amd.com/pod"  # container annotation: the pod this Allocate was matched to


class _Aborted(Exception):
    def __init__(self, code: int, details: str):
        super().__init__(details)
        self.code, self.details = code, details


class _NativeContext:
    """The slice of grpc.aio.ServicerContext the handlers use, for calls the native endpoint hands over."""

    async def abort(self, code, details=""):
        raise _Aborted(code.value[0] if isinstance(code, grpc.StatusCode) else int(code), details)


def native_grpc_available() -> tuple[bool, str]:
    """The native endpoint needs the engine module and the system's libnghttp2."""
    if os.environ.get("GSX_PLUGIN_GRPC", "native") == "grpcio":
        return False, "GSX_PLUGIN_GRPC=grpcio"
    try:
        from ..core.engine import native  # noqa: PLC0415

        return tuple(native().h2_available())
    except (ImportError, AttributeError) as e:
        return False, repr(e)

class _FeedInformer:
    """Stands in for the Python pod informer when the native endpoint's pod feed is the node's only watch: the
    Python side reads pods from the native state (:class:`.state._NativePods`) and decodes no pod event."""

    def __init__(self, plugin):
        self._plugin = plugin
        self.synced = asyncio.Event()
        self.synced.set()

    def _stat(self, k: str) -> int:
        n = self._plugin._native
        return int(n.stats().get(k, 0)) if n is not None else 0

    @property
    def relists(self) -> int:
        return self._stat("feed_relists")

    @property
    def rewatches(self) -> int:
        return self._stat("feed_rewatches")

    @property
    def events(self) -> int:
        return self._stat("feed_events")

    async def start(self):
        return None

    async def stop(self):
        return None

    async def wait_synced(self, timeout=None):
        return None

    def list(self) -> list[dict]:
        return [r.obj for r in self._plugin.state.pods.values()]


class GpuSharePlugin:
    def __init__(self, client: KubeClient, node: str, devices: list[Device], profile: NamingProfile, *,
                 unit: str = "GiB", socket_dir: str = api.DEVICE_PLUGIN_PATH, endpoint: str = "gpushare-amd.sock",
                 mount_mode: str = "isolated", health_backend: str | None = None, health_interval: float = 10.0,
                 reserve_bytes: int = 0, informer: Informer | None = None,
                 podresources_socket: str | None = None, reconcile_interval: float = 2.0,
                 isolation: IsolationManager | None = None, checkpoint: str | None = None,
                 extender: str | None = None):
        self.client = client
        # the scheduler extender: the one writer of *_IDX (reconciliation moves go through it, move_record)
        self.extender_url = extender or os.environ.get("GSX_EXTENDER_URL") or None
        self._ext = None
        self.node = node
        self.devices = {d.index: d for d in devices}
        self.profile = profile
        self.unit = unit
        self.socket_dir = socket_dir
        self.endpoint = endpoint
        self.mount_mode = mount_mode
        self.health_backend = health_backend
        self.health_interval = health_interval
        self.reserve_bytes = reserve_bytes
        self.isolation = isolation
        self._set_devices(devices)
        self.checkpoint = checkpoint if checkpoint is not None else os.path.join(socket_dir, "gsx-allocations.json")
        self.journal_path = (self.checkpoint or os.path.join(socket_dir, "gsx-allocations.json")) + ".journal"
        # early answer (default; GSX_PLUGIN_EARLY_ANSWER=0 turns it off): needs the journal next to the checkpoint
        # (the record must be durable before kubelet has the answer)
        self.early_answer = bool(self.checkpoint) and os.environ.get("GSX_PLUGIN_EARLY_ANSWER", "1") == "1"
        # GetPreferredAllocation: kubelet then asks before every Allocate, and the answer steers the pod's unit IDs
        # onto its GPU, so kubelet's per-ID accounting also bounds that GPU -- what lets an Allocate pass the
        # physical guard while the records still count containers kubelet has freed (DpCore: guard_by_ids).  With
        # one GPU every ID is on it anyway: "auto" (default) advertises it only on multi-GPU nodes, and a one-GPU
        # node's admissions skip that round trip (the reference's plugin never offered it); "1" / "0" force it
        pref = os.environ.get("GSX_PLUGIN_PREFERRED", "auto")
        self.preferred = len(self.devices) > 1 if pref == "auto" else pref == "1"
        # the records checkpoint: with early answer every Allocate is journaled first, so the checkpoint only bounds
        # how much journal a restart replays -- once a second (each one rotates the journal under the state lock
        # and writes a file: at 0.2 s it sat inside most of an 8-GPU node's busy seconds); without the journal the
        # checkpoint is the only record on disk, so it follows the Allocates closely
        self.checkpoint_interval = float(os.environ.get("GSX_PLUGIN_CHECKPOINT_S", "1.0" if self.early_answer else "0.2"))
        self._dirty = False
        self._persist_task: asyncio.Task | None = None
        # where an Allocate's time goes (plugin side, seconds summed over calls): matching, the ASSIGNED patch
        # (apiserver round trip), isolation files, the whole handler
        self.timing = {"n": 0, "match": 0.0, "assign_patch": 0.0, "isolate": 0.0, "handler": 0.0,
                       "preferred_n": 0, "preferred": 0.0}
        self._aid = 0
        self._tok = None  # (file stamp, service-account token) for the extender's endpoints
        self._phys_published: list | None = None  # the unaccounted use last published to the extender (None: none)
        self._phys_at = 0.0
        self._ext_epoch: str | None = None  # the extender epoch our last publication reached
        self.reconciler = None
        if podresources_socket:
            from .reconcile import Reconciler  # noqa: PLC0415

            self.reconciler = Reconciler(self, PodResourcesClient(podresources_socket), interval=reconcile_interval)
        # a kubelet stand-in in the same process may share its pod informer (one watch per node)
        self._own_informer = informer is None
        self.pods = informer or Informer(client, "pods", field_selector=f"spec.nodeName={node}")
        self._observed = asyncio.Event()  # set by every pod event: an Allocate waiting for its pod to arrive
        self.pods.add_handler(Handler(lambda o, raw: self._observe(o),
                                      lambda old, new, raw: self._observe(new),
                                      lambda o, raw: self.state.forget(o)))
        self._changed = asyncio.Event()
        self._version = 0
        self._stopped = False
        self._server: grpc.aio.Server | None = None
        self._native = None  # _engine.DpServer: the gRPC endpoint in native code (default)
        self._native_fd = -1  # what the loop watches for it (the serving thread's eventfd, or its epoll fd)
        self._native_serving = False
        self._feed = False  # the native endpoint's pod feed runs (the Python informer then mirrors only)
        self.grpc_impl = ""
        self._slow: set[asyncio.Task] = set()
        self._tasks: list[asyncio.Task] = []
        self.allocations = 0
        self.stats = {"allocate_ok": 0, "allocate_fail": 0, "allocate_retries": 0, "preferred": 0,
                      "registrations": 0, "refreshes": 0}
        self._debug = None

    def _observe(self, pod: dict):
        # with the native pod feed on, the native state has this event from its own watch: the Python informer
        # only keeps the Python views (the per-event native update from here cost the plugin's loop most of its
        # time at a few thousand pods/s)
        self.state.observe(pod, mirror_only=self._feed)
        self._observed.set()

    async def _await_informer(self, found, timeout: float = INFORMER_WAIT_S):
        """kubelet can call before this plugin's watch has delivered the pod it is admitting (they are separate
        processes with separate watches).  Waiting a few ms for the event is far cheaper than a full LIST."""
        deadline = time.monotonic() + timeout
        if self.state.native_views:  # the native feed applies events on its own thread: look again shortly
            while True:
                got = found()
                if got or time.monotonic() >= deadline:
                    return got
                await asyncio.sleep(0.001)
        while True:
            left = deadline - time.monotonic()
            if left <= 0:
                return found()
            self._observed.clear()
            try:
                await asyncio.wait_for(self._observed.wait(), left)
            except asyncio.TimeoutError:
                return found()
            got = found()
            if got:
                return got

    def _set_devices(self, devices: list[Device]):
        """(Re)build everything derived from the device layout: fake IDs per GPU and the allocation state."""
        self.devices = {d.index: d for d in devices}
        self.units = {d.index: d.units(self.unit, self.reserve_bytes) for d in devices}
        tags = device_tags(devices)
        self.ids = {d.index: fake_ids(d, self.units[d.index], tags[d.index]) for d in devices}
        self.id_owner = {i: d for d, ids in self.ids.items() for i in ids}
        self.state = AllocationState(self.node, self.devices, self.profile)
        self.state.core.set_linger(FORCE_DELETE != "report")
        self.state.on_drop.append(self._record_dropped)
        self.health_info: dict[int, dict] = {}
        native = getattr(self, "_native", None)
        if native is not None:
            native.set_state(self.state.core)
            self._sync_native()

    async def reload_devices(self, devices: list[Device] | None = None):
        """The node's GPUs were re-partitioned at run time (amd-smi set --compute-partition / --memory-partition):
        a new set of logical devices, so new fake IDs (ListAndWatch), new per-device totals (node annotation)
        and an allocation state rebuilt from the pods on the node."""
        if devices is None:
            from ..ops import mxdev  # noqa: PLC0415

            from .devices import apply_memory_pools  # noqa: PLC0415

            raw = await asyncio.get_running_loop().run_in_executor(None, mxdev.enumerate_devices, self.health_backend)
            devices = apply_memory_pools([Device(**d) for d in raw])
        old = sorted((d.index, d.partition, d.memory_partition) for d in self.devices.values())
        pods = self.pods.list()  # before the state is rebuilt (with the native feed, the pods live in it)
        native_views = self.state.native_views
        self._set_devices(devices)
        if native_views:
            self.state.use_native_views()
        if self.reconciler is not None:
            self.state.core.expect_owner_reports(True)
        self.state.resync(pods)
        self.stats["layout_changes"] = self.stats.get("layout_changes", 0) + 1
        log.warning("device layout changed: %s -> %s", old,
                    sorted((d.index, d.partition, d.memory_partition) for d in devices))
        self._devices_changed()
        try:
            await self.publish_node()
        except ApiError as e:
            log.warning("re-publishing node info failed: %s", e)

    # ------------------------------------------------------------ paths
    @property
    def socket_path(self) -> str:
        return os.path.join(self.socket_dir, self.endpoint)

    @property
    def kubelet_socket(self) -> str:
        return os.path.join(self.socket_dir, api.KUBELET_SOCKET)

    # ------------------------------------------------------------ device list
    def device_list(self) -> list:
        out = []
        for idx, ids in self.ids.items():
            d = self.devices[idx]
            health = api.HEALTHY if d.healthy else api.UNHEALTHY
            topo = api.TopologyInfo(nodes=[api.NUMANode(ID=d.numa_node)]) if d.numa_node >= 0 else None
            for i in ids:
                dev = api.Device(ID=i, health=health)
                if topo is not None:
                    dev.topology.CopyFrom(topo)
                out.append(dev)
        return out

    def set_health(self, index: int, healthy: bool, why: str = ""):
        d = self.devices.get(index)
        if d is None or d.healthy == healthy:
            return
        d.healthy = healthy
        log.warning("GPU %d (%s) is now %s %s", index, d.bdf, "Healthy" if healthy else "Unhealthy", why)
        self._devices_changed()

    def _devices_changed(self):
        """ListAndWatch streams (grpcio and native) send the new device list."""
        self._version += 1
        self._changed.set()
        self._sync_native()

    # ------------------------------------------------------------ native gRPC endpoint
    def _native_config(self) -> dict:
        from ..core.controller import api_dict  # noqa: PLC0415

        return {"node": self.node, "profile": {**self.profile.engine_dict(), "env_container": self.profile.env_container},
                "mount_mode": self.mount_mode, "unit_bytes": UNITS[self.unit],
                "iso_dir": str(self.isolation.host_dir) if self.isolation is not None else None,
                "guard": self.reconciler is not None, "api": api_dict(self.client.config),
                "fast": os.environ.get("GSX_PLUGIN_FAST", "1") == "1",
                # the serving thread polls this long after a pass before it sleeps (kubelet's calls come in bursts)
                "spin_us": float(os.environ.get("GSX_PLUGIN_SPIN_US", "1000")),
                "preferred": self.preferred,
                # answered Allocates reach this loop's bookkeeping at most this often (a pass takes the state lock)
                "py_event_ms": float(os.environ.get("GSX_PLUGIN_PY_EVENT_MS", "2")),
                # early answer (default; GSX_PLUGIN_EARLY_ANSWER=0 turns it off): answer a first container's Allocate
                # once its record is journaled, commit ASSIGNED=true behind it (kubelet's serial admission no longer
                # waits an apiserver round trip)
                "early_answer": self.early_answer, "journal": self.journal_path}

    def native_device(self, d: Device) -> dict:
        return {"index": d.index, "bdf": d.bdf, "cu_count": d.cu_count, "total_bytes": d.total_bytes,
                "share_bytes": d.share_bytes, "units": self.units.get(d.index, 0), "nodes": d.device_nodes(),
                "healthy": d.healthy}

    def _sync_native(self):
        if self._native is None:
            return
        self._native.set_devices([self.native_device(d) for d in self.devices.values()], self.id_owner)
        self._native.set_device_list(api.ListAndWatchResponse(devices=self.device_list()).SerializeToString())

    def _native_poll(self):
        srv = self._native
        if srv is None:
            return
        pending, events = srv.poll()
        served = [ev for ev in events if self._fast_allocated(ev)]
        if served and self.reconciler is not None:
            amb = sum(1 for ev in served if ev.get("ambiguous"))
            if amb:
                self.stats["ambiguous_allocates"] = self.stats.get("ambiguous_allocates", 0) + amb
            self.reconciler.kick(fast=amb > 0)
        self.state.flush_dropped()  # records the native pod feed dropped with their pods: isolation cleanup
        if pending:
            loop = asyncio.get_running_loop()
            for cid, method, payload in pending:
                t = loop.create_task(self._native_slow(srv, cid, method, payload))
                self._slow.add(t)
                t.add_done_callback(self._slow.discard)

    def _fast_allocated(self, ev: dict):
        """A native fast-path Allocate: what the Python handler would have done after it."""
        import json  # noqa: PLC0415

        native_views = self.state.native_views  # the native state observed the committed pod itself
        if ev.get("patch_only"):  # early answer: the commit of an Allocate answered before has landed
            if ev["pod_json"] and not native_views:
                self.state.observe(json.loads(ev["pod_json"]))
            return False
        if ev["pod_json"] and not native_views:
            self.state.observe(json.loads(ev["pod_json"]))  # the committed pod, before its watch event arrives
        if ev["iso"] and self.isolation is not None:
            self.isolation.note_prepared(ev["iso"])
        self.stats["allocate_ok"] += 1
        self.stats["allocate_native"] = self.stats.get("allocate_native", 0) + 1
        t = self.timing
        t["n"] += 1
        t["handler"] += ev["t_handler"]
        t["match"] += ev["t_match"]
        t["assign_patch"] += ev["t_patch"]
        t["isolate"] += ev["t_isolate"]
        self.persist_records()
        return True

    def _ambiguous(self, uids) -> bool:
        """kubelet may have admitted another pod than the one these Allocates were matched to: a pending pod of the
        same size waits for another GPU (a kubelet admission batch can serve the two each other's allocations).
        Then the reconciliation looks at once, so a swap is known -- and the extender told what the containers
        hold -- before either pod can be deleted.  One GPU: never (every allocation of a size is the same)."""
        if len(self.units) < 2:
            return False
        spread: dict[int, set] = {}
        for p in self.state.candidates():
            spread.setdefault(p.request, set()).add(p.dev)
        pods = self.state.pods
        for u in uids:
            p = pods.get(u)
            if p is not None and spread.get(p.request, set()) - {p.dev}:
                self.stats["ambiguous_allocates"] = self.stats.get("ambiguous_allocates", 0) + 1
                return True
        return False  # (the native fast path decides this at match time: DpEvent::ambiguous)

    async def _native_slow(self, srv, cid: int, method: str, payload: bytes):
        """A call the native fast path left to Python: the same handler grpcio would run."""
        try:
            if method == "Allocate":
                resp = await self.Allocate(api.AllocateRequest.FromString(payload), _NativeContext())
            else:
                resp = await self.GetPreferredAllocation(api.PreferredAllocationRequest.FromString(payload),
                                                         _NativeContext())
            srv.respond(cid, 0, resp.SerializeToString())
        except _Aborted as e:
            srv.respond(cid, e.code, e.details.encode())
        except Exception as e:  # noqa: BLE001 - kubelet gets an error, the plugin lives on
            log.exception("native %s slow path", method)
            srv.respond(cid, grpc.StatusCode.INTERNAL.value[0], repr(e).encode())

    def _close_native(self):
        if self._native is not None:
            try:
                asyncio.get_running_loop().remove_reader(self._native_fd)
            except RuntimeError:
                pass
            self._native.close()
            self._native = None
        self._native_serving = False
        self._feed = False

    # ------------------------------------------------------------ gRPC handlers
    async def GetDevicePluginOptions(self, request, context):
        return api.DevicePluginOptions(pre_start_required=False, get_preferred_allocation_available=self.preferred)

    async def ListAndWatch(self, request, context):
        seen = -1
        # the flag also ends the stream: before Python 3.12 asyncio.wait_for may swallow the cancellation
        # that grpc delivers when kubelet goes away
        while not self._stopped:
            if seen != self._version:
                seen = self._version
                yield api.ListAndWatchResponse(devices=self.device_list())
            self._changed.clear()
            try:
                await asyncio.wait_for(self._changed.wait(), 5.0)
            except asyncio.TimeoutError:
                pass

    async def refresh(self):
        """A fresh LIST of this node's pods into the state (the informer may lag an Allocate by a moment)."""
        lst = await self.client.list("pods", field_selector=f"spec.nodeName={self.node}")
        self.state.resync(lst.get("items") or [])
        self.stats["refreshes"] += 1

    async def GetPreferredAllocation(self, request, context):
        t0 = time.perf_counter()
        resp = api.PreferredAllocationResponse()
        for creq in request.container_requests:
            size = creq.allocation_size
            want_dev = self.state.preferred_device(size)
            if want_dev < 0 and await self._await_informer(lambda: self.state.preferred_device(size) >= 0):
                want_dev = self.state.preferred_device(size)
            if want_dev < 0:
                try:
                    await self.refresh()
                except (ApiError, OSError) as e:
                    log.warning("GetPreferredAllocation refresh: %s", e)
                want_dev = self.state.preferred_device(size)
            avail = list(creq.available_deviceIDs)
            chosen = list(creq.must_include_deviceIDs)
            pref = [i for i in avail if i not in chosen and self.id_owner.get(i) == want_dev]
            rest = [i for i in avail if i not in chosen and i not in pref]
            for i in pref + rest:
                if len(chosen) >= size:
                    break
                chosen.append(i)
            resp.container_responses.add(deviceIDs=chosen[:size])
            self.stats["preferred"] += 1
        self.timing["preferred_n"] += 1
        self.timing["preferred"] += time.perf_counter() - t0
        return resp

    # ------------------------------------------------------------ allocation records
    def _next_aid(self) -> str:
        self._aid += 1
        return f"{time.time_ns() // 1_000_000:x}-{os.getpid():x}-{self._aid}"

    def _record(self, rec: PodRec, ids, units: int, alloc: ContainerAllocation) -> AllocRecord:
        on_gpu = bool(ids) and all(self.id_owner.get(i) == rec.dev for i in ids)
        r = self.state.record(rec, ids, units, alloc.annotations.get("gpushare.amd.com/cu-mask", rec.cu_mask),
                              self._next_aid(), time.time(), alloc.iso, on_gpu=on_gpu)
        self.persist_records()
        return r

    def _record_dropped(self, r: AllocRecord):
        if self.isolation is not None and r.iso and not any(o.iso == r.iso for o in self.state.records.values()):
            self.isolation.release(r.iso)

    def persist_records(self):
        """Checkpoint of the Allocate records (a restarted plugin still knows what each set of IDs was): written
        by a background task at most every ``checkpoint_interval`` seconds, not on the Allocate path (a JSON dump
        + rename per Allocate cost ~1 ms of the plugin's ~2.8 ms admission on MI355X, profiles/r03_gpu)."""
        self._dirty = True
        if self._persist_task is None or self._persist_task.done():
            try:
                loop = asyncio.get_running_loop()
            except RuntimeError:
                self._write_checkpoint()
                return
            self._persist_task = loop.create_task(self._persist_later())

    async def _persist_later(self):
        await asyncio.sleep(self.checkpoint_interval)
        self._write_checkpoint()

    def _write_checkpoint(self):
        """The records snapshot, then the journal generations it covers go.  With the native endpoint journaling
        (early answer) the snapshot and the journal's rotation to ``<journal>.old`` are one step under the state
        lock; ``.old`` is deleted only once the checkpoint is in place, so a failed write or a crash in between
        loses no journaled record (the next start reads checkpoint, ``.old`` and journal)."""
        if not self.checkpoint or not self._dirty:
            return
        self._dirty = False
        import json  # noqa: PLC0415

        tmp = self.checkpoint + ".tmp"
        journaling = self._native is not None and self._native.stats().get("journaling", False)
        rotated = False
        if journaling:
            records, rotated, err = self._native.journal_checkpoint()
            if not rotated:
                log.warning("rotating the Allocate journal %s: %s (it keeps every line)", self.journal_path, err)
        else:
            records = [r.to_dict() for r in self.state.records.values()]
        try:
            with open(tmp, "w") as f:
                json.dump({"node": self.node, "records": records}, f)
            os.replace(tmp, self.checkpoint)
        except OSError as e:
            self._dirty = True  # the next pass tries again; the journal generations stay
            log.warning("checkpoint %s: %s", self.checkpoint, e)
            return
        # the checkpoint holds every record the journal generations held
        old = [self.journal_path + ".old"] if (rotated or not journaling) else []
        if not journaling:
            old.append(self.journal_path)  # nobody appends to it: lines from an earlier run, now checkpointed
        for path in old:
            try:
                os.unlink(path)
            except FileNotFoundError:
                pass
            except OSError as e:
                log.warning("removing %s: %s", path, e)

    def load_records(self) -> int:
        """Records of pods that are still on this node (after the informer's first sync): the checkpoint, then the
        early-answer journal of Allocates made after it."""
        import json  # noqa: PLC0415

        recs: list[dict] = []
        try:
            with open(self.checkpoint) as f:
                recs += list(json.load(f).get("records") or [])
        except (OSError, ValueError):
            pass
        journal_lines = 0
        # .old: a generation a checkpoint was about to cover when the plugin went away (plugin._write_checkpoint)
        for path in (self.journal_path + ".old", self.journal_path):
            try:
                with open(path) as f:
                    for line in f:
                        # a mapped journal is zero-padded past its lines: a generation appended after padding that
                        # was never trimmed starts with NULs (native dpcore trims .old first; this reads either)
                        line = line.strip("\x00")
                        if not line.strip():
                            continue
                        try:
                            recs.append(json.loads(line))
                            journal_lines += 1
                        except ValueError:
                            pass  # a torn last line
            except OSError:
                pass
        n, seen = 0, set()
        self._journaled = []
        for d in recs:
            r = AllocRecord.from_dict(d)
            if r.aid in seen or r.holder not in self.state.pods:
                continue
            seen.add(r.aid)
            self.state.restore_record(r)
            # whatever the early-answer setting was or is: a record is written once kubelet has (or is about to
            # have) the answer, so a pod it names that still reads ASSIGNED!=true has a commit that never landed
            self._journaled.append(r)
            n += 1
        if journal_lines:
            self.persist_records()  # the first checkpoint supersedes the journal lines read here
        return n

    async def commit_unlanded(self) -> int:
        """Early answer: an Allocate was answered before its ASSIGNED patch landed, and the plugin went away in between.
        The pod holds a journaled record but still reads ASSIGNED=false.  Claim it and land the commit before any
        Allocate is served, so it is never matched again; if the patch fails the claim stays."""
        n, late = 0, []
        for r in getattr(self, "_journaled", []):
            p = self.state.pods.get(r.uid)
            if p is None or p.assigned == "true" or not p.pending:
                continue
            self.state.inflight.add(p.uid)
            if await self._land_commit(p, r):
                n += 1
            else:
                late.append((p, r))
        self._journaled = []
        if late:  # the pods stay claimed; their commits are retried with backoff while the pods exist
            t = asyncio.get_running_loop().create_task(self._land_late(late))
            self._tasks.append(t)
        self.stats["commits_after_restart"] = self.stats.get("commits_after_restart", 0) + n
        return n

    async def _land_commit(self, p: PodRec, r: AllocRecord) -> bool:
        """One attempt at an answered Allocate's ASSIGNED commit, guarded by the pod's UID (never lands on a pod
        re-created under the name).  True when there is nothing left to do (landed, or the pod went away)."""
        ann = {self.profile.annotation_assigned: "true"}
        if r.cu_mask:
            ann[POD_CU_MASK_ANNOTATION] = r.cu_mask
        try:
            pod = await self.client.patch("pods", p.name, {"metadata": {"uid": p.uid, "annotations": ann}},
                                          p.namespace)
        except ApiError as e:
            # gone, or re-created under its name (kube-apiserver refuses the patch's changed metadata.uid: 422)
            if e.status == 404 or (e.status == 422 and "metadata.uid" in str(e)) or (
                    e.status == 409 and "UID in precondition" in str(e)):
                self.state.inflight.discard(p.uid)
                return True
            log.warning("committing the answered Allocate of %s: %s (the pod stays claimed; retrying)", p.key, e)
            return False
        except OSError as e:
            log.warning("committing the answered Allocate of %s: %s (the pod stays claimed; retrying)", p.key, e)
            return False
        self.state.inflight.discard(p.uid)
        self.state.observe(pod)
        return True

    async def _land_late(self, todo: list):
        delay = 0.01
        while todo and not self._stopped:
            await asyncio.sleep(delay)
            delay = min(2.0, delay * 2)
            still = []
            for p, r in todo:
                cur = self.state.pods.get(p.uid)
                if cur is None:
                    self.state.inflight.discard(p.uid)
                    continue
                if await self._land_commit(cur, r):
                    self.stats["commits_after_restart"] = self.stats.get("commits_after_restart", 0) + 1
                else:
                    still.append((cur, r))
            todo = still

    async def allocate_container(self, units: int, ids=()) -> tuple[PodRec, ContainerAllocation]:
        """Match one container request of ``units`` to its pod and build its allocation.

        For the pod's first container this commits ``ASSIGNED=true`` (with the pod's resourceVersion as a
        precondition, so two Allocates never claim one pod).  A 409 (the pod changed since we saw it) or an
        apiserver 5xx / transport error is retried from fresh state with capped backoff: failing Allocate makes
        kubelet reject the pod (UnexpectedAdmissionError) over a transient apiserver hiccup."""
        refreshed = False
        for attempt in range(ALLOCATE_ATTEMPTS):
            tm = time.perf_counter()
            rec, whole = self.state.match(units)
            self.timing["match"] += time.perf_counter() - tm
            if rec is None and not refreshed:
                m = await self._await_informer(lambda: self.state.match(units)[0] is not None)
                rec, whole = self.state.match(units) if m else (None, False)
            if rec is None and not refreshed:
                await self.refresh()
                refreshed = True
                rec, whole = self.state.match(units)
            if rec is None and self.state.unannotated(units):
                rec, whole = await self._wait_for_annotations(units)
            if rec is None and self.reconciler is not None and self.reconciler.pr.available():
                # kubelet may have started another pod's container with this pod's allocation (a swap the
                # reconciliation has not repaired yet): repair now, the exchange makes this pod a candidate again
                self.stats["reconcile_on_miss"] = self.stats.get("reconcile_on_miss", 0) + 1
                for k in range(8):
                    await self._reconcile_now(urgent=True)
                    rec, whole = self.state.match(units)
                    if rec is not None:
                        break
                    await asyncio.sleep(0.02 * (k + 1))
                # a pod of this size an exchange is about to make a candidate again: its hold is cleared once the
                # extender's informer has seen the exchange land, and a loaded extender's informer lags by seconds
                # (kubelet-restart chaos rows on MI355X: the 0.7 s above ran out).  Waiting fails no pod; bounded,
                # since kubelet admits serially
                deadline = time.monotonic() + MISS_EXCHANGE_WAIT_S
                while rec is None and time.monotonic() < deadline and self._exchange_due(units):
                    self.stats["miss_exchange_waits"] = self.stats.get("miss_exchange_waits", 0) + 1
                    await asyncio.sleep(0.1)
                    await self._reconcile_now(urgent=True)
                    rec, whole = self.state.match(units)
            if rec is None:
                keys = {p.uid: p.key for p in self.state.pods.values()}
                recs = self.state.records.values()
                busy = self.reconciler.busy() if self.reconciler is not None else set()

                def why(p):  # the records naming this pod, and who really holds them
                    held = [f"{keys.get(r.holder, r.holder[:8])}@gpu{r.dev}" for r in recs if r.uid == p.uid]
                    return f"{p.key}:{p.phase}:{p.assigned}:gpu{p.dev}" + (f"[{','.join(held)}]" if held else "") + (
                        "*" if p.uid in busy else "")
                same = [why(p) for p in self.state.pods.values() if p.request == units]
                raise AllocateError(f"no pending pod on {self.node} requests {units} {self.profile.resource} "
                                    f"with {self.profile.annotation_assigned}=false (pods of that size: "
                                    f"{', '.join(same[:8]) or 'none'})")
            device = self.devices.get(rec.dev)
            if device is None:
                raise AllocateError(f"pod {rec.key} annotated with GPU {rec.dev}, not on this node")
            cp = self.state.cus.get(rec.dev)
            had_cus = cp is not None and cp.holds(rec.uid)
            if rec.assigned == "true":  # a later container of a pod whose first container committed
                cus = self.state.claim_cus(rec)
                alloc = build_response(rec.obj, device, units, self.profile, mount_mode=self.mount_mode, cus=cus)
                self._isolate(rec, device, cus, alloc)
                self.state.later_container_allocated(rec, units)
                self._record(rec, ids, units, alloc)
                return rec, alloc
            if self.reconciler is not None:
                rec = await self._physical_guard(rec, units, ids)
                if rec is None:  # the repair it ran made the pod no candidate (it was served meanwhile): re-match
                    refreshed = True
                    continue
                device = self.devices[rec.dev]
                cp = self.state.cus.get(rec.dev)
                had_cus = cp is not None and cp.holds(rec.uid)
            self.state.inflight.add(rec.uid)
            try:
                cus = self.state.claim_cus(rec)
                alloc = build_response(rec.obj, device, units, self.profile, mount_mode=self.mount_mode, cus=cus)
                ti = time.perf_counter()
                self._isolate(rec, device, cus, alloc)
                tp = time.perf_counter()
                self.timing["isolate"] += tp - ti
                try:
                    pod = await self.client.patch("pods", rec.name, assigned_patch(rec.obj, self.profile,
                                                                                    alloc.annotations),
                                                  rec.namespace)
                except (ApiError, OSError) as e:
                    if cus and not had_cus:
                        cp.release(rec.uid)
                    # a conflict, a 5xx, or a 429 the client's own Retry-After retries did not get through; or the
                    # matched pod is gone (deleted after this view matched it): kubelet's pod is another one, so
                    # re-match rather than fail it (tests/interleave.py: swap-graceful seed 132)
                    gone = isinstance(e, ApiError) and e.not_found
                    if gone:
                        self.state.forget(rec.obj)
                    transient = not isinstance(e, ApiError) or e.transient or gone
                    if not transient or attempt == ALLOCATE_ATTEMPTS - 1:
                        raise AllocateError(f"marking {rec.key} assigned failed: {e}") from e
                    self.stats["allocate_retries"] += 1
                    await asyncio.sleep(min(0.2, 0.005 * 2 ** attempt))
                    await self.refresh()
                    refreshed = True
                    continue
            finally:
                self.state.inflight.discard(rec.uid)
            self.timing["assign_patch"] += time.perf_counter() - tp
            self.state.observe(pod)
            self.state.first_container_committed(rec, units, whole)
            self._record(rec, ids, units, alloc)
            return rec, alloc
        raise AllocateError("unreachable")

    def _exchange_due(self, units: int) -> bool:
        """Some unstarted pod requesting ``units`` is in an unfinished exchange, or another pod's container holds the
        allocation built for it (an exchange the next pass makes): it will be an Allocate candidate again."""
        busy = self.reconciler.busy() if self.reconciler is not None else set()
        pods = [p for p in self.state.pods.values() if p.request == units and p.pending and not p.complete]
        if any(p.uid in busy for p in pods):
            return True
        held_for = {r.uid for r in self.state.records.values() if r.holder and r.holder != r.uid}
        return any(p.uid in held_for and p.assigned == "true" for p in pods)

    async def _reconcile_now(self, urgent: bool = False):
        try:
            await self.reconciler.run_once(urgent)
        except Exception as e:  # noqa: BLE001 - an apiserver error: the caller retries
            log.debug("reconcile pass: %r", e)

    def _physical_used(self, dev: int) -> int:
        """Units kubelet has handed out on ``dev`` (the Allocate records of live pods: what really runs there)."""
        return self.state.core.physical_used(dev)

    def _gone_used(self, dev: int) -> int:
        """Units on ``dev`` held by containers of deleted pods: records kubelet still lists, and the allocations of
        force-deleted pods that linger for their termination grace (AllocState::deleted)."""
        from .reconcile import GONE  # noqa: PLC0415 - only with a reconciler, as the guard itself

        return (sum(r.units for r in self.state.records.values() if r.dev == dev and r.owner.startswith(GONE))
                + self.state.core.lingering(dev))

    def _annotated_used(self, dev: int, skip: str = "") -> int:
        """Units the pod annotations put on ``dev`` (what the extender's ledger accounts): the live pods, and the
        terminating ones -- the extender keeps their share charged until their objects are gone."""
        return (sum(p.request for p in self.state.pods.values() if p.dev == dev and p.uid != skip and not p.complete)
                + self.state.core.terminating_used(dev))

    def _kubelet_bounds(self, dev: int, ids) -> bool:
        """kubelet's own per-ID accounting bounds GPU ``dev``: this Allocate's IDs all lie on it and so do those of
        every recorded allocation whose container runs on ``dev`` (GetPreferredAllocation steered them), so every
        unit there holds one of ``dev``'s IDs and kubelet cannot have handed out more than it has, whatever records
        of containers it has since freed still say (native twin: dpcore.cc allocate)."""
        return (bool(ids) and all(self.id_owner.get(i) == dev for i in ids)
                and self.state.core.off_gpu_records_on(dev) == 0)

    async def _physical_guard(self, rec: PodRec, units: int, ids=()) -> PodRec | None:
        """Never start a container on a GPU that is physically full.  The extender placed ``rec`` by the
        annotations; after a swap kubelet has not told us about yet, a deletion can free the GPU the annotation
        names while the container that really ran there lives on.  Repair the records first; if the GPU is still
        full, move ``rec`` (not yet started) to a GPU of this node with room by both counts, hold-protected like a
        reconciliation exchange; with no such GPU, keep waiting (up to GUARD_GONE_WAIT_S) while containers of deleted
        pods hold the room, then fail the Allocate rather than over-commit."""
        cap = self.units.get(rec.dev, 0)
        if self._physical_used(rec.dev) + units <= cap or self._kubelet_bounds(rec.dev, ids):
            return rec
        self.stats["physical_guard"] = self.stats.get("physical_guard", 0) + 1
        # a deleted pod's container may still be stopping (its record goes once kubelet stops listing its IDs):
        # give it GUARD_WAIT_S before moving the pod or failing the Allocate
        t0 = time.monotonic()
        deadline, gone_deadline = t0 + GUARD_WAIT_S, t0 + GUARD_GONE_WAIT_S
        delay = 0.02
        refused = None
        while True:
            await self._reconcile_now(urgent=True)
            rec = self.state.fresh(self.state.pods.get(rec.uid))
            if (rec is None or rec.assigned != "false" or not rec.pending or rec.uid in self.state.inflight
                    or self.reconciler.exchange_pending(rec)):
                # served meanwhile, or an exchange the pass began is about to give it other fields: re-match
                return None
            used = self._physical_used(rec.dev)
            if used + units <= self.units.get(rec.dev, 0):
                return rec
            now = time.monotonic()
            # room will come, here or on another GPU, once containers of deleted pods have stopped
            stopping = (used - self._gone_used(rec.dev) + units <= self.units.get(rec.dev, 0)
                        or self.room_for(rec, units, soon=True) >= 0)
            if now >= deadline:
                # past the short wait: move the pod if another GPU has room; else keep waiting only for containers
                # that will stop -- deleted pods' (kubelet's view of a deletion can lag the plugin's by seconds
                # behind a dropped watch; a force-deleted pod's containers linger for their grace)
                best = self.room_for(rec, units) if rec.uid not in self.reconciler.busy() else -1
                if best >= 0:
                    log.warning("moving %s from GPU %d (physically full) to GPU %d before it starts", rec.key,
                                rec.dev, best)
                    try:
                        return await self.move_unstarted(rec, best)
                    except ApiError as e:
                        # the extender's ledger disagrees (a bind or publication this view has not seen), or its
                        # apiserver write failed: look again
                        refused = e
                        if not e.transient or now >= gone_deadline:
                            raise AllocateError(f"moving {rec.key} off a physically full GPU failed: {e}") from e
                elif now >= gone_deadline or not stopping:
                    break
                self.stats["physical_guard_gone_waits"] = self.stats.get("physical_guard_gone_waits", 0) + 1
            await asyncio.sleep(delay)
            delay = min(0.2, delay * 2)
        self.stats["physical_guard_failed"] = self.stats.get("physical_guard_failed", 0) + 1
        if rec.uid in self.reconciler.busy():
            raise AllocateError(f"GPU {rec.dev} of {self.node} is physically full and {rec.key} is in an unfinished "
                                f"reconciliation exchange")
        keys = {p.uid: p.key for p in self.state.pods.values()}
        held = [f"{keys.get(r.holder, r.holder)}:{r.units}" for r in self.state.records.values() if r.dev == rec.dev]
        raise AllocateError(f"GPU {rec.dev} of {self.node} is physically full ({self._physical_used(rec.dev)} of "
                            f"{self.units.get(rec.dev)} {self.unit} handed out: {', '.join(held)}) and no other "
                            f"GPU has room for {rec.key}" + (f" (last move refused: {refused})" if refused else ""))

    def room_for(self, rec: PodRec, units: int, exclude: int = -1, soon: bool = False) -> int:
        """Best-fit healthy GPU other than ``rec``'s (and ``exclude``) with room for ``rec`` by both counts: what the
        extender's ledger holds there -- the annotations plus the unaccounted use this plugin publishes (containers
        the annotations do not charge there, deleted pods' stopping ones included) -- and the Allocate records (what
        really runs).  ``soon``: as it will be once deleted pods' containers have stopped.  -1 if none."""
        extra = self.unaccounted() or []
        core = self.state.core
        best, best_free = -1, None
        for d, cap_d in self.units.items():
            if d in (rec.dev, exclude) or not self.devices[d].healthy:
                continue
            ex = extra[d] if d < len(extra) else 0
            phys = self._physical_used(d)
            if soon:
                ex = max(0, ex - core.gone_held(d) - core.lingering(d))
                phys -= self._gone_used(d)
            free_ann = cap_d - self._annotated_used(d, skip=rec.uid) - ex
            if free_ann >= rec.request and cap_d - phys >= units and (best < 0 or free_ann < best_free):
                best, best_free = d, free_ann
        return best

    async def move_unstarted(self, rec: PodRec, dev: int) -> PodRec:
        """Re-place a bound pod none of whose containers started onto GPU ``dev`` of this node, through the extender
        (it checks the room against its ledger and charges both GPUs until its informer sees the move).  Raises
        ApiError."""
        pod = await self.move_record(rec, dev, {})
        self.state.observe(pod)
        self.stats["moved_before_start"] = self.stats.get("moved_before_start", 0) + 1
        return self.state.pods.get(rec.uid, rec)

    async def move_record(self, rec: PodRec, to: int, annotations: dict, partner: str = "") -> dict:
        """Rewrite ``rec``'s allocation record (``*_IDX`` = ``to`` and the given allocation annotations, ``None``
        removing one) through the scheduler extender's ``POST /gpushare-scheduler/move``: the extender is the one
        writer of ``*_IDX`` (the reference's node lock, ``pkg/cache/nodeinfo.go:139-168``), so a move can never race
        a bind onto the same GPU.  The write is guarded by ``rec``'s resourceVersion; 409 when the extender refuses
        it (no room, stale view) or the pod changed.  Returns the updated pod.  Raises ApiError."""
        import json  # noqa: PLC0415

        if not self.extender_url:
            raise ApiError(409, "Conflict", "no scheduler extender configured (--extender / GSX_EXTENDER_URL): "
                                            "allocation records are written by the extender only")
        # the pod's container already runs on `to` (it holds an allocation there): the extender's physical account
        # (the use this plugin publishes) has it, only the annotations grow
        physical_on_to = any(r.owner == rec.uid and r.dev == int(to) for r in self.state.records.values())
        body = {"namespace": rec.namespace, "name": rec.name, "uid": rec.uid, "node": self.node,
                "resourceVersion": rec.rv, "from": rec.dev, "to": int(to), "partner": partner,
                "physical_on_to": physical_on_to, "annotations": annotations}
        r = await self._extender_post("/gpushare-scheduler/move", body)
        try:
            out = json.loads(r.body or b"{}")
        except ValueError:
            out = {}
        if r.status != 200:
            self.stats["moves_refused"] = self.stats.get("moves_refused", 0) + 1
            raise ApiError(r.status, "Conflict" if r.status == 409 else "", out.get("Error") or r.body[:200])
        self.stats["moves"] = self.stats.get("moves", 0) + 1
        if out.get("epoch") and out["epoch"] != self._ext_epoch and self.publishes_physical:
            self._schedule_republish()
        return out["pod"]

    @property
    def publishes_physical(self) -> bool:
        """This plugin tells the extender its unaccounted GPU use (it reconciles with kubelet's PodResources and
        knows the extender): advertised on the node (NODE_PHYSICAL_PUBLICATION_ANNOTATION)."""
        return bool(self.extender_url) and self.reconciler is not None

    def _schedule_republish(self):
        t = asyncio.get_running_loop().create_task(self.publish_physical(force=True))
        self._slow.add(t)
        t.add_done_callback(self._slow.discard)

    async def check_epoch(self) -> bool:
        """Read the extender's epoch; when it is not the one our last publication reached (a restarted extender,
        a new leader), publish again at once -- that extender holds binds to this node until then.  True when the
        publication is current."""
        import json  # noqa: PLC0415

        try:
            r = await self._extender_request("GET", "/gpushare-scheduler/epoch")
            d = json.loads(r.body or b"{}") if r.status == 200 else {}
        except (ApiError, ValueError):
            return False
        epoch = d.get("epoch")
        if not epoch or not d.get("leader", True):
            return False
        if epoch == self._ext_epoch:
            return True
        self.stats["epoch_changes"] = self.stats.get("epoch_changes", 0) + 1
        log.info("scheduler extender epoch %s -> %s: republishing the unaccounted GPU use", self._ext_epoch, epoch)
        return await self.publish_physical(force=True)

    async def _epoch_loop(self):
        while not self._stopped:
            try:
                await self.check_epoch()
            except asyncio.CancelledError:
                raise
            except Exception as e:  # noqa: BLE001 - the loop outlives a bad poll
                log.debug("extender epoch poll: %r", e)
            await asyncio.sleep(EPOCH_POLL_S)

    async def _extender_post(self, path: str, body: dict):
        import json  # noqa: PLC0415

        return await self._extender_request("POST", path, json.dumps(body).encode())

    async def _extender_request(self, method: str, path: str, data: bytes | None = None):
        """A request to the scheduler extender's device-plugin endpoints, with this plugin's service-account token
        when it has one (the extender reviews it: ``--plugin-auth tokenreview``).  Raises ApiError(503) on
        transport."""
        if self._ext is None:
            from ..k8s.fasthttp import Client as HttpClient  # noqa: PLC0415

            self._ext = HttpClient(self.extender_url)
        headers = None
        tok = self._extender_token()
        if tok:
            headers = {"Authorization": f"Bearer {tok}"}
        try:
            return await self._ext.request(method, path, data, content_type="application/json" if data else None,
                                           headers=headers)
        except OSError as e:
            raise ApiError(503, "ServiceUnavailable", f"scheduler extender: {e}") from e

    def _extender_token(self) -> str:
        """The plugin's service-account token (re-read when the kubelet rotates the projected file)."""
        path = os.environ.get("GSX_PLUGIN_TOKEN_FILE", SA_TOKEN_FILE)
        try:
            st = os.stat(path)
        except OSError:
            return ""
        if self._tok is None or self._tok[0] != (st.st_mtime_ns, st.st_size):
            try:
                with open(path) as f:
                    self._tok = ((st.st_mtime_ns, st.st_size), f.read().strip())
            except OSError:
                return ""
        return self._tok[1]

    # ------------------------------------------------------------ physical use -> the extender
    def unaccounted(self) -> list[int] | None:
        """Per GPU, the units kubelet's containers hold there that the annotations do not charge there: a record
        kubelet reports held by another, live pod than the one it was built for, and that pod is annotated with
        another GPU (a swap the exchange has not repaired); and what the containers of deleted pods still hold
        (listed by kubelet, or lingering for their grace).  None when every container is charged where it runs (the
        extender then uses the annotations alone).  On a one-GPU node only deleted pods' containers count: whoever
        holds an allocation there is annotated with that GPU too."""
        if not self.units:
            return None
        pods = self.state.pods
        out = [0] * (max(self.units) + 1)
        found = False
        for r in (self.state.records.values() if len(self.units) > 1 else ()):
            if not 0 <= r.dev < len(out) or not r.owner or r.owner == r.uid:
                # not reported by kubelet yet, or held by the pod it was built for: the annotations charge it (a
                # pod deleted before the first report: its container is stopping, as the extender assumes).  (Also
                # charging a pod's own record while its annotation names another GPU -- records exchanged, the
                # re-annotation refused -- double-charged both GPUs of every exchange in flight: kubelet-restart
                # chaos seeds then stalled with binds refused, 4 of 380 failing vs 0-2)
                continue
            if r.owner.startswith("~"):
                continue  # a holder whose object is gone: counted below (gone_held)
            p = pods.get(r.owner)
            if p is not None and not p.complete and p.dev != r.dev:
                out[r.dev] += r.units
                found = True
        # deleted pods' containers: those kubelet still lists, and (force deletes) those given their termination
        # grace although kubelet no longer lists them -- the extender freed their share when the objects went
        # (AllocState::gone_held / deleted)
        for d in range(len(out)):
            n = self.state.core.gone_held(d) + self.state.core.lingering(d)
            if n:
                out[d] += n
                found = True
        return out if found else None

    async def publish_physical(self, force: bool = False) -> bool:
        """Tell the extender what kubelet's containers hold where the annotations do not charge it
        (``unaccounted``), and withdraw it once they do: the extender charges it on top of the annotations, so a
        deleted pod whose allocation another pod's container holds (a kubelet batch swap not yet repaired) never
        frees that GPU for the next bind.  Refreshed while it lasts (the extender expires an unrefreshed
        publication).  False if the extender could not be told."""
        if not self.extender_url or not self.units:
            return True
        extra = self.unaccounted()
        now = time.monotonic()
        due = extra is not None and now - self._phys_at > PHYSICAL_REFRESH_S
        if not force and not due and extra == self._phys_published:
            return True
        try:
            r = await self._extender_post("/gpushare-scheduler/physical",
                                          {"node": self.node, "unaccounted": extra, "ttl": int(PHYSICAL_TTL_S)})
        except ApiError as e:
            log.warning("publishing the unaccounted GPU use to the extender failed: %s", e)
            return False
        if r.status != 200:
            log.warning("the extender refused the unaccounted GPU use: %s %s", r.status, r.body[:200])
            return False
        self._phys_published, self._phys_at = extra, now
        try:
            import json  # noqa: PLC0415

            self._ext_epoch = json.loads(r.body or b"{}").get("epoch") or self._ext_epoch
        except ValueError:
            pass
        self.stats["physical_published"] = self.stats.get("physical_published", 0) + 1
        log.debug("published unaccounted GPU use %s", extra)
        return True

    async def _wait_for_annotations(self, units: int, timeout: float = 10.0):
        """A pod of this size is bound to the node but carries no allocation record yet: the extender is writing
        it back (an apiserver that dropped the Binding's annotations).  Failing now would fail the pod."""
        self.stats["annotation_waits"] = self.stats.get("annotation_waits", 0) + 1
        deadline = time.monotonic() + timeout
        while time.monotonic() < deadline:
            await asyncio.sleep(0.02)
            rec, whole = self.state.match(units)
            if rec is not None:
                return rec, whole
            if not self.state.unannotated(units):
                break
        return self.state.match(units)

    def _isolate(self, rec: PodRec, device: Device, cus, alloc: ContainerAllocation):
        """Enforced isolation: the pod's config + ledger files, mounted (or named, for host processes)."""
        if self.isolation is None:
            return
        limit = rec.request * UNITS[self.unit]
        try:
            mounts, envs = self.isolation.prepare(rec.uid, cus, device.cu_count, limit,
                                                  host_process=self.mount_mode == "all")
        except OSError as e:
            raise AllocateError(f"isolation files for {rec.key}: {e}") from e
        alloc.mounts.extend(mounts)
        alloc.envs.update(envs)
        alloc.iso = rec.uid

    async def Allocate(self, request, context):
        resp = api.AllocateResponse()
        t0 = time.perf_counter()
        try:
            for creq in request.container_requests:
                rec, alloc = await self.allocate_container(len(creq.devices_ids), list(creq.devices_ids))
                c = resp.container_responses.add()
                for k, v in alloc.envs.items():
                    c.envs[k] = v
                for k, v in alloc.annotations.items():
                    c.annotations[k] = v
                c.annotations[POD_ANNOTATION] = f"{rec.key}/{rec.uid}"
                for dspec in alloc.devices:
                    c.devices.add(**dspec)
                for m in alloc.mounts:
                    c.mounts.add(**m)
            self.stats["allocate_ok"] += 1
            if self.reconciler is not None:
                self.reconciler.kick(fast=self._ambiguous([rec.uid]))
            self.timing["n"] += 1
            self.timing["handler"] += time.perf_counter() - t0
            return resp
        except (AllocateError, ApiError, OSError) as e:
            self.stats["allocate_fail"] += 1
            log.error("Allocate failed: %s", e)
            await context.abort(grpc.StatusCode.FAILED_PRECONDITION, str(e))

    async def PreStartContainer(self, request, context):
        return api.PreStartContainerResponse()

    # ------------------------------------------------------------ server / registration
    def _handlers(self):
        methods = {}
        for meth, (inp, out, stream) in api.SERVICES["DevicePlugin"].items():
            ic, oc, _ = api.io_types("DevicePlugin", meth)
            fn = getattr(self, meth)
            if stream:
                methods[meth] = grpc.unary_stream_rpc_method_handler(fn, request_deserializer=ic.FromString,
                                                                     response_serializer=oc.SerializeToString)
            else:
                methods[meth] = grpc.unary_unary_rpc_method_handler(fn, request_deserializer=ic.FromString,
                                                                    response_serializer=oc.SerializeToString)
        return grpc.method_handlers_generic_handler(f"{api.PKG}.DevicePlugin", methods)

    def _open_native(self) -> bool:
        """The native endpoint and (GSX_PLUGIN_FEED, default on) its pod feed, not serving yet: kubelet learns the
        socket only from the registration that follows start-up.  Switches the state to native views when the feed
        runs.  False if the native endpoint is unavailable."""
        ok, _why = native_grpc_available()
        if not ok:
            return False
        from ..core.engine import native  # noqa: PLC0415

        os.makedirs(self.socket_dir, exist_ok=True)
        try:
            os.unlink(self.socket_path)
        except FileNotFoundError:
            pass
        if self.isolation is not None:
            self.isolation.install()  # the fast path writes per-pod files next to the installed library
        cfg = self._native_config()
        self._native = native().DpServer(self.socket_path, self.state.core, cfg)
        self._native.set_ready(False)  # every call UNAVAILABLE until serve(): records and unlanded commits first
        self._native_serving = False
        if os.environ.get("GSX_PLUGIN_FEED", "1") == "1":
            self._native.start_feed(cfg["api"])  # this node's pods into the state from a native reflector
            self._feed = True
            if self._own_informer:
                self.state.use_native_views()
        return True

    async def serve(self):
        if self._server is not None:  # re-serving after a kubelet restart: retire the old server first
            await self._server.stop(0)
            self._server = None
        reuse = self._native is not None and not self._native_serving
        reserve = self._native is not None and self._native_serving  # kubelet restarted: a new endpoint
        if not reuse:
            self._close_native()
        if reserve:
            # commits of Allocates the closed endpoint answered early but had not landed (queued, or in flight and
            # cut off by the close) are in the journal; land them as a restarted plugin does
            self._journaled = list(self.state.records.values())
        ok, why = native_grpc_available()
        if ok:
            if not reuse:
                self._open_native()
            self._native_serving = True
            self._sync_native()
            if reserve:
                # in the background: the pods are still claimed in the state, so serving need not wait for a slow
                # apiserver (a commit that fails is retried with backoff while its pod exists)
                t = asyncio.get_running_loop().create_task(self.commit_unlanded())
                self._tasks.append(t)
            self._native.set_ready(True)
            if os.environ.get("GSX_PLUGIN_SERVE_THREAD", "1") == "1":
                # the endpoint is served from a native thread that never needs the GIL (a native lock guards the
                # allocation state shared with this loop), so a busy Python loop does not delay a fast Allocate
                self._native_fd = self._native.start_serving()
            else:
                self._native_fd = self._native.fd()
            asyncio.get_running_loop().add_reader(self._native_fd, self._native_poll)
            self.grpc_impl = "native"
            return
        # loud: the native endpoint is the product path (kubelet's serial admission pays every call's overhead)
        log.warning("device-plugin endpoint on grpc.aio, not the native endpoint (%s): Allocate admissions are "
                    "about 2x slower; install libnghttp2 (libnghttp2-14) to restore it", why)
        self.grpc_impl = "grpcio"
        os.makedirs(self.socket_dir, exist_ok=True)
        try:
            os.unlink(self.socket_path)
        except FileNotFoundError:
            pass
        self._server = grpc.aio.server()
        self._server.add_generic_rpc_handlers((self._handlers(),))
        self._server.add_insecure_port(f"unix://{self.socket_path}")
        await self._server.start()

    async def register(self, timeout: float = 10.0):
        async with grpc.aio.insecure_channel(f"unix://{self.kubelet_socket}") as ch:
            ic, oc, _ = api.io_types("Registration", "Register")
            call = ch.unary_unary(api.method_path("Registration", "Register"), request_serializer=ic.SerializeToString,
                                  response_deserializer=oc.FromString)
            await call(api.RegisterRequest(version=api.VERSION, endpoint=self.endpoint,
                                           resource_name=self.profile.resource,
                                           options=api.DevicePluginOptions(
                                               get_preferred_allocation_available=self.preferred)),
                       timeout=timeout)
        self.stats["registrations"] += 1
        log.info("registered %s with kubelet at %s", self.profile.resource, self.kubelet_socket)

    async def publish_node(self):
        """gpu-count capacity + per-device totals / inventory annotations (what kubelet does not publish), and
        the Allocate order this plugin matches in (landing order: the extender may bind concurrently)."""
        import json  # noqa: PLC0415

        totals = [self.units[i] for i in sorted(self.units)]
        inv = [{"index": d.index, "bdf": d.bdf, "uuid": d.uuid, "units": self.units[d.index],
                "total_bytes": d.total_bytes, "share_bytes": d.share_bytes, "cu": d.cu_count, "xcc": d.xcc_count,
                "partition": d.partition, "render": d.render_minor, "card": d.card_minor}
               for d in sorted(self.devices.values(), key=lambda d: d.index)]
        await self.client.patch("nodes", self.node, {"metadata": {"annotations": {
            NODE_DEVICE_MEMORY_ANNOTATION: ",".join(str(t) for t in totals),
            NODE_DEVICE_INFO_ANNOTATION: json.dumps(inv, separators=(",", ":")),
            NODE_ALLOCATE_ORDER_ANNOTATION: "landing",
            NODE_PHYSICAL_PUBLICATION_ANNOTATION: "true" if self.publishes_physical else None}}})
        await self.client.patch("nodes", self.node, {"status": {"capacity": {
            self.profile.count: str(len(self.devices))}}}, sub="status")

    def healthy(self) -> tuple[bool, str]:
        if self._stopped:
            return False, "stopped"
        if not self.pods.synced.is_set():
            return False, "pod informer not synced"
        if self._server is None:
            return False, "gRPC server not started"
        return True, "ok"

    def debug_state(self) -> dict:
        return {"node": self.node, "resource": self.profile.resource, "unit": self.unit,
                "devices": [{"index": d.index, "bdf": d.bdf, "healthy": d.healthy, "units": self.units[d.index],
                             "cu": d.cu_count, "partition": d.partition, "memory_partition": d.memory_partition,
                             "health": self.health_info.get(d.index)} for d in self.devices.values()],
                "informer": {"synced": self.pods.synced.is_set(), "relists": self.pods.relists,
                             "rewatches": self.pods.rewatches, "events": self.pods.events},
                "stats": dict(self.stats), "timing": dict(self.timing), **self.state.snapshot(),
                "reconcile": dict(self.reconciler.stats) if self.reconciler is not None else None,
                "grpc": {"impl": self.grpc_impl, **(self._native.stats() if self._native is not None else {})},
                "isolation": dict(self.isolation.stats) if self.isolation is not None else None}

    def metrics_text(self) -> str:
        lines = []
        for k, v in sorted(self.stats.items()):
            lines += [f"# TYPE gpushare_plugin_{k}_total counter", f"gpushare_plugin_{k}_total {v}"]
        if self.reconciler is not None:
            for k, v in sorted(self.reconciler.stats.items()):
                kind = "gauge" if k.endswith("_max") else "counter"
                name = f"gpushare_plugin_reconcile_{k}" + ("" if kind == "gauge" else "_total")
                lines += [f"# TYPE {name} {kind}", f"{name} {v}"]
        for k, v in sorted(self.state.stats.items()):
            lines += [f"# TYPE gpushare_plugin_state_{k}_total counter", f"gpushare_plugin_state_{k}_total {v}"]
        # 1: kubelet's calls are served by the native endpoint (h2.cc on libnghttp2); 0: the grpc.aio fallback
        lines += ["# TYPE gpushare_plugin_native_endpoint gauge",
                  f"gpushare_plugin_native_endpoint {int(self.grpc_impl == 'native')}"]
        lines.append("# TYPE gpushare_plugin_device_healthy gauge")
        lines += [f'gpushare_plugin_device_healthy{{device="{d.index}"}} {int(d.healthy)}' for d in self.devices.values()]
        for name, key in (("thermal_throttle", "thermal_throttle"), ("power_throttle", "power_throttle"),
                          ("xgmi_error", "xgmi_error"), ("ras_uncorrectable", None)):
            lines.append(f"# TYPE gpushare_plugin_device_{name} gauge")
            for i, h in sorted(self.health_info.items()):
                v = (h.get("ecc_uncorrectable", 0) + h.get("ras_umc_uncorrectable", 0) + h.get("ras_gfx_uncorrectable", 0)
                     + h.get("ras_sdma_uncorrectable", 0) + h.get("ras_xgmi_uncorrectable", 0)) if key is None \
                    else int(h.get(key, 0))
                lines.append(f'gpushare_plugin_device_{name}{{device="{i}"}} {v}')
        lines.append("# TYPE gpushare_plugin_cu_free gauge")
        lines += [f'gpushare_plugin_cu_free{{device="{i}"}} {cp.free_count()}' for i, cp in self.state.cus.items()]
        lines.append("# TYPE gpushare_plugin_allocate_candidates gauge")
        lines.append(f"gpushare_plugin_allocate_candidates {len(self.state.candidates())}")
        if self._native is not None:
            # the native gRPC endpoint: calls answered on its fast path vs handed to the Python handlers
            ns = self._native.stats()
            for k in ("fast_allocate", "fast_preferred", "slow_allocate", "slow_preferred", "patch_failures",
                      "commits_gone", "waited", "feed_events", "calls"):
                lines += [f"# TYPE gpushare_plugin_native_{k}_total counter", f"gpushare_plugin_native_{k}_total {ns.get(k, 0)}"]
        n = self.timing.get("n", 0)
        if n:
            # mean time per Allocate inside the plugin: handler total, match, ASSIGNED patch (seconds)
            for k in ("handler", "match", "assign_patch"):
                lines += [f"# TYPE gpushare_plugin_allocate_{k}_seconds gauge",
                          f"gpushare_plugin_allocate_{k}_seconds {self.timing.get(k, 0.0) / n:.9f}"]
        return "\n".join(lines) + "\n"

    async def serve_debug(self, host: str, port: int) -> int:
        """``/healthz``, ``/metrics`` (Prometheus text) and ``/debug/state`` (JSON) for problem determination."""
        import json  # noqa: PLC0415

        from aiohttp import web  # noqa: PLC0415

        async def healthz(_):
            ok, why = self.healthy()
            return web.Response(status=200 if ok else 503, text=why)

        async def metrics(_):
            return web.Response(text=self.metrics_text(), content_type="text/plain")

        async def state(_):
            return web.Response(text=json.dumps(self.debug_state(), indent=1), content_type="application/json")

        app = web.Application()
        app.router.add_get("/healthz", healthz)
        app.router.add_get("/metrics", metrics)
        app.router.add_get("/debug/state", state)
        self._debug = web.AppRunner(app, access_log=None)
        await self._debug.setup()
        site = web.TCPSite(self._debug, host, port)
        await site.start()
        return site._server.sockets[0].getsockname()[1]

    async def _watch_kubelet(self):
        """Re-register when kubelet restarts (it deletes and re-creates its socket)."""
        last = None
        while True:
            try:
                st = os.stat(self.kubelet_socket)
                ident = (st.st_ino, st.st_ctime)
                if last is not None and ident != last:
                    log.info("kubelet restarted; re-registering")
                    await self.serve()
                    await self.register()
                last = ident
            except FileNotFoundError:
                last = None
            except Exception as e:  # noqa: BLE001
                log.warning("re-register failed: %r", e)
            await asyncio.sleep(1.0)

    async def _health_loop(self):
        """Poll amdsmi health: uncorrectable ECC / RAS (HBM, GFX, SDMA, xGMI) or an xGMI link error makes a GPU's
        IDs Unhealthy in ListAndWatch; thermal / power throttling is exported as a metric; a compute or memory
        partition change re-shapes the advertised devices (:meth:`reload_devices`)."""
        from ..ops import mxdev  # noqa: PLC0415

        loop = asyncio.get_running_loop()
        while True:
            changed = False
            for idx in list(self.devices):
                d = self.devices.get(idx)
                try:
                    h = await loop.run_in_executor(None, mxdev.health, idx, self.health_backend)
                except Exception as e:  # noqa: BLE001
                    log.debug("health of GPU %d: %r", idx, e)
                    continue
                if d is None or self.devices.get(idx) is not d:
                    break  # re-shaped meanwhile
                self.health_info[idx] = h
                if h.get("partition") and (h["partition"] != d.partition or
                                           (h.get("memory_partition") or "") != (d.memory_partition or "")):
                    changed = True
                    break
                self.set_health(idx, bool(h["healthy"]), f"({h.get('reason') or 'ok'})")
            if changed:
                try:
                    await self.reload_devices()
                except Exception as e:  # noqa: BLE001
                    log.error("re-enumerating devices after a partition change failed: %r", e)
            await asyncio.sleep(self.health_interval)

    async def _event_loop(self):
        from ..ops import mxdev  # noqa: PLC0415

        sess = mxdev.session(self.health_backend)
        try:
            sess.watch_events()
        except Exception as e:  # noqa: BLE001
            log.info("amdsmi events unavailable: %r", e)
            return
        loop = asyncio.get_running_loop()
        while True:
            evs = await loop.run_in_executor(None, sess.poll_events, 1000)
            for ev in evs:
                if ev["name"] in ("GPU_PRE_RESET", "VMFAULT"):
                    self.set_health(ev["index"], False, f"({ev['name']}: {ev['message']})")
                elif ev["name"] == "GPU_POST_RESET":
                    h = self.health_info.get(ev["index"]) or {}
                    if h.get("healthy", True):  # a reset does not clear uncorrectable-error counters
                        self.set_health(ev["index"], True, "(post reset)")
                elif ev["name"] == "THERMAL_THROTTLE":
                    self.health_info.setdefault(ev["index"], {})["thermal_throttle"] = True

    async def start(self, register: bool = True, publish: bool = True, serve: bool = True,
                    sync_timeout: float = 30.0):
        # state first: CU partitions of running pods are rebuilt before the first Allocate can be served
        if self._own_informer and serve and self._open_native() and self._feed:
            # the native endpoint's pod feed is the node's one watch (no Python informer decodes pod events)
            loop = asyncio.get_running_loop()
            if not await loop.run_in_executor(None, self._native.feed_synced, sync_timeout):
                log.warning("pod feed of %s not synced after %.0fs; Allocate will LIST", self.node, sync_timeout)
            self._native.poll()  # apply the first LIST (the serving thread does this from now on)
            self.state.flush_dropped()
            self.pods = _FeedInformer(self)
        else:
            if self._own_informer:
                await self.pods.start()
            try:
                await self.pods.wait_synced(sync_timeout)
            except asyncio.TimeoutError:
                log.warning("pod informer of %s not synced after %.0fs; Allocate will LIST", self.node, sync_timeout)
        n = self.load_records()
        if n:
            log.info("restored %d allocation records from %s", n, self.checkpoint)
        if await self.commit_unlanded():
            log.warning("landed the ASSIGNED commits of Allocates answered before a restart")
        if self.isolation is not None and self.pods.synced.is_set():
            self.isolation.gc({r.iso for r in self.state.records.values() if r.iso} | set(self.state.pods))
        if self.reconciler is not None:
            self.reconciler.start()
        if self.publishes_physical:
            self._tasks.append(asyncio.get_running_loop().create_task(self._epoch_loop(), name="gsx-epoch"))
        if not serve:
            return
        await self.serve()
        if publish:
            try:
                await self.publish_node()
            except ApiError as e:
                log.warning("publishing node info failed: %s", e)
        if register:
            await self.register()
            self._tasks.append(asyncio.get_running_loop().create_task(self._watch_kubelet()))
        if self.health_backend:
            self._tasks.append(asyncio.get_running_loop().create_task(self._health_loop()))
            self._tasks.append(asyncio.get_running_loop().create_task(self._event_loop()))

    async def stop(self):
        self._stopped = True
        self._changed.set()
        if self._ext is not None:
            await self._ext.close()
            self._ext = None
        if self._persist_task is not None:
            self._persist_task.cancel()
        self._write_checkpoint()
        if self.reconciler is not None:
            await self.reconciler.stop()
        for t in self._tasks:
            t.cancel()
        if self._own_informer:
            await self.pods.stop()
        if self._debug is not None:
            await self._debug.cleanup()
            self._debug = None
        if self._server is not None:
            await self._server.stop(0.5)
        self._close_native()
        for t in list(self._slow):
            t.cancel()
        try:
            os.unlink(self.socket_path)
        except FileNotFoundError:
            pass


def now_ns() -> int:
    return time.time_ns()


UNIT_BYTES = UNITS
