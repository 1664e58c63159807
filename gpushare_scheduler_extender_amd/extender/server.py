"""kube-scheduler extender HTTP service: filter / bind / inspect / version / pprof / metrics.

Route table and status-code contract of ``pkg/routes/routes.go:18-182``:

=======================================  =========================================================
``POST /gpushare-scheduler/filter``      ExtenderArgs -> ExtenderFilterResult, **always 200**
                                         (``routes.go:58-99``); decided entirely in the native
                                         engine (``native/engine/ledger.cc: filter_body``)
``POST /gpushare-scheduler/bind``        ExtenderBindingArgs -> ExtenderBindingResult,
                                         **500 iff Error != ""** (``routes.go:101-148``)
``GET  /gpushare-scheduler/inspect``     all nodes (``pkg/scheduler/inspect.go``)
``GET  /gpushare-scheduler/inspect/:n``  one node; unknown node -> ``error`` field (the
                                         reference dereferences nil, ``inspect.go:19-24``)
``GET  /version``                        ``0.1.0`` (``routes.go:27-30,150-156``)
``GET  /debug/pprof/*``                  see :mod:`.pprof`
``GET  /metrics``, ``GET /healthz``       ours
=======================================  =========================================================

Bind (``pkg/scheduler/gpushare-bind.go`` + ``pkg/cache/nodeinfo.go:139-206``)
is re-designed for throughput while keeping its observable result (same
annotations, same best-fit device, same error strings):

1. the pod comes from the informer (lister); a UID mismatch triggers one live
   GET and the reference's UID error (``gpushare-bind.go:44-65``);
2. the native ledger *reserves* the best-fit device (``assume``) under its
   mutex for microseconds, instead of holding a node write lock across the
   apiserver round trips (``nodeinfo.go:141-142``), so binds to one node run
   concurrently and a concurrent filter already sees the reservation;
3. ``bind_mode="binding"`` (default) writes annotations and ``nodeName`` in
   one ``pods/binding`` POST whose annotations kube-apiserver copies onto the
   pod; ``bind_mode="update"`` reproduces the reference's two calls
   (annotate, then bind) with its retry-once-on-conflict
   (``nodeinfo.go:150-189``), detecting conflicts by HTTP 409.  Both modes
   run in the C++ front end (``server.cc: do_bind``; update mode writes the
   annotations as a merge patch guarded by the resourceVersion the scheduler
   saw); this Python path serves binds the front end did not filter, and
   every bind when a client-side QPS limit is set;
4. failure releases the reservation; success keeps it until the informer
   observes the annotated pod (then the annotations are the record).
"""
from __future__ import annotations

import asyncio
import json
import logging
import time

from aiohttp import web

from ..core.controller import Controller, NativeController, api_dict
from ..core.engine import new_engine
from ..k8s.client import ApiError, KubeClient
from ..models import pod as podutil
from ..models import wire
from ..models.profile import POD_CU_COUNT_ANNOTATION, SHARED_GPU, NamingProfile
from ..utils.metrics import Metrics
from .pprof import add_pprof

log = logging.getLogger("gsx.extender")

VERSION = "0.1.0"
API_PREFIX = "/gpushare-scheduler"


class BindError(Exception):
    pass


class ExtenderServer:
    def __init__(self, client: KubeClient, profile: NamingProfile = SHARED_GPU, *, workers: int = 1,
                 bind_mode: str = "binding", reservation_ttl: float = 60.0, resync_period: float = 30.0,
                 emit_events: bool = True, leader_elect: bool = False, lease_name: str = "gpushare-schd-extender",
                 lease_namespace: str = "kube-system", lease_duration: float = 15.0, renew_deadline: float = 10.0,
                 retry_period: float = 2.0, native_controller: bool = True, pprof: bool = True,
                 bind_order: str = "auto"):
        if bind_mode not in ("binding", "update"):
            raise ValueError("bind_mode must be 'binding' or 'update'")
        self.client = client
        self.profile = profile
        self.engine = new_engine(profile)
        if bind_order not in ("auto", "strict", "relaxed"):
            raise ValueError("bind_order must be 'auto', 'strict' or 'relaxed'")
        # strict: equal-size binds of one node for different GPUs reach the apiserver in ASSUME_TIME order (the
        # reference's node lock, pkg/cache/nodeinfo.go:141-189); auto: the same, except on nodes whose device
        # plugin matches Allocates in landing order (gpushare.amd.com/allocate-order=landing, native/engine/
        # allocstate.h), where binds need no order; relaxed: every bind is concurrent and the device plugin's
        # reconciliation with kubelet (deviceplugin/reconcile.py) repairs the swaps that can follow
        self.bind_order = bind_order
        self.engine.set_bind_order(bind_order)
        self.metrics = Metrics(self.engine)
        if native_controller:
            self.controller = NativeController(client, self.engine, profile, resync_period=resync_period)
        else:
            self.controller = Controller(client, self.engine, profile, workers=workers, resync_period=resync_period,
                                         metrics=self.metrics)
        self.bind_mode = bind_mode
        self.reservation_ttl = reservation_ttl
        self.emit_events = emit_events
        self.pprof = pprof
        self.app = self._make_app()
        self._gc_task: asyncio.Task | None = None
        self._repair_task: asyncio.Task | None = None
        self.annotation_repairs = 0
        self._bg: set[asyncio.Task] = set()
        self.native_server = False
        self.elector = None
        if leader_elect:
            from ..k8s.leader import LeaderElector  # noqa: PLC0415

            self.elector = LeaderElector(client, lease_name, lease_namespace, lease_duration=lease_duration,
                                         renew_deadline=renew_deadline, retry_period=retry_period,
                                         on_started=self._became_leader, on_stopped=self._lost_leadership)
            self.engine.set_binds_enabled(False)  # standby until the Lease is ours

    @property
    def is_leader(self) -> bool:
        return self.elector is None or self.elector.is_leader

    def _became_leader(self):
        self.engine.set_binds_enabled(True)

    def _lost_leadership(self):
        self.engine.set_binds_enabled(False)

    # ------------------------------------------------------------ lifecycle
    async def start(self):
        await self.controller.start()
        self._gc_task = asyncio.get_running_loop().create_task(self._gc_loop())
        self._repair_task = asyncio.get_running_loop().create_task(self._repair_loop())
        self.metrics.bind_mode.set(1 if self.bind_mode == "update" else 0)
        if self.elector is not None:
            await self.elector.start()  # informers + ledger are warm before we can win

    async def stop(self):
        if self.elector is not None:
            await self.elector.stop()
        if self._gc_task:
            self._gc_task.cancel()
        if self._repair_task:
            self._repair_task.cancel()
        await self.controller.stop()

    async def _gc_loop(self):
        """Expire bind reservations the pod informer never confirmed -- but only on the evidence of a LIST
        begun after the binding was written; a stalled watch forces a re-list instead (never over-commit)."""
        while True:
            await asyncio.sleep(min(5.0, max(0.05, self.reservation_ttl / 4)))
            n, relist = self.controller.gc_reservations()
            if n:
                log.warning("expired %d bind reservations a fresh LIST did not confirm", n)
            if relist:
                log.info("bind reservations overdue: forcing a pod re-list to confirm them")

    async def _repair_loop(self):
        """Self-check of the ``binding`` bind mode.  It relies on kube-apiserver copying the Binding's
        ``metadata.annotations`` onto the pod; an apiserver or admission webhook that drops them leaves the pod
        bound without ``*_IDX`` -- the device plugin then has no candidate and every Allocate fails.  The ledger
        flags such pods (bound by us, observed on the node, annotations missing); here the annotations are
        written back with the reference's pod update (``pkg/cache/nodeinfo.go:150-189``), later binds switch to
        ``update`` mode (annotate, then bind), and a metric and a Warning event record it."""
        while True:
            await asyncio.sleep(0.05)
            for a in self.engine.drain_annotation_repairs():
                ann = podutil.bind_annotations(self.profile, a["dev"], a["dev_total"], a["mem"], now_ns=a["assume_ns"])
                pod = {"kind": "Pod", "metadata": {"name": a["name"], "namespace": a["namespace"], "uid": a["uid"]}}
                if self.bind_mode != "update":
                    self.bind_mode = "update"
                    self.engine.set_update_mode(True)
                    self.metrics.bind_mode.set(1)
                    log.warning("the apiserver dropped the annotations of a Binding (pod %s/%s): binds now write "
                                "the annotations first (bind mode 'update')", a["namespace"], a["name"])
                    self._event(pod, "BindingAnnotationsDropped",
                                "the apiserver did not keep the Binding's annotations; switched to annotate-then-bind")
                for attempt in range(20):
                    try:
                        await self.client.patch("pods", a["name"], {"metadata": {"annotations": ann}}, a["namespace"])
                        self.annotation_repairs += 1
                        self.metrics.annotation_repairs.labels("ok").inc()
                        break
                    except ApiError as e:
                        if e.not_found:
                            self.metrics.annotation_repairs.labels("gone").inc()
                            break
                        await asyncio.sleep(min(0.5, 0.01 * 2 ** attempt))
                    except OSError:
                        await asyncio.sleep(min(0.5, 0.01 * 2 ** attempt))
                else:
                    self.metrics.annotation_repairs.labels("failed").inc()
                    log.error("could not write the allocation annotations back onto %s/%s", a["namespace"], a["name"])

    # ------------------------------------------------------------ verbs
    def filter(self, body: bytes) -> bytes:
        """predicate.go:15-39 + gpushare-predicate.go:13-40, in C++."""
        return self.engine.filter(body)

    async def _get_pod(self, name: str, ns: str, uid: str) -> dict:
        """gpushare-bind.go:44-65."""
        pod = self.controller.get_pod(name, ns)
        if pod is not None and (pod.get("metadata") or {}).get("uid") == uid:
            return pod
        t0 = time.perf_counter()
        try:
            pod = await self.client.get("pods", name, ns)
        except ApiError as e:
            raise BindError(e.message or str(e)) from e
        finally:
            self.metrics.api_latency.labels("get_pod").observe(time.perf_counter() - t0)
        puid = (pod.get("metadata") or {}).get("uid")
        if puid != uid:
            raise BindError(f"The pod {name} in ns {ns}'s uid is {puid}, and it's not equal with expected {uid}")
        return pod

    async def bind(self, args: wire.ExtenderBindingArgs) -> str:
        """Returns "" on success or the error string of ExtenderBindingResult."""
        name, ns, uid, node = args.pod_name, args.pod_namespace, args.pod_uid, args.node
        if not self.is_leader:
            self.metrics.bind_results.labels("standby").inc()
            return "this extender replica is not the leader"
        try:
            pod = await self._get_pod(name, ns, uid)
        except BindError as e:
            self.metrics.bind_results.labels("pod_lookup_failed").inc()
            return str(e)
        req = podutil.gpu_mem_request(pod, self.profile)
        # reservation + ASSUME_TIME + entry in the bind-order set shared with the native front end
        cu_count = ((pod.get("metadata") or {}).get("annotations") or {}).get(POD_CU_COUNT_ANNOTATION, "")
        dev, dev_total, seq, assume_ns = self.engine.assume_ordered(uid, ns, name, node, req, str(cu_count))
        if dev < 0:
            self.metrics.bind_results.labels("no_device").inc()
            if dev == -2:
                msg = f'node "{node}" not found'
            elif dev == -3:
                msg = f"The node {node} is not for GPU share, need skip"
            elif dev == -4:
                msg = f"bind of pod {name} in ns {ns} is already in progress"
            else:
                msg = f"The node {node} can't place the pod {name} in ns {ns}"  # nodeinfo.go:170
            self._event(pod, "FailedBinding", msg)
            return msg
        ann = podutil.bind_annotations(self.profile, dev, dev_total, req, now_ns=assume_ns)
        t0 = time.perf_counter()
        try:
            # kubelet admits a node's pods in binding order and the device plugin hands a request of N
            # units to the earliest-ASSUME_TIME pod of that size: an equal-size pod for another GPU of the
            # same node must not overtake an earlier one, whichever path (native or this one) binds it
            # (the reference's node lock across the API calls, pkg/cache/nodeinfo.go:141-189)
            if self.bind_mode == "update":
                # the reference's first call; not ordered: a pod without spec.nodeName is no plugin candidate
                await self._annotate(pod, ann)
            if self.engine.bind_blocked(seq):
                # shielded: if this handler is cancelled (server shutdown), the finally below must not run
                # bind_leave before the executor thread has left bind_wait (use-after-free)
                fut = asyncio.get_running_loop().run_in_executor(None, self.engine.bind_wait, seq)
                try:
                    await asyncio.shield(fut)
                except asyncio.CancelledError:
                    self.engine.bind_leave(seq)  # wakes the waiter, which then finds its entry gone
                    await asyncio.wait_for(asyncio.shield(fut), 5.0)
                    raise
            if self.bind_mode == "binding":
                await self._bind_with_annotations(pod, node, ann)
            else:
                md = pod["metadata"]
                await self.client.bind_pod(md["namespace"], md["name"], node, md.get("uid"))
        except (ApiError, BindError, OSError, asyncio.TimeoutError) as e:
            self.engine.finish_bind(uid, False, 0.0)
            self.metrics.bind_results.labels("api_error").inc()
            msg = e.message if isinstance(e, ApiError) and e.message else str(e)
            self._event(pod, "FailedBinding", msg)
            return msg
        finally:
            self.metrics.api_latency.labels("bind").observe(time.perf_counter() - t0)
            self.engine.bind_leave(seq)
        self.engine.finish_bind(uid, True, self.reservation_ttl)
        self.metrics.bind_results.labels("ok").inc()
        return ""

    async def _bind_with_annotations(self, pod: dict, node: str, ann: dict, retries: int = 2):
        md = pod["metadata"]
        for attempt in range(retries + 1):
            try:
                await self.client.bind_pod(md["namespace"], md["name"], node, md.get("uid"), ann)
                return
            except ApiError as e:
                # only a transient (injected / storage) conflict is retried; an
                # "already assigned" conflict is final
                if e.conflict and "already assigned" not in e.message and attempt < retries:
                    continue
                raise

    async def _annotate(self, pod: dict, ann: dict):
        """nodeinfo.go:145-168: PUT the annotated pod; on a conflict retry once on a fresh GET.  The Binding
        (nodeinfo.go:174-189) follows in :meth:`bind`, after the bind-order wait."""
        md = pod["metadata"]
        new = podutil.with_annotations(pod, ann)
        try:
            await self.client.replace("pods", new)
        except ApiError as e:
            if not e.conflict:
                raise
            fresh = await self.client.get("pods", md["name"], md["namespace"])
            await self.client.replace("pods", podutil.with_annotations(fresh, ann))

    def _event(self, pod: dict, reason: str, msg: str):
        if not self.emit_events:
            return
        ns = (pod.get("metadata") or {}).get("namespace", "default")

        async def go():
            try:
                await self.client.create_event(ns, {"kind": "Pod", **pod}, reason, msg, "Warning")
            except Exception as e:  # noqa: BLE001 - events are best effort
                log.debug("event emit failed: %r", e)
        t = asyncio.get_running_loop().create_task(go())
        self._bg.add(t)
        t.add_done_callback(self._bg.discard)

    # ------------------------------------------------------------ HTTP
    def _make_app(self) -> web.Application:
        app = web.Application(client_max_size=64 * 1024 * 1024)
        r = app.router
        r.add_post(API_PREFIX + "/filter", self.h_filter)
        r.add_post(API_PREFIX + "/bind", self.h_bind)
        r.add_post(API_PREFIX + "/prioritize", self.h_prioritize)
        r.add_get(API_PREFIX + "/inspect", self.h_inspect)
        r.add_get(API_PREFIX + "/inspect/", self.h_inspect)
        r.add_get(API_PREFIX + "/inspect/{nodename}", self.h_inspect)
        r.add_get("/version", self.h_version)
        r.add_get("/metrics", self.h_metrics)
        r.add_get("/healthz", self.h_healthz)
        r.add_get("/debug/engine", self.h_debug_engine)
        if self.pprof:
            add_pprof(app, self.engine)
        return app

    async def h_filter(self, request: web.Request):
        t0 = time.perf_counter()
        body = await request.read()
        out = self.filter(body)
        self.metrics.latency.labels("filter").observe(time.perf_counter() - t0)
        self.metrics.requests.labels("filter", "200").inc()
        return web.Response(body=out, content_type="application/json")

    async def h_prioritize(self, request: web.Request):
        """Ours (the reference has no prioritize verb): binpack-first node scores, HostPriorityList."""
        body = await request.read()
        self.metrics.requests.labels("prioritize", "200").inc()
        return web.Response(body=self.engine.prioritize(body), content_type="application/json")

    async def h_bind(self, request: web.Request):
        t0 = time.perf_counter()
        body = await request.read()
        try:
            args = wire.ExtenderBindingArgs.decode(body)
            err = await self.bind(args)
        except wire.WireError as e:
            err = str(e)
        status = 500 if err else 200
        self.metrics.latency.labels("bind").observe(time.perf_counter() - t0)
        self.metrics.requests.labels("bind", str(status)).inc()
        return web.Response(body=wire.binding_result(err), status=status, content_type="application/json")

    async def h_inspect(self, request: web.Request):
        node = request.match_info.get("nodename", "")
        body, _found = self.engine.inspect(node)
        self.metrics.requests.labels("inspect", "200").inc()
        return web.Response(body=body, content_type="application/json")

    async def h_version(self, request):
        return web.Response(text=VERSION)

    async def h_healthz(self, request):
        ok = self.controller.is_synced()
        if ok and not self.is_leader:
            return web.Response(text="standby (not the leader)", status=503)
        return web.Response(text="ok" if ok else "not synced", status=200 if ok else 503)

    async def h_debug_engine(self, request):
        """Ledger, controller (LIST pages, watch errors) and native front-end counters as JSON."""
        out = {"ledger": self.engine.stats()}
        st = getattr(self.controller, "stats", None)
        if st is not None:
            out["controller"] = st()
        if self.native_server:
            out["server"] = self.engine.server_stats()
        return web.Response(text=json.dumps(out), content_type="application/json")

    async def h_metrics(self, request):
        return web.Response(body=self.metrics.render(), content_type="text/plain")


class ExtenderRunner:
    """Serve an :class:`ExtenderServer` on host:port (port 0 = ephemeral).

    ``native=True`` (default) puts the C++ front end (``native/engine/server.cc``)
    on the public port: filter / bind / inspect / version never touch Python;
    every other route is proxied to the aiohttp app on a loopback port.
    ``native=False`` serves everything from aiohttp (reference-equivalent path,
    used to A/B the native one).
    """

    def __init__(self, server: ExtenderServer, host: str = "127.0.0.1", port: int = 0, *, native: bool = True,
                 http_threads: int = 2, pool_threads: int = 16):
        self.server = server
        self.host = host
        self.port = port
        self.native = native
        self.http_threads = http_threads
        self.pool_threads = pool_threads
        self.internal_port = 0
        self._runner: web.AppRunner | None = None
        self._drain: asyncio.Task | None = None

    @property
    def url(self) -> str:
        return f"http://{self.host}:{self.port}"

    async def start(self) -> "ExtenderRunner":
        await self.server.start()
        self._runner = web.AppRunner(self.server.app, access_log=None, handle_signals=False, shutdown_timeout=1.0)
        await self._runner.setup()
        if self.native:
            site = web.TCPSite(self._runner, "127.0.0.1", 0, backlog=1024, reuse_address=True)
            await site.start()
            self.internal_port = site._server.sockets[0].getsockname()[1]  # noqa: SLF001
            api = api_dict(self.server.client.config)
            # a client-side QPS limit (--kube-qps) lives in the Python client: binds then take that path
            native_bind = self.server.client.limiter.qps <= 0
            self.port = self.server.engine.serve(self.host, self.port, self.http_threads, self.pool_threads,
                                                 self.internal_port, native_bind, self.server.reservation_ttl, api,
                                                 update_mode=self.server.bind_mode == "update")
            self.server.native_server = True
            self._drain = asyncio.get_running_loop().create_task(self._drain_failures())
        else:
            site = web.TCPSite(self._runner, self.host, self.port, backlog=1024, reuse_address=True)
            await site.start()
            if self.port == 0:
                self.port = site._server.sockets[0].getsockname()[1]  # noqa: SLF001
        return self

    async def _drain_failures(self):
        """Native bind failures -> Warning events + metrics (the C++ path does not call Python)."""
        while True:
            await asyncio.sleep(0.2)
            for f in self.server.engine.drain_bind_failures():
                self.server.metrics.bind_results.labels("native_fail").inc()
                pod = {"kind": "Pod", "metadata": {"name": f["name"], "namespace": f["namespace"], "uid": f["uid"]}}
                self.server._event(pod, "FailedBinding", f["message"])  # noqa: SLF001

    async def stop(self):
        if self._drain:
            self._drain.cancel()
        if self.native:
            await asyncio.get_running_loop().run_in_executor(None, self.server.engine.stop_server)
        if self._runner:
            await self._runner.cleanup()
        await self.server.stop()


def dumps(o) -> bytes:
    return json.dumps(o, separators=(",", ":")).encode()
