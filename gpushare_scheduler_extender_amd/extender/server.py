"""kube-scheduler extender HTTP service: filter / bind / inspect / version / pprof / metrics.

Route table and status-code contract of ``pkg/routes/routes.go:18-182``, served by the C++ front end
(``native/engine/server.cc``) on the public port:

=======================================  =========================================================
``POST /gpushare-scheduler/filter``      ExtenderArgs -> ExtenderFilterResult, **always 200**
                                         (``routes.go:58-99``; ``ledger.cc: filter_body``)
``POST /gpushare-scheduler/bind``        ExtenderBindingArgs -> ExtenderBindingResult,
                                         **500 iff Error != ""** (``routes.go:101-148``;
                                         ``server.cc: do_bind``)
``POST /gpushare-scheduler/move``        the device plugin's allocation-record moves (ours;
                                         ``server.cc: do_move``): the extender is the one writer
                                         of ``*_IDX``
``GET  /gpushare-scheduler/inspect``     all nodes (``pkg/scheduler/inspect.go``)
``GET  /gpushare-scheduler/inspect/:n``  one node; unknown node -> ``error`` field (the
                                         reference dereferences nil, ``inspect.go:19-24``)
``GET  /version``                        ``0.1.0`` (``routes.go:27-30,150-156``)
``GET  /debug/pprof/*``                  see :mod:`.pprof` (proxied to this module's aiohttp app)
``GET  /metrics``, ``GET /healthz``       ours (proxied to this module's aiohttp app)
=======================================  =========================================================

Bind (``pkg/scheduler/gpushare-bind.go`` + ``pkg/cache/nodeinfo.go:139-206``) runs entirely in C++: the pod
comes from the filter request the scheduler just sent, else the controller's lister, else one live GET (with
the reference's UID error); the ledger reserves the best-fit device under its mutex for microseconds; one
``pods/binding`` POST carries the annotations (``bind_mode="binding"``) or the reference's annotate-then-bind
pair runs (``bind_mode="update"``).  This module owns what is not on the request path: the controller's
lifecycle, reservation GC, the annotation self-repair, Warning events for failed binds, leader election, and
the metrics / health / pprof routes.
"""
from __future__ import annotations

import asyncio
import json
import logging

from aiohttp import web

from ..core.controller import NativeController, api_dict
from ..core.engine import new_engine
from ..k8s.client import ApiError, KubeClient
from ..models import pod as podutil
from ..models.profile import SHARED_GPU, NamingProfile
from ..utils.metrics import Metrics
from .pprof import add_pprof

log = logging.getLogger("gsx.extender")

VERSION = "0.1.0"
API_PREFIX = "/gpushare-scheduler"


class ExtenderServer:
    def __init__(self, client: KubeClient, profile: NamingProfile = SHARED_GPU, *,
                 bind_mode: str = "binding", reservation_ttl: float = 60.0, resync_period: float = 30.0,
                 emit_events: bool = True, leader_elect: bool = False, lease_name: str = "gpushare-schd-extender",
                 lease_namespace: str = "kube-system", lease_duration: float = 15.0, renew_deadline: float = 10.0,
                 retry_period: float = 2.0, pprof: bool = True, bind_order: str = "auto"):
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
        self.controller = NativeController(client, self.engine, profile, resync_period=resync_period)
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

    def get_pod(self, name: str, ns: str | None = None) -> dict | None:
        """The controller's lister (raw JSON of gpu-share pods)."""
        return self.controller.get_pod(name, ns)

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
        r.add_get("/metrics", self.h_metrics)
        r.add_get("/healthz", self.h_healthz)
        r.add_get("/debug/engine", self.h_debug_engine)
        if self.pprof:
            add_pprof(app, self.engine)
        return app

    async def h_healthz(self, request):
        ok = self.controller.is_synced()
        if ok and not self.is_leader:
            return web.Response(text="standby (not the leader)", status=503)
        return web.Response(text="ok" if ok else "not synced", status=200 if ok else 503)

    async def h_debug_engine(self, request):
        """Ledger, controller (LIST pages, watch errors) and native front-end counters as JSON."""
        out = {"ledger": self.engine.stats(), "controller": self.controller.stats()}
        if self.native_server:
            out["server"] = self.engine.server_stats()
        return web.Response(text=json.dumps(out), content_type="application/json")

    async def h_metrics(self, request):
        return web.Response(body=self.metrics.render(), content_type="text/plain")


class ExtenderRunner:
    """Serve an :class:`ExtenderServer` on host:port (port 0 = ephemeral).

    The C++ front end (``native/engine/server.cc``) owns the public port: filter / prioritize / bind / move /
    inspect / version never touch Python; every other route is proxied to the aiohttp app on a loopback port.
    A client-side QPS limit (``KubeClient(qps=, burst=)``, ``--kube-qps``) becomes the front end's token bucket.
    """

    def __init__(self, server: ExtenderServer, host: str = "127.0.0.1", port: int = 0, *, http_threads: int = 2,
                 pool_threads: int = 16, plugin_auth: str = "none", plugin_users: list[str] | None = None):
        self.server = server
        # the device plugin's endpoints (/move, /physical): "tokenreview" = only a bearer token the apiserver
        # authenticates as one of plugin_users (the plugin's service account)
        self.plugin_auth = plugin_auth
        self.plugin_users = list(plugin_users or [])
        self.host = host
        self.port = port
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
        site = web.TCPSite(self._runner, "127.0.0.1", 0, backlog=1024, reuse_address=True)
        await site.start()
        self.internal_port = site._server.sockets[0].getsockname()[1]  # noqa: SLF001
        client = self.server.client
        self.port = self.server.engine.serve(self.host, self.port, self.http_threads, self.pool_threads,
                                             self.internal_port, self.server.reservation_ttl, api_dict(client.config),
                                             update_mode=self.server.bind_mode == "update",
                                             qps=float(client.limiter.qps), burst=int(client.limiter.burst),
                                             plugin_auth=self.plugin_auth, plugin_users=self.plugin_users)
        self.server.native_server = True
        self._drain = asyncio.get_running_loop().create_task(self._drain_failures())
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
        await asyncio.get_running_loop().run_in_executor(None, self.server.engine.stop_server)
        if self._runner:
            await self._runner.cleanup()
        await self.server.stop()


def dumps(o) -> bytes:
    return json.dumps(o, separators=(",", ":")).encode()
