"""Test fixture: in-process kube-scheduler simulator speaking the extender protocol.

Not shipped: ``gsxtools/`` and ``bench.py`` run the compiled ``gsx-schedsim`` (``native/schedsim``), which replays the
same cycle with C++ reflectors and bind threads; this asyncio twin stays for tests that drive scheduling from
their own event loop.

There is no kube-scheduler, kind or kubectl in this environment (SURVEY.md
§4), so this replays what kube-scheduler does for a pod that requests a
managed extended resource (``config/scheduler-policy-config.json:4-19``):

1. **scheduling cycle** (serial, one pod at a time): the default
   ``NodeResourcesFit`` predicate on the node *aggregate* of ``gpu-mem``
   (``ignoredByScheduler: false``), then ``POST <urlPrefix>/filter`` with
   ``NodeNames`` (``nodeCacheCapable: true``) or full ``Nodes``; pick a node
   (``first`` / ``binpack`` / ``spread``); assume the pod on it;
2. **binding cycle** (asynchronous, many in flight): ``POST <urlPrefix>/bind``;
   on any error the assumption is dropped and the pod is retried with
   backoff, exactly like a failed extender bind (``routes.go:139-143`` returns
   500).

Per-pod timings (queue -> bound, filter RTT, bind RTT) are recorded for the
benchmark's p50/p99 bind latency.
"""
from __future__ import annotations

import asyncio
import collections
import json
import logging
import time
from dataclasses import dataclass, field

from gpushare_scheduler_extender_amd.k8s.client import KubeClient
from gpushare_scheduler_extender_amd.k8s.fasthttp import Client
from gpushare_scheduler_extender_amd.k8s.informer import Handler, Informer, obj_key
from gpushare_scheduler_extender_amd.models import pod as podutil
from gpushare_scheduler_extender_amd.models import wire
from gpushare_scheduler_extender_amd.models.profile import NamingProfile

log = logging.getLogger("gsx.sim")


@dataclass
class PodTiming:
    key: str
    seen: float = 0.0
    filtered: float = 0.0
    bound: float = 0.0
    filter_rtt: float = 0.0
    bind_rtt: float = 0.0
    attempts: int = 0
    node: str = ""
    error: str = ""


@dataclass
class SimStats:
    scheduled: int = 0
    bound: int = 0
    bind_errors: int = 0
    unschedulable: int = 0
    filter_calls: int = 0
    timings: dict = field(default_factory=dict)


class SchedulerSim:
    def __init__(self, client: KubeClient, extender_url: str, profile: NamingProfile, *,
                 scheduler_name: str = "default-scheduler", node_cache_capable: bool = True,
                 node_policy: str = "binpack", max_inflight_binds: int = 64, retry_backoff: float = 0.05,
                 http_limit: int = 128, namespace: str | None = None, use_prioritize: bool = False):
        self.client = client
        self.url = extender_url.rstrip("/") + "/gpushare-scheduler"
        self.profile = profile
        self.scheduler_name = scheduler_name
        self.node_cache_capable = node_cache_capable
        self.node_policy = node_policy
        self.use_prioritize = use_prioritize  # call the extender's prioritize verb when >1 node passes
        self.retry_backoff = retry_backoff
        self.pods = Informer(client, "pods", namespace=namespace)
        self.nodes = Informer(client, "nodes")
        self.queue: asyncio.Queue = asyncio.Queue()
        self.bind_sem = asyncio.Semaphore(max_inflight_binds)
        self.stats = SimStats()
        self._assumed: dict[str, tuple[str, int]] = {}  # pod key -> (node, request), bind in flight
        self._placed: dict[str, tuple[str, int]] = {}  # pod key -> (node, request), observed bound & live
        self._used: dict[str, int] = collections.defaultdict(int)  # node -> placed + assumed requests
        self._req: dict[str, int] = {}  # pod uid -> gpu-mem request (pod specs are immutable)
        self._queued: set[str] = set()
        self._pod_json: dict[str, bytes] = {}  # pending pod -> its bytes from the watch event (no re-encode)
        self._http: Client | None = None
        self._http_limit = http_limit
        self._tasks: list[asyncio.Task] = []
        self._bg: set[asyncio.Task] = set()
        self._waiters: list[asyncio.Future] = []  # woken on every pod event and every bind (event-driven waits)
        self.pods.add_handler(Handler(self._on_pod, lambda o, n, r: self._on_pod(n, r), self._on_pod_delete))

    # ------------------------------------------------------------ pod intake
    def _pending(self, pod: dict) -> bool:
        return (not podutil.node_name(pod) and (pod.get("spec") or {}).get("schedulerName",
                                                                           "default-scheduler") == self.scheduler_name
                and not podutil.is_complete(pod))

    def _request(self, pod: dict) -> int:
        uid = (pod.get("metadata") or {}).get("uid", "")
        r = self._req.get(uid)
        if r is None:
            r = self._req[uid] = podutil.gpu_mem_request(pod, self.profile)
        return r

    def _account(self, key: str, pod: dict | None):
        """Incremental NodeResourcesFit bookkeeping (the scheduler cache's view of node usage)."""
        old = self._placed.pop(key, None)
        if old is not None:
            self._used[old[0]] -= old[1]
        if pod is None:
            return
        n = podutil.node_name(pod)
        if n and not podutil.is_terminal(pod):
            req = self._request(pod)
            self._placed[key] = (n, req)
            self._used[n] += req
            a = self._assumed.pop(key, None)  # now observed: stop counting the assumption
            if a is not None:
                self._used[a[0]] -= a[1]

    def _assume(self, key: str, node: str, req: int):
        self._assumed[key] = (node, req)
        self._used[node] += req

    def _unassume(self, key: str):
        a = self._assumed.pop(key, None)
        if a is not None:
            self._used[a[0]] -= a[1]

    def _on_pod(self, pod: dict, raw):
        key = obj_key(pod)
        self._account(key, pod)
        self._notify()
        if self._pending(pod) and key not in self._queued and key not in self._assumed:
            ob = wire.watch_object_bytes(raw)
            if ob is not None:
                self._pod_json[key] = ob
            else:
                self._pod_json.pop(key, None)
            self._queued.add(key)
            t = self.stats.timings.get(key)
            if t is None:
                self.stats.timings[key] = PodTiming(key, seen=time.perf_counter())
            self.queue.put_nowait(key)

    @staticmethod
    def _rv_of(ob: bytes) -> str | None:
        i = ob.find(b'"resourceVersion":"')
        if i < 0:
            return None
        j = ob.find(b'"', i + 19)
        return ob[i + 19:j].decode() if j > 0 else None

    def _on_pod_delete(self, pod: dict, raw):
        key = obj_key(pod)
        self._account(key, None)
        self._notify()
        self._unassume(key)
        self._pod_json.pop(key, None)
        self._req.pop((pod.get("metadata") or {}).get("uid", ""), None)

    # ------------------------------------------------------------ aggregate fit (NodeResourcesFit)
    def _node_used(self) -> dict[str, int]:
        return self._used

    def _prefilter(self, req: int) -> list[dict]:
        used = self._node_used()
        out = []
        for n in self.nodes.list():
            alloc = podutil.node_allocatable(n, self.profile.resource)
            name = n["metadata"]["name"]
            if req == 0 or alloc - used.get(name, 0) >= req:
                out.append(n)
        return out

    def _pick(self, names: list[str], req: int) -> str:
        if self.node_policy == "first" or len(names) == 1:
            return names[0]
        used = self._node_used()

        def free(nm):
            n = self.nodes.get(nm)
            return podutil.node_allocatable(n, self.profile.resource) - used.get(nm, 0) if n else 0
        if self.node_policy == "spread":
            return max(names, key=lambda nm: (free(nm), nm))
        return min(names, key=lambda nm: (free(nm), nm))

    # ------------------------------------------------------------ cycles
    def _sess(self) -> Client:
        if self._http is None:
            self._http = Client(self.url, limit=self._http_limit, timeout=60.0)
        return self._http

    async def _schedule_one(self, key: str):
        pod = self.pods.get(key)
        self._queued.discard(key)
        if pod is None or not self._pending(pod):
            return
        tm = self.stats.timings.setdefault(key, PodTiming(key, seen=time.perf_counter()))
        tm.attempts += 1
        req = self._request(pod)
        cands = self._prefilter(req)
        if not cands:
            self.stats.unschedulable += 1
            tm.error = "0 nodes available: Insufficient " + self.profile.resource
            self._retry_later(key)
            return
        if req > 0:
            ob = self._pod_json.pop(key, None)
            if self.node_cache_capable and ob is not None and (pod.get("metadata") or {}).get(
                    "resourceVersion") == self._rv_of(ob):
                body = wire.filter_args_raw(ob, [n["metadata"]["name"] for n in cands])
            elif self.node_cache_capable:
                body = wire.filter_args(pod, [n["metadata"]["name"] for n in cands])
            else:
                body = wire.filter_args(pod, nodes=cands)
            t0 = time.perf_counter()
            r = await self._sess().request("POST", "/filter", body)
            res = wire.ExtenderFilterResult.decode(r.body)
            tm.filter_rtt = time.perf_counter() - t0
            self.stats.filter_calls += 1
            if res.error:
                tm.error = res.error
                self._retry_later(key)
                return
            names = res.passing()
        else:
            names = [n["metadata"]["name"] for n in cands]
        if not names:
            self.stats.unschedulable += 1
            tm.error = "extender filtered all nodes"
            self._retry_later(key)
            return
        if self.use_prioritize and len(names) > 1:
            r = await self._sess().request("POST", "/prioritize", wire.filter_args(pod, names))
            scores = {h["Host"]: h["Score"] for h in json.loads(r.body)}
            node = max(names, key=lambda nm: (scores.get(nm, 0), [-ord(ch) for ch in nm]))
        else:
            node = self._pick(names, req)
        tm.filtered = time.perf_counter()
        self._assume(key, node, req)
        self.stats.scheduled += 1
        await self.bind_sem.acquire()
        t = asyncio.get_running_loop().create_task(self._bind(key, pod, node, tm))
        self._bg.add(t)
        t.add_done_callback(self._bg.discard)

    async def _bind(self, key: str, pod: dict, node: str, tm: PodTiming):
        try:
            md = pod["metadata"]
            args = wire.ExtenderBindingArgs(md["name"], md.get("namespace", "default"), md.get("uid", ""), node)
            t0 = time.perf_counter()
            r = await self._sess().request("POST", "/bind", args.encode())
            body, status = r.body, r.status
            tm.bind_rtt = time.perf_counter() - t0
            err = json.loads(body).get("Error", "") if body else f"HTTP {status}"
            if status != 200 or err:
                self.stats.bind_errors += 1
                tm.error = err
                self._unassume(key)
                self._retry_later(key)
                return
            tm.bound = time.perf_counter()
            tm.node = node
            tm.error = ""
            self.stats.bound += 1
            self._notify()
        except Exception as e:  # noqa: BLE001
            self.stats.bind_errors += 1
            tm.error = repr(e)
            self._unassume(key)
            self._retry_later(key)
        finally:
            self.bind_sem.release()

    def _retry_later(self, key: str):
        def again():
            pod = self.pods.get(key)
            if pod is not None and self._pending(pod) and key not in self._queued:
                self._queued.add(key)
                self.queue.put_nowait(key)
        asyncio.get_running_loop().call_later(self.retry_backoff, again)

    async def _loop(self):
        while True:
            key = await self.queue.get()
            try:
                await self._schedule_one(key)
            except asyncio.CancelledError:
                raise
            except Exception as e:  # noqa: BLE001
                log.warning("schedule %s failed: %r", key, e)
                self._retry_later(key)

    # ------------------------------------------------------------ lifecycle
    async def start(self):
        await self.nodes.start()
        await self.pods.start()
        await self.nodes.wait_synced(30)
        await self.pods.wait_synced(30)
        self._tasks.append(asyncio.get_running_loop().create_task(self._loop(), name="sim-scheduler"))

    async def stop(self):
        for t in self._tasks:
            t.cancel()
        for t in list(self._bg):
            t.cancel()
        await self.pods.stop()
        await self.nodes.stop()
        if self._http:
            await self._http.close()
            self._http = None

    def forget(self, keys):
        for k in keys:
            self.stats.timings.pop(k, None)

    def _notify(self):
        ws, self._waiters = self._waiters, []
        for f in ws:
            if not f.done():
                f.set_result(None)

    async def _changed(self, timeout: float):
        """Sleep until the next pod event / bind or ``timeout`` (a bare future: no task per wait)."""
        loop = asyncio.get_running_loop()
        f = loop.create_future()
        self._waiters.append(f)
        h = loop.call_later(timeout, lambda: f.done() or f.set_result(None))
        try:
            await f
        finally:
            h.cancel()

    async def wait_for(self, cond, timeout: float = 30.0):
        """Wait until ``cond()`` holds, re-checking on every pod event the informer delivers."""
        deadline = time.perf_counter() + timeout
        while not cond():
            rem = deadline - time.perf_counter()
            if rem <= 0:
                raise TimeoutError("condition not reached")
            await self._changed(min(rem, 0.05))

    async def wait_bound(self, keys: list[str], timeout: float = 30.0):
        deadline = time.perf_counter() + timeout
        pending = set(keys)
        while pending:
            pending = {k for k in pending if not (self.stats.timings.get(k) and self.stats.timings[k].bound)}
            if not pending:
                return
            if time.perf_counter() > deadline:
                raise TimeoutError(f"{len(pending)} pods not bound, e.g. {sorted(pending)[:3]}: "
                                   f"{[self.stats.timings.get(k).error if self.stats.timings.get(k) else '?' for k in sorted(pending)[:3]]}")
            await self._changed(0.05)
