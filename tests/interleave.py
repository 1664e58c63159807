"""Deterministic interleaving harness for the device plugin's swap / guard / exchange protocol.

The chaos rows (tests/test_chaos.py) run the real processes and find protocol races by seed sweeps: a failure shows
up in a few seeds out of a thousand, and a run does not replay.  This harness runs the same protocol code -- the
device plugin's Allocate / GetPreferredAllocation handlers (deviceplugin/plugin.py), its physical guard, the
PodResources reconciler with its three-step exchange and holds (deviceplugin/reconcile.py), the physical publication,
and the extender's native ledger (``_engine.Engine``: assume / bind order / begin_move / end_move / set_unaccounted /
epochs) -- in ONE thread, on one asyncio loop, with every point where the real system can interleave turned into a
*gate* that a seeded scheduler opens:

* every apiserver call (the fixture's in-memory store, tests/fixtures/fakeapi.py -- no HTTP),
* every extender endpoint call (move / physical / epoch: the ledger halves of server.cc do_move / do_physical, with
  the move's PATCH a separate gate as it is an apiserver round trip there too),
* every ``asyncio.sleep`` of the plugin (the guard's waits, the miss path's retries), on a virtual clock,
* kubelet's PodResources answer,
* the delivery of each watch event, separately to the extender's informer, the plugin's informer and kubelet.

Actors (each a task or a step the scheduler may start whenever it is enabled): the extender binding a pending pod
(assume_ordered, the Binding POST, finish_bind); kubelet admitting the earliest-created pod it has seen bound
(GetPreferredAllocation, Allocate, the IDs recorded as the call returns: kubelet's podDevices), stopping the
container of a pod being deleted and finalising its graceful deletion (DELETE grace 0, UID precondition); a
reconciliation pass; the plugin's epoch poll; a user deleting a pod (graceful or force) or creating one; the
extender restarting (a new ledger from a LIST, a new epoch, binds held until the plugin republishes).

Checked after EVERY step (safety): no GPU runs more than its capacity -- the sum of the units of the containers
kubelet runs on a GPU (the GPU the Allocate answer told the container to use) never exceeds the GPU -- and the
annotations never promise a GPU past it (an exchange in flight read as its protocol defines it, as
tests/test_chaos.py reads it).  Checked once
the schedule is drained with only fair system actions left (convergence): every running pod is annotated with the
GPU its container runs on, no exchange hold is left, the extender's ledger equals the annotations with nothing
unaccounted, no Allocate failed, and every pod bound to the node was admitted.

A schedule is a function of (scenario, seed): ``python -m tests.interleave --scenario swap-graceful --seeds 0-999``
replays or sweeps; a failure prints the step trace.  ``--systematic 1|2`` enumerates instead of sampling: every
schedule that departs from a fair default order at no more than that many of the first ``--window`` steps (a
preemption bound, as CHESS does), each replayable from its script of departures.  Scenarios with ``faults`` answer a
share of the apiserver writes with an injected 409 or 500, as the chaos rows' fake apiserver does.  The ``mutation``
argument re-introduces a known bug class (MUTATIONS) so the tests can show the harness finds it.
"""
from __future__ import annotations

import argparse
import asyncio
import collections
import dataclasses
import json
import logging
import random
import sys
import time as _time

from gpushare_scheduler_extender_amd.core.engine import new_engine
from gpushare_scheduler_extender_amd.deviceplugin import api as dpapi
from gpushare_scheduler_extender_amd.deviceplugin import plugin as plugin_mod
from gpushare_scheduler_extender_amd.deviceplugin import reconcile as reconcile_mod
from gpushare_scheduler_extender_amd.deviceplugin import state as state_mod
from gpushare_scheduler_extender_amd.deviceplugin.devices import fake_devices
from gpushare_scheduler_extender_amd.k8s.client import ApiError
from gpushare_scheduler_extender_amd.k8s.fasthttp import HTTPError
from gpushare_scheduler_extender_amd.k8s.objects import make_node, make_pod
from gpushare_scheduler_extender_amd.models.pod import bind_annotations
from gpushare_scheduler_extender_amd.models.profile import (NODE_PHYSICAL_PUBLICATION_ANNOTATION,
                                                            POD_HOLD_IDX_ANNOTATION, POD_HOLD_PARTNER_ANNOTATION,
                                                            SHARED_GPU)
from tests.fixtures.fakeapi import FakeApiServer

_real_sleep = asyncio.sleep
NODE = "n"
PROFILE = SHARED_GPU
TERM_GRACE_S = 5  # the pods' spec.terminationGracePeriodSeconds: a force-deleted pod's container is gone by then


@dataclasses.dataclass
class Scenario:
    name: str
    sizes: tuple = (8, 8, 8, 8)      # pods created at the start, in this creationTimestamp order
    extra: tuple = (8,)              # pods a user creates later (one per "create" step)
    deletes: int = 1                 # user deletions
    grace: str = "graceful"          # graceful | force | mixed
    gpus: int = 2
    gpu_units: int = 16
    passes: int = 10                 # reconciliation passes the scheduler may start before the drain
    restarts: int = 0                # extender restarts
    stop_after: int = 0              # steps before kubelet may stop a deleted pod's container (a slow runtime)
    # kubelet lists a force-deleted pod's container until it has stopped (the node agent stand-in), and the plugin
    # runs GSX_PLUGIN_FORCE_DELETE=report; False: real kubelet (drops it at once) and the default "grace" policy
    truthful: bool = False
    # share of apiserver writes (the plugin's PATCHes, the extender's move PATCH) answered 409 or 500 (the chaos rows'
    # injected faults), decided by the schedule's seed
    faults: float = 0.0
    max_steps: int = 4000


SCENARIOS = {s.name: s for s in (
    Scenario("swap-graceful"),
    Scenario("swap-force", grace="force"),
    Scenario("mixed-sizes", sizes=(8, 4, 4, 8, 8), extra=(4, 4), deletes=2, grace="mixed"),
    Scenario("restart", deletes=1, grace="mixed", restarts=1),
    Scenario("churn", sizes=(8, 8, 8, 8), extra=(8, 8, 8), deletes=3, grace="mixed", passes=14),
    # containers of deleted pods outlive their objects (a force delete) or their deletion (graceful) for a while:
    # the binds and admissions that meet them go through the physical guard
    Scenario("slow-stop", sizes=(8, 8, 8, 8), extra=(8, 8), deletes=2, grace="mixed", passes=14, stop_after=60),
    # force deletes whose containers run out their whole termination grace, new pods bound meanwhile
    Scenario("force-grace", sizes=(8, 8, 8, 8), extra=(8, 8), deletes=2, grace="force", passes=14,
             stop_after=10 ** 9),
    # the same against a kubelet whose report is the truth, with the plugin taking it as such (bench.py's setting)
    Scenario("force-report", sizes=(8, 8, 8, 8), extra=(8, 8), deletes=2, grace="force", passes=14,
             stop_after=10 ** 9, truthful=True),
    # the chaos rows' apiserver: writes refused (409) or failing (500) at random, sizes mixed, deletes of both kinds
    Scenario("faults", sizes=(8, 8, 4, 4, 8), extra=(8, 4), deletes=2, grace="mixed", passes=16, faults=0.2),
    # a chaos row's node in small: four GPUs, three sizes, a full first batch, deletes and new pods racing it
    Scenario("batch-faults", sizes=(8, 16, 8, 16, 8, 8, 16, 8, 4, 4), extra=(8, 16, 4), deletes=3, grace="mixed",
             gpus=4, gpu_units=24, passes=20, faults=0.15, max_steps=8000),
)}


class Clock:
    """Virtual time for the plugin, its state and the reconciler (their ``time`` module attribute is swapped for
    this; the native state takes its times from them)."""

    def __init__(self):
        self.t = 1_000_000.0

    def time(self):
        return self.t

    monotonic = perf_counter = time

    def time_ns(self):
        return int(self.t * 1e9)


class Gate:
    __slots__ = ("label", "fut", "wake")

    def __init__(self, label, fut, wake):
        self.label, self.fut, self.wake = label, fut, wake


class Resp:
    __slots__ = ("status", "body")

    def __init__(self, status: int, body: dict):
        self.status, self.body = status, json.dumps(body).encode()


class Violation(AssertionError):
    pass


def _api_error(e: HTTPError) -> ApiError:
    try:
        b = json.loads(e.body or b"{}")
    except ValueError:
        b = {}
    return ApiError(e.status, b.get("reason", ""), b.get("message", ""), b)


class _Store(FakeApiServer):
    """The fixture's apiserver state, its watch events fanned out to the three watchers' queues."""

    def __init__(self, harness):
        super().__init__()
        self.h = harness

    def _emit(self, kind, etype, obj):
        super()._emit(kind, etype, obj)
        if kind != "pods":
            return
        self.h.ext_q.append((etype, obj))
        if (obj.get("spec") or {}).get("nodeName") == NODE:
            self.h.plugin_q.append((etype, obj))
            self.h.kubelet_q.append((etype, obj))


class _Client:
    """The slice of KubeClient the plugin uses, every call a gate."""

    def __init__(self, h):
        self.h = h

    async def patch(self, kind, name, patch, ns=None, sub=None, **_):
        await self.h.point(f"api PATCH {name}")
        f = self.h.fault()
        if f:
            raise ApiError(f, "Conflict" if f == 409 else "InternalError", "injected")
        try:
            return self.h.api.patch(kind, ns or "default", name, patch, sub or "")
        except HTTPError as e:
            raise _api_error(e) from None

    async def list(self, kind, ns=None, field_selector="", label_selector="", **_):
        await self.h.point("api LIST")
        return {"items": self.h.api.list(kind, ns or "", field_selector, label_selector),
                "metadata": {"resourceVersion": str(self.h.api.rv)}}

    async def get(self, kind, name, ns=None):
        await self.h.point(f"api GET {name}")
        try:
            return self.h.api._get(kind, ns or "default", name)
        except HTTPError as e:
            raise _api_error(e) from None


class _PodResources:
    """kubelet's PodResources List: the device IDs of every container it runs, answered at a gate."""

    def __init__(self, h):
        self.h = h

    def available(self):
        return True

    async def device_ids(self, resource, timeout=2.0):
        await self.h.point("podresources List")
        # a pod kubelet saw deleted outright is out of its pod manager: not listed, though its container may still
        # stop (a truthful kubelet lists it until it has)
        return {tuple(c.key.split("/", 1)): [tuple(sorted(c.ids))] for uid, c in self.h.active.items()
                if self.h.sc.truthful or uid not in self.h.kgone}

    async def close(self):
        pass


# Known bug classes, re-introduced on demand so the tests can show the harness finds each:
MUTATIONS = {
    "free_on_deleting": "the extender frees a pod's share at its deletionTimestamp (round 5's controller)",
    "no_guard": "the device plugin starts containers without its physical guard",
    "no_publication": "the device plugin never tells the extender its unaccounted use",
    "no_linger": "a force-deleted pod's share is freed as soon as kubelet stops listing it",
    "no_stand_in": "no unstarted pod stands in for a swapped partner that is gone (round 5's fix)",
    "serve_partner": "the matcher serves the partner of an unfinished exchange (fixed in round 6)",
    "strict_finish": "finishing an exchange re-applies step 2 over a partner served on the fields it gave it since "
                     "(fixed in round 6; with serve_partner, the bug the harness first found)",
    "fail_on_gone": "an Allocate whose matched pod was deleted meanwhile fails kubelet's pod (fixed in round 6)",
}


@dataclasses.dataclass
class Container:
    key: str
    ids: list
    dev: int
    units: int


class Harness:
    def __init__(self, scenario: Scenario, seed: int, mutation: str = "", script: dict | None = None):
        self.sc, self.seed, self.mutation = scenario, seed, mutation
        # systematic mode (``script``, see systematic()): the first enabled action at every step but the steps the
        # script names, where it takes the one at that index; ``widths`` records how many were enabled at each step
        self.script = script
        self.widths: list[int] = []
        self.muts = set(filter(None, mutation.split(",")))
        unknown = self.muts - set(MUTATIONS)
        if unknown:
            raise ValueError(f"unknown mutations {sorted(unknown)}; known: {sorted(MUTATIONS)}")
        self.rng = random.Random(seed)
        self.clock = Clock()
        self.gates: list[Gate] = []
        self.trace: list[str] = []
        self.errors: list[str] = []
        self.ext_q, self.plugin_q, self.kubelet_q = collections.deque(), collections.deque(), collections.deque()
        self.api = _Store(self)
        # kubelet
        self.kview: dict[str, dict] = {}          # uid -> pod as kubelet last saw it (bound to NODE)
        self.kgone: set[str] = set()               # uids kubelet saw DELETED
        self.active: dict[str, Container] = {}     # uid -> running container (kubelet's podDevices)
        self.reserved: dict[str, list] = {}        # uid -> IDs kubelet set aside for an Allocate in flight
        self.admitted: set[str] = set()
        self.failed: dict[str, str] = {}
        self.refused: dict[str, str] = {}
        self.lingered, self._lc = 0, 0                # force-deleted containers' shares the plugin kept counted
        self.admitting = False
        self.k_deleted_at: dict[str, int] = {}     # uid -> step kubelet saw its deletion
        self.stop_due: dict[str, float] = {}       # uid -> virtual time a force-deleted pod's container is dead by
        # extender
        self.binding: set[str] = set()
        self.gen = 1
        self.epoch = "boot1.1"
        self.eng = None
        # budgets
        self.passes_left = scenario.passes
        self.deletes_left = scenario.deletes
        self.extra = list(scenario.extra)
        self.restarts_left = scenario.restarts
        self.polls_left = 4
        self.pass_running = False
        self.poll_running = False
        self.tasks: list[asyncio.Task] = []
        self.n_pods = 0
        self.steps = 0
        self.max_used = [0] * scenario.gpus
        self.faults = 0

    def fault(self) -> int:
        """An injected apiserver answer for this write (409 or 500), or 0."""
        if self.sc.faults and self.rng.random() < self.sc.faults:
            self.faults += 1
            return 409 if self.rng.random() < 0.6 else 500
        return 0

    # ------------------------------------------------------------ gates
    async def point(self, label: str, wake: float | None = None):
        fut = asyncio.get_running_loop().create_future()
        self.gates.append(Gate(label, fut, wake))
        await fut

    async def vsleep(self, delay, result=None):
        if delay <= 0:
            await _real_sleep(0)
            return result
        await self.point("sleep", wake=self.clock.t + delay)
        return result

    async def settle(self):
        loop = asyncio.get_running_loop()
        for _ in range(100000):
            await _real_sleep(0)
            if not loop._ready:  # every task is parked at a gate (or done)
                break
        for t in list(self.tasks):
            if t.done():
                self.tasks.remove(t)
                if t.exception() is not None:
                    e = t.exception()
                    raise RuntimeError(f"actor {t.get_name()} raised {e!r}") from e

    def spawn(self, name: str, coro):
        self.tasks.append(asyncio.get_running_loop().create_task(coro, name=name))

    # ------------------------------------------------------------ setup
    def pod(self, size: int) -> dict:
        i = self.n_pods
        self.n_pods += 1
        p = make_pod(f"p{i}", size, uid=f"u{i}", profile=PROFILE)
        p["metadata"]["creationTimestamp"] = f"2026-01-01T00:{i // 60:02d}:{i % 60:02d}Z"
        p["spec"]["terminationGracePeriodSeconds"] = TERM_GRACE_S
        return self.api.create("pods", p)

    def node_obj(self) -> dict:
        return make_node(NODE, self.sc.gpu_units * self.sc.gpus, self.sc.gpus, profile=PROFILE,
                         annotations={NODE_PHYSICAL_PUBLICATION_ANNOTATION: "true"})

    def new_ledger(self):
        eng = new_engine(PROFILE)
        eng.upsert_node_json(json.dumps(self.api.store["nodes"][("", NODE)]).encode())
        for p in self.api.list("pods"):
            if not _terminal(p):
                eng.upsert_pod_json(json.dumps(p).encode())
        return eng

    def setup(self, tmpdir: str):
        self.api.create("nodes", self.node_obj())
        self.eng = self.new_ledger()
        self.ext_q.clear()
        pl = plugin_mod.GpuSharePlugin(_Client(self), NODE, fake_devices(f"{self.sc.gpus}x{self.sc.gpu_units}GiB"),
                                       PROFILE, socket_dir=tmpdir, checkpoint="", extender="http://harness")
        pl.reconciler = reconcile_mod.Reconciler(pl, _PodResources(self))
        pl.state.core.expect_owner_reports(True)
        pl.state.core.set_linger(not self.sc.truthful)
        pl._extender_request = self.ext_request

        async def informer_wait(found, timeout=0.0):  # the pod event may still be on its way: a gate, then look
            await self.point("plugin informer wait")
            return found()

        pl._await_informer = informer_wait
        if "no_publication" in self.muts:
            async def _no_pub(force=False):
                pl._ext_epoch = self.epoch  # (no epoch poll keeps asking)
                return True
            pl.publish_physical = _no_pub
        if "no_guard" in self.muts:
            async def _no_guard(rec, units, ids=()):
                return rec
            pl._physical_guard = _no_guard
        if "no_linger" in self.muts:
            st = pl.state

            def _forget(pod, st=st):  # a force-deleted pod's share lingers until t=3: gone at the next pass
                uid = pod["metadata"].get("uid", "")
                st.core.deleted(uid, 1.0)
                st._recs.pop(uid, None)
                st._flush()
            st.forget = _forget
        if "no_stand_in" in self.muts:
            pl.reconciler._stand_in_partner = lambda dev, p, started: None
        if "serve_partner" in self.muts:
            pl.state.core.set_skip_partners(False)
        if "strict_finish" in self.muts:
            reconcile_mod._took = lambda q, want: reconcile_mod.fields(q) == {
                k: want.get(k) for k in ("idx", "assigned", "cu_mask")}
        self.plugin = pl
        self.all_ids = [i for d in sorted(pl.ids) for i in pl.ids[d]]
        for s in self.sc.sizes:
            self.pod(s)

    # ------------------------------------------------------------ the extender
    async def ext_request(self, method: str, path: str, data: bytes | None = None):
        await self.point(f"ext {path.rsplit('/', 1)[-1]}")
        if path.endswith("/epoch"):
            return Resp(200, {"epoch": self.epoch, "leader": True})
        body = json.loads(data or b"{}")
        eng = self.eng
        if path.endswith("/physical"):
            eng.set_unaccounted(body["node"], body.get("unaccounted") or [], float(body.get("ttl") or 60))
            return Resp(200, {"Error": "", "epoch": self.epoch})
        assert path.endswith("/move"), path
        ann = body.get("annotations") or {}
        hold = ann.get(POD_HOLD_IDX_ANNOTATION)
        req_hold = int(hold) if isinstance(hold, str) and hold.isdigit() else -1
        hp = ann.get(POD_HOLD_PARTNER_ANNOTATION)
        try:
            hp_uid = json.loads(hp).get("uid", "") if isinstance(hp, str) else ""
        except ValueError:
            hp_uid = ""
        rc, to, why = eng.begin_move(body["uid"], body["node"], int(body["from"]), int(body.get("to", -1)),
                                     body.get("partner", ""), bool(body.get("physical_on_to")), req_hold, hp_uid)
        if rc != 0:
            return Resp(404 if rc == 1 else 409, {"Error": why})
        await self.point(f"ext move PATCH {body['name']}")
        f = self.fault()
        if f:
            eng.end_move(body["uid"], False)
            return Resp(f, {"Error": f"apiserver {f} (injected)"})
        patch = {"metadata": {"resourceVersion": body["resourceVersion"],
                              "annotations": {PROFILE.annotation_idx: str(to), **ann}}}
        try:
            pod = self.api.patch("pods", body["namespace"], body["name"], patch)
        except HTTPError as e:
            eng.end_move(body["uid"], False)
            return Resp(409 if e.status == 409 else e.status, {"Error": f"apiserver {e.status}"})
        eng.end_move(body["uid"], True)
        return Resp(200, {"Error": "", "epoch": self.epoch, "to": to, "pod": pod})

    async def bind_task(self, uid: str):
        try:
            p = _by_uid(self.api, uid)
            if p is None:
                return
            md = p["metadata"]
            req = _request(p)
            eng = self.eng
            dev, total, seq, assume_ns = eng.assume_ordered(uid, md["namespace"], md["name"], NODE, req, "")
            if dev < 0:
                return
            while eng.bind_blocked(seq):
                await self.point("bind order wait")
            await self.point(f"Binding POST {md['name']}")
            ann = bind_annotations(PROFILE, dev, total, req, now_ns=assume_ns)
            try:
                self.api.bind(md["namespace"], md["name"], {"metadata": {"uid": uid, "annotations": ann},
                                                            "target": {"name": NODE}})
                ok = True
            except HTTPError:
                ok = False
            eng.bind_leave(seq)
            eng.finish_bind(uid, ok, 30.0)
        finally:
            self.binding.discard(uid)

    def deliver_ext(self):
        etype, obj = self.ext_q.popleft()
        uid = obj["metadata"]["uid"]
        deleting = bool(obj["metadata"].get("deletionTimestamp"))
        if etype == "DELETED" or _terminal(obj) or (deleting and "free_on_deleting" in self.muts):
            self.eng.remove_pod(uid)
        else:
            self.eng.upsert_pod_json(json.dumps(obj).encode())

    def restart_extender(self):
        """The extender process restarts (or another replica takes the lease): a ledger built from a LIST, a new
        epoch, binds to the publishing node held until its plugin publishes to this epoch."""
        self.gen += 1
        self.epoch = f"boot{self.gen}.1"
        self.eng = self.new_ledger()
        self.eng.begin_epoch(3600.0)
        self.ext_q.clear()

    # ------------------------------------------------------------ the plugin's informer
    def deliver_plugin(self):
        etype, obj = self.plugin_q.popleft()
        if etype == "DELETED":
            self.plugin.state.forget(obj)
        else:
            self.plugin._observe(obj)

    # ------------------------------------------------------------ kubelet
    def deliver_kubelet(self):
        etype, obj = self.kubelet_q.popleft()
        uid = obj["metadata"]["uid"]
        if etype == "DELETED":
            self.kgone.add(uid)
            self.kview.pop(uid, None)
        else:
            self.kview[uid] = obj
        if etype == "DELETED" or obj["metadata"].get("deletionTimestamp"):
            self.k_deleted_at.setdefault(uid, self.steps)

    def admission_candidate(self) -> str | None:
        cands = [p for uid, p in self.kview.items()
                 if uid not in self.admitted and not p["metadata"].get("deletionTimestamp")
                 and not _terminal(p)]
        if not cands:
            return None
        return min(cands, key=lambda p: (p["metadata"]["creationTimestamp"], p["metadata"]["name"]))["metadata"]["uid"]

    async def admit_task(self, uid: str):
        try:
            p = self.kview[uid]
            key = f"{p['metadata']['namespace']}/{p['metadata']['name']}"
            units = _request(p)
            # kubelet frees a force-deleted pod's device IDs as soon as it sees the delete (its container may still
            # run); a truthful one when the container has stopped
            taken = ({i for u, c in self.active.items() if self.sc.truthful or u not in self.kgone for i in c.ids}
                     | {i for ids in self.reserved.values() for i in ids})
            avail = [i for i in self.all_ids if i not in taken]
            if len(avail) < units and self.sc.truthful:
                return  # the node agent stand-in re-queues the pod until the stopping containers' IDs are free
            self.admitted.add(uid)
            if len(avail) < units:
                self.failed[uid] = "kubelet: not enough device IDs"
                return
            ids = avail[:units]
            if self.plugin.preferred:
                req = dpapi.PreferredAllocationRequest()
                req.container_requests.add(available_deviceIDs=avail, allocation_size=units)
                resp = await self.plugin.GetPreferredAllocation(req, None)
                ids = list(resp.container_responses[0].deviceIDs)
            self.reserved[uid] = ids
            areq = dpapi.AllocateRequest()
            areq.container_requests.add(devices_ids=ids)
            try:
                resp = await self.plugin.Allocate(areq, plugin_mod._NativeContext())
            except plugin_mod._Aborted as e:
                if "physically full" in e.details:
                    # the physical guard refusing to start a container on a GPU a stopping container still holds
                    # (a bind raced a force delete): the protocol's safe outcome, counted apart
                    self.refused[uid] = e.details
                else:
                    self.failed[uid] = e.details
                return
            finally:
                self.reserved.pop(uid, None)
            dev = int(resp.container_responses[0].envs[PROFILE.annotation_idx])
            # kubelet records the IDs as the Allocate call returns (podDevices): the container runs on `dev`
            self.active[uid] = Container(key, ids, dev, units)
        finally:
            self.admitting = False

    def stoppable(self) -> list[str]:
        return [uid for uid in self.active if uid in self.k_deleted_at
                and self.steps - self.k_deleted_at[uid] >= self.sc.stop_after]

    def finalizable(self) -> list[str]:
        return [uid for uid, p in self.kview.items()
                if p["metadata"].get("deletionTimestamp") and uid not in self.active and uid not in self.reserved]

    def stop(self, uid: str):
        self.active.pop(uid)
        self.stop_due.pop(uid, None)

    def finalize(self, uid: str):
        p = self.kview[uid]
        try:
            self.api.delete("pods", p["metadata"]["namespace"], p["metadata"]["name"], grace=0, uid=uid)
        except HTTPError:
            pass
        self.kview.pop(uid, None)

    # ------------------------------------------------------------ plugin background actors
    async def pass_task(self):
        try:
            await self.plugin.reconciler.run_once()
        except ApiError:
            pass  # the reconciler's loop outlives a pass an apiserver error cut short (Reconciler.run)
        finally:
            self.pass_running = False

    async def poll_task(self):
        try:
            await self.plugin.check_epoch()
        finally:
            self.poll_running = False

    # ------------------------------------------------------------ users
    def user_delete(self, uid: str, force: bool):
        p = _by_uid(self.api, uid)
        if p is None:
            return
        md = p["metadata"]
        if force:
            # the container gets its termination grace, then the runtime kills it (stop_due)
            self.stop_due[uid] = self.clock.t + TERM_GRACE_S
        self.api.delete("pods", md["namespace"], md["name"], grace=0 if force else 30)

    # ------------------------------------------------------------ the scheduler
    def enabled(self, users: bool, passes: bool = True) -> list[tuple[str, object]]:
        acts: list[tuple[str, object]] = []
        for g in self.gates:
            acts.append((f"resume {g.label}", lambda g=g: self._open(g)))
        if self.ext_q:
            acts.append(("deliver extender", self.deliver_ext))
        if self.plugin_q:
            acts.append(("deliver plugin", self.deliver_plugin))
        if self.kubelet_q:
            acts.append(("deliver kubelet", self.deliver_kubelet))
        if self.eng.publication_wait(NODE) <= 0:
            for p in self.api.list("pods"):
                md = p["metadata"]
                if ((p.get("spec") or {}).get("nodeName") or md.get("deletionTimestamp") or md["uid"] in self.binding
                        or _terminal(p) or self.eng.check(NODE, _request(p)) != 0):
                    continue
                acts.append((f"bind {md['name']}", lambda uid=md["uid"]: self._start_bind(uid)))
        if not self.admitting:
            c = self.admission_candidate()
            if c is not None:
                acts.append((f"admit {self.kview[c]['metadata']['name']}", lambda c=c: self._start_admit(c)))
        for uid in self.stoppable():
            acts.append((f"stop {uid}", lambda uid=uid: self.stop(uid)))
        for uid in self.finalizable():
            acts.append((f"finalize {uid}", lambda uid=uid: self.finalize(uid)))
        if passes and not self.pass_running and self.passes_left > 0:
            acts.append(("reconcile pass", self._start_pass))
        if not self.poll_running and ((users and self.polls_left > 0) or self.plugin._ext_epoch != self.epoch):
            acts.append(("epoch poll", self._start_poll))
        if users:
            if self.deletes_left > 0:
                live = [p for p in self.api.list("pods") if not p["metadata"].get("deletionTimestamp")]
                for p in live:
                    force = self.sc.grace == "force" or (self.sc.grace == "mixed" and self.rng.random() < 0.5)
                    acts.append((f"delete {p['metadata']['name']}{' force' if force else ''}",
                                 lambda uid=p["metadata"]["uid"], f=force: self._delete(uid, f)))
            if self.extra:
                acts.append(("create", self._create))
            if self.restarts_left > 0 and not self.binding:
                acts.append(("restart extender", self._restart))
        return acts

    def _open(self, g: Gate):
        self.gates.remove(g)
        if g.wake is not None:
            self.clock.t = max(self.clock.t, g.wake)
        g.fut.set_result(None)

    def _start_bind(self, uid):
        self.binding.add(uid)
        self.spawn(f"bind {uid}", self.bind_task(uid))

    def _start_admit(self, uid):
        self.admitting = True
        self.spawn(f"admit {uid}", self.admit_task(uid))

    def _start_pass(self):
        self.pass_running = True
        self.passes_left -= 1
        self.spawn("reconcile", self.pass_task())

    def _start_poll(self):
        self.poll_running = True
        self.polls_left -= 1
        self.spawn("epoch poll", self.poll_task())

    def _delete(self, uid, force):
        self.deletes_left -= 1
        self.user_delete(uid, force)

    def _create(self):
        self.pod(self.extra.pop(0))

    def _restart(self):
        self.restarts_left -= 1
        self.restart_extender()

    # ------------------------------------------------------------ invariants
    def committed(self) -> list[int]:
        """Per-GPU units the annotations promise (bound, non-terminal pods), an exchange in flight read as its
        protocol defines it: until the partner has taken P's old fields P's committed GPU is its hold-idx."""
        pods = [p for p in self.api.list("pods") if (p.get("spec") or {}).get("nodeName") == NODE and not _terminal(p)]
        by_uid = {p["metadata"]["uid"]: p for p in pods}
        used = [0] * self.sc.gpus
        for p in pods:
            a = p["metadata"].get("annotations") or {}
            try:
                dev = int(a.get(PROFILE.annotation_idx, "-1"))
            except ValueError:
                dev = -1
            if POD_HOLD_IDX_ANNOTATION in a:
                want = json.loads(a.get(POD_HOLD_PARTNER_ANNOTATION) or "{}")
                q = by_uid.get(want.get("uid", ""))
                qa = (q or {}).get("metadata", {}).get("annotations") or {}
                if q is not None and qa.get(PROFILE.annotation_idx) != str(want.get("idx")):
                    dev = int(a[POD_HOLD_IDX_ANNOTATION])
            if 0 <= dev < self.sc.gpus:
                used[dev] += _request(p)
        return used

    def check_safety(self):
        for d, u in enumerate(self.committed()):
            if u > self.sc.gpu_units:
                raise Violation(f"the annotations promise GPU {d} {u} > {self.sc.gpu_units} units")
        used = [0] * self.sc.gpus
        for c in self.active.values():
            used[c.dev] += c.units
        for d, u in enumerate(used):
            self.max_used[d] = max(self.max_used[d], u)
            if u > self.sc.gpu_units:
                held = ", ".join(f"{c.key}:{c.units}" for c in self.active.values() if c.dev == d)
                raise Violation(f"GPU {d} runs {u} > {self.sc.gpu_units} units ({held})")

    def check_converged(self):
        ann_used = [0] * self.sc.gpus
        for p in self.api.list("pods"):
            md, a = p["metadata"], p["metadata"].get("annotations") or {}
            uid = md["uid"]
            if POD_HOLD_IDX_ANNOTATION in a or POD_HOLD_PARTNER_ANNOTATION in a:
                raise Violation(f"{md['name']} still carries an exchange hold: {a}")
            if (p.get("spec") or {}).get("nodeName") == NODE and not _terminal(p):
                idx = int(a.get(PROFILE.annotation_idx, "-1"))
                if 0 <= idx < self.sc.gpus:
                    ann_used[idx] += _request(p)
                if uid in self.active:
                    c = self.active[uid]
                    if idx != c.dev or a.get(PROFILE.annotation_assigned) != "true":
                        raise Violation(f"{md['name']} runs on GPU {c.dev} but is annotated {idx} / "
                                        f"{a.get(PROFILE.annotation_assigned)}")
                elif not md.get("deletionTimestamp") and uid not in self.failed and uid not in self.refused:
                    raise Violation(f"{md['name']} is bound to the node and was never admitted")
        # an Allocate for a pod being deleted (kubelet admitted it before its view had the delete) may fail: the pod
        # goes anyway
        def live(uid):
            p = _by_uid(self.api, uid)
            return p is not None and not p["metadata"].get("deletionTimestamp")
        failed = {u: w for u, w in self.failed.items() if live(u)}
        refused = {u: w for u, w in self.refused.items() if live(u)}
        if failed or refused:
            raise Violation(f"Allocate failed: {failed or ''} refused by the physical guard: {refused or ''}")
        ledger = [used for _, used in self.eng.node_devices(NODE)]
        if ledger != ann_used:
            raise Violation(f"extender ledger {ledger} != annotations {ann_used}")
        un = self.eng.node_unaccounted(NODE)
        if any(un):
            raise Violation(f"unaccounted use {un} still published after convergence")

    # ------------------------------------------------------------ run
    async def _step(self, users: bool, passes: bool = True) -> bool:
        await self.settle()
        for uid, due in list(self.stop_due.items()):
            # the end of a force-deleted pod's grace: its container is gone (one admitted since -- kubelet's view
            # lagged the delete -- dies the moment it starts)
            if self.clock.t >= due and uid in self.active:
                self.stop_due.pop(uid)
                self.active.pop(uid)
        lc = self.plugin.state.core.linger_count()
        self.lingered += max(0, lc - self._lc)
        self._lc = lc
        self.check_safety()
        acts = self.enabled(users, passes)
        if not acts:
            if self.tasks:
                import traceback  # noqa: PLC0415
                where = []
                for t in self.tasks:
                    fr = t.get_stack(limit=1)
                    where.append(f"{t.get_name()} @ " + (traceback.format_stack(fr[0])[-1].strip().replace("\n", " ")
                                                          if fr else "?"))
                raise Violation(f"stuck: actors blocked outside any gate: {where}")
            return False
        self.widths.append(len(acts))
        if self.script is None:
            k = self.rng.randrange(len(acts))
        else:
            # the default order is a fair one: a sleep ends after the work already due (a delivery, a call's
            # answer), so an actor sleeping in a loop cannot starve the others but by the script's departures
            acts.sort(key=lambda a: a[0] == "resume sleep")
            k = self.script.get(self.steps, 0)
            k = k if k < len(acts) else 0
        name, fn = acts[k]
        self.trace.append(name)
        self.steps += 1
        self.clock.t += 0.001
        fn()
        return True

    async def run(self, tmpdir: str):
        self.setup(tmpdir)
        for _ in range(self.sc.max_steps):
            if not await self._step(users=True):
                break
            if not (self.deletes_left or self.extra or self.restarts_left or self.passes_left):
                break
        # drain: no more user actions.  Everything else runs (random order) until nothing is enabled but a
        # reconciliation pass; then one whole pass; converged once passes in a row change nothing
        quiet = 0
        for _ in range(60):
            self.clock.t += 1.0  # time passes: force-deleted pods' lingering shares expire
            for _ in range(self.sc.max_steps):
                if not await self._step(users=False, passes=False):
                    break
            rv = self.api.rv
            self._start_pass()
            for _ in range(self.sc.max_steps):
                if not (self.tasks or self.gates) or not await self._step(users=False, passes=False):
                    break
            # (a deleting pod's container kubelet has yet to stop: the drain waits for it)
            stopping = any(u in self.k_deleted_at or u in self.stop_due for u in self.active)
            settled = (not self.enabled(False, passes=False) and self.plugin._phys_published is None
                       and not stopping)
            quiet = quiet + 1 if self.api.rv == rv and settled else 0
            if quiet >= 3:
                break
        await self.settle()
        self.check_safety()
        self.check_converged()


def _terminal(p: dict) -> bool:
    return (p.get("status") or {}).get("phase") in ("Succeeded", "Failed")


def _request(p: dict) -> int:
    n = 0
    for c in (p.get("spec") or {}).get("containers") or []:
        v = ((c.get("resources") or {}).get("limits") or {}).get(PROFILE.resource)
        n += int(v or 0)
    return n


def _by_uid(api, uid):
    for p in api.store["pods"].values():
        if p["metadata"]["uid"] == uid:
            return p
    return None


def run_one(scenario: str | Scenario, seed: int, mutation: str = "", tmpdir: str = "/tmp/gsx-interleave",
            script: dict | None = None) -> Harness:
    """One schedule.  Raises Violation (with the trace attached) if an invariant breaks."""
    sc = SCENARIOS[scenario] if isinstance(scenario, str) else scenario
    h = Harness(sc, seed, mutation, script)
    saved = (plugin_mod.time, reconcile_mod.time, state_mod.time, asyncio.sleep, ApiError.not_found,
             reconcile_mod._took)
    plugin_mod.time = reconcile_mod.time = state_mod.time = h.clock
    if "fail_on_gone" in h.muts:
        ApiError.not_found = property(lambda self: False)
    asyncio.sleep = h.vsleep
    lg = logging.getLogger("gsx")
    level = lg.level
    lg.setLevel(logging.CRITICAL)
    try:
        loop = asyncio.new_event_loop()
        try:
            loop.run_until_complete(h.run(tmpdir))
        except Violation as e:
            e.args = (f"[{sc.name} seed {seed}{' ' + mutation if mutation else ''}"
                      f"{' script ' + json.dumps(script) if script is not None else ''}] {e.args[0]}\n  trace: "
                      + " | ".join(h.trace[-60:]),)
            raise
        finally:
            async def _cancel():
                rest = [t for t in asyncio.all_tasks() if t is not asyncio.current_task()]
                for t in rest:
                    t.cancel()
                await asyncio.gather(*rest, return_exceptions=True)

            loop.run_until_complete(_cancel())
            loop.close()
    finally:
        (plugin_mod.time, reconcile_mod.time, state_mod.time, asyncio.sleep, ApiError.not_found,
         reconcile_mod._took) = saved
        lg.setLevel(level)
    return h


def sweep(scenario: str, seeds, mutation: str = "") -> dict:
    out = {"scenario": scenario, "mutation": mutation, "runs": 0, "violations": [], "steps": 0, "swaps": 0,
           "guards": 0, "holds": 0, "moves": 0, "guard_refusals": 0, "lingered": 0, "faults": 0,
           "unequal_partners": 0, "unreconcilable": 0}
    for s in seeds:
        out["runs"] += 1
        try:
            h = run_one(scenario, s, mutation)
        except Violation as e:
            out["violations"].append(str(e))
            continue
        out["steps"] += h.steps
        rs = h.plugin.reconciler.stats
        out["swaps"] += rs.get("swaps", 0)
        out["holds"] += rs.get("holds_finished", 0)
        out["guards"] += h.plugin.stats.get("physical_guard", 0)
        out["moves"] += h.plugin.stats.get("moves", 0)
        out["guard_refusals"] += len(h.refused)
        out["lingered"] += h.lingered
        out["faults"] += h.faults
        out["unequal_partners"] += rs.get("unequal_partners", 0)
        out["unreconcilable"] += rs.get("unreconcilable", 0)
    return out


def systematic(scenario: str, bound: int = 1, window: int = 60, seed: int = 0, mutation: str = "",
               limit: int | None = None) -> dict:
    """Every schedule that departs from the default order -- the first enabled action at each step -- at no more than
    ``bound`` steps (1 or 2) among the first ``window`` (a preemption bound, as CHESS does): small bugs of ordering
    need few departures, and the bound makes the search exhaustive instead of sampled.  ``seed`` only fixes the
    other choices (which deletes are force deletes, injected faults)."""
    out = {"scenario": scenario, "bound": bound, "window": window, "runs": 0, "violations": [], "steps": 0}

    def one(script):
        out["runs"] += 1
        try:
            h = run_one(scenario, seed, mutation, script=script)
        except Violation as e:
            out["violations"].append(str(e))
            return None
        out["steps"] += h.steps
        return h

    base = one({})
    if base is None:
        return out
    firsts = [(i, j) for i, n in enumerate(base.widths[:window]) for j in range(1, n)]
    for i, j in firsts:
        if limit is not None and out["runs"] >= limit:
            break
        h = one({i: j})
        if bound < 2 or h is None:
            continue
        for i2, n2 in enumerate(h.widths[:window]):
            if i2 <= i:
                continue
            for j2 in range(1, n2):
                if limit is not None and out["runs"] >= limit:
                    break
                one({i: j, i2: j2})
    return out


def _seeds(spec: str):
    out = []
    for part in spec.split(","):
        a, _, b = part.partition("-")
        out.extend(range(int(a), int(b or a) + 1))
    return out


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n", 1)[0])
    ap.add_argument("--scenario", default="all", help=f"one of {sorted(SCENARIOS)} or all")
    ap.add_argument("--seeds", default="0-99")
    ap.add_argument("--mutation", default="", help=f"comma-separated, of {sorted(MUTATIONS)}")
    ap.add_argument("--systematic", type=int, default=0, metavar="BOUND",
                    help="instead of seeded random schedules: every schedule departing from the default order at <= "
                         "BOUND (1 or 2) of the first --window steps")
    ap.add_argument("--window", type=int, default=60)
    a = ap.parse_args(argv)
    if a.systematic:
        bad = 0
        for n in (sorted(SCENARIOS) if a.scenario == "all" else [a.scenario]):
            t0 = _time.perf_counter()
            r = systematic(n, a.systematic, a.window, mutation=a.mutation)
            r["seconds"] = round(_time.perf_counter() - t0, 1)
            viol = r.pop("violations")
            r["violations"] = len(viol)
            print(json.dumps(r), flush=True)
            for v in viol[:3]:
                print("  " + v, flush=True)
            bad += len(viol)
        return 1 if bad and not a.mutation else 0
    names = sorted(SCENARIOS) if a.scenario == "all" else [a.scenario]
    bad = 0
    for n in names:
        t0 = _time.perf_counter()
        r = sweep(n, _seeds(a.seeds), a.mutation)
        r["seconds"] = round(_time.perf_counter() - t0, 1)
        viol = r.pop("violations")
        r["violations"] = len(viol)
        print(json.dumps(r), flush=True)
        for v in viol[:3]:
            print("  " + v, flush=True)
        bad += len(viol)
    return 1 if bad and not a.mutation else 0


if __name__ == "__main__":
    sys.exit(main())
