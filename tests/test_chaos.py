"""Whole-stack fault injection: the fake apiserver answers 409 / 500 at random, drops watch streams and
expires watch resourceVersions while pods of mixed sizes are created and deleted; afterwards every
surviving pod must be bound, admitted and Running, no device over-committed, and the extender's ledger
equal to what the pod annotations record (the reference's durable state, pkg/utils/pod.go:192-206)."""
import asyncio
import json
import os
import random
import time

import pytest

from gpushare_scheduler_extender_amd.k8s.client import ApiError
from gpushare_scheduler_extender_amd.k8s.fasthttp import Client as HttpClient
from gpushare_scheduler_extender_amd.models.profile import (ALIYUN, POD_HOLD_IDX_ANNOTATION,
                                                            POD_HOLD_PARTNER_ANNOTATION)
from gsxtools.configs import NODE, Cluster


# kubelet's restart case (--batch-window: pods met within 20 ms admitted as one creationTimestamp-sorted batch) swaps
# equal-size pods nearly every batch while pods are deleted mid-admission.  The rows below run it through the compiled
# stand-in (native-plugin-batch) and the Python faithful kubelet over several seeds each: every surviving pod must end
# Running with physical == *_IDX.  What makes that hold: the plugin publishes to the extender the GPU use its
# containers hold where the annotations do not charge it (a deleted pod's allocation held by a swapped container),
# the extender charges it on top of the annotations, and an exchange of two unequal pods is checked on its final state
# (docs/ROUND5.md).
BATCH_SEEDS = (43, 47, 53, 59, 61)
if os.environ.get("GSX_CHAOS_BATCH_SEEDS"):  # a sweep: "first-last" (inclusive)
    _lo, _hi = (int(x) for x in os.environ["GSX_CHAOS_BATCH_SEEDS"].split("-"))
    BATCH_SEEDS = tuple(range(_lo, _hi + 1))


async def _retry(fn, *a, tries=50, **kw):
    for i in range(tries):
        try:
            return await fn(*a, **kw)
        except ApiError as e:
            if e.status == 409 and "already exists" in str(e):
                return None
            if e.status not in (409, 500) or i == tries - 1:
                raise
            await asyncio.sleep(0.002)


def _committed_use(cl, bound: dict) -> tuple[list[int], int]:
    """Per-device units from the annotations, reading a reconciliation exchange in flight the way its protocol
    defines it (``deviceplugin/reconcile.py``): until the partner Q has taken P's old fields, P's committed device
    is its ``hold-idx`` (P's new fields duplicate Q's); once Q has them, P's new ``*_IDX`` is.  Returns the
    per-device sums and the number of holds outstanding."""
    by_uid = {p["metadata"]["uid"]: p for p in bound.values()}
    used, holds = [0] * len(cl.totals), 0
    for p in bound.values():
        ann = p["metadata"]["annotations"]
        dev = cl.device_of(p)
        if POD_HOLD_IDX_ANNOTATION in ann:
            holds += 1
            want = json.loads(ann.get(POD_HOLD_PARTNER_ANNOTATION) or "{}")
            q = by_uid.get(want.get("uid", ""))
            if q is not None and cl.device_of(q) != want.get("idx"):
                dev = int(ann[POD_HOLD_IDX_ANNOTATION])
        used[dev] += int(ann[ALIYUN.annotation_pod])
    return used, holds


@pytest.mark.parametrize("seed,agent,bind_mode,early", [(7, "plugin", "binding", True),
                                                        (11, "plugin", "binding", False),
                                                        (23, "native", "binding", True),
                                                        (11, "native", "binding", True),
                                                        (17, "native-plugin", "binding", True),
                                                        (19, "native-plugin", "update", True),
                                                        (41, "native-plugin", "binding", False),
                                                        *[(sd, "native-plugin-batch", "binding", True)
                                                          for sd in BATCH_SEEDS],
                                                        *[(sd, "faithful", "binding", True) for sd in BATCH_SEEDS[1:]],
                                                        (13, "plugin", "update", True),
                                                        (7, "faithful", "binding", True),
                                                        (29, "faithful", "update", False),
                                                        (13, "faithful-event", "binding", True),
                                                        (31, "faithful-event", "update", True)])
def test_chaos_whole_stack_converges_without_overcommit(seed, agent, bind_mode, early, monkeypatch):
    """``agent``: kubelet + the shipped gRPC device plugin
    (the product path), the same behind a *faithful* kubelet (no re-routing, PodResources reconciliation; here
    with 20 ms creationTimestamp-sorted admission batches, kubelet's restart case, so swaps do happen), or the
    compiled node agent (``native``: its in-process matcher; ``native-plugin``: kubelet-faithful, calling the shipped
    plugin process over gRPC and serving it PodResources; ``-batch``: with 20 ms creationTimestamp batches);
    ``faithful-event``: the faithful kubelet admitting one pod per watch event (its steady state) with every bind
    concurrent (landing-order node); ``bind_mode``: one annotated Binding, or the reference's annotation write +
    Binding (two calls, the first guarded by resourceVersion); ``early``: the plugin answers an Allocate once its
    record is journaled and commits ASSIGNED behind it (the default), or after the commit.

    On every poll the annotations -- the allocation record the extender's ledger is built from -- never promise a
    GPU past its capacity (the extender is the one writer of ``*_IDX``: the plugin's reconciliation moves go through
    it), and behind a faithful kubelet neither do the containers physically."""
    faithful = agent.startswith("faithful")
    kubelet_args = ["--faithful"] + (["--batch-window", "0.02"] if agent == "faithful" else [])
    monkeypatch.setenv("GSX_PLUGIN_EARLY_ANSWER", "1" if early else "0")
    cl_agent = "plugin" if faithful else ("native-plugin" if agent.startswith("native-plugin") else agent)
    args = kubelet_args if faithful else (["--batch-window", "0.02"] if agent == "native-plugin-batch" else [])

    async def go():
        rnd = random.Random(seed)
        cl = Cluster(ALIYUN, [96] * 4, gpu=False, agent=cl_agent, bind_mode=bind_mode, agent_args=args)
        try:
            await cl.start()
            api = HttpClient(cl.api.url)
            faults = {"conflict_rate": 0.15, "error_rate": 0.1, "drop_watch_after": 40, "expire_watches": 2,
                      "seed": seed}
            await api.request("POST", "/fake/faults", json.dumps(faults).encode())
            sizes = [8, 16, 24, 32]
            live, deleted = {}, set()
            for wave in range(4):
                names = [f"c{wave}-{i}" for i in range(10)]
                for n in names:
                    live[n] = rnd.choice(sizes)
                    await _retry(cl.create, n, live[n])
                await asyncio.sleep(0.05)
                for n in rnd.sample(sorted(live), 4):  # delete some, bound or not
                    await _retry(cl.c.delete, "pods", n, "default")
                    deleted.add(n)
                    live.pop(n)
            await api.request("POST", "/fake/faults", json.dumps({"conflict_rate": 0, "error_rate": 0,
                                                                  "drop_watch_after": 0}).encode())
            # capacity 4 x 96 GiB: whatever fits is bound and Running; the rest stays Pending (never Failed)
            deadline = time.monotonic() + 30
            while True:
                pods = {p["metadata"]["name"]: p for p in (await cl.c.list("pods", "default"))["items"]}
                assert set(pods) == set(live), (sorted(set(pods) ^ set(live)))
                bound = {n: p for n, p in pods.items() if p["spec"].get("nodeName")}
                running = [n for n, p in bound.items() if p["status"].get("phase") == "Running"]
                failed = [n for n, p in pods.items() if p["status"].get("phase") == "Failed"]
                if failed:
                    raise AssertionError((failed, [ch.tail(20) for ch in cl.children if ch.name == "node-agent"],
                                          await _plugin_state(cl), await _physical_use(cl, bound, running)))
                used, holds = _committed_use(cl, bound)
                assert all(u <= 96 for u in used), ("annotations", used)
                if faithful or agent.startswith("native-plugin"):
                    # kubelet's real env: two containers' shares never past a GPU's capacity either
                    phys = await _physical_use(cl, bound, running)
                    assert all(u <= 96 for u in phys), ("physical", phys)
                pending = [live[n] for n in live if n not in bound]
                free = [96 - u for u in used]
                settled = not holds and len(running) == len(bound) and all(s > max(free) for s in pending)
                insp = await cl.inspect()
                ledger = [d["usedGPU"] for d in insp["nodes"][0]["devs"]]
                if settled and ledger == used:
                    assert all(u <= 96 for u in used), used
                    break
                if time.monotonic() >= deadline:  # (a string: pytest shortens a dict message)
                    raise AssertionError(json.dumps({"used": used, "ledger": ledger, "pending": pending,
                                                     "running": len(running), "bound": len(bound), "holds": holds,
                                                     "hold_pods": {n: {k: v for k, v in (p["metadata"].get(
                                                         "annotations") or {}).items() if "hold" in k or k in (
                                                         ALIYUN.annotation_idx, ALIYUN.annotation_assigned)}
                                                         for n, p in bound.items() if POD_HOLD_IDX_ANNOTATION in (
                                                             p["metadata"].get("annotations") or {})},
                                                     "node": insp["nodes"][0], "plugin": await _plugin_state(cl)},
                                                    default=str))
                await asyncio.sleep(0.05)
            # every running container is on the GPU its annotation names (physical == *_IDX), holds cleared
            drift, drifted = await cl.physical_drift(sorted(live), timeout=15)
            assert drift == 0, drifted

            st = json.loads((await api.request("GET", "/fake/stats")).body)
            assert st["counts"].get("injected_conflict", 0) > 0 and st["counts"].get("injected_error", 0) > 0
            await api.close()
            ext = HttpClient(cl.ext.url)
            srv = json.loads((await ext.request("GET", "/debug/engine")).body)["server"]
            await ext.close()

            # update mode writes the annotations before each Binding: at least two apiserver calls per bind
            assert srv["bind_ok"] > 0
            # (the plugin's reconciliation moves are extender apiserver calls too)
            assert (srv["api_calls"] - srv.get("moves", 0) >= 2 * srv["bind_ok"]) == (bind_mode == "update"), srv
        finally:
            await cl.close()
    asyncio.run(go())


async def _plugin_state(cl) -> dict:
    """The spawned plugin's /debug/state (physical account, records, counters), for a failure message."""
    try:
        url = (await cl.agent_stats()).get("plugin_debug")
        if not url:
            return {}
        h = HttpClient(url)
        try:
            r = await h.request("GET", "/debug/state")
            d = json.loads(r.body)
        finally:
            await h.close()
        return {k: d.get(k) for k in ("physical", "held", "records", "cu_free", "reconcile", "grpc", "stats")}
    except Exception as e:  # noqa: BLE001 - diagnostics only
        return {"error": repr(e)}


async def _physical_use(cl, bound: dict, running: list) -> list[int]:
    """Per-device units of the running containers, from the GPU kubelet's Allocate env gave each."""
    out = [0] * len(cl.totals)
    for n in running:
        p = bound[n]
        env = (await cl.allocation(p["metadata"]["uid"])).get("envs", {})
        if env:
            out[int(env[ALIYUN.annotation_idx])] += int(p["metadata"]["annotations"][ALIYUN.annotation_pod])
    return out


async def _settled(cl, names, timeout=30.0):
    """All ``names`` bound and Running; returns per-device GiB from the annotations of the bound pods once
    the extender's ledger reports exactly that."""
    deadline = time.monotonic() + timeout
    while True:
        pods = {p["metadata"]["name"]: p for p in (await cl.c.list("pods", "default"))["items"]}
        ok = all(n in pods and pods[n]["status"].get("phase") == "Running" for n in names)
        used = [0] * len(cl.totals)
        for p in pods.values():
            if p["spec"].get("nodeName"):
                used[cl.device_of(p)] += int(p["metadata"]["annotations"][ALIYUN.annotation_pod])
        try:
            ledger = [d["usedGPU"] for d in (await cl.inspect())["nodes"][0]["devs"]]
        except (OSError, ValueError, KeyError, IndexError):
            ledger = None
        if ok and ledger == used:
            return used
        assert time.monotonic() < deadline, {"used": used, "ledger": ledger}
        await asyncio.sleep(0.05)


def test_extender_crash_restart_rebuilds_ledger_from_annotations():
    """Checkpoint / resume: the durable state is the pod annotations (pkg/utils/pod.go:192-206).  The
    extender is SIGKILLed with pods placed, more pods arrive while it is down (kube-scheduler's filter and
    bind calls fail and are retried), a new process on the same port rebuilds the ledger from the
    annotations and placement resumes without over-committing a device."""
    async def go():
        cl = Cluster(ALIYUN, [96] * 4, gpu=False)
        try:
            await cl.start()
            first = [f"a{i}" for i in range(8)]
            for n in first:
                await cl.create(n, 24)
            assert await _settled(cl, first) == [96, 96, 0, 0]  # binpack: best fit fills a device first
            cl.kill_extender()
            second = [f"b{i}" for i in range(6)]
            for n in second:
                await cl.create(n, 16)
            await asyncio.sleep(0.3)
            pods = {p["metadata"]["name"]: p for p in (await cl.c.list("pods", "default"))["items"]}
            assert not any(pods[n]["spec"].get("nodeName") for n in second)  # nothing binds without it
            cl.restart_extender()
            assert await _settled(cl, first + second) == [96, 96, 96, 0]
        finally:
            await cl.close()
    asyncio.run(go())


def test_reservation_gc_never_frees_a_device_behind_a_stalled_watch():
    """a bound reservation the informer has not confirmed within its TTL must not be dropped
    while the pod watch is stalled and LISTs fail (the device would look free while the pod holds it); once
    a LIST begun after the binding succeeds it decides: confirmed -> kept, absent -> expired."""
    from gpushare_scheduler_extender_amd.extender.server import ExtenderRunner, ExtenderServer
    from gpushare_scheduler_extender_amd.k8s.client import KubeClient
    from tests.fixtures.fakeapi import FakeApiServerRunner
    from gpushare_scheduler_extender_amd.k8s.objects import make_node, make_pod
    from gpushare_scheduler_extender_amd.models import wire
    from gpushare_scheduler_extender_amd.models.profile import SHARED_GPU

    async def go():
        api = await FakeApiServerRunner().start()
        c = KubeClient(api.url)
        await c.create("nodes", make_node("n", 100, 1))
        srv = ExtenderServer(KubeClient(api.url), SHARED_GPU, reservation_ttl=0.2)
        ext = await ExtenderRunner(srv).start()
        http = HttpClient(ext.url)
        eng = srv.engine
        try:
            for _ in range(200):
                if eng.has_node("n"):
                    break
                await asyncio.sleep(0.01)

            async def filter_(pod):
                r = await http.request("POST", "/gpushare-scheduler/filter", wire.filter_args(pod, ["n"]))
                return json.loads(r.body)

            async def bind(pod):
                args = wire.ExtenderBindingArgs(pod["metadata"]["name"], "default", pod["metadata"]["uid"], "n")
                r = await http.request("POST", "/gpushare-scheduler/bind", args.encode())
                return r.status

            # the extender's pod watch stalls (dropped, new watches never answered) and LISTs fail
            fa = HttpClient(api.url)
            await fa.request("POST", "/fake/faults", json.dumps({"hold_watches": True, "fail_lists": True,
                                                                 "drop_watches_now": True}).encode())
            await fa.close()
            await asyncio.sleep(0.1)
            a = await c.create("pods", make_pod("a", 60))
            assert (await filter_(a))["NodeNames"] == ["n"]
            assert await bind(a) == 200
            await asyncio.sleep(1.0)  # 5 x the TTL, GC runs every 0.05 s
            assert eng.node_devices("n") == [(100, 60)], "reservation dropped behind a stalled watch"
            b = make_pod("b", 60)
            assert (await filter_(b))["NodeNames"] == []  # still no room: never over-committed
            assert eng.stats()["expired"] == 0 and eng.stats()["expiry_deferred"] > 0
            # LISTs work again (watches still held): the forced re-list confirms the binding -> kept
            api.server.faults.fail_lists = False
            await asyncio.sleep(0.6)
            assert eng.node_devices("n") == [(100, 60)] and eng.stats()["expired"] == 0
            # a binding the apiserver no longer has (pod deleted unseen): the next LIST proves it -> expired
            await c.delete("pods", "a", "default")
            await asyncio.sleep(0.05)
            p2 = await c.create("pods", make_pod("p2", 30))
            await filter_(p2)
            assert await bind(p2) == 200
            await c.delete("pods", "p2", "default")
            for _ in range(200):
                if eng.node_devices("n") == [(100, 0)]:
                    break
                await asyncio.sleep(0.02)
            assert eng.node_devices("n") == [(100, 0)]
            assert eng.stats()["expired"] >= 1
        finally:
            api.server.faults.hold_watches = False
            await http.close()
            await ext.stop()
            await srv.client.close()
            await c.close()
            await api.stop()
    asyncio.run(go())


@pytest.mark.parametrize("agent", ["plugin", "faithful"])
def test_binding_annotations_dropped_by_apiserver_self_heals(agent):
    """``binding`` mode trusts kube-apiserver to copy Binding.metadata.annotations onto the pod.
    An apiserver that drops them leaves pods bound without ``*_IDX``; the extender must notice, write the
    annotations back (the reference's update call), switch to annotate-then-bind, and nothing may fail."""
    async def go():
        cl = Cluster(ALIYUN, [96] * 4, gpu=False, agent="plugin", agent_args=["--faithful"] if agent == "faithful" else [])
        try:
            await cl.start()
            api = HttpClient(cl.api.url)
            await api.request("POST", "/fake/faults", json.dumps({"drop_binding_annotations": True}).encode())
            names = [f"d{i}" for i in range(10)]
            sizes = [48, 24, 24, 48, 32, 16, 64, 8, 24, 40]
            for n, g in zip(names, sizes):
                await cl.create(n, g)
            pods = await cl.wait(names, timeout=60)
            for _ in range(500):  # early answer (default): Running can come before the ASSIGNED commit lands
                if all(p["metadata"]["annotations"].get(ALIYUN.annotation_assigned) == "true" for p in pods.values()):
                    break
                await asyncio.sleep(0.02)
                pods = {p["metadata"]["name"]: p for p in (await cl.c.list("pods", "default"))["items"]
                        if p["metadata"]["name"] in names}
            used = [0] * 4
            for p in pods.values():
                ann = p["metadata"]["annotations"]
                assert ALIYUN.annotation_idx in ann and ann[ALIYUN.annotation_assigned] == "true", ann
                used[cl.device_of(p)] += int(ann[ALIYUN.annotation_pod])
            assert all(u <= 96 for u in used), used
            insp = await cl.inspect()
            assert [d["usedGPU"] for d in insp["nodes"][0]["devs"]] == used
            st = await cl.agent_stats()
            assert st["allocate_errors"] == 0 and st["failed"] == 0, st
            ext = HttpClient(cl.ext.url)
            metrics = (await ext.request("GET", "/metrics")).body.decode()
            await ext.close()
            assert "gpushare_bind_mode_update 1.0" in metrics
            assert 'gpushare_bind_annotation_repairs_total{result="ok"}' in metrics
            # after the switch, binds write the annotations first: new pods arrive annotated without repair
            await cl.create("late", 8)
            late = (await cl.wait(["late"]))["late"]
            assert ALIYUN.annotation_idx in late["metadata"]["annotations"]
            await api.close()
        finally:
            await cl.close()
    asyncio.run(go())


GRACE_SEEDS = (3, 5, 8)
if os.environ.get("GSX_CHAOS_GRACE_SEEDS"):  # a sweep: "first-last" (inclusive)
    _lo, _hi = (int(x) for x in os.environ["GSX_CHAOS_GRACE_SEEDS"].split("-"))
    GRACE_SEEDS = tuple(range(_lo, _hi + 1))


@pytest.mark.parametrize("agent", ["native-plugin", "faithful"])
@pytest.mark.parametrize("seed", GRACE_SEEDS)
def test_chaos_graceful_deletes_on_a_full_node(seed, agent, monkeypatch):
    """pods are deleted the way users delete them -- gracefully, ``gracePeriodSeconds`` 2-3 s -- on a
    node whose GPUs are full, with containers that take that long to stop (``--stop-delay``), while new pods wait
    for the room.  kube-apiserver only marks such a pod; its kubelet stops the containers, reports the terminal phase
    and deletes the object with grace 0.  The extender keeps a terminating pod's share charged until then, so no
    pod is bound into room a stopping container still fills: no pod fails, the plugin's physical guard never takes
    its fail-closed branch, and neither the annotations nor the containers ever promise a GPU past its capacity."""
    monkeypatch.setenv("GSX_PLUGIN_GUARD_WAIT_S", "0.5")
    monkeypatch.setenv("GSX_PLUGIN_GUARD_GONE_WAIT_S", "1.0")
    faithful = agent == "faithful"
    cl_agent = "plugin" if faithful else "native-plugin"
    args = (["--faithful"] if faithful else []) + ["--stop-delay", "2.0"]

    async def go():
        rnd = random.Random(seed)
        cl = Cluster(ALIYUN, [96] * 4, gpu=False, agent=cl_agent, agent_args=args)
        try:
            await cl.start()
            live: dict[str, int] = {}
            for i in range(16):  # full: 4 x 24 GiB per GPU
                live[f"f{i}"] = 24
                await cl.create(f"f{i}", 24)
            await cl.wait(sorted(live), timeout=30)
            terminating: set[str] = set()
            for rnd_no in range(3):
                victims = rnd.sample(sorted(live), 4)
                for n in victims:
                    await cl.c.delete("pods", n, "default", grace_seconds=rnd.choice([2, 3]))
                    live.pop(n)
                    terminating.add(n)
                new = [f"r{rnd_no}-{k}" for k in range(4)]
                for n in new:  # the same room again, in other sizes: they wait for the stopping containers
                    live[n] = rnd.choice([8, 16, 24])
                    await cl.create(n, live[n])
                deadline = time.monotonic() + 30
                while True:
                    pods = {p["metadata"]["name"]: p for p in (await cl.c.list("pods", "default"))["items"]}
                    failed = [n for n, p in pods.items() if p["status"].get("phase") == "Failed"]
                    assert not failed, (failed, await _plugin_state(cl))
                    bound = {n: p for n, p in pods.items() if p["spec"].get("nodeName")}
                    running = [n for n, p in bound.items() if p["status"].get("phase") == "Running"]
                    used, holds = _committed_use(cl, bound)
                    assert all(u <= 96 for u in used), ("annotations", used)
                    phys = await _physical_use(cl, bound, running)
                    assert all(u <= 96 for u in phys), ("physical", phys)
                    terminating &= set(pods)
                    if not terminating and all(n in running for n in live) and not holds:
                        break
                    assert time.monotonic() < deadline, {"terminating": sorted(terminating), "used": used,
                                                         "running": len(running), "live": len(live)}
                    await asyncio.sleep(0.05)
            drift, drifted = await cl.physical_drift(sorted(live), timeout=15)
            assert drift == 0, drifted
            insp = await cl.inspect()
            assert [d["usedGPU"] for d in insp["nodes"][0]["devs"]] == _committed_use(cl, {
                n: p for n, p in pods.items() if n in live})[0]
            st = await cl.agent_stats()
            assert st["failed"] == 0 and st.get("finalized", 0) >= 12, st
            ps = (await _plugin_debug(cl)).get("stats") or {}
            assert ps.get("physical_guard_failed", 0) == 0 and ps.get("allocate_fail", 0) == 0, ps
        finally:
            await cl.close()
    asyncio.run(go())


@pytest.mark.parametrize("agent", ["native-plugin", "plugin"])
def test_chaos_apiserver_throttling_every_call_retried(agent):
    """API Priority and Fairness answers 20 % of the stack's apiserver calls 429 with Retry-After
    (scheduler, extender binds and reflectors, plugin commits, kubelet status).  Every client waits the server's
    Retry-After and sends again (client-go's contract), so every pod ends bound and Running and no bind fails."""
    async def go():
        cl = Cluster(ALIYUN, [96] * 4, gpu=False, agent=agent)
        try:
            await cl.start()
            api = HttpClient(cl.api.url)
            await api.request("POST", "/fake/faults", json.dumps({"throttle_rate": 0.2, "retry_after": 0.01,
                                                                  "seed": 9}).encode())
            names = [f"t{i}" for i in range(24)]
            rnd = random.Random(9)
            for n in names:
                await cl.create(n, rnd.choice([8, 12, 16]))
            await cl.wait(names, timeout=60)
            for n in names[:8]:
                await cl.c.delete("pods", n, "default")
            more = [f"u{i}" for i in range(8)]
            for n in more:
                await cl.create(n, 8)
            await cl.wait(more, timeout=60)
            st = json.loads((await api.request("GET", "/fake/stats")).body)
            await api.request("POST", "/fake/faults", json.dumps({"throttle_rate": 0}).encode())
            await api.close()
            assert st["counts"].get("injected_throttle", 0) >= 15, st["counts"]
            ext = HttpClient(cl.ext.url)
            srv = json.loads((await ext.request("GET", "/debug/engine")).body)["server"]
            await ext.close()
            assert srv["bind_fail"] == 0 and srv["bind_ok"] >= 32, srv
            ast = await cl.agent_stats()
            assert ast["failed"] == 0 and ast.get("allocate_errors", 0) == 0, ast
        finally:
            await cl.close()
    asyncio.run(go())


async def _plugin_debug(cl) -> dict:
    try:
        url = (await cl.agent_stats()).get("plugin_debug")
        if not url:
            return {}
        h = HttpClient(url)
        try:
            return json.loads((await h.request("GET", "/debug/state")).body)
        finally:
            await h.close()
    except (OSError, ValueError):
        return {}


def test_extender_restart_holds_binds_until_the_node_republishes_its_physical_use():
    """VERDICT r5 #3 / ADVICE r5: the device plugin's publication of its unaccounted GPU use (containers holding room
    the annotations put elsewhere) lives only in the extender's memory.  A SIGKILLed extender comes back in a new
    epoch; binds to a node whose plugin publishes (node annotation) wait for that plugin's first publication of the
    epoch, so no bind lands in room a swapped container still fills, and binds resume as soon as it arrives.  A
    standby answers /physical 503 (the plugin must not count it delivered)."""
    from gpushare_scheduler_extender_amd.models.profile import NODE_PHYSICAL_PUBLICATION_ANNOTATION
    from gsxtools.configs import NODE as N

    async def go():
        cl = Cluster(ALIYUN, [96, 96], gpu=False, agent="inproc")
        try:
            await cl.start()
            await cl.c.patch("nodes", N, {"metadata": {"annotations": {NODE_PHYSICAL_PUBLICATION_ANNOTATION: "true"}}})

            async def ext(method, path, body=None):
                h = HttpClient(cl.ext.url)
                try:
                    r = await h.request(method, path, json.dumps(body).encode() if body is not None else None)
                    return r.status, json.loads(r.body or b"{}")
                finally:
                    await h.close()

            async def publish(extra):
                return await ext("POST", "/gpushare-scheduler/physical", {"node": N, "unaccounted": extra, "ttl": 60})

            async def node_of(name):
                return (await cl.c.get("pods", name, "default"))["spec"].get("nodeName")

            st, e1 = await ext("GET", "/gpushare-scheduler/epoch")
            assert st == 200 and e1["leader"] and e1["epoch"]
            st, body = await publish(None)  # the plugin's first publication of the epoch: nothing unaccounted
            assert st == 200 and body["epoch"] == e1["epoch"]
            await cl.create("a", 60)  # best fit: GPU 0 (36 free after)
            await cl.wait(["a"])
            assert cl.device_of(await cl.c.get("pods", "a", "default")) == 0
            # a swapped container physically fills 90 of GPU 1 that no annotation charges there
            assert (await publish([0, 90]))[0] == 200
            cl.kill_extender()
            cl.restart_extender()  # rebuilt from the annotations: the publication is gone
            for _ in range(400):
                st, e2 = await ext("GET", "/gpushare-scheduler/epoch")
                if st == 200:
                    break
                await asyncio.sleep(0.01)
            assert e2["epoch"] != e1["epoch"]
            # 48 GiB fits GPU 1 by the annotations only: held while the node has not republished
            await cl.create("b", 48)
            await asyncio.sleep(1.0)
            assert await node_of("b") is None, "bound before the node republished its physical use"
            t0 = time.monotonic()
            st, body = await publish([0, 90])  # the plugin saw the epoch change and republishes
            assert st == 200 and body["epoch"] == e2["epoch"]
            await asyncio.sleep(1.0)
            assert await node_of("b") is None  # no room anywhere: never into the unaccounted room
            t1 = time.monotonic()
            assert (await publish(None))[0] == 200  # the swapped container stopped: withdrawn
            for _ in range(200):
                if await node_of("b"):
                    break
                await asyncio.sleep(0.01)
            assert await node_of("b") == N and time.monotonic() - t1 < 1.0
            assert cl.device_of(await cl.c.get("pods", "b", "default")) == 1
            srv = (await ext("GET", "/debug/engine"))[1]["server"]
            assert srv["publication_waits"] >= 1, srv
            assert t1 - t0 >= 1.0
        finally:
            await cl.close()
    asyncio.run(go())
