"""End-to-end slice A: fake apiserver + extender + controller + scheduler simulator.

BASELINE.json config 1: one node with one fake device, two pods requesting
gpu-mem binpack onto device 0, annotations written, /inspect shows it.
"""
import asyncio
import json

import aiohttp
import pytest

from gpushare_scheduler_extender_amd.extender.server import ExtenderRunner, ExtenderServer
from gpushare_scheduler_extender_amd.k8s.client import KubeClient
from tests.fixtures.fakeapi import FakeApiServerRunner
from gpushare_scheduler_extender_amd.k8s.objects import make_node, make_pod
from gpushare_scheduler_extender_amd.models import wire
from gpushare_scheduler_extender_amd.models.profile import ALIYUN, SHARED_GPU
from tests.fixtures.schedsim import SchedulerSim


class Cluster:
    def __init__(self, profile=SHARED_GPU, bind_mode="binding", **ext_kw):
        self.profile = profile
        self.bind_mode = bind_mode
        self.ext_kw = ext_kw

    async def __aenter__(self):
        self.api = await FakeApiServerRunner().start()
        self.client = KubeClient(self.api.url)
        self.ext = await ExtenderRunner(ExtenderServer(KubeClient(self.api.url), self.profile,
                                                       bind_mode=self.bind_mode, **self.ext_kw)).start()
        self.sim = None
        self.http = aiohttp.ClientSession()
        return self

    async def start_sim(self, **kw):
        self.sim = SchedulerSim(KubeClient(self.api.url), self.ext.url, self.profile, **kw)
        await self.sim.start()
        return self.sim

    async def __aexit__(self, *exc):
        if self.sim:
            await self.sim.stop()
            await self.sim.client.close()
        await self.ext.stop()
        await self.ext.server.client.close()
        await self.client.close()
        await self.http.close()
        await self.api.stop()

    async def settle(self, cond, timeout=5.0):
        for _ in range(int(timeout / 0.005)):
            if cond():
                return
            await asyncio.sleep(0.005)
        raise TimeoutError("condition not reached")

    async def get(self, path):
        async with self.http.get(self.ext.url + path) as r:
            return r.status, await r.read()

    async def post(self, path, body: bytes):
        async with self.http.post(self.ext.url + path, data=body) as r:
            return r.status, await r.read()


def run(coro):
    return asyncio.run(coro)


def test_slice_a_two_pods_binpack_one_device():
    async def go():
        async with Cluster() as c:
            await c.client.create("nodes", make_node("node-1", 30, 1))
            eng = c.ext.server.engine
            await c.settle(lambda: eng.has_node("node-1"))
            await c.start_sim()
            for i in range(2):
                await c.client.create("pods", make_pod(f"binpack-{i}", 2))
            await c.sim.wait_bound(["default/binpack-0", "default/binpack-1"], 10)
            await c.settle(lambda: eng.node_devices("node-1") == [(30, 4)])
            for i in range(2):
                p = await c.client.get("pods", f"binpack-{i}", "default")
                ann = p["metadata"]["annotations"]
                assert p["spec"]["nodeName"] == "node-1"
                assert ann["SHARED_GPU_MEM_IDX"] == "0" and ann["SHARED_GPU_MEM_POD"] == "2"
                assert ann["SHARED_GPU_MEM_DEV"] == "30" and ann["SHARED_GPU_MEM_ASSIGNED"] == "false"
                assert int(ann["SHARED_GPU_MEM_ASSUME_TIME"]) > 0
            # reservations are confirmed by the informer (not left as "assumed")
            await c.settle(lambda: all(eng.pod_state(c.sim.pods.get(f"default/binpack-{i}")["metadata"]["uid"])[0] == 1
                                       for i in range(2)))
            st, body = await c.get("/gpushare-scheduler/inspect")
            assert st == 200
            res = wire.InspectResult.decode(body)
            assert res.nodes[0].usedGPU == 4
            assert sorted(p.name for p in res.nodes[0].devs[0].pods) == ["binpack-0", "binpack-1"]
            st, body = await c.get("/gpushare-scheduler/inspect/node-1")
            assert st == 200 and json.loads(body)["nodes"][0]["name"] == "node-1"
    run(go())


def test_routes_version_and_status_codes():
    async def go():
        async with Cluster() as c:
            st, body = await c.get("/version")
            assert (st, body) == (200, b"0.1.0")
            st, body = await c.post("/gpushare-scheduler/filter", b"garbage")
            assert st == 200 and json.loads(body)["Error"]  # filter: always 200 (routes.go:94-96)
            st, body = await c.post("/gpushare-scheduler/bind", b"garbage")
            assert st == 500 and json.loads(body)["Error"]  # bind: 500 iff Error (routes.go:139-143)
            args = wire.ExtenderBindingArgs("ghost", "default", "uid-x", "n").encode()
            st, body = await c.post("/gpushare-scheduler/bind", args)
            assert st == 500 and json.loads(body)["Error"] == 'pods "ghost" not found'
            st, body = await c.get("/gpushare-scheduler/inspect/nope")
            assert st == 200 and json.loads(body) == {"nodes": [], "error": 'node "nope" not found'}
            st, body = await c.get("/debug/pprof/")
            assert st == 200 and b"goroutine" in body
            st, body = await c.get("/debug/pprof/goroutine/")
            assert st == 200 and b"asyncio tasks" in body
            st, body = await c.get("/metrics")
            assert st == 200 and b"gpushare_binpack_utilization" in body
    run(go())


def test_pprof_can_be_turned_off():
    async def go():
        async with Cluster(pprof=False) as c:
            st, _ = await c.get("/debug/pprof/")
            assert st == 404
            st, body = await c.get("/version")
            assert (st, body) == (200, b"0.1.0")
    run(go())


def test_bind_uid_mismatch_error_string():
    async def go():
        async with Cluster() as c:
            await c.client.create("nodes", make_node("n", 10, 1))
            await c.client.create("pods", make_pod("p", 2, uid="real-uid"))
            await c.settle(lambda: c.ext.server.engine.has_node("n"))
            args = wire.ExtenderBindingArgs("p", "default", "other-uid", "n").encode()
            st, body = await c.post("/gpushare-scheduler/bind", args)
            assert st == 500
            assert json.loads(body)["Error"] == ("The pod p in ns default's uid is real-uid, and it's not equal "
                                                 "with expected other-uid")
    run(go())


@pytest.mark.parametrize("mode", ["binding", "update"])
def test_bind_modes_and_cant_place(mode):
    async def go():
        async with Cluster(bind_mode=mode) as c:
            await c.client.create("nodes", make_node("n", 20, 2))
            for nm, m in (("a", 8), ("b", 8), ("c", 8)):
                await c.client.create("pods", make_pod(nm, m, uid=f"u-{nm}"))
            eng = c.ext.server.engine
            await c.settle(lambda: eng.has_node("n") and c.ext.server.controller.get_pod("c", "default") is not None)
            for nm in ("a", "b"):
                st, body = await c.post("/gpushare-scheduler/bind",
                                        wire.ExtenderBindingArgs(nm, "default", f"u-{nm}", "n").encode())
                assert st == 200, body
            assert [u for _, u in eng.node_devices("n")] == [8, 8]
            st, body = await c.post("/gpushare-scheduler/bind",
                                    wire.ExtenderBindingArgs("c", "default", "u-c", "n").encode())
            assert st == 500 and json.loads(body)["Error"] == "The node n can't place the pod c in ns default"
            p = await c.client.get("pods", "b", "default")
            assert p["spec"]["nodeName"] == "n" and p["metadata"]["annotations"]["SHARED_GPU_MEM_IDX"] == "1"
    run(go())


def test_bind_conflict_retry_and_release_on_error():
    async def go():
        async with Cluster() as c:
            await c.client.create("nodes", make_node("n", 10, 1))
            await c.client.create("pods", make_pod("a", 6, uid="ua"))
            eng = c.ext.server.engine
            await c.settle(lambda: eng.has_node("n") and c.ext.server.controller.get_pod("a", "default") is not None)
            c.api.server.faults.update({"error_rate": 1.0})
            st, body = await c.post("/gpushare-scheduler/bind", wire.ExtenderBindingArgs("a", "default", "ua", "n").encode())
            assert st == 500
            assert eng.node_devices("n") == [(10, 0)]  # reservation released on failure
            c.api.server.faults.update({"error_rate": 0.0, "conflict_rate": 0.5, "seed": 3})
            st, body = await c.post("/gpushare-scheduler/bind", wire.ExtenderBindingArgs("a", "default", "ua", "n").encode())
            assert st == 200, body
            assert eng.node_devices("n") == [(10, 6)]
    run(go())


def test_pod_lifecycle_frees_memory_and_restart_recovery():
    async def go():
        async with Cluster() as c:
            await c.client.create("nodes", make_node("n", 10, 1))
            await c.start_sim()
            await c.client.create("pods", make_pod("a", 6))
            await c.sim.wait_bound(["default/a"], 10)
            eng = c.ext.server.engine
            await c.settle(lambda: eng.node_devices("n") == [(10, 6)])
            # a second extender started now rebuilds the ledger from annotations (cache.go:49-74)
            srv2 = ExtenderServer(KubeClient(c.api.url), SHARED_GPU)
            await srv2.start()
            assert srv2.engine.node_devices("n") == [(10, 6)]
            await srv2.stop()
            await srv2.client.close()
            # completion frees the device
            await c.client.patch("pods", "a", {"status": {"phase": "Succeeded"}}, "default", sub="status")
            await c.settle(lambda: eng.node_devices("n") == [(10, 0)])
            await c.client.create("pods", make_pod("b", 6))
            await c.sim.wait_bound(["default/b"], 10)
            await c.settle(lambda: eng.node_devices("n") == [(10, 6)])
            await c.client.delete("pods", "b", "default")
            await c.settle(lambda: eng.node_devices("n") == [(10, 0)])
    run(go())


def test_concurrent_binds_never_overcommit():
    async def go():
        async with Cluster() as c:
            await c.client.create("nodes", make_node("n", 8 * 100, 8))
            await c.start_sim(max_inflight_binds=64)
            keys = []
            for i in range(32):  # 4 x 25 fills each 100-unit device exactly (BASELINE config 3 shape)
                await c.client.create("pods", make_pod(f"p{i}", 25))
                keys.append(f"default/p{i}")
            await c.sim.wait_bound(keys, 20)
            eng = c.ext.server.engine
            await c.settle(lambda: eng.node_devices("n") == [(100, 100)] * 8)
            await c.client.create("pods", make_pod("extra", 1))
            await asyncio.sleep(0.2)
            assert not c.sim.stats.timings["default/extra"].bound
    run(go())


def test_fragmentation_guard_end_to_end():
    """BASELINE config 4: mixed 200/100/50 GiB requests fit the node total but no single device."""
    async def go():
        async with Cluster(profile=ALIYUN) as c:
            await c.client.create("nodes", make_node("n", 2 * 268, 2, profile=ALIYUN))
            await c.start_sim()
            for nm, m in (("a", 200), ("b", 200), ("c", 50)):
                await c.client.create("pods", make_pod(nm, m, profile=ALIYUN))
            await c.sim.wait_bound(["default/a", "default/b", "default/c"], 10)
            eng = c.ext.server.engine
            await c.settle(lambda: sorted(u for _, u in eng.node_devices("n")) == [200, 250])
            # 86 GiB free in total, but at most 68 on one device: a 70 GiB pod must be filtered
            big = make_pod("big", 70, profile=ALIYUN)
            st, body = await c.post("/gpushare-scheduler/filter", wire.filter_args(big, ["n"]))
            assert json.loads(body)["FailedNodes"] == {"n": "Insufficient GPU Memory in one device"}
    run(go())


def test_recovery_consistency_check_flags_overcommit():
    """Annotations that over-commit a device (e.g. capacity shrank) are reported, not wrapped (nodeinfo.go:260)."""
    async def go():
        async with Cluster() as c:
            await c.client.create("nodes", make_node("n", 10, 1))
            for nm in ("a", "b"):
                await c.client.create("pods", make_pod(nm, 8, node="n", phase="Running", annotations={
                    "SHARED_GPU_MEM_IDX": "0", "SHARED_GPU_MEM_POD": "8"}))
            srv2 = ExtenderServer(KubeClient(c.api.url), SHARED_GPU)
            await srv2.start()
            try:
                assert srv2.controller.overcommitted == [("n", 0, 16, 10)]
                st, body = await c.post("/gpushare-scheduler/filter", wire.filter_args(make_pod("p", 1), ["n"]))
                assert json.loads(body)["NodeNames"] == []
            finally:
                await srv2.stop()
                await srv2.client.close()
    run(go())


def test_prioritize_packs_nodes_before_spreading():
    """With the prioritize verb the scheduler fills the partly used node first (binpack across nodes)."""
    async def go():
        async with Cluster() as c:
            for n in ("n1", "n2", "n3"):
                await c.client.create("nodes", make_node(n, 100, 1))
            await c.start_sim(use_prioritize=True, node_policy="spread")
            keys = []
            for i in range(6):
                await c.client.create("pods", make_pod(f"p{i}", 30))
                keys.append(f"default/p{i}")
                await c.sim.wait_bound([keys[-1]], 10)
            nodes = [c.sim.stats.timings[k].node for k in keys]
            # 3 pods of 30 fit one 100-unit device: the first node fills before the next is opened
            assert nodes[:3] == [nodes[0]] * 3 and nodes[3:] == [nodes[3]] * 3 and nodes[0] != nodes[3]
            st, body = await c.post("/gpushare-scheduler/prioritize", wire.filter_args(make_pod("q", 10), ["n1", "n2", "n3"]))
            assert st == 200 and len(json.loads(body)) == 3
    run(go())


def test_leader_election_failover():
    """HA (reference roadmap): two hot replicas, only the Lease holder binds; the standby takes over on loss."""
    async def go():
        async with Cluster() as c:
            await c.client.create("nodes", make_node("n", 100, 1))
            kw = dict(leader_elect=True, lease_namespace="default", lease_duration=2.0, renew_deadline=1.2,
                      retry_period=0.05)
            a = await ExtenderRunner(ExtenderServer(KubeClient(c.api.url), SHARED_GPU, **kw)).start()
            await asyncio.sleep(0.2)
            b = await ExtenderRunner(ExtenderServer(KubeClient(c.api.url), SHARED_GPU, **kw)).start()
            try:
                await c.settle(lambda: a.server.is_leader, 3)
                await asyncio.sleep(0.3)
                assert not b.server.is_leader
                async with c.http.get(b.url + "/healthz") as r:
                    assert r.status == 503 and "standby" in await r.text()
                p = await c.client.create("pods", make_pod("x", 10))
                args = wire.ExtenderBindingArgs("x", "default", p["metadata"]["uid"], "n").encode()
                await c.settle(lambda: b.server.controller.get_pod("x", "default") is not None)
                async with c.http.post(b.url + "/gpushare-scheduler/bind", data=args) as r:
                    assert r.status == 500 and "not the leader" in json.loads(await r.read())["Error"]
                # the leader goes away (Lease released on stop); the standby takes over and binds
                await a.stop()
                await a.server.client.close()
                await c.settle(lambda: b.server.is_leader, 5)
                async with c.http.get(b.url + "/healthz") as r:
                    assert r.status == 200
                async with c.http.post(b.url + "/gpushare-scheduler/bind", data=args) as r:
                    assert r.status == 200, await r.read()
                lease = await c.client.get("leases", "gpushare-schd-extender", "default")
                assert lease["spec"]["holderIdentity"] == b.server.elector.identity
                assert lease["spec"]["leaseTransitions"] >= 1
            finally:
                await b.stop()
                await b.server.client.close()
    run(go())
