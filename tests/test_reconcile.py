"""Allocate swaps under a faithful kubelet, and their reconciliation with kubelet's PodResources record (VERDICT r2
"what's missing" #1).

kubelet admits a batch of pods in creationTimestamp order and the device plugin serves an Allocate of N units
with the earliest-ASSUME_TIME pending pod of that size (``docs/designs/designs.md:93-103``).  Pods bound in
the reverse of their creation order and met by kubelet in one batch therefore start on each other's GPUs.
The kubelet stand-in here does what kubelet does (``--faithful``: no re-routing, sorted batches, PodResources
served), so the swap really happens; every container's real env is read back from it.
"""
import asyncio
import time

import pytest

from gpushare_scheduler_extender_amd.k8s.client import ApiError
from gpushare_scheduler_extender_amd.k8s.objects import make_pod
from gpushare_scheduler_extender_amd.models.profile import ALIYUN, POD_HOLD_IDX_ANNOTATION
from gsxtools.configs import Cluster


async def _pods(cl) -> dict:
    return {p["metadata"]["name"]: p for p in (await cl.c.list("pods", "default"))["items"]}


async def _physical(cl, pods: dict) -> dict:
    """GPU each pod's container was started with (the env kubelet passed to it)."""
    out = {}
    for n, p in pods.items():
        env = (await cl.allocation(p["metadata"]["uid"])).get("envs", {})
        if env:
            out[n] = int(env[ALIYUN.annotation_idx])
    return out


async def _wait(pred, timeout=30.0, what=""):
    deadline = time.monotonic() + timeout
    while True:
        r = await pred()
        if r:
            return r
        assert time.monotonic() < deadline, what
        await asyncio.sleep(0.05)


async def _swap_scenario(reconcile: bool, plugin: str = "grpc"):
    # kubelet restarting meets the pods of its initial LIST as one creationTimestamp-sorted batch
    args = ["--faithful", "--batch-window", "0.02", "--plugin", plugin] + ([] if reconcile else ["--no-reconcile"])
    cl = Cluster(ALIYUN, [96] * 4, gpu=False, agent="plugin", agent_args=args)
    try:
        await cl.start()
        cl.stop_agent()  # kubelet is down while the pods are bound (its restart: it meets them as one batch)
        names = [f"p{i}" for i in range(4)]
        pods = []
        for n in names:  # created p0..p3
            pod = make_pod(n, 64, profile=ALIYUN, scheduler_name="manual")
            del pod["metadata"]["uid"]
            pods.append(await cl.c.create("pods", pod))
        for pod in reversed(pods):  # bound p3..p0: p3 -> GPU 0, ..., p0 -> GPU 3 (ASSUME_TIME p3 < ... < p0)
            assert await cl.bind(pod) == 200
        bound = await _pods(cl)
        assert [cl.device_of(bound[n]) for n in names] == [3, 2, 1, 0]
        await cl.start_agent()
        running = await cl.wait(names)
        phys = await _physical(cl, running)
        # kubelet admitted p0 first and the plugin served it p3's allocation (earliest ASSUME_TIME): a real swap.
        # Without a reconcile pass inside the batch the pattern is {p0: 0, p1: 1, p2: 2, p3: 3}; a pass that lands
        # between two of its Allocates (the plugin's loop is busy elsewhere for a moment) repairs the first swaps
        # before the later admissions, which then swap among themselves -- either way containers run on other GPUs
        # than their pods were bound to, one per GPU
        assert sorted(phys.values()) == [0, 1, 2, 3], phys
        assert sum(phys[n] != cl.device_of(bound[n]) for n in names) >= 2, (phys, bound)
        st = await cl.agent_stats()
        assert st["faithful"] and st["mismatch"] >= 2, st

        async def consistent():
            cur = await _pods(cl)
            ok = all(cl.device_of(cur[n]) == phys[n] for n in names) and not any(
                POD_HOLD_IDX_ANNOTATION in cur[n]["metadata"]["annotations"] for n in names)
            return cur if ok else None
        if reconcile:
            cur = await _wait(consistent, 15, "annotations never matched the GPUs kubelet gave the containers")
            insp = await cl.inspect()
            assert [d["usedGPU"] for d in insp["nodes"][0]["devs"]] == [64] * 4
            st = await cl.agent_stats()
            assert st["reconcile"]["swaps"] >= 2 and st["reconcile"]["unreconcilable"] == 0, st
        else:
            await asyncio.sleep(1.0)
            assert await consistent() is None  # the hole: annotations keep the extender's reservation
        # delete two pods: the extender frees the GPUs their annotations name
        for n in ("p0", "p1"):
            await cl.c.delete("pods", n, "default")
        for n in ("c0", "c1"):
            await cl.create(n, 64)
        deadline = time.monotonic() + 20
        while True:
            cur = await _pods(cl)
            new = {n: cur[n] for n in ("c0", "c1") if n in cur}
            phases = {n: p["status"].get("phase") for n, p in new.items()}
            if all(ph in ("Running", "Failed") for ph in phases.values()) and len(phases) == 2:
                break
            assert time.monotonic() < deadline, phases
            await asyncio.sleep(0.05)
        live = {n: cur[n] for n in ("p2", "p3", "c0", "c1")}
        phys = await _physical(cl, live)
        if reconcile:
            # the new pods may have been served each other's allocations too: the repair is asynchronous
            async def settled():
                now = await _pods(cl)
                ok = all(int(now[n]["metadata"]["annotations"][ALIYUN.annotation_idx]) == phys[n] for n in live
                         if now[n]["status"].get("phase") == "Running")
                return now if ok else None
            cur = await _wait(settled, 10, "the new pods' annotations never matched their containers' GPUs")
            live = {n: cur[n] for n in ("p2", "p3", "c0", "c1")}
        per_gpu = [0] * 4
        for n, g in phys.items():
            if live[n]["status"].get("phase") == "Running":
                per_gpu[g] += 64
        return phases, per_gpu, phys, live
    finally:
        await cl.close()


@pytest.mark.parametrize("plugin", ["grpc", "process"])
def test_kubelet_batch_swap_is_reconciled_and_deletes_free_the_right_gpu(plugin):
    """``process``: the plugin runs as deployed (``python -m ...deviceplugin``, registered with the stand-in's
    Registration service), so the reconciliation works across the process boundary kubelet really has."""
    phases, per_gpu, phys, live = asyncio.run(_swap_scenario(reconcile=True, plugin=plugin))
    assert phases == {"c0": "Running", "c1": "Running"}, phases
    assert all(u <= 96 for u in per_gpu), per_gpu  # never two 64 GiB containers on one 96 GiB GPU
    assert sorted(phys.values()) == [0, 1, 2, 3]
    for n, p in live.items():  # every annotation names the GPU its container runs on
        assert int(p["metadata"]["annotations"][ALIYUN.annotation_idx]) == phys[n], (n, phys)


def test_without_reconciliation_a_swap_lets_a_pod_land_on_a_physically_full_gpu():
    """The hole the reconciliation closes, reproduced: the new pods are placed on GPUs whose annotated pods were
    deleted, but the containers there belong to the pods that were not."""
    phases, per_gpu, phys, live = asyncio.run(_swap_scenario(reconcile=False))
    assert "Failed" in phases.values(), (phases, per_gpu)  # the node's runtime could not fit them physically


def test_pod_resources_api_roundtrip(tmp_path):
    """The hand-built v1 PodResourcesLister descriptor: our kubelet-side server and the plugin's client agree."""
    from gpushare_scheduler_extender_amd.deviceplugin.podresources import PodResourcesClient, PodResourcesServer

    async def go():
        sock = str(tmp_path / "pr" / "kubelet.sock")
        data = [("default", "a", [("main", "aliyun.com/gpu-mem", ["g0-_-1", "g0-_-0"])]),
                ("kube-system", "b", [("c1", "other/res", ["x"]), ("c2", "aliyun.com/gpu-mem", ["g1-_-0"])])]
        srv = PodResourcesServer(sock, lambda: data)
        await srv.start()
        cli = PodResourcesClient(sock)
        try:
            got = await cli.device_ids("aliyun.com/gpu-mem")
            assert got == {("default", "a"): [("g0-_-0", "g0-_-1")], ("kube-system", "b"): [("g1-_-0",)]}
            one = await cli.get("b", "kube-system")
            assert [c.name for c in one.pod_resources.containers] == ["c1", "c2"]
        finally:
            await cli.close()
            await srv.stop()
    asyncio.run(go())


@pytest.mark.parametrize("seed", [3, 5])
def test_reconcile_state_exchange_cycles(seed):
    """A 3-cycle (P holds Q's record, Q holds R's, R holds P's) resolves as a chain of exchanges: every record
    ends described by the pod that holds it, and the CU partitions follow."""
    import random

    from gpushare_scheduler_extender_amd.deviceplugin.devices import Device
    from gpushare_scheduler_extender_amd.deviceplugin.state import AllocationState
    from gpushare_scheduler_extender_amd.models.profile import SHARED_GPU

    rnd = random.Random(seed)
    devs = {i: Device(index=i, total_bytes=96 << 30) for i in range(3)}
    st = AllocationState("n", devs, SHARED_GPU)
    pods = {}
    for i, n in enumerate("PQR"):
        p = make_pod(n, 64, node="n", uid=f"u{n}", annotations={SHARED_GPU.annotation_idx: str(i),
                                                                 SHARED_GPU.annotation_assigned: "false"})
        p["metadata"]["resourceVersion"] = "1"
        st.observe(p)
        pods[n] = p
    recs = {n: st.record(st.pods[f"u{n}"], [f"g{i}-_-0"], 64, "", f"a{n}") for i, n in enumerate("PQR")}
    for n in "PQR":
        st.cus[recs[n].dev].allocate(f"u{n}", 8)
    holds = {"P": recs["Q"].aid, "Q": recs["R"].aid, "R": recs["P"].aid}  # who physically holds which record
    order = list("PQR")
    rnd.shuffle(order)
    ann = {n: recs[n].dev for n in "PQR"}  # annotation device per pod
    for _ in range(3):
        for n in order:
            r = st.records[holds[n]]
            if r.uid == f"u{n}":
                continue
            q = r.uid[1:]
            ann[n], ann[q] = r.dev, ann[n]
            st.move_records(f"u{n}", r.uid, r)
    for n in "PQR":
        r = st.records[holds[n]]
        assert r.uid == f"u{n}" and ann[n] == r.dev
        assert st.cus[r.dev].holds(f"u{n}")


def test_unowned_record_outlives_the_pod_it_was_built_for_while_kubelet_reports_owners():
    """A record built for Q may be running in P's container (a swap no pass has seen yet).  Once PodResources is
    reconciled, deleting Q must not drop it -- only kubelet no longer listing its IDs does."""
    from gpushare_scheduler_extender_amd.deviceplugin.devices import Device
    from gpushare_scheduler_extender_amd.deviceplugin.state import AllocationState
    from gpushare_scheduler_extender_amd.models.profile import SHARED_GPU

    def make():
        st = AllocationState("n", {0: Device(index=0, total_bytes=96 << 30)}, SHARED_GPU)
        q = make_pod("q", 32, node="n", uid="uQ", annotations={SHARED_GPU.annotation_idx: "0",
                                                                SHARED_GPU.annotation_assigned: "false"})
        q["metadata"]["resourceVersion"] = "1"
        st.observe(q)
        st.record(st.pods["uQ"], ["g0-_-0"], 32, "", "aQ")
        return st

    st = make()  # no PodResources: the pod's records go with it
    st.release("uQ")
    assert "aQ" not in st.records
    st = make()
    st.core.set_owners_reported(True)
    st.release("uQ")
    assert "aQ" in st.records  # kept until kubelet's report decides
    st.set_owner("aQ", "uP")
    st.release("uP")  # its owner's deletion does drop it
    assert "aQ" not in st.records


def test_off_gpu_records_are_counted_per_gpu_their_container_runs_on():
    """The guard's ID bound (dpcore.cc allocate, plugin.py _kubelet_bounds) holds for a GPU while every allocation
    whose container runs there has its IDs there: a record off its GPU elsewhere on the node does not lift it."""
    from gpushare_scheduler_extender_amd.deviceplugin.devices import Device
    from gpushare_scheduler_extender_amd.deviceplugin.state import AllocationState
    from gpushare_scheduler_extender_amd.models.profile import SHARED_GPU

    st = AllocationState("n", {i: Device(index=i, total_bytes=96 << 30) for i in range(2)}, SHARED_GPU)
    for n, dev in (("P", 0), ("Q", 1)):
        p = make_pod(n, 32, node="n", uid=f"u{n}", annotations={SHARED_GPU.annotation_idx: str(dev),
                                                                 SHARED_GPU.annotation_assigned: "false"})
        p["metadata"]["resourceVersion"] = "1"
        st.observe(p)
    st.record(st.pods["uP"], ["g0-_-0"], 32, "", "aP", on_gpu=True)
    st.record(st.pods["uQ"], ["g0-_-1"], 32, "", "aQ", on_gpu=False)  # Q runs on GPU 1 with an ID of GPU 0
    core = st.core
    assert core.off_gpu_records() == 1
    assert core.off_gpu_records_on(0) == 0 and core.off_gpu_records_on(1) == 1
    core.mark_on_gpu("aQ", True)
    assert core.off_gpu_records() == 0 and core.off_gpu_records_on(1) == 0
    core.mark_on_gpu("aQ", False)
    st.release("uQ")  # no PodResources: the record goes with its pod
    assert core.off_gpu_records() == 0 and core.off_gpu_records_on(1) == 0


def test_annotations_edited_behind_the_plugins_back_are_repaired():
    """Any cause (an operator's edit, a half-applied exchange from an older plugin): a pod whose annotation names
    another GPU than its container's allocation is re-annotated from kubelet's record, by exchanging with the
    pod that carries its real GPU."""
    async def go():
        cl = Cluster(ALIYUN, [96] * 4, gpu=False, agent="plugin", agent_args=["--faithful"])
        try:
            await cl.start()
            for n in ("a", "b"):
                await cl.create(n, 64)
            pods = await cl.wait(["a", "b"])
            phys = await _physical(cl, pods)
            assert phys["a"] != phys["b"]
            for n, other in (("a", "b"), ("b", "a")):  # swap the two pods' *_IDX behind everyone's back
                await cl.c.patch("pods", n, {"metadata": {"annotations": {
                    ALIYUN.annotation_idx: str(phys[other])}}}, "default")
            drift, drifted = await cl.physical_drift(["a", "b"], timeout=15)
            assert drift == 0, drifted
            st = await cl.agent_stats()
            assert st["reconcile"]["drift_repaired"] >= 1, st["reconcile"]
            insp = await cl.inspect()
            used = [d["usedGPU"] for d in insp["nodes"][0]["devs"]]
            assert sorted(used) == [0, 0, 64, 64] and used[phys["a"]] == 64 and used[phys["b"]] == 64
        finally:
            await cl.close()
    asyncio.run(go())


def test_a_bind_into_an_unrepaired_drift_trades_gpus_with_the_drifted_pod():
    """reconcile.py drift repair: P's container runs on GPU X while P is annotated GPU Y, and before a pass finds it
    the extender binds a larger pod C into the room P's container fills on X.  P cannot be re-annotated onto X (C's
    annotation fills it) and C cannot move to Y alone (P's annotation holds it); the repair trades their GPUs (C is
    the stand-in partner, any size with which both GPUs fit afterwards), so C's Allocate starts it on Y instead of
    failing at the physical guard."""
    async def go():
        cl = Cluster(ALIYUN, [96] * 2, gpu=False, agent="plugin", agent_args=["--faithful"])
        try:
            await cl.start()
            await cl.create("p", 32)
            pods = await cl.wait(["p"])
            x = (await _physical(cl, pods))["p"]
            y = 1 - x
            await cl.c.patch("pods", "p", {"metadata": {"annotations": {ALIYUN.annotation_idx: str(y)}}}, "default")
            for _ in range(500):  # the extender's ledger follows the edit: X looks empty
                used = [d["usedGPU"] for d in (await cl.inspect())["nodes"][0]["devs"]]
                if used[x] == 0:
                    break
                await asyncio.sleep(0.002)
            await cl.create("c", 80)  # fits only X by the annotations; X physically holds P's 32
            pods = await cl.wait(["p", "c"], timeout=20)
            assert all(q["status"].get("phase") == "Running" for q in pods.values())
            drift, drifted = await cl.physical_drift(["p", "c"], timeout=15)
            assert drift == 0, drifted
            phys = await _physical(cl, pods)
            assert phys == {"p": x, "c": y}, phys
        finally:
            await cl.close()
    asyncio.run(go())


def test_unaccounted_use_is_a_live_holder_on_another_gpu_and_reaches_the_extender():
    """plugin.py unaccounted / publish_physical: a record kubelet reports held by another live pod annotated with
    another GPU is charged where the container runs; nothing while the record is unreported or held by its own pod;
    one held by a pod that is gone is charged while kubelet lists it; withdrawn once the annotations agree.  The
    extender charges what is published."""
    import asyncio
    import json as _json

    from gpushare_scheduler_extender_amd.deviceplugin.devices import fake_devices
    from gpushare_scheduler_extender_amd.deviceplugin.plugin import GpuSharePlugin
    from gpushare_scheduler_extender_amd.extender.server import ExtenderRunner, ExtenderServer
    from gpushare_scheduler_extender_amd.k8s.client import KubeClient
    from gpushare_scheduler_extender_amd.k8s.objects import make_node
    from gpushare_scheduler_extender_amd.models.profile import SHARED_GPU
    from tests.fixtures.fakeapi import FakeApiServerRunner

    async def go():
        api = await FakeApiServerRunner().start()
        c = KubeClient(api.url)
        await c.create("nodes", make_node("n", 32, 2))
        ext = await ExtenderRunner(ExtenderServer(KubeClient(api.url))).start()
        plugin = GpuSharePlugin(c, "n", fake_devices("2x16GiB"), SHARED_GPU, socket_dir="/tmp/gsx-unacc-test",
                                extender=f"http://127.0.0.1:{ext.port}")
        st = plugin.state
        try:
            for _ in range(200):
                if ext.server.engine.has_node("n"):
                    break
                await asyncio.sleep(0.01)

            def pod(name, dev):
                p = make_pod(name, 4, node="n", uid=f"u{name}", annotations={SHARED_GPU.annotation_idx: str(dev),
                                                                             SHARED_GPU.annotation_assigned: "true"})
                p["metadata"]["resourceVersion"] = "1"
                st.observe(p)

            pod("P", 0)
            pod("Q", 1)
            st.core.set_owners_reported(True)
            st.record(st.pods["uQ"], ["g1-_-0"], 4, "", "aQ")  # built for Q, on GPU 1
            assert plugin.unaccounted() is None  # kubelet has not reported who holds it
            st.set_owner("aQ", "uQ")
            assert plugin.unaccounted() is None  # its own pod: the annotations charge it
            st.set_owner("aQ", "uP")  # P's container runs with it (a swap), P annotated GPU 0
            assert plugin.unaccounted() == [0, 4]
            assert await plugin.publish_physical()
            assert ext.server.engine.node_unaccounted("n") == [0, 4]
            pod("P", 1)  # the exchange landed: P is annotated where its container runs
            assert plugin.unaccounted() is None
            assert await plugin.publish_physical()
            assert ext.server.engine.node_unaccounted("n") == []
            pod("P", 0)
            st.set_owner("aQ", "~default/gone")  # kubelet lists it for a pod that is gone: its container is stopping
            st.core.prune_held([["g1-_-0"]], 0.0, 0.0)
            st.core.prune_held([["g1-_-0"]], 1.0, 0.0)
            assert plugin.unaccounted() == [0, 4]  # charged until kubelet stops listing it (the extender freed it)
            st.core.prune_held([], 1e12, 0.0)
            assert plugin.unaccounted() is None
            one = GpuSharePlugin(c, "n", fake_devices("1x16GiB"), SHARED_GPU, socket_dir="/tmp/gsx-unacc-test1")
            assert one.unaccounted() is None  # one GPU: whoever holds it is annotated with it
        finally:
            await ext.stop()
            await ext.server.client.close()
            await c.close()
            await api.stop()
    asyncio.run(go())


def test_stand_in_partner_prefers_equal_size_then_the_largest_that_fits():
    """reconcile.py _stand_in_partner: P's container runs on GPU 1 while P is annotated GPU 0 (the pod its allocation
    was built for is gone).  An unstarted pod the extender placed on GPU 1 exchanges GPUs with P: one of P's size
    first (every GPU's sum unchanged), else the largest one with which both GPUs fit after the exchange."""
    import asyncio

    from gpushare_scheduler_extender_amd.deviceplugin.devices import fake_devices
    from gpushare_scheduler_extender_amd.deviceplugin.plugin import GpuSharePlugin
    from gpushare_scheduler_extender_amd.deviceplugin.reconcile import Reconciler
    from gpushare_scheduler_extender_amd.models.profile import SHARED_GPU

    async def go():
        plugin = GpuSharePlugin(None, "n", fake_devices("2x16GiB"), SHARED_GPU, socket_dir="/tmp/gsx-standin-test")
        st = plugin.state
        rec = Reconciler(plugin, None)

        def pod(name, mem, dev, rv):
            p = make_pod(name, mem, node="n", uid=f"u{name}", annotations={SHARED_GPU.annotation_idx: str(dev),
                                                                           SHARED_GPU.annotation_assigned: "false"})
            p["metadata"]["resourceVersion"] = str(rv)
            st.observe(p)
            return st.pods[f"u{name}"]

        p = pod("P", 4, 0, 1)
        pod("Q8", 8, 1, 2)
        pod("Q2", 2, 1, 3)
        got = rec._stand_in_partner(1, p, set())
        assert got is not None and got.name == "Q8"  # no equal size: the largest that fits both GPUs
        assert rec.stats.get("unequal_partners") == 1
        pod("Q4", 4, 1, 4)
        assert rec._stand_in_partner(1, p, set()).name == "Q4"  # equal size first
        assert rec._stand_in_partner(1, p, {"default/Q4"}).name == "Q8"  # a started pod never stands in
        pod("Big", 14, 0, 5)  # GPU 0 now holds P 4 + Big 14 by the annotations: Q8 no longer fits there
        st.release("uQ4")
        assert rec._stand_in_partner(1, p, set()).name == "Q2"

    asyncio.run(go())


def test_physical_guard_waits_for_a_deleted_pods_container_when_no_gpu_has_room(monkeypatch):
    """plugin.py _physical_guard: the GPU a pending pod is annotated with is physically full by a container of a
    deleted pod that kubelet still lists (owner ``~ns/name``), and no other GPU has room.  Past the short wait the
    Allocate keeps waiting for that container (up to GUARD_GONE_WAIT_S) and proceeds once it is gone; a GPU full by
    live containers fails it after the short wait."""
    import asyncio

    from gpushare_scheduler_extender_amd.deviceplugin import plugin as plugin_mod
    from gpushare_scheduler_extender_amd.deviceplugin.devices import fake_devices
    from gpushare_scheduler_extender_amd.deviceplugin.plugin import AllocateError, GpuSharePlugin
    from gpushare_scheduler_extender_amd.models.profile import SHARED_GPU

    monkeypatch.setattr(plugin_mod, "GUARD_WAIT_S", 0.05)
    monkeypatch.setattr(plugin_mod, "GUARD_GONE_WAIT_S", 5.0)

    async def go():
        plugin = GpuSharePlugin(None, "n", fake_devices("2x16GiB"), SHARED_GPU, socket_dir="/tmp/gsx-guard-test")
        st = plugin.state

        class _Rec:  # the guard's reconciler: passes are no-ops here, nothing in an exchange
            def busy(self):
                return set()

            def exchange_pending(self, q):
                return False

        async def _no_pass(urgent=False):
            return None

        plugin.reconciler = _Rec()
        plugin._reconcile_now = _no_pass

        def pod(name, mem, dev, assigned):
            p = make_pod(name, mem, node="n", uid=f"u{name}", annotations={SHARED_GPU.annotation_idx: str(dev),
                                                                           SHARED_GPU.annotation_assigned: assigned})
            p["metadata"]["resourceVersion"] = "1"
            st.observe(p)
            return st.pods[f"u{name}"]

        st.core.set_owners_reported(True)
        old = pod("old", 12, 0, "true")
        st.record(old, [f"g0-_-{i}" for i in range(12)], 12, "", "aold")
        st.set_owner("aold", "uold")
        full = pod("full", 16, 1, "true")  # GPU 1 full by a live container: no room to move to
        st.record(full, [f"g1-_-{i}" for i in range(16)], 16, "", "afull")
        st.set_owner("afull", "ufull")
        new = pod("new", 8, 0, "false")
        # a live container fills the room: the guard fails after its short wait
        t0 = time.monotonic()
        with pytest.raises(AllocateError, match="physically full"):
            await plugin._physical_guard(new, 8)
        assert time.monotonic() - t0 < 2.0
        # the same container, its pod deleted and kubelet still listing it: the guard waits, then proceeds
        st.set_owner("aold", "~default/old")
        task = asyncio.ensure_future(plugin._physical_guard(st.pods["unew"], 8))
        await asyncio.sleep(0.4)
        assert not task.done()
        # kubelet stops listing it: the reconciliation prunes the physical account and drops the record
        st.core.prune_held([], time.time(), 0.0)
        st.drop_record(st.records["aold"])
        got = await asyncio.wait_for(task, 3.0)
        assert got is not None and got.uid == "unew" and got.dev == 0
        assert plugin.stats.get("physical_guard_gone_waits", 0) >= 1

    asyncio.run(go())


def test_plugin_republishes_on_a_new_extender_epoch_and_counts_terminating_holders():
    """a publishing plugin reads the extender's epoch and republishes the moment it changes (a new
    leader knows nothing of what the old one was told); a standby answers /physical 503, never counted as delivered.
    VERDICT r5 #1: the plugin's annotated view (where it may move a pod) counts terminating pods as the extender
    does: charged until their objects are gone."""
    import asyncio

    from gpushare_scheduler_extender_amd.deviceplugin.devices import fake_devices
    from gpushare_scheduler_extender_amd.deviceplugin.plugin import GpuSharePlugin
    from gpushare_scheduler_extender_amd.deviceplugin.reconcile import Reconciler
    from gpushare_scheduler_extender_amd.extender.server import ExtenderRunner, ExtenderServer
    from gpushare_scheduler_extender_amd.k8s.client import KubeClient
    from gpushare_scheduler_extender_amd.k8s.objects import make_node
    from gpushare_scheduler_extender_amd.models.profile import SHARED_GPU
    from tests.fixtures.fakeapi import FakeApiServerRunner

    async def go():
        api = await FakeApiServerRunner().start()
        c = KubeClient(api.url)
        await c.create("nodes", make_node("n", 32, 2))
        ext = await ExtenderRunner(ExtenderServer(KubeClient(api.url))).start()
        plugin = GpuSharePlugin(c, "n", fake_devices("2x16GiB"), SHARED_GPU, socket_dir="/tmp/gsx-epoch-test",
                                extender=f"http://127.0.0.1:{ext.port}")
        plugin.reconciler = Reconciler(plugin, None)  # publishing (PodResources reconciled)
        st = plugin.state
        eng = ext.server.engine
        try:
            assert plugin.publishes_physical
            for _ in range(200):
                if eng.has_node("n"):
                    break
                await asyncio.sleep(0.01)

            def pod(name, dev, deleting=False):
                p = make_pod(name, 4, node="n", uid=f"u{name}", annotations={SHARED_GPU.annotation_idx: str(dev),
                                                                             SHARED_GPU.annotation_assigned: "true"})
                p["metadata"]["resourceVersion"] = "2" if deleting else "1"
                if deleting:
                    p["metadata"]["deletionTimestamp"] = "2026-01-01T00:00:00Z"
                    p["status"]["phase"] = "Running"
                st.observe(p)

            pod("P", 0)
            pod("Q", 1)
            st.core.set_owners_reported(True)
            st.record(st.pods["uQ"], ["g1-_-0"], 4, "", "aQ")
            st.set_owner("aQ", "uP")  # P's container runs with Q's allocation on GPU 1
            assert await plugin.check_epoch()  # first sight of the epoch: published
            assert eng.node_unaccounted("n") == [0, 4]
            n0 = plugin.stats["physical_published"]
            assert await plugin.check_epoch() and plugin.stats["physical_published"] == n0  # same epoch: nothing
            # a standby: /physical is refused and the epoch says "not leader"
            eng.set_binds_enabled(False)
            assert not await plugin.publish_physical(force=True)
            assert not await plugin.check_epoch()
            eng.set_binds_enabled(True)  # leader again: a new epoch
            assert await plugin.check_epoch()
            assert plugin.stats["physical_published"] == n0 + 1 and plugin.stats["epoch_changes"] >= 2
            assert eng.node_unaccounted("n") == [0, 4]  # republished at once
            # P is being deleted gracefully while its container stops: the extender charges P's annotated GPU 0
            # until the object goes, and so does the plugin's annotated view
            pod("P", 0, deleting=True)
            assert st.core.terminating_dev("uP") == 0 and st.core.terminating_used(0) == 4
            assert plugin._annotated_used(0) == 4 and "uP" not in st.pods
            gone = make_pod("P", 4, node="n", uid="uP")
            st.forget(gone)  # kubelet's grace-0 delete
            assert st.core.terminating_used(0) == 0 and plugin._annotated_used(0) == 0
        finally:
            await ext.stop()
            await ext.server.client.close()
            await c.close()
            await api.stop()
    asyncio.run(go())


def test_a_force_deleted_pods_share_lingers_until_its_containers_are_killed():
    """AllocState::deleted / prune_held (force deletes): kubelet stops listing a pod deleted outright
    and frees its device IDs at once, but its containers get their termination grace.  Their share stays counted on
    its GPU -- physical_used, no per-ID bound there, published as unaccounted -- until the kill deadline; a graceful
    deletion (seen terminating first) ends with the containers and lingers nothing; an entry kubelet never reported
    lingers while a force-deleted pod could be running it; so does one whose IDs kubelet re-used while its reported
    holder was still live here."""
    from gpushare_scheduler_extender_amd.deviceplugin.devices import fake_devices
    from gpushare_scheduler_extender_amd.deviceplugin.plugin import GpuSharePlugin
    from gpushare_scheduler_extender_amd.models.profile import SHARED_GPU

    def make(gpus="2x16GiB"):
        plugin = GpuSharePlugin(None, "n", fake_devices(gpus), SHARED_GPU, socket_dir="/tmp/gsx-linger-test",
                                checkpoint="")
        plugin.state.core.expect_owner_reports(True)
        return plugin, plugin.state

    def pod(st, name, dev, grace=5, deleting=False, rv="1"):
        p = make_pod(name, 8, node="n", uid=f"u{name}", annotations={SHARED_GPU.annotation_idx: str(dev),
                                                                     SHARED_GPU.annotation_assigned: "true"})
        p["metadata"]["resourceVersion"] = rv
        p["spec"]["terminationGracePeriodSeconds"] = grace
        if deleting:
            p["metadata"]["deletionTimestamp"] = "2026-01-01T00:00:00Z"
        st.observe(p)
        return p

    plugin, st = make()
    core = st.core
    a = pod(st, "A", 0)
    st.record(st.pods["uA"], [f"g0-_-{i}" for i in range(8)], 8, "", "aA", 100.0, on_gpu=True)
    core.set_owner("aA", "uA")
    assert core.physical_used(0) == 8 and core.off_gpu_records_on(0) == 0
    core.deleted("uA", 101.0)  # force delete: kill deadline 101 + 5 + 2
    assert core.linger_count() == 1 and core.lingering(0) == 8 and core.physical_used(0) == 8
    assert core.off_gpu_records_on(0) == 1  # kubelet's per-ID count no longer bounds GPU 0
    assert plugin.unaccounted() == [8, 0]  # the extender charges it too
    core.prune_held([], 107.5, 0.5)
    assert core.lingering(0) == 8
    core.prune_held([], 108.5, 0.5)
    assert core.linger_count() == 0 and core.physical_used(0) == 0 and plugin.unaccounted() is None
    del a
    # graceful: seen terminating, then deleted once kubelet finalised it -- nothing lingers
    pod(st, "B", 1)
    st.record(st.pods["uB"], [f"g1-_-{i}" for i in range(8)], 8, "", "aB", 200.0, on_gpu=True)
    core.set_owner("aB", "uB")
    pod(st, "B", 1, deleting=True, rv="2")
    core.deleted("uB", 201.0)
    core.prune_held([], 201.5, 0.1)
    assert core.linger_count() == 0 and core.physical_used(1) == 0
    # an entry kubelet never reported while a force-deleted pod may still run it (kubelet gave it the IDs before
    # its view had the delete): it lingers until that pod's deadline, then goes
    pod(st, "C", 0, grace=10)
    pod(st, "D", 0)
    core.deleted("uC", 300.0)  # C had no container yet: deadline 312
    st.record(st.pods["uD"], [f"g0-_-{i}" for i in range(8)], 8, "", "aD", 300.5, on_gpu=True)
    core.prune_held([], 301.5, 0.5)  # kubelet lists nothing: the ghost may be running D's allocation
    assert core.lingering(0) == 8
    core.prune_held([], 312.5, 0.5)
    assert core.lingering(0) == 0
    # kubelet re-used IDs whose reported holder this view still has live (its delete not seen yet)
    pod(st, "E", 1)
    ids = [f"g1-_-{i}" for i in range(8)]
    st.record(st.pods["uE"], ids, 8, "", "aE", 400.0, on_gpu=True)
    core.set_owner("aE", "uE")
    pod(st, "F", 1)
    st.record(st.pods["uF"], ids, 8, "", "aF", 401.0, on_gpu=True)
    assert core.lingering(1) == 8 and core.physical_used(1) == 16
    # a LIST without a pod that was live here: deleted outright
    st.resync([p for p in []])
    assert core.linger_count() >= 2
    # one GPU: lingering is the only unaccounted use, and it is published
    one, st1 = make("1x16GiB")
    pod(st1, "G", 0)
    st1.record(st1.pods["uG"], [f"g0-_-{i}" for i in range(8)], 8, "", "aG", 500.0, on_gpu=True)
    st1.core.set_owner("aG", "uG")
    st1.core.deleted("uG", 501.0)
    assert one.unaccounted() == [8]
    # nobody reports owners (no PodResources reconciliation): a pod's going ends its allocations, as before
    bare = GpuSharePlugin(None, "n", fake_devices("2x16GiB"), SHARED_GPU, socket_dir="/tmp/gsx-linger-test2",
                          checkpoint="")
    pod(bare.state, "H", 0)
    bare.state.record(bare.state.pods["uH"], [f"g0-_-{i}" for i in range(8)], 8, "", "aH", 600.0, on_gpu=True)
    bare.state.core.deleted("uH", 601.0)
    assert bare.state.core.linger_count() == 0 and bare.state.core.physical_used(0) == 0


def test_with_kubelets_report_as_the_truth_a_deleted_pods_container_counts_while_listed():
    """GSX_PLUGIN_FORCE_DELETE=report (a kubelet that lists a container until it has stopped, like the node agent):
    a pod deleted outright keeps its held entry while kubelet lists its IDs -- counted on its GPU and published as
    unaccounted use (the extender freed the share with the object) -- and it goes with the first report that no
    longer lists it.  A completed pod's entry is not published (a finished Job's object stays)."""
    from gpushare_scheduler_extender_amd.deviceplugin.devices import fake_devices
    from gpushare_scheduler_extender_amd.deviceplugin.plugin import GpuSharePlugin
    from gpushare_scheduler_extender_amd.models.profile import SHARED_GPU

    plugin = GpuSharePlugin(None, "n", fake_devices("2x16GiB"), SHARED_GPU, socket_dir="/tmp/gsx-report-test",
                            checkpoint="")
    st, core = plugin.state, plugin.state.core
    core.expect_owner_reports(True)
    core.set_linger(False)

    def pod(name, dev, phase="Running"):
        p = make_pod(name, 8, node="n", uid=f"u{name}", annotations={SHARED_GPU.annotation_idx: str(dev),
                                                                     SHARED_GPU.annotation_assigned: "true"})
        p["metadata"]["resourceVersion"] = "1"
        p["status"]["phase"] = phase
        st.observe(p)
        return p

    pod("A", 0)
    ids = [f"g0-_-{i}" for i in range(8)]
    st.record(st.pods["uA"], ids, 8, "", "aA", 100.0, on_gpu=True)
    core.set_owner("aA", "uA")
    core.deleted("uA", 101.0)
    assert core.linger_count() == 0 and core.physical_used(0) == 8
    assert core.gone_held(0) == 0  # kubelet has not reported it yet: nothing to publish
    core.prune_held([ids], 102.0, 0.5)  # kubelet lists it: counted; published once a second report still does
    assert core.physical_used(0) == 8 and core.gone_held(0) == 0
    core.prune_held([ids], 102.5, 0.5)
    assert core.gone_held(0) == 8
    assert plugin.unaccounted() == [8, 0]
    core.prune_held([], 103.0, 0.5)  # kubelet stopped listing it: its container has stopped
    assert core.physical_used(0) == 0 and plugin.unaccounted() is None
    # a completed pod kubelet keeps listing is not published
    pod("B", 1)
    ids_b = [f"g1-_-{i}" for i in range(8)]
    st.record(st.pods["uB"], ids_b, 8, "", "aB", 200.0, on_gpu=True)
    core.set_owner("aB", "uB")
    pod("B", 1, phase="Succeeded")
    assert core.gone_held(1) == 0
