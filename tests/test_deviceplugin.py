"""Device plugin: kubelet gRPC API against a fake kubelet + fake apiserver; Allocate semantics; CU partitions."""
import asyncio
import json
import tempfile

import pytest

from gpushare_scheduler_extender_amd.deviceplugin import api
from gpushare_scheduler_extender_amd.deviceplugin.allocator import CU_COUNT_ANNOTATION, CUPartitioner, build_response
from gsxtools.agent import NodeAgent
from gpushare_scheduler_extender_amd.deviceplugin.devices import Device, discover, fake_devices
from gpushare_scheduler_extender_amd.deviceplugin.plugin import GpuSharePlugin, fake_ids
from gsxtools.kubeletapi import FakeKubelet, PluginClient
from gpushare_scheduler_extender_amd.deviceplugin.runtime import AdmissionError, LedgerRuntime
from gpushare_scheduler_extender_amd.deviceplugin.state import AllocationState
from gpushare_scheduler_extender_amd.k8s.client import KubeClient
from tests.fixtures.fakeapi import FakeApiServerRunner
from gpushare_scheduler_extender_amd.k8s.objects import make_node, make_pod
from gpushare_scheduler_extender_amd.models.profile import ALIYUN, SHARED_GPU

P = SHARED_GPU
GIB = 1 << 30


def bound_pod(name, mem, node="n1", dev=0, assume=1, assigned="false", dev_total=268, **kw):
    ann = {P.annotation_idx: str(dev), P.annotation_pod: str(mem if not isinstance(mem, list) else sum(mem)),
           P.annotation_dev: str(dev_total), P.annotation_assigned: assigned, P.annotation_assume_time: str(assume)}
    ann.update(kw.pop("annotations", {}))
    return make_pod(name, mem, node=node, annotations=ann, **kw)


async def assigned_value(client, name, want="true", ns="default", timeout=3.0):
    """The pod's ASSIGNED annotation once it reads ``want`` (or the last value after ``timeout``): with early answer
    (the default) an Allocate's commit lands just after kubelet has the answer."""
    import time as _time

    deadline = _time.monotonic() + timeout
    while True:
        v = (await client.get("pods", name, ns))["metadata"]["annotations"].get(P.annotation_assigned)
        if v == want or _time.monotonic() > deadline:
            return v
        await asyncio.sleep(0.01)


# ---------------------------------------------------------------- allocator (pure)

def _state(spec="2x16GiB"):
    return AllocationState("n1", {d.index: d for d in fake_devices(spec)}, P)


def test_candidate_order_and_pick_by_size():
    st = _state()
    pods = [bound_pod("late", 8, assume=30), bound_pod("early", 8, assume=10), bound_pod("other", 4, assume=5),
            bound_pod("done", 8, assume=1, assigned="true"), bound_pod("elsewhere", 8, node="n2", assume=1),
            bound_pod("running", 8, assume=2, phase="Running"), bound_pod("gpu7", 8, dev=7, assume=0)]
    st.resync(pods)
    assert [r.name for r in st.candidates()] == ["other", "early", "late"]
    assert st.match(8)[0].name == "early"
    assert st.match(4)[0].name == "other"
    assert st.match(3) == (None, False)
    st.inflight.add(st.match(8)[0].uid)  # a claim in flight is never matched twice
    assert st.match(8)[0].name == "late"


def test_candidates_follow_landing_order_not_assume_time():
    """kubelet admits a node's pods one at a time in the order its watch delivers them (resourceVersion order), so
    the plugin serves the earliest *landed* candidate: the resourceVersion at which it was first seen bound here,
    kept across later copies of the pod (annotation patches); ASSUME_TIME only breaks ties."""
    st = _state()

    def at(pod, rv):
        pod["metadata"]["resourceVersion"] = str(rv)
        return pod

    late = at(bound_pod("late", 8, assume=30, uid="u-late"), 5)   # assumed last, landed first
    early = at(bound_pod("early", 8, assume=10, uid="u-early"), 9)
    st.observe(late)
    st.observe(early)
    assert [r.name for r in st.candidates()] == ["late", "early"]
    # a later copy of "late" (e.g. an annotation written back after the binding) keeps its landing
    st.observe(at(bound_pod("late", 8, assume=30, uid="u-late", annotations={"x": "y"}), 12))
    assert st.match(8)[0].name == "late"
    # a pod first seen unbound and then bound lands when it is bound
    st.observe(at(bound_pod("mid", 8, assume=1, uid="u-mid", node=""), 3))
    st.observe(at(bound_pod("mid", 8, assume=1, uid="u-mid"), 14))
    assert [r.name for r in st.candidates()] == ["late", "early", "mid"]


def test_state_releases_cus_and_partial_on_completion_and_delete():
    st = _state("1x64GiB")
    a = bound_pod("a", 16, annotations={CU_COUNT_ANNOTATION: "64"})
    mc = bound_pod("mc", [8, 4], assume=2)
    st.resync([a, mc])
    rec, whole = st.match(16)
    assert rec.name == "a" and whole and len(st.claim_cus(rec)) == 64 and st.cus[0].free_count() == 192
    rec2, whole2 = st.match(8)
    assert rec2.name == "mc" and not whole2
    st.first_container_committed(rec2, 8, whole2)
    assert st.partial[rec2.uid] == [4]
    # a completes (Succeeded): its CUs come back; mc is deleted: its partial entry goes
    st.observe(bound_pod("a", 16, phase="Succeeded", uid=rec.uid, annotations={CU_COUNT_ANNOTATION: "64"}))
    assert st.cus[0].free_count() == 256 and st.stats["cu_released"] == 64
    st.forget(mc)
    assert not st.partial and not st.pods


def test_state_rebuilds_cu_ownership_from_annotations():
    """After a plugin restart the running pods' partitions are taken from their cu-mask annotations."""
    from gpushare_scheduler_extender_amd.models.profile import POD_CU_MASK_ANNOTATION

    first = _state("1x64GiB")
    run = []
    for i in range(3):
        p = bound_pod(f"r{i}", 8, assume=i, annotations={CU_COUNT_ANNOTATION: "64"})
        first.observe(p)
        rec, _ = first.match(8)
        words = build_response(p, first.devices[0], 8, P, cus=first.claim_cus(rec)).envs["GSX_CU_MASK"]
        run.append(bound_pod(f"r{i}", 8, assume=i, assigned="true", phase="Running", uid=rec.uid,
                             annotations={CU_COUNT_ANNOTATION: "64", POD_CU_MASK_ANNOTATION: words}))
        first.observe(run[-1])
    fresh = _state("1x64GiB")
    new = bound_pod("new", 8, assume=9, annotations={CU_COUNT_ANNOTATION: "64"})
    fresh.resync(run + [new])
    assert fresh.cus[0].free_count() == 64 and fresh.stats["cu_adopted"] == 3
    rec, _ = fresh.match(8)
    got = set(fresh.claim_cus(rec))
    held = {c for u, cs in fresh.cus[0].held().items() if u != rec.uid for c in cs}
    assert len(got) == 64 and not got & held
    # a pending ASSIGNED=true multi-container pod: progress unknown after restart, all sizes accepted
    mc = bound_pod("mc", [8, 4], assume=3, assigned="true")
    fresh.observe(mc)
    assert sorted(fresh.partial[mc["metadata"]["uid"]]) == [4, 8]


def test_build_response_env_and_devices():
    dev = fake_devices("8x288GB")[3]
    pod = bound_pod("p", 64, dev=3, dev_total=268)
    r = build_response(pod, dev, 64, P)
    assert r.envs["HIP_VISIBLE_DEVICES"] == "0" and r.envs["ROCR_VISIBLE_DEVICES"] == "0"
    assert r.envs["SHARED_GPU_MEM_IDX"] == "3" and r.envs["SHARED_GPU_MEM_DEV"] == "268"
    assert r.envs["SHARED_GPU_MEM_CONTAINER"] == "64" and r.envs["SHARED_GPU_MEM_POD"] == "64"
    assert abs(float(r.envs["GSX_GPU_MEM_FRACTION"]) - 64 / 268) < 1e-6
    paths = [d["host_path"] for d in r.devices]
    assert paths == ["/dev/kfd", f"/dev/dri/renderD{128 + 24}", "/dev/dri/card4"]
    r2 = build_response(pod, dev, 64, P, mount_mode="all")
    assert r2.envs["HIP_VISIBLE_DEVICES"] == "3" and r2.devices == []
    r3 = build_response(bound_pod("q", 8, dev=0), dev, 8, ALIYUN)
    assert "ALIYUN_COM_GPU_MEM_CONTAINER" in r3.envs


def test_cu_partitioner_spreads_over_xcds_and_releases():
    cp = CUPartitioner(256, 8)
    a = cp.allocate("a", 64)
    assert len(a) == 64 and len({c // 32 for c in a}) == 8  # 8 CUs on each of the 8 XCDs
    b = cp.allocate("b", 64)
    assert not set(a) & set(b)
    assert cp.allocate("a", 64) == a  # idempotent
    cp.allocate("c", 64)
    cp.allocate("d", 64)
    with pytest.raises(Exception):
        cp.allocate("e", 1)
    assert cp.release("b") == 64 and cp.free_count() == 64
    assert CUPartitioner.ranges([0, 1, 2, 5, 7, 8]) == "0-2,5,7-8"
    w = CUPartitioner.words(list(range(32, 40)))
    assert w[1] == 0xFF and w[0] == 0


def test_build_response_cu_mask_env():
    dev = fake_devices("1x288GB")[0]
    r = build_response(bound_pod("p", 8), dev, 8, P, cus=[0, 1, 2, 3, 32, 33])
    assert r.envs["HSA_CU_MASK"] == "0:0-3,32-33"
    assert r.envs["GSX_CU_MASK"].startswith("0x0000000f,0x00000003")


def test_fake_devices_and_discover(monkeypatch):
    devs = fake_devices("4x288GB")
    assert [d.units("GiB") for d in devs] == [268] * 4
    monkeypatch.setenv("GSX_FAKE_DEVICES", "2x64GiB")
    backend, d2 = discover()
    assert backend == "fake" and [d.units("GiB") for d in d2] == [64, 64]


def test_native_mxdev_fake_backend_matches_python():
    from gpushare_scheduler_extender_amd.ops import mxdev

    recs = mxdev.enumerate_devices("fake:8x288GB")
    assert len(recs) == 8
    devs = [Device(**r) for r in recs]
    py = fake_devices("8x288GB")
    assert [(d.bdf, d.total_bytes, d.render_minor) for d in devs] == [(d.bdf, d.total_bytes, d.render_minor) for d in py]
    assert devs[0].links[1] == "XGMI" and devs[0].links[0] == "SELF"
    with pytest.raises(RuntimeError):
        mxdev.native().Session("fake:nonsense")


@pytest.mark.parametrize("spec", ["2x288GB:CPX:NPS1", "2x288GB:CPX:NPS2", "1x288GB:DPX", "1x288GB:QPX:NPS4"])
def test_native_mxdev_partition_spec_matches_python(spec):
    from gpushare_scheduler_extender_amd.ops import mxdev

    nat = [Device(**r) for r in mxdev.enumerate_devices("fake:" + spec)]
    py = fake_devices(spec)
    key = lambda d: (d.index, d.bdf, d.pool, d.total_bytes, d.cu_count, d.xcc_count, d.partition,  # noqa: E731
                     d.memory_partition, d.partition_id, d.render_minor)
    assert [key(d) for d in nat] == [key(d) for d in py]
    with pytest.raises(RuntimeError):
        mxdev.native().Session("fake:1x288GB:SPX:NPS2")  # more memory pools than compute partitions


def test_memory_pools_split_shared_hbm(monkeypatch):
    from gpushare_scheduler_extender_amd.deviceplugin.devices import apply_memory_pools

    # CPX / NPS1: 8 partitions per GPU, each reporting the whole 288 GB pool
    devs = apply_memory_pools(fake_devices("2x288GB:CPX:NPS1"))
    assert len(devs) == 16 and all(d.total_bytes == 288 * 10**9 for d in devs)
    assert all(d.cu_count == 32 and d.xcc_count == 1 for d in devs)
    assert sum(d.usable_bytes for d in devs) == 2 * 288 * 10**9  # the pool is advertised once
    assert {d.usable_bytes for d in devs} == {36 * 10**9}
    # CPX / NPS2: two 144 GB pools per GPU, four partitions each
    d2 = apply_memory_pools(fake_devices("1x288GB:CPX:NPS2"))
    assert sum(d.usable_bytes for d in d2) == 288 * 10**9 and {d.usable_bytes for d in d2} == {36 * 10**9}
    # QPX / NPS4: one pool per partition, nothing to split; SPX untouched
    assert all(d.share_bytes == 0 for d in apply_memory_pools(fake_devices("1x288GB:QPX:NPS4")))
    assert all(d.share_bytes == 0 for d in apply_memory_pools(fake_devices("8x288GB")))
    # uneven pool: the remainder goes to the lowest partition ids
    odd = fake_devices("1x288GB:DPX")
    for d in odd:
        d.total_bytes = 101
    assert [d.usable_bytes for d in apply_memory_pools(odd)] == [51, 50]
    # off: raw totals (a driver that already reports per-partition VRAM)
    assert all(d.share_bytes == 0 for d in apply_memory_pools(fake_devices("1x288GB:CPX"), "off"))
    monkeypatch.setenv("GSX_FAKE_DEVICES", "1x288GB:CPX:NPS1")
    _, d3 = discover()
    assert sum(d.units("GiB") for d in d3) == 8 * (36 * 10**9 // 2**30)


def test_partitioned_device_plugin_advertises_pool_once_and_scales_fraction():
    from gpushare_scheduler_extender_amd.deviceplugin.devices import apply_memory_pools

    devs = apply_memory_pools(fake_devices("1x288GB:CPX:NPS1"))
    plugin = GpuSharePlugin(None, "n1", devs, P)
    assert sum(plugin.units.values()) == 8 * 33 and len(plugin.device_list()) == 8 * 33
    dev = devs[5]
    r = build_response(bound_pod("p", 16, dev=5, dev_total=33), dev, 16, P)
    # the partition's process sees the whole 288 GB pool: 16 of its 33 GiB is 16/33 * 36/288 of that
    assert abs(float(r.envs["GSX_GPU_MEM_FRACTION"]) - (16 / 33) * (36 / 288)) < 1e-6
    assert r.envs["SHARED_GPU_MEM_DEV"] == "33"
    # CU masks stay inside the partition's one XCD
    cp = CUPartitioner(dev.cu_count, dev.xcc_count)
    a = cp.allocate("a", 16)
    assert len(a) == 16 and all(0 <= c < 32 for c in a)
    with pytest.raises(Exception):
        cp.allocate("b", 17)


def test_runtime_slices_first_fit():
    rt = LedgerRuntime({0: 256 * GIB})
    offs = [rt.start(f"p{i}", 0, 64 * GIB) for i in range(4)]
    assert offs == [0, 64 * GIB, 128 * GIB, 192 * GIB]
    with pytest.raises(AdmissionError):
        rt.start("p5", 0, GIB)
    rt.stop("p1")
    assert rt.start("p6", 0, 32 * GIB) == 64 * GIB
    assert rt.resident_bytes(0) == 224 * GIB


def test_runtime_slices_span_holes_when_fragmented():
    """The extender admits by free bytes per device; a fragmented arena must still hold the pod (extents)."""
    rt = LedgerRuntime({0: 96 * GIB})
    for n in ("a", "b", "c"):
        rt.start(n, 0, 32 * GIB)
    rt.stop("a")
    rt.stop("c")
    assert rt.start("d", 0, 48 * GIB) == 0
    assert rt.slices[0].used["d"] == [(0, 32 * GIB), (64 * GIB, 16 * GIB)]
    assert rt.resident_bytes(0) == 80 * GIB
    with pytest.raises(AdmissionError):
        rt.start("e", 0, 20 * GIB)
    rt.stop("b")
    assert rt.start("e", 0, 20 * GIB) == 32 * GIB and rt.resident_bytes(0) == 68 * GIB


def test_native_pod_runtime_extents_match_python():
    """_engine.PodRuntime (accounting only) carves the same extents: a fragmented device still admits."""
    from gpushare_scheduler_extender_amd.core.engine import native

    rt = native().PodRuntime(0, 96 * GIB)
    for n in ("a", "b", "c"):
        assert rt.admit(n, 32 * GIB, True) == 0
    rt.release("a")
    rt.release("c")
    assert rt.admit("d", 48 * GIB, True) == 0
    assert rt.stats()["resident_bytes"] == 80 * GIB
    with pytest.raises(RuntimeError, match="arena exhausted"):
        rt.admit("e", 20 * GIB, True)


# ---------------------------------------------------------------- gRPC plugin with fake kubelet

def run(coro):
    return asyncio.run(coro)


def test_plugin_register_listandwatch_allocate(monkeypatch):
    monkeypatch.setenv("GSX_PLUGIN_PREFERRED", "1")  # GetPreferredAllocation advertised (off by default)

    async def go():
        api_srv = await FakeApiServerRunner().start()
        client = KubeClient(api_srv.url)
        d = tempfile.mkdtemp(prefix="gsx-dp-")
        kubelet = FakeKubelet(d)
        await kubelet.start()
        devs = fake_devices("2x16GiB")
        await client.create("nodes", make_node("n1", 32, 0))
        plugin = GpuSharePlugin(client, "n1", devs, P, socket_dir=d)
        await plugin.start()
        try:
            await asyncio.wait_for(kubelet.registered.wait(), 5)
            reg = kubelet.registrations[0]
            assert reg.resource_name == "shared-gpu/gpu-mem" and reg.version == "v1beta1"
            assert reg.endpoint == "gpushare-amd.sock" and reg.options.get_preferred_allocation_available
            node = await client.get("nodes", "n1")
            assert node["status"]["capacity"]["shared-gpu/gpu-count"] == "2"
            assert node["metadata"]["annotations"]["gpushare.amd.com/device-memory"] == "16,16"
            pc = PluginClient(plugin.socket_path)
            stream = pc.list_and_watch()
            first = await stream.read()
            assert len(first.devices) == 32 and all(x.health == "Healthy" for x in first.devices)
            # two bound pods of 8 on GPU1: "b" lands first (its ASSUME_TIME is the later one).  kubelet admits pods
            # in the order they land, so the first Allocate is b's (landing order, native/engine/allocstate.h)
            await client.create("pods", bound_pod("b", 8, dev=1, assume=20, dev_total=16))
            await client.create("pods", bound_pod("a", 8, dev=1, assume=10, dev_total=16))
            ids = fake_ids(devs[0], 16) + fake_ids(devs[1], 16)
            pref = await pc.preferred(ids, 8)
            assert all(i in plugin.ids[1] for i in pref.container_responses[0].deviceIDs)
            r = await pc.allocate([list(pref.container_responses[0].deviceIDs)])
            env = dict(r.container_responses[0].envs)
            assert env["SHARED_GPU_MEM_IDX"] == "1" and env["SHARED_GPU_MEM_CONTAINER"] == "8"
            assert [x.host_path for x in r.container_responses[0].devices][0] == "/dev/kfd"
            assert await assigned_value(client, "b") == "true"
            a = await client.get("pods", "a", "default")
            assert a["metadata"]["annotations"]["SHARED_GPU_MEM_ASSIGNED"] == "false"
            await pc.allocate([ids[:8]])
            assert await assigned_value(client, "a") == "true"
            node = await client.get("nodes", "n1")
            assert node["metadata"]["annotations"]["gpushare.amd.com/allocate-order"] == "landing"
            # nothing left to match
            with pytest.raises(Exception) as ei:
                await pc.allocate([ids[:8]])
            assert "no pending pod" in str(ei.value)
            # health change re-sends the list with Unhealthy IDs of GPU0
            plugin.set_health(0, False, "test")
            nxt = await asyncio.wait_for(stream.read(), 5)
            bad = [x.ID for x in nxt.devices if x.health == "Unhealthy"]
            assert sorted(bad) == sorted(plugin.ids[0])
            stream.cancel()
            await pc.close()
        finally:
            await plugin.stop()
            await kubelet.stop()
            await client.close()
            await api_srv.stop()

    run(go())


def test_plugin_reregisters_after_kubelet_restart():
    """kubelet re-creates its socket on restart: the plugin re-serves (old server retired) and registers again."""
    async def go():
        api_srv = await FakeApiServerRunner().start()
        client = KubeClient(api_srv.url)
        d = tempfile.mkdtemp(prefix="gsx-dp-")
        kubelet = FakeKubelet(d)
        await kubelet.start()
        await client.create("nodes", make_node("n1", 32, 0))
        plugin = GpuSharePlugin(client, "n1", fake_devices("2x16GiB"), P, socket_dir=d)
        await plugin.start(publish=False)
        kubelet2 = None
        try:
            await asyncio.wait_for(kubelet.registered.wait(), 5)
            first_server = plugin._native or plugin._server
            await kubelet.stop()
            kubelet2 = FakeKubelet(d)
            await kubelet2.start()  # new socket inode: the plugin's watcher notices within ~1 s
            await asyncio.wait_for(kubelet2.registered.wait(), 10)
            for _ in range(100):  # the kubelet side sees Register before the plugin's call returns
                if plugin.stats["registrations"] == 2:
                    break
                await asyncio.sleep(0.01)
            assert plugin.stats["registrations"] == 2
            assert (plugin._native or plugin._server) is not first_server
            pc = PluginClient(plugin.socket_path)
            opts = await pc.options()
            # "auto" (default): advertised on multi-GPU nodes, where steering the unit IDs onto the pod's GPU lets
            # kubelet's per-ID accounting bound each GPU; a one-GPU node skips the round trip
            assert opts.get_preferred_allocation_available == (len(plugin.devices) > 1)
            assert not opts.pre_start_required
            first = await pc.list_and_watch().read()
            assert len(first.devices) == 32
            await pc.close()
        finally:
            await plugin.stop()
            if kubelet2 is not None:
                await kubelet2.stop()
            await client.close()
            await api_srv.stop()

    run(go())


def test_kubelet_restart_lands_an_early_answered_commit_the_old_endpoint_dropped(monkeypatch):
    """An Allocate answered early, its ASSIGNED commit still failing (retried with backoff by the endpoint's worker)
    when kubelet restarts: the plugin's re-serve closes the old endpoint, whose queued retries go with it, and lands
    the journaled commit itself."""
    monkeypatch.setenv("GSX_PLUGIN_EARLY_ANSWER", "1")

    async def go():
        api_srv = await FakeApiServerRunner().start()
        client = KubeClient(api_srv.url)
        d = tempfile.mkdtemp(prefix="gsx-dp-")
        kubelet = FakeKubelet(d)
        await kubelet.start()
        await client.create("nodes", make_node("n1", 32, 0))
        plugin = GpuSharePlugin(client, "n1", fake_devices("2x16GiB"), P, socket_dir=d)
        await plugin.start(publish=False)
        kubelet2 = None
        try:
            await asyncio.wait_for(kubelet.registered.wait(), 5)
            if plugin.grpc_impl != "native":
                pytest.skip("the early answer is the native endpoint's")
            await client.create("pods", bound_pod("a", 4, dev=0, assume=1, dev_total=16))
            await asyncio.sleep(0.3)
            api_srv.server.faults.error_rate = 1.0  # the commit's PATCH fails: the endpoint retries it with backoff
            pc = PluginClient(plugin.socket_path)
            r = (await pc.allocate([fake_ids(plugin.devices[0], 16)[0:4]])).container_responses[0]
            assert dict(r.annotations)["gpushare.amd.com/pod"].split("/")[1] == "a"
            await pc.close()
            await asyncio.sleep(0.1)  # the commit is queued for its next attempt
            await kubelet.stop()
            kubelet2 = FakeKubelet(d)
            await kubelet2.start()
            await asyncio.wait_for(kubelet2.registered.wait(), 10)
            api_srv.server.faults.error_rate = 0.0
            ann = {}
            for _ in range(100):  # within ~5 s (the old endpoint's retries went with it)
                ann = (await client.get("pods", "a", "default"))["metadata"]["annotations"]
                if ann.get(P.annotation_assigned) == "true":
                    break
                await asyncio.sleep(0.05)
            assert ann.get(P.annotation_assigned) == "true", ann
        finally:
            api_srv.server.faults.error_rate = 0.0
            await plugin.stop()
            if kubelet2 is not None:
                await kubelet2.stop()
            await client.close()
            await api_srv.stop()

    run(go())


def test_plugin_allocate_retries_conflicts_and_apiserver_errors():
    """kubelet's Allocate must not fail over transient apiserver trouble: 409s and 500s on the ASSIGNED patch
    are retried from a fresh LIST; every pod still ends up ASSIGNED=true exactly once."""
    async def go():
        api_srv = await FakeApiServerRunner().start()
        client = KubeClient(api_srv.url)
        d = tempfile.mkdtemp(prefix="gsx-dp-")
        kubelet = FakeKubelet(d)
        await kubelet.start()
        devs = fake_devices("2x16GiB")
        await client.create("nodes", make_node("n1", 32, 0))
        plugin = GpuSharePlugin(client, "n1", devs, P, socket_dir=d)
        await plugin.start()
        try:
            await asyncio.wait_for(kubelet.registered.wait(), 5)
            pc = PluginClient(plugin.socket_path)
            for i in range(4):
                await client.create("pods", bound_pod(f"p{i}", 4, dev=0, assume=10 + i, dev_total=16))
            # every commit meets a 500 or a 409 while the faults are on (early answer: the Allocate is answered first)
            api_srv.server.faults.update({"conflict_rate": 0.5, "error_rate": 1.0, "seed": 5})
            ids = fake_ids(devs[0], 16)
            for i in range(4):
                r = await pc.allocate([ids[4 * i: 4 * i + 4]])
                assert dict(r.container_responses[0].envs)["SHARED_GPU_MEM_IDX"] == "0"
            api_srv.server.faults.update({"conflict_rate": 0, "error_rate": 0})
            for i in range(4):  # early answer (default): a commit that hit a fault lands on its backoff retry
                for _ in range(200):
                    p = await client.get("pods", f"p{i}", "default")
                    if p["metadata"]["annotations"]["SHARED_GPU_MEM_ASSIGNED"] == "true":
                        break
                    await asyncio.sleep(0.01)
                assert p["metadata"]["annotations"]["SHARED_GPU_MEM_ASSIGNED"] == "true"
            # retried: by the Python handler, or a native fast-path patch that failed and was handed to it
            native_failures = plugin.debug_state()["grpc"].get("patch_failures", 0)
            assert plugin.stats["allocate_retries"] + native_failures > 0 and plugin.stats["allocate_fail"] == 0
            await pc.close()
        finally:
            await plugin.stop()
            await kubelet.stop()
            await client.close()
            await api_srv.stop()
    run(go())


def test_plugin_multi_container_pod_and_cu_partition():
    async def go():
        api_srv = await FakeApiServerRunner().start()
        client = KubeClient(api_srv.url)
        d = tempfile.mkdtemp(prefix="gsx-dp-")
        devs = fake_devices("1x64GiB")
        await client.create("nodes", make_node("n1", 64, 1))
        plugin = GpuSharePlugin(client, "n1", devs, P, socket_dir=d)
        await plugin.start(register=False)
        try:
            pc = PluginClient(plugin.socket_path)
            await client.create("pods", bound_pod("mc", [10, 20], dev=0, dev_total=64,
                                                  annotations={CU_COUNT_ANNOTATION: "64"}))
            ids = plugin.ids[0]
            r1 = await pc.allocate([ids[:20]])
            r2 = await pc.allocate([ids[20:30]])
            e1, e2 = dict(r1.container_responses[0].envs), dict(r2.container_responses[0].envs)
            assert e1["SHARED_GPU_MEM_CONTAINER"] == "20" and e2["SHARED_GPU_MEM_CONTAINER"] == "10"
            assert e1["HSA_CU_MASK"] == e2["HSA_CU_MASK"] and e1["HSA_CU_MASK"].startswith("0:")
            p = await client.get("pods", "mc", "default")
            assert p["metadata"]["annotations"]["gpushare.amd.com/cu-mask"] == e1["GSX_CU_MASK"]
            await pc.close()
        finally:
            await plugin.stop()
            await client.close()
            await api_srv.stop()
    run(go())


def test_node_agent_admits_and_releases():
    async def go():
        api_srv = await FakeApiServerRunner().start()
        client = KubeClient(api_srv.url)
        devs = fake_devices("2x16GiB")
        rt = LedgerRuntime({0: 16 * GIB, 1: 16 * GIB})
        agent = NodeAgent(client, "n1", devs, P, rt)
        await agent.start()
        try:
            for i, dev in enumerate([0, 0, 1]):
                await client.create("pods", bound_pod(f"p{i}", 8, dev=dev, assume=i, dev_total=16))
            for _ in range(400):
                if agent.admitted == 3:
                    break
                await asyncio.sleep(0.01)
            assert agent.admitted == 3 and rt.resident_bytes(0) == 16 * GIB and rt.resident_bytes(1) == 8 * GIB
            p = await client.get("pods", "p0", "default")
            assert p["status"]["phase"] == "Running"
            assert p["metadata"]["annotations"]["SHARED_GPU_MEM_ASSIGNED"] == "true"
            await client.delete("pods", "p1", "default")
            for _ in range(400):
                if rt.resident_bytes(0) == 8 * GIB:
                    break
                await asyncio.sleep(0.01)
            assert rt.resident_bytes(0) == 8 * GIB
            # an over-committed pod (the ledger would never do this) is refused at admission
            await client.create("pods", bound_pod("big", 12, dev=0, assume=9, dev_total=16))
            for _ in range(400):
                if agent.failed:
                    break
                await asyncio.sleep(0.01)
            assert agent.failed == 1
            big = await client.get("pods", "big", "default")
            assert big["status"]["phase"] == "Failed"
        finally:
            await agent.stop()
            await client.close()
            await api_srv.stop()
    run(go())


def test_api_messages_roundtrip():
    r = api.ContainerAllocateResponse()
    r.envs["HIP_VISIBLE_DEVICES"] = "0"
    r.devices.add(container_path="/dev/kfd", host_path="/dev/kfd", permissions="rw")
    b = r.SerializeToString()
    assert api.ContainerAllocateResponse.FromString(b).envs["HIP_VISIBLE_DEVICES"] == "0"
    # field numbers match the upstream proto: envs=1 (map), devices=3
    assert b[0] == 0x0A and b"\x1a" in b
    assert api.method_path("DevicePlugin", "Allocate") == "/v1beta1.DevicePlugin/Allocate"
    assert json.dumps(list(api.SERVICES["DevicePlugin"]))


def test_process_runtime_starts_container_with_allocate_env():
    """Slice B plumbing on CPU: bind -> Allocate -> the launcher runs the container with Allocate's env."""
    import asyncio
    import sys as _sys

    from gpushare_scheduler_extender_amd.deviceplugin.devices import fake_devices
    from gpushare_scheduler_extender_amd.deviceplugin.runtime import ProcessRuntime
    from gpushare_scheduler_extender_amd.extender.server import ExtenderRunner, ExtenderServer
    from tests.fixtures.fakeapi import FakeApiServerRunner
    from tests.fixtures.schedsim import SchedulerSim

    code = "import json,os;print(json.dumps({k:v for k,v in os.environ.items() if k.startswith(('SHARED_','HIP_','ROCR_'))}))"

    async def go():
        api = await FakeApiServerRunner().start()
        client = KubeClient(api.url)
        ext = await ExtenderRunner(ExtenderServer(KubeClient(api.url), P)).start()
        devs = fake_devices("2x288GB")
        rt = ProcessRuntime([_sys.executable, "-c", code])
        agent = NodeAgent(KubeClient(api.url), "n1", devs, P, rt, unit="GiB")
        sim = SchedulerSim(KubeClient(api.url), ext.url, P)
        try:
            totals = [d.units("GiB") for d in devs]
            await client.create("nodes", make_node("n1", sum(totals), 2, device_totals=totals))
            await agent.start()
            await sim.start()
            await client.create("pods", make_pod("b1", 200))
            await client.create("pods", make_pod("b2", 200))
            await sim.wait_bound(["default/b1", "default/b2"], 20)
            for _ in range(2000):
                if len(rt.procs) == 2:
                    break
                await asyncio.sleep(0.005)
            outs = {}
            for uid in list(rt.procs):
                rc, so, _se = await rt.wait(uid, 60)
                assert rc == 0
                outs[uid] = json.loads(so.strip().splitlines()[-1])
            pods = {p["metadata"]["uid"]: p for p in (await client.list("pods"))["items"]}
            return outs, pods
        finally:
            await sim.stop()
            await sim.client.close()
            await agent.stop()
            await agent.client.close()
            rt.close()
            await ext.stop()
            await ext.server.client.close()
            await client.close()
            await api.stop()

    outs, pods = asyncio.run(go())
    assert len(outs) == 2
    used = set()
    for uid, env in outs.items():
        ann = pods[uid]["metadata"]["annotations"]
        assert ann[P.annotation_assigned] == "true"
        assert env["HIP_VISIBLE_DEVICES"] == ann[P.annotation_idx] == env["SHARED_GPU_MEM_IDX"]
        assert env["SHARED_GPU_MEM_CONTAINER"] == "200"
        used.add(env["HIP_VISIBLE_DEVICES"])
    assert used == {"0", "1"}  # 200 + 200 GiB cannot share one 288 GB device


# ---------------------------------------------------------------- plugin lifecycle

class _PluginStack:
    """fake apiserver + the shipped gRPC plugin + the kubelet stand-in talking to it over its unix socket."""

    def __init__(self, spec="1x268GiB"):
        self.spec = spec

    async def __aenter__(self):
        self.api = await FakeApiServerRunner().start()
        self.client = KubeClient(self.api.url)
        self.dir = tempfile.mkdtemp(prefix="gsx-dp-")
        self.devs = fake_devices(self.spec)
        totals = [d.units("GiB") for d in self.devs]
        await self.client.create("nodes", make_node("n1", sum(totals), len(totals), device_totals=totals))
        self.plugin = await self.start_plugin()
        self.rt = LedgerRuntime({d.index: d.units("GiB") * GIB for d in self.devs})
        self.agent = NodeAgent(KubeClient(self.api.url), "n1", self.devs, P, self.rt,
                               plugin_socket=self.plugin.socket_path)
        await self.agent.start()
        return self

    async def start_plugin(self):
        plugin = GpuSharePlugin(KubeClient(self.api.url), "n1", self.devs, P, socket_dir=self.dir)
        await plugin.start(register=False)
        return plugin

    async def restart_plugin(self):
        await self.plugin.stop()
        await self.plugin.client.close()
        self.plugin = await self.start_plugin()  # same socket path: the kubelet stand-in reconnects

    async def wait(self, pred, timeout=10.0):
        for _ in range(int(timeout / 0.01)):
            if pred():
                return
            await asyncio.sleep(0.01)
        st = self.plugin.state
        raise TimeoutError(f"condition not reached: cu holders {[sorted(c.held()) for c in st.cus.values()]}, "
                           f"pods {sorted(st.pods)}, records {[(r.uid, r.dev) for r in st.records.values()] if not callable(st.records) else [(r.uid, r.dev) for r in st.records().values()]}, "
                           f"stats {self.plugin.stats}")

    async def phase(self, name):
        return (await self.client.get("pods", name, "default"))["status"].get("phase")

    async def wait_phase(self, name, phase="Running", timeout=10.0):
        for _ in range(int(timeout / 0.01)):
            if await self.phase(name) == phase:
                return await self.client.get("pods", name, "default")
            await asyncio.sleep(0.01)
        raise TimeoutError(f"{name} not {phase}: {await self.phase(name)}")

    async def wait_committed(self, name, timeout=10.0):
        """Running, and the plugin's commit (ASSIGNED=true with the CU mask) landed: with early answer (the
        default) kubelet starts the container before the commit is written."""
        await self.wait_phase(name, timeout=timeout)
        for _ in range(int(timeout / 0.01)):
            pod = await self.client.get("pods", name, "default")
            if pod["metadata"].get("annotations", {}).get("SHARED_GPU_MEM_ASSIGNED") == "true":
                return pod
            await asyncio.sleep(0.01)
        raise TimeoutError(f"{name}: the ASSIGNED commit never landed")

    async def __aexit__(self, *exc):
        await self.agent.stop()
        await self.agent.client.close()
        await self.plugin.stop()
        await self.plugin.client.close()
        await self.client.close()
        await self.api.stop()


def _cus_of(pod):
    from gpushare_scheduler_extender_amd.deviceplugin.state import parse_cu_mask
    from gpushare_scheduler_extender_amd.models.profile import POD_CU_MASK_ANNOTATION

    return set(parse_cu_mask(pod["metadata"]["annotations"][POD_CU_MASK_ANNOTATION]))


def test_cu_partitions_are_released_when_pods_go_away():
    """Done-criterion (a): 64-CU pods keep allocating across deletes; before the fix the fifth failed forever."""
    async def go():
        async with _PluginStack() as s:
            cu = {CU_COUNT_ANNOTATION: "64"}
            for i in range(4):
                await s.client.create("pods", bound_pod(f"p{i}", 16, assume=i, annotations=cu))
            pods = [await s.wait_committed(f"p{i}") for i in range(4)]
            sets = [_cus_of(p) for p in pods]
            assert all(len(x) == 64 for x in sets) and len(set().union(*sets)) == 256
            assert s.plugin.state.cus[0].free_count() == 0
            # the node's CUs are all taken: a fifth partition needs a pod to go away first
            await s.client.delete("pods", "p1", "default")
            await s.wait(lambda: s.plugin.state.cus[0].free_count() == 64)
            await s.client.create("pods", bound_pod("p4", 16, assume=4, annotations=cu))
            p4 = await s.wait_committed("p4")
            assert _cus_of(p4) == sets[1]
            # five sequential pods, each deleted before the next: all allocate
            for i in (0, 2, 3, 4):
                await s.client.delete("pods", f"p{i}", "default")
            await s.wait(lambda: s.plugin.state.cus[0].free_count() == 256)
            for i in range(5):
                await s.client.create("pods", bound_pod(f"s{i}", 16, assume=10 + i, annotations=cu))
                assert len(_cus_of(await s.wait_committed(f"s{i}"))) == 64
                await s.client.delete("pods", f"s{i}", "default")
            await s.wait(lambda: s.plugin.state.cus[0].free_count() == 256 and not s.plugin.state.pods)
            assert s.plugin.stats["allocate_fail"] == 0 and s.agent.failed == 0
            # a Succeeded pod (not deleted) also gives its partition back
            await s.client.create("pods", bound_pod("job", 16, assume=30, annotations=cu))
            await s.wait_phase("job")
            await s.client.patch("pods", "job", {"status": {"phase": "Succeeded"}}, "default", sub="status")
            await s.wait(lambda: s.plugin.state.cus[0].free_count() == 256)
    run(go())


def test_plugin_restart_rebuilds_partitions_from_annotations():
    """Done-criterion (b): after a restart the new pod's CU mask is disjoint from every running pod's."""
    async def go():
        async with _PluginStack() as s:
            cu = {CU_COUNT_ANNOTATION: "64"}
            for i in range(3):
                await s.client.create("pods", bound_pod(f"r{i}", 16, assume=i, annotations=cu))
            running = [_cus_of(await s.wait_committed(f"r{i}")) for i in range(3)]
            await s.restart_plugin()
            assert s.plugin.state.cus[0].free_count() == 64  # rebuilt before serving
            assert s.plugin.state.stats["cu_adopted"] == 3
            await s.client.create("pods", bound_pod("new", 16, assume=9, annotations=cu))
            new = _cus_of(await s.wait_committed("new"))
            assert len(new) == 64 and all(not new & r for r in running)
            # and a fifth partition does not exist until one goes away
            await s.client.create("pods", bound_pod("extra", 16, assume=10, annotations=cu))
            await s.wait_phase("extra", "Failed")
            assert s.plugin.stats["allocate_fail"] >= 1
    run(go())


def test_multi_container_progress_survives_restart_and_is_released():
    async def go():
        async with _PluginStack() as s:
            await s.client.create("pods", bound_pod("mc", [10, 20], assume=1))
            await s.wait_phase("mc")
            env = s.agent.allocations[(await s.client.get("pods", "mc", "default"))["metadata"]["uid"]]
            assert env["SHARED_GPU_MEM_POD"] == "30"
            assert not s.plugin.state.partial  # both containers allocated, pod Running
            await s.client.delete("pods", "mc", "default")
            await s.wait(lambda: not s.plugin.state.pods)
    run(go())
