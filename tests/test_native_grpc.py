"""The device plugin's native gRPC endpoint (``native/engine/h2.cc`` on libnghttp2, ``dpcore.cc``): interop with
grpcio in both directions, the fast Allocate path against the Python handler it stands in for, and the hand-off
of everything else to Python."""
import asyncio
import json
import os
import tempfile

import grpc
import pytest

from gpushare_scheduler_extender_amd.core.engine import native
from gpushare_scheduler_extender_amd.deviceplugin import api
from gpushare_scheduler_extender_amd.deviceplugin.devices import fake_devices
from gpushare_scheduler_extender_amd.deviceplugin.isolation import IsolationManager
from gpushare_scheduler_extender_amd.deviceplugin.plugin import GpuSharePlugin, fake_ids
from gsxtools.kubeletapi import FakeKubelet, PluginClient
from gpushare_scheduler_extender_amd.k8s.client import KubeClient
from gpushare_scheduler_extender_amd.k8s.objects import make_node
from gpushare_scheduler_extender_amd.models.profile import POD_CU_COUNT_ANNOTATION, SHARED_GPU
from tests.fixtures.fakeapi import FakeApiServerRunner
from tests.test_deviceplugin import bound_pod

P = SHARED_GPU

pytestmark = pytest.mark.skipif(not native().h2_available()[0], reason="libnghttp2 not on this system")


async def _plugin(tmp, fast: bool, isolation: bool = False, spec: str = "2x16GiB"):
    api_srv = await FakeApiServerRunner().start()
    client = KubeClient(api_srv.url)
    await client.create("nodes", make_node("n1", 32, 0))
    iso = IsolationManager(os.path.join(tmp, "iso")) if isolation else None
    os.environ["GSX_PLUGIN_FAST"] = "1" if fast else "0"
    try:
        plugin = GpuSharePlugin(client, "n1", fake_devices(spec), P, socket_dir=os.path.join(tmp, "dp"), isolation=iso)
        await plugin.start(register=False)
    finally:
        os.environ.pop("GSX_PLUGIN_FAST", None)
    assert plugin.grpc_impl == "native"
    return api_srv, client, plugin


async def _close(api_srv, client, plugin, *clients):
    for c in clients:
        await c.close()
    await plugin.stop()
    await client.close()
    await api_srv.stop()


def test_grpcio_kubelet_against_the_native_endpoint(monkeypatch):
    monkeypatch.setenv("GSX_PLUGIN_PREFERRED", "1")  # GetPreferredAllocation advertised (off by default)

    async def go():
        tmp = tempfile.mkdtemp()
        api_srv, client, plugin = await _plugin(tmp, fast=True)
        pc = PluginClient(plugin.socket_path)
        try:
            opts = await pc._call("GetDevicePluginOptions")(api.Empty())
            assert opts.get_preferred_allocation_available and not opts.pre_start_required
            stream = pc.list_and_watch()
            first = await asyncio.wait_for(stream.read(), 5)
            assert len(first.devices) == 32 and {d.health for d in first.devices} == {api.HEALTHY}
            plugin.set_health(1, False, "test")  # the stream gets the new list
            second = await asyncio.wait_for(stream.read(), 5)
            assert sum(d.health == api.UNHEALTHY for d in second.devices) == 16
            stream.cancel()
            for i in range(3):
                await client.create("pods", bound_pod(f"p{i}", 4, dev=0, assume=10 + i, dev_total=16))
            await asyncio.sleep(0.2)
            ids = fake_ids(plugin.devices[0], 16)
            pref = await pc.preferred(ids + fake_ids(plugin.devices[1], 16), 4)
            assert all(i.startswith(ids[0].split("-")[0]) for i in pref.container_responses[0].deviceIDs)
            for i in range(3):
                r = await pc.allocate([ids[4 * i: 4 * i + 4]])
                envs = dict(r.container_responses[0].envs)
                assert envs["SHARED_GPU_MEM_IDX"] == "0" and envs["SHARED_GPU_MEM_CONTAINER"] == "4"
                assert dict(r.container_responses[0].annotations)["gpushare.amd.com/pod"].startswith(f"default/p{i}/")
            with pytest.raises(grpc.aio.AioRpcError) as e:  # no pod left: the Python handler says why
                await pc.allocate([ids[12:16]])
            assert e.value.code() == grpc.StatusCode.FAILED_PRECONDITION and "no pending pod" in e.value.details()
            st = plugin.debug_state()["grpc"]
            assert st["fast_allocate"] == 3 and st["slow_allocate"] >= 1 and st["fast_preferred"] >= 1, st
            for i in range(3):  # committed exactly like the Python path: ASSIGNED=true, a record per Allocate
                assert (await client.get("pods", f"p{i}", "default"))["metadata"]["annotations"][
                    P.annotation_assigned] == "true"
            assert len(plugin.state.records) == 3 and plugin.stats["allocate_native"] == 3
            # the endpoint's own counters and the plugin's per-Allocate times on /metrics
            m = plugin.metrics_text()
            assert "gpushare_plugin_native_fast_allocate_total 3" in m, m
            assert "gpushare_plugin_native_slow_allocate_total" in m and "gpushare_plugin_allocate_handler_seconds" in m
            assert st["serving_thread"], st  # served from the native thread, not the event loop
        finally:
            await _close(api_srv, client, plugin, pc)
    asyncio.run(go())


def test_preferred_allocation_steers_ids_onto_the_pods_gpu(monkeypatch):
    """GetPreferredAllocation on the native endpoint: kubelet's usual request (one container, every free ID, in any
    order) gets the pod's GPU's IDs first and others only when that GPU has too few; a request with must_include
    IDs (the general path) keeps them."""
    monkeypatch.setenv("GSX_PLUGIN_PREFERRED", "1")

    async def go():
        tmp = tempfile.mkdtemp()
        api_srv, client, plugin = await _plugin(tmp, fast=True)
        pc = PluginClient(plugin.socket_path)
        try:
            await client.create("pods", bound_pod("a", 4, dev=1, assume=1, dev_total=16))
            await asyncio.sleep(0.2)
            ids0, ids1 = fake_ids(plugin.devices[0], 16), fake_ids(plugin.devices[1], 16)
            on1 = set(ids1)
            got = list((await pc.preferred(ids0 + ids1[::-1], 4)).container_responses[0].deviceIDs)
            assert len(got) == 4 and set(got) <= on1 and got == ids1[::-1][:4], got
            got = list((await pc.preferred(ids0[:8] + ids1[:2] + ids0[8:], 4)).container_responses[0].deviceIDs)
            assert got[:2] == ids1[:2] and got[2:] == ids0[:2], got  # GPU 1 has two free: the rest in list order
            got = list((await pc.preferred(ids0 + ids1, 4, must=[ids0[5]])).container_responses[0].deviceIDs)
            assert got[0] == ids0[5] and set(got[1:]) <= on1 and len(got) == 4, got
            assert plugin.debug_state()["grpc"]["fast_preferred"] >= 3
        finally:
            await _close(api_srv, client, plugin, pc)
    asyncio.run(go())


@pytest.mark.parametrize("isolation", [False, True])
def test_fast_path_answers_exactly_what_the_python_handler_answers(isolation):
    """The same pods through the native fast path and through the Python handler (fast path off): identical
    container responses (env contract, device nodes, CU partition, isolation mounts)."""
    async def run(fast):
        tmp = tempfile.mkdtemp()
        api_srv, client, plugin = await _plugin(tmp, fast=fast, isolation=isolation, spec="1x64GiB")
        pc = PluginClient(plugin.socket_path)
        try:
            pods = [bound_pod("a", 16, dev=0, assume=1, dev_total=64, uid="u-a",
                              annotations={POD_CU_COUNT_ANNOTATION: "64"}),
                    bound_pod("b", [8, 4], dev=0, assume=2, dev_total=64, uid="u-b")]
            for p in pods:
                await client.create("pods", p)
            await asyncio.sleep(0.2)
            ids = fake_ids(plugin.devices[0], 64)
            out = []
            for chunk in (ids[0:16], ids[16:24], ids[24:28]):
                r = (await pc.allocate([chunk])).container_responses[0]
                out.append({"envs": dict(r.envs), "annotations": dict(r.annotations),
                            "devices": sorted((d.container_path, d.host_path, d.permissions) for d in r.devices),
                            "mounts": sorted((m.container_path, m.host_path.replace(tmp, "<tmp>"), m.read_only)
                                             for m in r.mounts)})
            st = plugin.debug_state()["grpc"]
            return out, st
        finally:
            await _close(api_srv, client, plugin, pc)
    fast, st_fast = asyncio.run(run(True))
    slow, st_slow = asyncio.run(run(False))
    assert st_fast["fast_allocate"] == 3 and st_slow["fast_allocate"] == 0
    assert fast == slow
    assert fast[0]["envs"]["HSA_CU_MASK"].startswith("0:") and "GSX_CU_MASK" in fast[0]["envs"]
    assert fast[1]["envs"]["SHARED_GPU_MEM_CONTAINER"] == "8" and fast[2]["envs"]["SHARED_GPU_MEM_CONTAINER"] == "4"
    if isolation:
        assert any(m[0] == "/etc/ld.so.preload" for m in fast[0]["mounts"])


def test_native_client_against_a_grpcio_server():
    """h2::Client (the compiled kubelet stand-in's side) registering with a grpcio Registration service."""
    async def go():
        tmp = tempfile.mkdtemp()
        kubelet = FakeKubelet(tmp)
        await kubelet.start()
        try:
            req = api.RegisterRequest(version=api.VERSION, endpoint="x.sock", resource_name=P.resource).SerializeToString()
            status, body = await asyncio.get_running_loop().run_in_executor(
                None, native().h2_call, os.path.join(tmp, api.KUBELET_SOCKET), "/v1beta1.Registration/Register", req,
                5.0)
            assert status == 0, body
            assert kubelet.registrations[0].endpoint == "x.sock"
            status, body = await asyncio.get_running_loop().run_in_executor(
                None, native().h2_call, os.path.join(tmp, api.KUBELET_SOCKET), "/v1beta1.Registration/Nope", b"", 5.0)
            assert status == 12, (status, body)  # UNIMPLEMENTED from grpcio
        finally:
            await kubelet.stop()
    asyncio.run(go())


def test_early_answer_claims_the_pod_until_its_commit_lands():
    """Opt-in early answer (GSX_PLUGIN_EARLY_ANSWER=1): an Allocate is answered once its record is journaled and
    the ASSIGNED patch follows.  With a slow apiserver the answer comes first, the pod stays claimed (a second
    Allocate of that size gets the other pod), both commits land, and the checkpoint takes over the journal."""
    async def go():
        tmp = tempfile.mkdtemp()
        os.environ["GSX_PLUGIN_EARLY_ANSWER"] = "1"
        try:
            api_srv, client, plugin = await _plugin(tmp, fast=True)
        finally:
            os.environ.pop("GSX_PLUGIN_EARLY_ANSWER", None)
        pc = PluginClient(plugin.socket_path)
        try:
            assert plugin.early_answer
            await client.create("pods", bound_pod("a", 4, dev=0, assume=1, dev_total=16))
            await client.create("pods", bound_pod("b", 4, dev=1, assume=2, dev_total=16))
            await asyncio.sleep(0.3)
            api_srv.server.faults.latency_ms = 400.0  # every apiserver call now takes 0.4 s
            ids = fake_ids(plugin.devices[0], 16) + fake_ids(plugin.devices[1], 16)
            t0 = asyncio.get_running_loop().time()
            got = []
            for chunk in (ids[0:4], ids[16:20]):
                r = (await pc.allocate([chunk])).container_responses[0]
                got.append(dict(r.annotations)["gpushare.amd.com/pod"].split("/")[1])
            assert asyncio.get_running_loop().time() - t0 < 0.35, "answers waited for the apiserver"
            assert got == ["a", "b"], got  # a stayed claimed while its commit was in flight
            assert len(_journal_lines(plugin.journal_path)) == 2
            api_srv.server.faults.latency_ms = 0.0
            for _ in range(200):  # both commits land
                anns = [(await client.get("pods", n, "default"))["metadata"]["annotations"] for n in ("a", "b")]
                if all(a[P.annotation_assigned] == "true" for a in anns):
                    break
                await asyncio.sleep(0.02)
            assert all(a[P.annotation_assigned] == "true" for a in anns), anns
            for _ in range(100):  # the debounced checkpoint took the records and emptied the journal
                if os.path.exists(plugin.checkpoint) and not _journal_lines(plugin.journal_path):
                    break
                await asyncio.sleep(0.02)
            assert not _journal_lines(plugin.journal_path)
            with open(plugin.checkpoint) as f:
                assert len(json.load(f)["records"]) == 2
        finally:
            await _close(api_srv, client, plugin, pc)
    asyncio.run(go())


def _journal_lines(path: str) -> list:
    """The journal's lines: the native side maps the file in 1 MiB steps, so zeros follow the last line while it runs."""
    with open(path, "rb") as f:
        return [ln for ln in f.read().rstrip(b"\0").splitlines() if ln.strip(b"\0")]


def test_mapped_journal_survives_a_torn_tail_and_is_trimmed_on_close():
    """The journal is a shared mapping sized ahead (dpcore.cc journal_map): a crash can leave a line torn mid-copy
    and zeros after it.  A restarted plugin keeps the whole lines, writes over the torn one, and a closed endpoint
    leaves the file trimmed to whole JSON lines."""
    async def go():
        tmp = tempfile.mkdtemp()
        os.environ["GSX_PLUGIN_EARLY_ANSWER"] = "1"
        try:
            api_srv, client, plugin = await _plugin(tmp, fast=True)
            a = await client.create("pods", bound_pod("a", 4, dev=0, assume=1, dev_total=16))
            await client.create("pods", bound_pod("b", 4, dev=0, assume=2, dev_total=16))
            await plugin.stop()
            ids = fake_ids(plugin.devices[0], 16)
            whole = json.dumps({"aid": "x-1", "uid": a["metadata"]["uid"], "ids": sorted(ids[0:4]), "dev": 0,
                                "units": 4, "cu_mask": "", "owner": "", "t": 0.0, "iso": ""}) + "\n"
            with open(plugin.journal_path, "wb") as f:  # a whole line, a line torn by a crash, the mapping's zeros
                f.write(whole.encode() + b'{"aid":"x-2","uid":"torn-line-with-no-end' + b"\0" * 4096)
            again = GpuSharePlugin(client, "n1", fake_devices("2x16GiB"), P, socket_dir=os.path.join(tmp, "dp"))
            await again.start(register=False)
        finally:
            os.environ.pop("GSX_PLUGIN_EARLY_ANSWER", None)
        pc = PluginClient(again.socket_path)
        try:
            assert again.stats.get("commits_after_restart") == 1  # the whole line was read, the torn one skipped
            r = (await pc.allocate([ids[4:8]])).container_responses[0]
            assert dict(r.annotations)["gpushare.amd.com/pod"].split("/")[1] == "b"
            lines = _journal_lines(again.journal_path)
            assert all(json.loads(ln)["uid"] != "torn-line-with-no-end" for ln in lines)
        finally:
            await _close(api_srv, client, again, pc)
        with open(again.journal_path, "rb") as f:
            raw = f.read()
        assert b"\0" not in raw and b"torn-line" not in raw, raw[-200:]
        assert all(json.loads(ln) for ln in raw.splitlines())
    asyncio.run(go())


def test_closing_the_endpoint_does_not_wait_out_a_commit_in_flight():
    """An early-answered commit stuck on a slow apiserver: closing the native endpoint shuts its socket
    (ApiClient::abort) instead of waiting for the request to time out; the record stays in the journal."""
    async def go():
        tmp = tempfile.mkdtemp()
        os.environ["GSX_PLUGIN_EARLY_ANSWER"] = "1"
        try:
            api_srv, client, plugin = await _plugin(tmp, fast=True)
        finally:
            os.environ.pop("GSX_PLUGIN_EARLY_ANSWER", None)
        pc = PluginClient(plugin.socket_path)
        try:
            await client.create("pods", bound_pod("a", 4, dev=0, assume=1, dev_total=16))
            await asyncio.sleep(0.3)
            api_srv.server.faults.latency_ms = 30000.0  # the commit's PATCH now waits 30 s for its answer
            r = (await pc.allocate([fake_ids(plugin.devices[0], 16)[0:4]])).container_responses[0]
            assert dict(r.annotations)["gpushare.amd.com/pod"].split("/")[1] == "a"
            await asyncio.sleep(0.2)  # the commit is in flight
            t0 = asyncio.get_running_loop().time()
            await pc.close()
            await plugin.stop()
            assert asyncio.get_running_loop().time() - t0 < 5.0
            lines = _journal_lines(plugin.journal_path) + _journal_lines(plugin.journal_path + ".old") \
                if os.path.exists(plugin.journal_path + ".old") else _journal_lines(plugin.journal_path)
            with open(plugin.checkpoint) as f:
                recs = json.load(f)["records"]
            assert recs or lines  # the answered Allocate is on disk for the next start
        finally:
            api_srv.server.faults.latency_ms = 0.0
            await client.close()
            await api_srv.stop()
    asyncio.run(go())


def test_early_answer_commit_lands_after_a_restart():
    """The plugin went away between an early answer and its commit: the journal still holds the record, the pod
    still reads ASSIGNED=false.  A restarted plugin lands the commit before it serves, and never offers the pod
    to another Allocate."""
    async def go():
        tmp = tempfile.mkdtemp()
        os.environ["GSX_PLUGIN_EARLY_ANSWER"] = "1"
        try:
            api_srv, client, plugin = await _plugin(tmp, fast=True)
            a = await client.create("pods", bound_pod("a", 4, dev=0, assume=1, dev_total=16))
            await client.create("pods", bound_pod("b", 4, dev=0, assume=2, dev_total=16))
            await plugin.stop()
            ids = fake_ids(plugin.devices[0], 16)
            with open(plugin.journal_path, "w") as f:  # the answered Allocate of "a", its commit never sent
                f.write(json.dumps({"aid": "x-1", "uid": a["metadata"]["uid"], "ids": sorted(ids[0:4]), "dev": 0,
                                    "units": 4, "cu_mask": "", "owner": "", "t": 0.0, "iso": ""}) + "\n")
            again = GpuSharePlugin(client, "n1", fake_devices("2x16GiB"), P, socket_dir=os.path.join(tmp, "dp"))
            await again.start(register=False)
        finally:
            os.environ.pop("GSX_PLUGIN_EARLY_ANSWER", None)
        pc = PluginClient(again.socket_path)
        try:
            assert again.stats.get("commits_after_restart") == 1
            assert (await client.get("pods", "a", "default"))["metadata"]["annotations"][P.annotation_assigned] == "true"
            r = (await pc.allocate([ids[4:8]])).container_responses[0]
            assert dict(r.annotations)["gpushare.amd.com/pod"].split("/")[1] == "b"
            assert any(rec.uid == a["metadata"]["uid"] for rec in again.state.records.values())
        finally:
            await _close(api_srv, client, again, pc)
    asyncio.run(go())


def test_early_answer_is_the_default_and_commits_with_a_uid_precondition():
    """Early answer is on by default; its commit is guarded by the pod's UID, not the resourceVersion the match was
    made on, so kubelet's status updates landing first do not make it conflict."""
    async def go():
        tmp = tempfile.mkdtemp()
        api_srv, client, plugin = await _plugin(tmp, fast=True)
        pc = PluginClient(plugin.socket_path)
        try:
            assert plugin.early_answer and plugin.debug_state()["grpc"]["journaling"]
            await client.create("pods", bound_pod("a", 4, dev=0, assume=1, dev_total=16))
            await asyncio.sleep(0.2)
            api_srv.server.faults.latency_ms = 200.0
            ids = fake_ids(plugin.devices[0], 16)
            r = (await pc.allocate([ids[0:4]])).container_responses[0]
            assert dict(r.annotations)["gpushare.amd.com/pod"].split("/")[1] == "a"
            # kubelet's status update lands before the commit: it moves the resourceVersion
            api_srv.server.faults.latency_ms = 0.0
            await client.patch("pods", "a", {"status": {"phase": "Running"}}, "default", sub="status")
            for _ in range(100):
                a = await client.get("pods", "a", "default")
                if a["metadata"]["annotations"][P.annotation_assigned] == "true":
                    break
                await asyncio.sleep(0.02)
            assert a["metadata"]["annotations"][P.annotation_assigned] == "true"
            assert plugin.debug_state()["grpc"]["patch_failures"] == 0  # no 409 from the moved resourceVersion
        finally:
            await _close(api_srv, client, plugin, pc)
    asyncio.run(go())


def test_early_answer_commit_retries_with_backoff_until_the_apiserver_recovers():
    """an answered Allocate's commit that hits 5xx is retried with capped backoff for as long as the pod
    exists (not 8 times in a few ms): an apiserver outage of a second still ends with ASSIGNED=true."""
    async def go():
        tmp = tempfile.mkdtemp()
        api_srv, client, plugin = await _plugin(tmp, fast=True)
        pc = PluginClient(plugin.socket_path)
        try:
            await client.create("pods", bound_pod("a", 4, dev=0, assume=1, dev_total=16))
            await asyncio.sleep(0.2)
            api_srv.server.faults.error_rate = 1.0  # every mutating pod call answers 500
            ids = fake_ids(plugin.devices[0], 16)
            await pc.allocate([ids[0:4]])
            await asyncio.sleep(1.0)
            st = plugin.debug_state()["grpc"]
            assert st["patch_failures"] >= 8 and st["early_answer_backlog"] == 1, st
            assert (await client.get("pods", "a", "default"))["metadata"]["annotations"][P.annotation_assigned] == "false"
            assert plugin.state.match(4) == (None, False)  # still claimed: never offered to another Allocate
            api_srv.server.faults.error_rate = 0.0
            for _ in range(200):
                a = await client.get("pods", "a", "default")
                if a["metadata"]["annotations"][P.annotation_assigned] == "true":
                    break
                await asyncio.sleep(0.02)
            assert a["metadata"]["annotations"][P.annotation_assigned] == "true"
            assert plugin.debug_state()["grpc"]["early_answer_backlog"] == 0
        finally:
            api_srv.server.faults.error_rate = 0.0
            await _close(api_srv, client, plugin, pc)
    asyncio.run(go())


def test_early_answer_commit_of_a_deleted_pod_releases_it_before_the_feed_does():
    """The pod was deleted while its early-answered commit was in flight, and the plugin's watch has not delivered
    the deletion yet: the commit's 404 releases the pod at once.  Unclaimed but still pending ASSIGNED=false in the
    state it would be the next Allocate's match -- kubelet has started its container and is admitting the next
    pod, which would get an allocation built for a deleted pod (seen on an 8-GPU rehearsal, profiles/r04_scale)."""
    async def go():
        tmp = tempfile.mkdtemp()
        api_srv, client, plugin = await _plugin(tmp, fast=True)
        pc = PluginClient(plugin.socket_path)
        try:
            await client.create("pods", bound_pod("a", 4, dev=0, assume=1, dev_total=16))
            await client.create("pods", bound_pod("b", 4, dev=0, assume=2, dev_total=16))
            await asyncio.sleep(0.3)
            api_srv.server.faults.latency_ms = 300.0  # the commit of "a" is in flight for 0.3 s
            ids = fake_ids(plugin.devices[0], 16)
            r = (await pc.allocate([ids[0:4]])).container_responses[0]
            assert dict(r.annotations)["gpushare.amd.com/pod"].split("/")[1] == "a"
            del api_srv.server.store["pods"][("default", "a")]  # gone, and no watch event says so
            for _ in range(100):
                if plugin.debug_state()["grpc"].get("commits_gone") == 1:
                    break
                await asyncio.sleep(0.02)
            assert plugin.debug_state()["grpc"]["commits_gone"] == 1
            api_srv.server.faults.latency_ms = 0.0
            r = (await pc.allocate([ids[4:8]])).container_responses[0]
            assert dict(r.annotations)["gpushare.amd.com/pod"].split("/")[1] == "b"
        finally:
            api_srv.server.faults.latency_ms = 0.0
            await _close(api_srv, client, plugin, pc)
    asyncio.run(go())


def test_early_answer_checkpoint_failure_keeps_the_journal_generation():
    """the journal is rotated (not truncated) with the records snapshot; a checkpoint that fails to land
    leaves the rotated generation in place, and a restarted plugin still finds the record.  ADVICE r5: a second
    failed checkpoint appends the next generation to .old after trimming its zero padding, so both records are
    recovered (a NUL run before the appended line made the loader skip it as torn)."""
    async def go():
        tmp = tempfile.mkdtemp()
        api_srv, client, plugin = await _plugin(tmp, fast=True)
        pc = PluginClient(plugin.socket_path)
        try:
            a = await client.create("pods", bound_pod("a", 4, dev=0, assume=1, dev_total=16))
            b = await client.create("pods", bound_pod("b", 4, dev=0, assume=2, dev_total=16))
            await client.create("pods", bound_pod("c", 4, dev=0, assume=3, dev_total=16))
            await asyncio.sleep(0.2)
            os.makedirs(plugin.checkpoint + ".tmp")  # the checkpoint write fails (a directory where its file goes)
            api_srv.server.faults.error_rate = 1.0  # and the commit never lands before the plugin goes away
            ids = fake_ids(plugin.devices[0], 16)
            await pc.allocate([ids[0:4]])
            for _ in range(100):  # the debounced checkpoint ran and failed
                if os.path.exists(plugin.journal_path + ".old"):
                    break
                await asyncio.sleep(0.02)
            with open(plugin.journal_path + ".old") as f:
                assert a["metadata"]["uid"] in f.read()
            assert not os.path.exists(plugin.checkpoint)
            await pc.allocate([ids[4:8]])  # b: a second generation, and a second checkpoint that fails
            for _ in range(200):
                with open(plugin.journal_path + ".old", "rb") as f:
                    raw = f.read()
                if b["metadata"]["uid"].encode() in raw:
                    break
                await asyncio.sleep(0.02)
            lines = [ln for ln in raw.rstrip(b"\x00").split(b"\n") if ln]
            assert len(lines) == 2 and all(ln.startswith(b"{") for ln in lines), raw[:400]
            assert not os.path.exists(plugin.checkpoint)
            await pc.close()
            pc = None
            await plugin.stop()
            os.rmdir(plugin.checkpoint + ".tmp")
            api_srv.server.faults.error_rate = 0.0
            os.environ["GSX_PLUGIN_EARLY_ANSWER"] = "0"  # restarted with the knob off: still lands the commit
            try:
                again = GpuSharePlugin(client, "n1", fake_devices("2x16GiB"), P, socket_dir=os.path.join(tmp, "dp"))
                await again.start(register=False)
            finally:
                os.environ.pop("GSX_PLUGIN_EARLY_ANSWER", None)
            plugin = again
            assert again.stats.get("commits_after_restart") == 2
            for n in ("a", "b"):
                assert (await client.get("pods", n, "default"))["metadata"]["annotations"][P.annotation_assigned] == "true"
            pc = PluginClient(again.socket_path)
            r = (await pc.allocate([ids[8:12]])).container_responses[0]
            assert dict(r.annotations)["gpushare.amd.com/pod"].split("/")[1] == "c"
            for _ in range(100):  # the first checkpoint supersedes both journal generations
                if os.path.exists(again.checkpoint) and not os.path.exists(again.journal_path + ".old"):
                    break
                await asyncio.sleep(0.02)
            with open(again.checkpoint) as f:
                assert len(json.load(f)["records"]) == 3
            assert not os.path.exists(again.journal_path + ".old")
        finally:
            api_srv.server.faults.error_rate = 0.0
            await _close(api_srv, client, plugin, *([pc] if pc else []))
    asyncio.run(go())


def test_missing_libnghttp2_falls_back_loudly():
    """without libnghttp2 the plugin serves kubelet from grpc.aio; it must say so -- a WARNING at
    startup and gpushare_plugin_native_endpoint 0 on /metrics (1 with the library)."""
    import subprocess
    import sys

    script = r'''
import asyncio, logging, os, sys, tempfile
sys.path.insert(0, os.getcwd())
from gpushare_scheduler_extender_amd.deviceplugin.devices import fake_devices
from gpushare_scheduler_extender_amd.deviceplugin.plugin import GpuSharePlugin
from gpushare_scheduler_extender_amd.k8s.client import KubeClient
from gpushare_scheduler_extender_amd.k8s.objects import make_node
from gpushare_scheduler_extender_amd.models.profile import SHARED_GPU
from tests.fixtures.fakeapi import FakeApiServerRunner
logging.basicConfig(level=logging.WARNING, stream=sys.stdout, format="%(levelname)s %(message)s")
async def go():
    tmp = tempfile.mkdtemp()
    api = await FakeApiServerRunner().start()
    c = KubeClient(api.url)
    await c.create("nodes", make_node("n1", 16, 0))
    p = GpuSharePlugin(c, "n1", fake_devices("1x16GiB"), SHARED_GPU, socket_dir=os.path.join(tmp, "dp"))
    await p.start(register=False)
    print("IMPL", p.grpc_impl)
    print([l for l in p.metrics_text().splitlines() if l.startswith("gpushare_plugin_native_endpoint ")][0])
    await p.stop(); await c.close(); await api.stop()
asyncio.run(go())
'''
    import pathlib

    root = str(pathlib.Path(__file__).resolve().parents[1])
    out = {}
    for hide in (True, False):
        env = dict(os.environ)
        env.pop("GSX_PLUGIN_GRPC", None)
        if hide:
            env["GSX_NGHTTP2_LIB"] = "/nonexistent/libnghttp2.so.14"
        r = subprocess.run([sys.executable, "-c", script], env=env, cwd=root, capture_output=True, text=True,
                           timeout=120)
        assert r.returncode == 0, r.stderr[-2000:]
        out[hide] = r.stdout
    assert "IMPL grpcio" in out[True] and "gpushare_plugin_native_endpoint 0" in out[True], out[True]
    assert "WARNING device-plugin endpoint on grpc.aio" in out[True] and "libnghttp2" in out[True], out[True]
    assert "IMPL native" in out[False] and "gpushare_plugin_native_endpoint 1" in out[False], out[False]


def test_plugin_process_sigkilled_between_answer_and_commit():
    """the plugin process (as deployed, ``python -m ...deviceplugin``) answers an Allocate early and
    is SIGKILLed before its ASSIGNED commit reaches a slow apiserver.  A new plugin process on the same socket
    directory lands the commit from its journal before it serves, the pod is never served to a second Allocate, and
    the other pending pod of that size is."""
    import signal
    import subprocess
    import sys

    async def go():
        tmp = tempfile.mkdtemp()
        api_srv = await FakeApiServerRunner().start()
        client = KubeClient(api_srv.url)
        await client.create("nodes", make_node("n1", 32, 0))
        spec = os.path.join(tmp, "devices.json")
        devs = fake_devices("2x16GiB")
        with open(spec, "w") as f:
            json.dump([{"index": d.index, "bdf": d.bdf, "uuid": d.uuid, "total_bytes": d.total_bytes,
                        "share_bytes": d.share_bytes, "cu_count": d.cu_count, "xcc_count": d.xcc_count}
                       for d in devs], f)
        sock_dir = os.path.join(tmp, "dp")
        env = dict(os.environ, GSX_FAKE_DEVICES=spec, GSX_PLUGIN_EARLY_ANSWER="1")

        async def start_plugin():
            p = subprocess.Popen([sys.executable, "-m", "gpushare_scheduler_extender_amd.deviceplugin", "--node", "n1",
                                  "--apiserver", api_srv.url, "--backend", "fake", "--socket-dir", sock_dir,
                                  "--no-register", "--no-publish", "--podresources-socket", "", "--isolation",
                                  "advisory", "--log-level", "warning"], env=env, cwd=os.getcwd())
            sock = os.path.join(sock_dir, "gpushare-amd.sock")
            for _ in range(600):
                if os.path.exists(sock):
                    try:
                        pc = PluginClient(sock)
                        await asyncio.wait_for(pc.options(), 1.0)
                        return p, pc
                    except Exception:  # noqa: BLE001 - not serving yet
                        await pc.close()
                await asyncio.sleep(0.05)
            raise TimeoutError("plugin never served")

        a = await client.create("pods", bound_pod("a", 4, dev=0, assume=1, dev_total=16))
        await client.create("pods", bound_pod("b", 4, dev=0, assume=2, dev_total=16))
        proc, pc = await start_plugin()
        try:
            await asyncio.sleep(0.3)
            # the commit cannot land before the kill: every pod write fails (a commit the dead plugin had already
            # sent may be read by the apiserver after the kill, so the writes keep failing until after the check)
            api_srv.server.faults.update({"error_rate": 1.0})
            ids = fake_ids(devs[0], 16)
            r = (await pc.allocate([ids[0:4]])).container_responses[0]
            assert dict(r.annotations)["gpushare.amd.com/pod"].split("/")[1] == "a"
            proc.send_signal(signal.SIGKILL)
            proc.wait(10)
            await pc.close()
            await asyncio.sleep(0.05)  # whatever the dead plugin had sent is read (and refused) now
            assert (await client.get("pods", "a", "default"))["metadata"]["annotations"][P.annotation_assigned] == "false"
            api_srv.server.faults.update({"error_rate": 0.0})
            proc, pc = await start_plugin()  # serves only after landing the journaled commit
            assert (await client.get("pods", "a", "default"))["metadata"]["annotations"][P.annotation_assigned] == "true"
            r = (await pc.allocate([ids[4:8]])).container_responses[0]
            assert dict(r.annotations)["gpushare.amd.com/pod"].split("/")[1] == "b"  # a is never served twice
            with pytest.raises(grpc.aio.AioRpcError):
                await pc.allocate([ids[8:12]])
        finally:
            api_srv.server.faults.update({"error_rate": 0.0})
            await pc.close()
            if proc.poll() is None:
                proc.terminate()
                proc.wait(10)
            await client.close()
            await api_srv.stop()
    asyncio.run(go())


@pytest.mark.parametrize("feed", ["1", "0"])
def test_native_endpoint_with_and_without_its_pod_feed(feed, monkeypatch):
    """GSX_PLUGIN_FEED=1 (default): the native reflector is the node's only pod watch and the Python views read the
    native state; 0: the Python informer feeds the state.  Either way an Allocate is answered on the fast path for
    the earliest pod of its size, and the views see the committed pod."""
    monkeypatch.setenv("GSX_PLUGIN_FEED", feed)

    async def go():
        tmp = tempfile.mkdtemp()
        api_srv, client, plugin = await _plugin(tmp, fast=True, spec="1x16GiB")
        pc = PluginClient(plugin.socket_path)
        try:
            assert plugin.state.native_views == (feed == "1")
            for i in range(3):
                await client.create("pods", bound_pod(f"f{i}", 4, dev=0, assume=i + 1, dev_total=16))
            ids = fake_ids(plugin.devices[0], 16)
            for _ in range(300):
                if len(plugin.state.candidates()) == 3:
                    break
                await asyncio.sleep(0.01)
            r = (await pc.allocate([ids[0:4]])).container_responses[0]
            assert dict(r.annotations)["gpushare.amd.com/pod"].split("/")[1] == "f0"
            for _ in range(300):
                rec = plugin.state.pods.get(next(u for u, p in plugin.state.pods.items() if p.name == "f0"))
                if rec is not None and rec.assigned == "true":
                    break
                await asyncio.sleep(0.01)
            assert rec.assigned == "true" and rec.obj["metadata"]["name"] == "f0"
            assert plugin.debug_state()["grpc"]["fast_allocate"] == 1
        finally:
            await _close(api_srv, client, plugin, pc)
    asyncio.run(go())
