"""C++ front end of the extender (native/engine/server.cc): HTTP edge cases, concurrency, unfiltered binds, proxied routes."""
import asyncio
import json
import socket
import threading

import pytest

from gpushare_scheduler_extender_amd.extender.server import ExtenderRunner, ExtenderServer
from gpushare_scheduler_extender_amd.k8s.client import KubeClient
from tests.fixtures.fakeapi import FakeApiServerRunner
from gpushare_scheduler_extender_amd.k8s.objects import make_node, make_pod
from gpushare_scheduler_extender_amd.models import wire


async def _stack():
    api = await FakeApiServerRunner().start()
    c = KubeClient(api.url)
    await c.create("nodes", make_node("n", 8 * 100, 8))
    ext = await ExtenderRunner(ExtenderServer(KubeClient(api.url)), http_threads=2).start()
    for _ in range(200):
        if ext.server.engine.has_node("n"):
            break
        await asyncio.sleep(0.01)
    return api, c, ext


async def _teardown(api, c, ext):
    await ext.stop()
    await ext.server.client.close()
    await c.close()
    await api.stop()


def _raw(port, payload: bytes, expect_responses: int) -> bytes:
    s = socket.create_connection(("127.0.0.1", port), timeout=5)
    s.sendall(payload)
    data = b""
    while data.count(b"HTTP/1.1 ") < expect_responses or not data.rstrip().endswith(b"}"):
        chunk = s.recv(65536)
        if not chunk:
            break
        data += chunk
    s.close()
    return data


def test_pipelined_and_chunked_requests():
    async def go():
        api, c, ext = await _stack()
        try:
            body = wire.filter_args(make_pod("p", 50), ["n"])
            one = (b"POST /gpushare-scheduler/filter HTTP/1.1\r\nHost: x\r\nContent-Length: %d\r\n\r\n" % len(body)) + body
            chunked = (b"POST /gpushare-scheduler/filter HTTP/1.1\r\nHost: x\r\nTransfer-Encoding: chunked\r\n\r\n" +
                       b"%x\r\n" % 10 + body[:10] + b"\r\n" + b"%x\r\n" % (len(body) - 10) + body[10:] + b"\r\n0\r\n\r\n")
            loop = asyncio.get_running_loop()
            data = await loop.run_in_executor(None, _raw, ext.port, one + chunked + one, 3)
            assert data.count(b'"NodeNames":["n"]') == 3
            # garbage request line -> 400 and close
            bad = await loop.run_in_executor(None, _raw, ext.port, b"NOPE\r\n\r\n", 1)
            assert bad.startswith(b"HTTP/1.1 400")
        finally:
            await _teardown(api, c, ext)
    asyncio.run(go())


def test_hostile_chunk_sizes_do_not_stop_the_server():
    """a chunk size that wraps ``body.size() + sz`` used to abort the extender process."""
    async def go():
        api, c, ext = await _stack()
        try:
            loop = asyncio.get_running_loop()
            head = b"POST /gpushare-scheduler/filter HTTP/1.1\r\nHost: x\r\nTransfer-Encoding: chunked\r\n\r\n"
            for tail in (b"5\r\nhello\r\nfffffffffffffffb\r\n", b"5\r\nhello\r\n-1\r\n", b"ffffffffffffffffffff\r\n"):
                r = await loop.run_in_executor(None, _raw, ext.port, head + tail, 1)
                assert r.startswith(b"HTTP/1.1 400"), r[:80]
            # the server is still up and answers a normal filter
            body = wire.filter_args(make_pod("p", 50), ["n"])
            one = (b"POST /gpushare-scheduler/filter HTTP/1.1\r\nHost: x\r\nContent-Length: %d\r\n\r\n" % len(body)) + body
            data = await loop.run_in_executor(None, _raw, ext.port, one, 1)
            assert b'"NodeNames":["n"]' in data
        finally:
            await _teardown(api, c, ext)
    asyncio.run(go())


def _trickle(port, payload: bytes, piece: int) -> bytes:
    s = socket.create_connection(("127.0.0.1", port), timeout=10)
    s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
    for i in range(0, len(payload), piece):
        s.sendall(payload[i:i + piece])
    data = b""
    while not data.rstrip().endswith(b"}"):
        chunk = s.recv(65536)
        if not chunk:
            break
        data += chunk
    s.close()
    return data


def test_trickled_chunked_filter_while_another_client_is_served():
    """A filter body sent as one-byte chunks in small writes is answered, and a normal client on the same loop is
    served meanwhile (the connection parser resumes instead of re-parsing the whole buffer on every read)."""
    async def go():
        api, c, ext = await _stack()
        try:
            loop = asyncio.get_running_loop()
            body = wire.filter_args(make_pod("p", 50), ["n"])
            framed = b"".join(b"1\r\n" + body[i:i + 1] + b"\r\n" for i in range(len(body))) + b"0\r\n\r\n"
            slow = (b"POST /gpushare-scheduler/filter HTTP/1.1\r\nHost: x\r\nTransfer-Encoding: chunked\r\n\r\n" +
                    framed)
            one = (b"POST /gpushare-scheduler/filter HTTP/1.1\r\nHost: x\r\nContent-Length: %d\r\n\r\n" % len(body)) + body
            slow_f = loop.run_in_executor(None, _trickle, ext.port, slow, 7)
            fast = await loop.run_in_executor(None, _raw, ext.port, one, 1)
            assert b'"NodeNames":["n"]' in fast
            assert b'"NodeNames":["n"]' in await slow_f
        finally:
            await _teardown(api, c, ext)
    asyncio.run(go())


def test_concurrent_filters_from_threads_and_stats():
    async def go():
        api, c, ext = await _stack()
        try:
            body = wire.filter_args(make_pod("p", 10), ["n", "ghost"])
            req = (b"POST /gpushare-scheduler/filter HTTP/1.1\r\nHost: x\r\nContent-Length: %d\r\n\r\n" % len(body)) + body
            errs = []

            def worker():
                try:
                    s = socket.create_connection(("127.0.0.1", ext.port), timeout=5)
                    for _ in range(50):
                        s.sendall(req)
                        data = b""
                        while not data.endswith(b'"Error":""}'):
                            data += s.recv(65536)
                        assert b'"NodeNames":["n"]' in data
                    s.close()
                except Exception as e:  # noqa: BLE001
                    errs.append(e)
            ts = [threading.Thread(target=worker) for _ in range(8)]
            loop = asyncio.get_running_loop()
            await loop.run_in_executor(None, lambda: ([t.start() for t in ts], [t.join() for t in ts]))
            assert not errs, errs
            st = ext.server.engine.server_stats()
            assert st["filters"] >= 400 and st["filter_latency"]["n"] >= 400
        finally:
            await _teardown(api, c, ext)
    asyncio.run(go())


def test_native_bind_fast_path_and_unfiltered_bind():
    async def go():
        api, c, ext = await _stack()
        try:
            import aiohttp

            eng = ext.server.engine
            p1 = await c.create("pods", make_pod("fast", 30))
            p2 = await c.create("pods", make_pod("slow", 20))
            for _ in range(200):
                if ext.server.controller.get_pod("slow", "default"):
                    break
                await asyncio.sleep(0.01)
            async with aiohttp.ClientSession() as s:
                # filter first: the pod is remembered natively, bind never touches Python
                async with s.post(ext.url + "/gpushare-scheduler/filter", data=wire.filter_args(p1, ["n"])) as r:
                    assert json.loads(await r.read())["NodeNames"] == ["n"]
                before = eng.server_stats()["proxied"]
                async with s.post(ext.url + "/gpushare-scheduler/bind", data=wire.ExtenderBindingArgs(
                        "fast", "default", p1["metadata"]["uid"], "n").encode()) as r:
                    assert r.status == 200 and json.loads(await r.read()) == {"Error": ""}
                assert eng.server_stats()["proxied"] == before
                # never filtered here -> the request comes from the controller's lister, still in C++
                async with s.post(ext.url + "/gpushare-scheduler/bind", data=wire.ExtenderBindingArgs(
                        "slow", "default", p2["metadata"]["uid"], "n").encode()) as r:
                    assert r.status == 200, await r.read()
                st = eng.server_stats()
                assert st["proxied"] == before and st["unfiltered_binds"] == 1 and st["live_gets"] == 0
                # non-native routes are served through the proxy
                async with s.get(ext.url + "/metrics") as r:
                    text = await r.text()
                    assert r.status == 200 and "gpushare_binpack_utilization" in text
                async with s.get(ext.url + "/healthz") as r:
                    assert r.status == 200
            fast = await c.get("pods", "fast", "default")
            slow = await c.get("pods", "slow", "default")
            assert fast["spec"]["nodeName"] == "n" and slow["spec"]["nodeName"] == "n"
            # best fit: both land on device 0 (30 + 20 <= 100)
            assert fast["metadata"]["annotations"]["SHARED_GPU_MEM_IDX"] == "0"
            assert slow["metadata"]["annotations"]["SHARED_GPU_MEM_IDX"] == "0"
            assert eng.node_devices("n")[0] == (100, 50)
            assert eng.server_stats()["bind_ok"] == 2
        finally:
            await _teardown(api, c, ext)
    asyncio.run(go())


def test_native_bind_failure_becomes_event():
    async def go():
        api, c, ext = await _stack()
        try:
            import aiohttp

            p = await c.create("pods", make_pod("huge", 500))
            async with aiohttp.ClientSession() as s:
                async with s.post(ext.url + "/gpushare-scheduler/filter", data=wire.filter_args(p, ["n"])) as r:
                    assert json.loads(await r.read())["FailedNodes"] == {"n": "Insufficient GPU Memory in one device"}
                async with s.post(ext.url + "/gpushare-scheduler/bind", data=wire.ExtenderBindingArgs(
                        "huge", "default", p["metadata"]["uid"], "n").encode()) as r:
                    assert r.status == 500
                    assert json.loads(await r.read())["Error"] == "The node n can't place the pod huge in ns default"
            for _ in range(100):
                evs = (await c.list("events", "default"))["items"]
                if evs:
                    break
                await asyncio.sleep(0.05)
            assert evs and evs[0]["reason"] == "FailedBinding" and evs[0]["type"] == "Warning"
        finally:
            await _teardown(api, c, ext)
    asyncio.run(go())


@pytest.mark.parametrize("filtered", [True, False], ids=["filtered", "unfiltered"])
def test_equal_size_binds_for_different_gpus_land_in_assume_order(filtered):
    """kubelet admits pods in binding order and the device plugin serves a request of N units with the
    earliest-ASSUME_TIME pod of that size: two equal-size pods bound to different GPUs of one node must
    commit in ASSUME_TIME order even when the first binding is slow; other binds do not wait."""
    async def go():
        import aiohttp

        api = await FakeApiServerRunner().start()
        c = KubeClient(api.url)
        await c.create("nodes", make_node("n", 2 * 16, 2))
        ext = await ExtenderRunner(ExtenderServer(KubeClient(api.url)), http_threads=2).start()
        try:
            pods = {}
            for name, mem in (("a", 10), ("b", 10), ("x", 6), ("y", 5)):
                pods[name] = await c.create("pods", make_pod(name, mem))
            for _ in range(300):
                if ext.server.engine.has_node("n") and ext.server.controller.get_pod("y", "default"):
                    break
                await asyncio.sleep(0.01)
            async with aiohttp.ClientSession() as s:
                async def bind(name):
                    p = pods[name]
                    if filtered:
                        async with s.post(ext.url + "/gpushare-scheduler/filter", data=wire.filter_args(p, ["n"])) as r:
                            assert json.loads(await r.read())["NodeNames"] == ["n"]
                    async with s.post(ext.url + "/gpushare-scheduler/bind", data=wire.ExtenderBindingArgs(
                            name, "default", p["metadata"]["uid"], "n").encode()) as r:
                        assert r.status == 200, await r.read()

                # a (10 GiB) -> GPU0, b (10 GiB) -> GPU1; a's binding takes 300 ms: b must wait for it
                api.server.faults.slow_bindings = {"a": 300.0, "x": 300.0}
                ta = asyncio.create_task(bind("a"))
                await asyncio.sleep(0.05)
                await asyncio.gather(ta, bind("b"))
                # x (6 GiB) -> GPU0, y (5 GiB) -> GPU1: different sizes, y does not wait for slow x
                tx = asyncio.create_task(bind("x"))
                await asyncio.sleep(0.05)
                await asyncio.gather(tx, bind("y"))
            assert api.server.binding_log == ["a", "b", "y", "x"]
            got = {n: (await c.get("pods", n, "default"))["metadata"]["annotations"] for n in pods}
            assert [got[n]["SHARED_GPU_MEM_IDX"] for n in ("a", "b", "x", "y")] == ["0", "1", "0", "1"]
            assert int(got["a"]["SHARED_GPU_MEM_ASSUME_TIME"]) < int(got["b"]["SHARED_GPU_MEM_ASSUME_TIME"])
            assert ext.server.engine.server_stats()["bind_order_waits"] == 1
        finally:
            await _teardown(api, c, ext)
    asyncio.run(go())


@pytest.mark.parametrize("filtered", [True, False], ids=["filtered", "unfiltered"])
def test_same_gpu_binds_with_different_cu_partitions_land_in_assume_order(filtered):
    """Equal-size pods for the same GPU are interchangeable for the device plugin unless their CU-partition
    requests differ (gpushare.amd.com/cu-count): then a swap would start one pod's container with the other's
    partition size, so they are ordered too. Equal-size, same-class pods still bind concurrently."""
    async def go():
        import aiohttp

        api = await FakeApiServerRunner().start()
        c = KubeClient(api.url)
        await c.create("nodes", make_node("n", 64, 1))
        ext = await ExtenderRunner(ExtenderServer(KubeClient(api.url)), http_threads=2).start()
        try:
            cu = {"gpushare.amd.com/cu-count": "64"}
            pods = {}
            for name, ann in (("c", cu), ("d", None), ("e", cu), ("f", cu)):
                pods[name] = await c.create("pods", make_pod(name, 8, annotations=ann))
            for _ in range(300):
                if ext.server.engine.has_node("n") and ext.server.controller.get_pod("f", "default"):
                    break
                await asyncio.sleep(0.01)
            async with aiohttp.ClientSession() as s:
                async def bind(name):
                    p = pods[name]
                    if filtered:
                        async with s.post(ext.url + "/gpushare-scheduler/filter", data=wire.filter_args(p, ["n"])) as r:
                            assert json.loads(await r.read())["NodeNames"] == ["n"]
                    async with s.post(ext.url + "/gpushare-scheduler/bind", data=wire.ExtenderBindingArgs(
                            name, "default", p["metadata"]["uid"], "n").encode()) as r:
                        assert r.status == 200, await r.read()

                api.server.faults.slow_bindings = {"c": 300.0, "e": 300.0}
                tc = asyncio.create_task(bind("c"))
                await asyncio.sleep(0.05)
                await asyncio.gather(tc, bind("d"))  # d has no partition request: waits for c
                te = asyncio.create_task(bind("e"))
                await asyncio.sleep(0.05)
                await asyncio.gather(te, bind("f"))  # f asks for the same partition size: does not wait
            assert api.server.binding_log == ["c", "d", "f", "e"]
            assert ext.server.engine.stats()["bind_order_waits"] == 1  # d
            async with aiohttp.ClientSession() as s:
                async with s.get(ext.url + "/metrics") as r:
                    assert "gpushare_bind_order_waits_total 1.0" in await r.text()
        finally:
            await _teardown(api, c, ext)
    asyncio.run(go())


def test_native_update_mode_annotates_then_binds_with_one_conflict_retry():
    """bind_mode="update" on the C++ front end: the reference's two calls (annotate, then a plain Binding,
    pkg/cache/nodeinfo.go:145-189). The annotation write is guarded by the resourceVersion the scheduler saw.
    On the optimistic-lock conflict it is retried once on the latest version."""
    async def go():
        import aiohttp

        api = await FakeApiServerRunner().start()
        c = KubeClient(api.url)
        await c.create("nodes", make_node("n", 2 * 16, 2))
        ext = await ExtenderRunner(ExtenderServer(KubeClient(api.url), bind_mode="update"),
                                   http_threads=2).start()
        try:
            pa = await c.create("pods", make_pod("a", 10))
            pb = await c.create("pods", make_pod("b", 10))
            for _ in range(300):
                if ext.server.engine.has_node("n") and ext.server.controller.get_pod("b", "default"):
                    break
                await asyncio.sleep(0.01)
            async with aiohttp.ClientSession() as s:
                async def bind(p):
                    async with s.post(ext.url + "/gpushare-scheduler/filter", data=wire.filter_args(p, ["n"])) as r:
                        assert json.loads(await r.read())["NodeNames"] == ["n"]
                    async with s.post(ext.url + "/gpushare-scheduler/bind", data=wire.ExtenderBindingArgs(
                            p["metadata"]["name"], "default", p["metadata"]["uid"], "n").encode()) as r:
                        assert r.status == 200, await r.read()

                before = ext.server.engine.server_stats()
                await bind(pa)
                # b changes after the scheduler saw it: its annotation write meets a conflict, retried once
                await c.patch("pods", "b", {"metadata": {"labels": {"touched": "1"}}}, "default")
                await bind(pb)
                after = ext.server.engine.server_stats()
            assert after["proxied"] == before["proxied"]  # both bound natively
            assert after["api_calls"] - before["api_calls"] == 5  # PATCH + POST, PATCH (409) + PATCH + POST
            assert after["conflicts_retried"] - before["conflicts_retried"] == 1
            for n, dev in (("a", "0"), ("b", "1")):
                got = await c.get("pods", n, "default")
                assert got["spec"]["nodeName"] == "n"
                ann = got["metadata"]["annotations"]
                assert ann["SHARED_GPU_MEM_IDX"] == dev and ann["SHARED_GPU_MEM_ASSIGNED"] == "false"
                assert ann["SHARED_GPU_MEM_POD"] == "10" and ann["SHARED_GPU_MEM_DEV"] == "16"
            assert (await c.get("pods", "b", "default"))["metadata"]["labels"]["touched"] == "1"
        finally:
            await _teardown(api, c, ext)
    asyncio.run(go())


def test_pprof_sees_native_threads():
    """/debug/pprof covers the C++ threads that serve filter / bind (names, native stacks, CPU
    time, verb latency histograms, ledger mutex profile), not only the Python loop."""
    async def go():
        api, c, ext = await _stack()
        stop = threading.Event()
        body = wire.filter_args(make_pod("p", 50), ["n"])
        req = (b"POST /gpushare-scheduler/filter HTTP/1.1\r\nHost: x\r\nContent-Length: %d\r\n\r\n" % len(body)) + body

        def storm():
            s = socket.create_connection(("127.0.0.1", ext.port), timeout=5)
            while not stop.is_set():
                s.sendall(req)
                buf = b""
                while not buf.endswith(b"}"):
                    buf += s.recv(65536)
            s.close()
        ts = [threading.Thread(target=storm, daemon=True) for _ in range(3)]
        for t in ts:
            t.start()
        try:
            from aiohttp import ClientSession

            async with ClientSession() as http:
                async with http.get(ext.url + "/debug/pprof/goroutine/") as r:
                    g = await r.text()
                async with http.get(ext.url + "/debug/pprof/profile?seconds=1&hz=200") as r:
                    prof = await r.text()
                async with http.get(ext.url + "/debug/pprof/mutex") as r:
                    mtx = await r.text()
                async with http.get(ext.url + "/debug/pprof/threadcreate/") as r:
                    tc = await r.text()
        finally:
            stop.set()
            for t in ts:
                t.join(5)
            await _teardown(api, c, ext)
        # thread names and symbolised native stacks of the epoll loops, bind pool and reflectors
        for name in ("gsx-http-0", "gsx-bind-0", "gsx-refl-pods", "gsx-refl-nodes"):
            assert f"[{name}] native" in g, name
        assert "NativeServer::run_loop" in g and "Reflector::run" in g
        # on-CPU profile of the whole process: native frames of the filter path, per-thread CPU, histograms
        assert "# native filter_latency: n=" in prof and "# ledger mutex: acquisitions=" in prof
        assert any(ln.startswith("#   gsx-http") for ln in prof.splitlines())
        stacks = [ln for ln in prof.splitlines() if ln.startswith("gsx-http")]
        assert stacks and any("NativeServer" in ln for ln in stacks)
        assert "acquisitions=" in mtx and "native" in tc
    asyncio.run(go())


def test_bind_order_spans_filtered_and_unfiltered_binds():
    """one in-flight set for every bind.  a is filtered here and has a slow binding; b, equal-size for
    the other GPU, was never filtered by this process (e.g. a restart between filter and bind) and must still
    commit after a."""
    async def go():
        import aiohttp

        api = await FakeApiServerRunner().start()
        c = KubeClient(api.url)
        await c.create("nodes", make_node("n", 2 * 16, 2))
        ext = await ExtenderRunner(ExtenderServer(KubeClient(api.url)), http_threads=2).start()
        try:
            pa = await c.create("pods", make_pod("a", 10))
            pb = await c.create("pods", make_pod("b", 10))
            for _ in range(300):
                if ext.server.engine.has_node("n") and ext.server.controller.get_pod("b", "default"):
                    break
                await asyncio.sleep(0.01)
            async with aiohttp.ClientSession() as s:
                async with s.post(ext.url + "/gpushare-scheduler/filter", data=wire.filter_args(pa, ["n"])) as r:
                    assert json.loads(await r.read())["NodeNames"] == ["n"]

                async def bind(p):
                    async with s.post(ext.url + "/gpushare-scheduler/bind", data=wire.ExtenderBindingArgs(
                            p["metadata"]["name"], "default", p["metadata"]["uid"], "n").encode()) as r:
                        assert r.status == 200, await r.read()

                api.server.faults.slow_bindings = {"a": 300.0}
                ta = asyncio.create_task(bind(pa))
                await asyncio.sleep(0.05)
                await asyncio.gather(ta, bind(pb))
                assert ext.server.engine.server_stats()["unfiltered_binds"] == 1  # b
            assert api.server.binding_log == ["a", "b"]
            got = {n: (await c.get("pods", n, "default"))["metadata"]["annotations"] for n in ("a", "b")}
            assert [got[n]["SHARED_GPU_MEM_IDX"] for n in ("a", "b")] == ["0", "1"]
            assert int(got["a"]["SHARED_GPU_MEM_ASSUME_TIME"]) < int(got["b"]["SHARED_GPU_MEM_ASSUME_TIME"])
        finally:
            await _teardown(api, c, ext)
    asyncio.run(go())


@pytest.mark.parametrize("order,landing,want", [("auto", True, ["b", "a"]), ("auto", False, ["a", "b"]),
                                                ("strict", True, ["a", "b"]), ("relaxed", False, ["b", "a"])])
def test_bind_order_follows_the_nodes_allocate_order(order, landing, want):
    """``--bind-order auto`` (default): equal-size binds for different GPUs of a node wait for each other (ASSUME_TIME
    order, for a plugin that matches by ASSUME_TIME) unless the node's device plugin advertises landing-order
    matching (``gpushare.amd.com/allocate-order=landing``, native/engine/allocstate.h): then b, bound while a's
    binding is slow, lands first.  ``strict`` orders every node, ``relaxed`` none."""
    async def go():
        import aiohttp

        from gpushare_scheduler_extender_amd.models.profile import NODE_ALLOCATE_ORDER_ANNOTATION

        api = await FakeApiServerRunner().start()
        c = KubeClient(api.url)
        node = make_node("n", 2 * 16, 2)
        if landing:
            node["metadata"].setdefault("annotations", {})[NODE_ALLOCATE_ORDER_ANNOTATION] = "landing"
        await c.create("nodes", node)
        ext = await ExtenderRunner(ExtenderServer(KubeClient(api.url), bind_order=order),
                                   http_threads=2).start()
        try:
            pa = await c.create("pods", make_pod("a", 10))
            pb = await c.create("pods", make_pod("b", 10))
            for _ in range(300):
                if ext.server.engine.has_node("n") and ext.server.controller.get_pod("b", "default"):
                    break
                await asyncio.sleep(0.01)
            async with aiohttp.ClientSession() as s:
                for p in (pa, pb):
                    async with s.post(ext.url + "/gpushare-scheduler/filter", data=wire.filter_args(p, ["n"])) as r:
                        assert json.loads(await r.read())["NodeNames"] == ["n"]

                async def bind(p):
                    async with s.post(ext.url + "/gpushare-scheduler/bind", data=wire.ExtenderBindingArgs(
                            p["metadata"]["name"], "default", p["metadata"]["uid"], "n").encode()) as r:
                        assert r.status == 200, await r.read()

                api.server.faults.slow_bindings = {"a": 300.0}
                ta = asyncio.create_task(bind(pa))
                await asyncio.sleep(0.05)
                await asyncio.gather(ta, bind(pb))
            assert api.server.binding_log == want
            got = {n: (await c.get("pods", n, "default"))["metadata"]["annotations"] for n in ("a", "b")}
            assert [got[n]["SHARED_GPU_MEM_IDX"] for n in ("a", "b")] == ["0", "1"]
            assert ext.server.engine.bind_order == order
        finally:
            await _teardown(api, c, ext)
    asyncio.run(go())


def test_move_endpoint_is_the_one_writer_of_the_gpu_index():
    """the device plugin's allocation-record moves go through POST /gpushare-scheduler/move.  Under
    the ledger mutex the extender checks the move (pod where the caller thinks, room on the target unless an
    equal-size partner makes it an exchange), charges the target until its informer shows the pod there, and writes
    *_IDX with a resourceVersion precondition."""
    from gpushare_scheduler_extender_amd.k8s.fasthttp import Client as HttpClient
    from gpushare_scheduler_extender_amd.models.profile import SHARED_GPU as P

    async def go():
        api = await FakeApiServerRunner().start()
        c = KubeClient(api.url)
        await c.create("nodes", make_node("n", 2 * 100, 2))
        ext = await ExtenderRunner(ExtenderServer(KubeClient(api.url)), http_threads=2).start()
        eng = ext.server.engine
        http = HttpClient(f"http://127.0.0.1:{ext.port}")

        def bound(name, mem, dev):
            ann = {P.annotation_idx: str(dev), P.annotation_pod: str(mem), P.annotation_dev: "100",
                   P.annotation_assigned: "false", P.annotation_assume_time: "1"}
            return make_pod(name, mem, node="n", annotations=ann)

        async def move(pod, to, frm=None, partner="", annotations=None):
            md = pod["metadata"]
            body = {"namespace": "default", "name": md["name"], "uid": md["uid"], "node": "n",
                    "resourceVersion": md["resourceVersion"], "from": frm if frm is not None else int(
                        md["annotations"][P.annotation_idx]), "to": to, "partner": partner,
                    "annotations": annotations or {}}
            # the extender refuses a move while the pod's previous one is in flight (until its watch event lands in
            # the ledger); the plugin's reconciliation retries on its next pass, this waits for it
            for _ in range(200):
                r = await http.request("POST", "/gpushare-scheduler/move", json.dumps(body).encode())
                out = json.loads(r.body)
                if r.status != 409 or "in flight" not in out.get("Error", ""):
                    break
                await asyncio.sleep(0.01)
            return r.status, out

        async def settle(want):
            for _ in range(200):
                if eng.node_devices("n") == want:
                    return
                await asyncio.sleep(0.01)
            assert eng.node_devices("n") == want

        try:
            for _ in range(200):
                if eng.has_node("n"):
                    break
                await asyncio.sleep(0.01)
            a = await c.create("pods", bound("a", 60, 0))
            b = await c.create("pods", bound("b", 60, 1))
            q = await c.create("pods", bound("q", 30, 0))
            await settle([(100, 90), (100, 60)])
            # no room: GPU 1 has 40 free, a needs 60
            st, out = await move(a, 1)
            assert st == 409 and "free" in out["Error"], out
            # stale view: a is on GPU 0, not 1
            st, out = await move(a, 0, frm=1)
            assert st == 409 and "stale" in out["Error"], out
            # a partner claim the ledger cannot verify (no hold on a's old GPU naming b) earns no credit
            st, out = await move(a, 1, partner=b["metadata"]["uid"], annotations={P.annotation_assigned: "true"})
            assert st == 409 and "free" in out["Error"], out
            assert eng.stats()["partner_claims_refused"] >= 1
            # an exchange step with a partner on the target: a holds its old GPU and names b as the hold's partner,
            # so b's share is credited on GPU 1 (b leaves it in step 2): allowed
            hp = json.dumps({"uid": b["metadata"]["uid"], "key": "default/b", "idx": 0, "assigned": "false",
                             "cu_mask": None})
            st, out = await move(a, 1, partner=b["metadata"]["uid"],
                                 annotations={"gpushare.amd.com/hold-idx": "0", "gpushare.amd.com/hold-partner": hp,
                                              P.annotation_assigned: "true"})
            assert st == 200, out
            ann = out["pod"]["metadata"]["annotations"]
            assert ann[P.annotation_idx] == "1" and ann["gpushare.amd.com/hold-idx"] == "0"
            assert ann[P.annotation_assigned] == "true"
            b = await c.get("pods", "b", "default")
            st, out = await move(b, 0, partner=a["metadata"]["uid"])  # step 2: b takes a's old GPU (a holds it)
            assert st == 200, out
            a = await c.get("pods", "a", "default")
            st, out = await move(a, 1, annotations={"gpushare.amd.com/hold-idx": None,
                                                    "gpushare.amd.com/hold-partner": None})  # step 3: the hold goes
            assert st == 200 and "gpushare.amd.com/hold-idx" not in out["pod"]["metadata"]["annotations"], out
            await settle([(100, 90), (100, 60)])
            # a plain move with room: best fit picked by the extender (to = -1), the target charged at once
            q = await c.get("pods", "q", "default")
            st, out = await move(q, -1)
            assert st == 200 and out["to"] == 1, out
            await settle([(100, 60), (100, 90)])
            # the resourceVersion precondition: a stale copy of q conflicts (and its reservation is rolled back)
            st, out = await move(q, 0, frm=1)
            assert st == 409, out
            await settle([(100, 60), (100, 90)])
            # *_IDX (and the pod's share) are never written through the annotations map
            q = await c.get("pods", "q", "default")
            st, out = await move(q, 1, annotations={P.annotation_idx: "0"})
            assert st == 400, out
            # ... and nothing outside the allocation fields a move rewrites (no arbitrary annotation writes)
            st, out = await move(q, 1, annotations={"example.com/owner": "x"})
            assert st == 400 and "writes only" in out["Error"], out
            assert eng.stats()["moves_ok"] == 4 and eng.stats()["moves_refused"] >= 2
            # an exchange of two sizes is checked on the final state: c (20, GPU 0) and q (30, GPU 1);
            # GPU 0 holds a 60 + c 20 = 80, GPU 1 holds b 60 + q 30 = 90.  q -> GPU 0 alone needs 30 (20 free) ...
            cpod = await c.create("pods", bound("c", 20, 0))
            await settle([(100, 80), (100, 90)])
            q = await c.get("pods", "q", "default")
            st, out = await move(q, 0)
            assert st == 409, out
            # ... as an exchange with c (c leaves GPU 0 for GPU 1): GPU 0 ends at 90, GPU 1 at 80 -- allowed
            hp = json.dumps({"uid": cpod["metadata"]["uid"], "key": "default/c", "idx": 1, "assigned": "false",
                             "cu_mask": None})
            st, out = await move(q, 0, partner=cpod["metadata"]["uid"],
                                 annotations={"gpushare.amd.com/hold-idx": "1", "gpushare.amd.com/hold-partner": hp})
            assert st == 200, out
            cpod = await c.get("pods", "c", "default")
            st, out = await move(cpod, 1, partner=q["metadata"]["uid"])  # step 2, verified by q's hold
            assert st == 200, out
            q = await c.get("pods", "q", "default")
            st, out = await move(q, 0, annotations={"gpushare.amd.com/hold-idx": None,
                                                    "gpushare.amd.com/hold-partner": None})
            assert st == 200, out
            await settle([(100, 90), (100, 80)])
        finally:
            await http.close()
            await ext.stop()
            await ext.server.client.close()
            await c.close()
            await api.stop()
    asyncio.run(go())


def test_unfiltered_bind_errors_match_the_reference_and_qps_limits_native_binds():
    """Binds the filter never saw are decided in C++ too (the Python bind path is gone): Go's decoder error for
    a mistyped field, the reference's UID error after one live GET (gpushare-bind.go:44-65), and a client-side
    QPS limit (--kube-qps) paces the front end's apiserver calls."""
    async def go():
        import time

        import aiohttp

        api = await FakeApiServerRunner().start()
        c = KubeClient(api.url)
        await c.create("nodes", make_node("n", 8 * 100, 8))
        ext = await ExtenderRunner(ExtenderServer(KubeClient(api.url, qps=20, burst=1)), http_threads=2).start()
        try:
            pods = [await c.create("pods", make_pod(f"q{i}", 10)) for i in range(6)]
            for _ in range(300):
                if ext.server.engine.has_node("n") and ext.server.controller.get_pod("q5", "default"):
                    break
                await asyncio.sleep(0.01)
            url = ext.url + "/gpushare-scheduler/bind"
            async with aiohttp.ClientSession() as s:
                async with s.post(url, data=b'{"PodName":"q0","PodNamespace":"default","PodUID":7,"Node":"n"}') as r:
                    assert r.status == 500
                    assert json.loads(await r.read())["Error"] == (
                        "json: cannot unmarshal number into Go struct field ExtenderBindingArgs.PodUID of type string")
                async with s.post(url, data=wire.ExtenderBindingArgs("q0", "default", "not-its-uid", "n").encode()) as r:
                    assert r.status == 500
                    assert json.loads(await r.read())["Error"] == (
                        f"The pod q0 in ns default's uid is {pods[0]['metadata']['uid']}, and it's not equal with "
                        "expected not-its-uid")
                async with s.post(url, data=wire.ExtenderBindingArgs("gone", "default", "u", "n").encode()) as r:
                    assert r.status == 500 and "not found" in json.loads(await r.read())["Error"]

                async def bind(p):
                    async with s.post(url, data=wire.ExtenderBindingArgs(
                            p["metadata"]["name"], "default", p["metadata"]["uid"], "n").encode()) as r:
                        assert r.status == 200, await r.read()
                t0 = time.monotonic()
                await asyncio.gather(*(bind(p) for p in pods))
                dt = time.monotonic() - t0
            st = ext.server.engine.server_stats()
            assert st["unfiltered_binds"] == 8 and st["live_gets"] == 2 and st["bind_ok"] == 6
            assert st["qps_waits"] >= 5 and dt >= 0.2, (st, dt)  # 6 bindings at 20 qps, burst 1
        finally:
            await _teardown(api, c, ext)
    asyncio.run(go())


def test_plugin_endpoints_take_only_the_plugin_token_and_the_physical_floor_steers_binds():
    """the device plugin's endpoints (/move, /physical) write allocation records with the extender's
    rights, so with ``plugin_auth="tokenreview"`` only a bearer token the apiserver's TokenReview authenticates as
    the plugin's service account gets in (401 without one, 403 for another user; a reviewed token is cached).  The
    unaccounted use the plugin publishes (containers on a device whose pods the annotations put elsewhere) is
    charged on top of the annotations: a device those containers fill takes no bind while the annotations still
    show room."""
    from gsxtools.cluster import start_apiserver
    from gpushare_scheduler_extender_amd.k8s.fasthttp import Client as HttpClient

    plugin_user = "system:serviceaccount:kube-system:gpushare-device-plugin"

    async def go():
        api = start_apiserver()
        c = KubeClient(api.url)
        fa = HttpClient(api.url)
        for tok, user, node in (("tok-plugin", plugin_user, None), ("tok-other", "system:serviceaccount:default:app", None),
                                ("tok-node-m", plugin_user, "m"), ("tok-node-n", plugin_user, "n")):
            await fa.request("POST", "/fake/tokens", json.dumps({"token": tok, "user": user, "node": node}).encode())
        await c.create("nodes", make_node("n", 2 * 100, 2))
        ext = await ExtenderRunner(ExtenderServer(KubeClient(api.url)), plugin_auth="tokenreview",
                                   plugin_users=[plugin_user]).start()
        eng = ext.server.engine
        http = HttpClient(f"http://127.0.0.1:{ext.port}")

        async def physical(used, tok=None):
            h = {"Authorization": f"Bearer {tok}"} if tok else None
            r = await http.request("POST", "/gpushare-scheduler/physical",
                                   json.dumps({"node": "n", "unaccounted": used, "ttl": 30}).encode(), headers=h)
            return r.status

        try:
            for _ in range(200):
                if eng.has_node("n"):
                    break
                await asyncio.sleep(0.01)
            assert await physical([100, 0]) == 401
            assert await physical([100, 0], "tok-other") == 403
            assert await physical([100, 0], "nobody") == 401
            r = await http.request("POST", "/gpushare-scheduler/move", b"{}", headers={"Authorization": "Bearer x"})
            assert r.status == 401
            assert await physical([100, 0], "tok-plugin") == 200
            assert await physical([100, 0], "tok-plugin") == 200
            srv = json.loads((await http.request("GET", "/debug/engine")).body)["server"]
            assert srv["plugin_auth_denied"] == 4 and srv["token_reviews"] == 4  # the plugin's token reviewed once
            # a denial is cached too: the same bad token again costs the apiserver no review
            assert await physical([100, 0], "tok-other") == 403
            # a token bound to a node (its pod's node-name claim) writes that node's records only
            assert await physical([100, 0], "tok-node-m") == 403
            assert await physical([100, 0], "tok-node-n") == 200
            srv = json.loads((await http.request("GET", "/debug/engine")).body)["server"]
            assert srv["token_reviews"] == 6 and srv["plugin_auth_denied"] == 6, srv
            # made-up tokens: the reviews the cache cannot answer are rate limited (20 a second, bursts of 40)
            codes = [await physical([100, 0], f"junk-{i}") for i in range(80)]
            assert codes.count(401) <= 45 and 429 in codes, codes
            assert await physical([100, 0], "tok-plugin") == 200  # a cached good token is not limited
            assert eng.node_unaccounted("n") == [100, 0]
            metrics = (await http.request("GET", "/metrics")).body.decode()
            assert 'gpushare_device_unaccounted_gpu_mem{device="0",node="n"} 100.0' in metrics, metrics[-2000:]
            # GPU 0's containers fill it (the annotations say empty): the bind goes to GPU 1, and after it a
            # 95-unit pod fits nowhere
            assert eng.assume("u1", "default", "p1", "n", 10)[0] == 1
            assert eng.assume("u2", "default", "p2", "n", 95)[0] < 0
            # withdrawn: the annotations alone again -- GPU 0 takes it
            assert await physical(None, "tok-plugin") == 200
            assert eng.node_unaccounted("n") == []
            assert eng.assume("u3", "default", "p3", "n", 95)[0] == 0
        finally:
            await http.close()
            await fa.close()
            await ext.stop()
            await ext.server.client.close()
            await c.close()
            api.stop()
    asyncio.run(go())


def test_published_unaccounted_use_expires_unless_refreshed():
    """A plugin that stops refreshing its publication (it died) cannot pin a device: the charge lapses after its
    ttl (Ledger::gc), and a refresh before that keeps it."""
    from gpushare_scheduler_extender_amd.k8s.fasthttp import Client as HttpClient

    async def go():
        api = await FakeApiServerRunner().start()
        c = KubeClient(api.url)
        await c.create("nodes", make_node("n", 2 * 100, 2))
        ext = await ExtenderRunner(ExtenderServer(KubeClient(api.url))).start()
        eng = ext.server.engine
        http = HttpClient(f"http://127.0.0.1:{ext.port}")

        async def physical(used, ttl):
            r = await http.request("POST", "/gpushare-scheduler/physical",
                                   json.dumps({"node": "n", "unaccounted": used, "ttl": ttl}).encode())
            return r.status

        try:
            for _ in range(200):
                if eng.has_node("n"):
                    break
                await asyncio.sleep(0.01)
            assert await physical([100, 0], 0.3) == 200
            eng.gc()
            assert eng.node_unaccounted("n") == [100, 0]  # within its ttl
            assert eng.assume("u1", "default", "p1", "n", 95)[0] == 1
            await asyncio.sleep(0.2)
            assert await physical([100, 0], 0.3) == 200  # refreshed: a fresh ttl
            await asyncio.sleep(0.2)
            eng.gc()
            assert eng.node_unaccounted("n") == [100, 0]
            await asyncio.sleep(0.25)
            eng.gc()
            assert eng.node_unaccounted("n") == []  # lapsed
            assert eng.stats()["unaccounted_expired"] == 1
            assert eng.assume("u2", "default", "p2", "n", 95)[0] == 0  # GPU 0 takes binds again
        finally:
            await http.close()
            await ext.stop()
            await ext.server.client.close()
            await c.close()
            await api.stop()
    asyncio.run(go())
