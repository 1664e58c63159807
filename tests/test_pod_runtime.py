"""Native per-GPU pod runtime (native/engine/podruntime.cc).

CPU part: slice accounting (2 MiB aligned first fit, arena exhaustion, release,
idempotent admit) through the HTTP endpoint the node agent uses.  GPU part
(``-m gpu``): the request path launches the HIP admission (stamp the new slice,
verify every resident slice) on a real MI355X, and a slice overwritten behind
the runtime's back is reported as bad stamps.
"""
import json
import urllib.request

import pytest

from gpushare_scheduler_extender_amd.core.engine import native

MiB = 1 << 20


def _req(url, method, body=None):
    r = urllib.request.Request(url, data=json.dumps(body).encode() if body is not None else None, method=method)
    try:
        with urllib.request.urlopen(r) as resp:
            return resp.status, resp.read()
    except urllib.error.HTTPError as e:
        return e.code, e.read()


def test_pod_runtime_accounting_over_http():
    rt = native().PodRuntime(0, 64 * MiB)
    url = f"http://127.0.0.1:{rt.serve('127.0.0.1', 0)}"
    try:
        assert _req(url + "/v1/pods/a", "POST", {"dev": 0, "bytes": 10 * MiB, "verify": True}) == (200, b'{"bad":0}')
        assert _req(url + "/v1/pods/b", "POST", {"dev": 0, "bytes": 30 * MiB})[0] == 200  # 12 MiB aligned + 30
        assert _req(url + "/v1/pods/a", "POST", {"dev": 0, "bytes": 10 * MiB})[0] == 200  # idempotent
        st, body = _req(url + "/v1/pods/c", "POST", {"dev": 0, "bytes": 30 * MiB})
        assert st == 409 and b"arena exhausted" in body
        assert _req(url + "/v1/pods/a", "DELETE")[0] == 200
        assert _req(url + "/v1/pods/a", "DELETE")[0] == 404
        # the freed 10 MiB hole (aligned to 10 MiB) is reused first-fit
        assert _req(url + "/v1/pods/d", "POST", {"dev": 0, "bytes": 8 * MiB})[0] == 200
        st = json.loads(_req(url + "/v1/stats", "GET")[1])
        assert st["admitted"] == 3 and st["failed"] == 1 and st["resident"] == 2
        s = rt.stats()
        assert s["resident_bytes"] == (8 + 30) * MiB
        assert _req(url + "/v1/pods/e", "POST", {"dev": 0, "bytes": 0})[0] == 400
    finally:
        rt.stop()


@pytest.mark.gpu
def test_pod_runtime_hip_admission_detects_overlap():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.fail("gpu tests need a GPU")
    from gpushare_scheduler_extender_amd.ops import hip

    arena = 1 << 30
    buf = hip.DeviceBuffer(0, arena)
    s = hip.Stream(0)
    rt = native().PodRuntime(0, arena, buf.addr(0), s.ptr, 1 << 16, hip.lib()._name)
    url = f"http://127.0.0.1:{rt.serve('127.0.0.1', 0)}"
    try:
        for uid in ("p0", "p1", "p2"):
            st, body = _req(url + f"/v1/pods/{uid}", "POST", {"dev": 0, "bytes": 256 * MiB, "verify": True})
            assert (st, json.loads(body)["bad"]) == (200, 0)
        assert rt.verify() == 0
        # something writes into p1's slice (offset 256 MiB) behind the runtime's back
        hip.hbm_fill(s, buf.addr(256 * MiB), 4 * MiB, 0)
        s.sync()
        assert rt.verify() == 4 * MiB // (1 << 16)
        # an idempotent re-admission of p1 (kubelet retrying) re-verifies its own slice and reports the damage
        st, body = _req(url + "/v1/pods/p1", "POST", {"dev": 0, "bytes": 256 * MiB, "verify": False})
        assert st == 200 and json.loads(body)["bad"] == 64
        # a new admission verifies every resident slice and reports the damage
        st, body = _req(url + "/v1/pods/p3", "POST", {"dev": 0, "bytes": 128 * MiB, "verify": True})
        assert st == 200 and json.loads(body)["bad"] == 64
        assert rt.release("p1")
        assert rt.verify() == 0
        assert rt.admit("p4", 200 * MiB, True) == 0  # reuses p1's hole, restamped
        assert rt.stats()["resident"] == 4
    finally:
        rt.stop()
        s.sync()
        s.destroy()
        buf.free()


def _concurrent_admit(url, n, size):
    import threading

    go = threading.Barrier(n)
    out = {}

    def one(i):
        go.wait()
        out[i] = _req(url + f"/v1/pods/c{i}", "POST", {"dev": 0, "bytes": size, "verify": True})

    ts = [threading.Thread(target=one, args=(i,)) for i in range(n)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(60)
    return out


def test_pod_runtime_concurrent_admissions_group_commit():
    """Admissions arriving together are carved and admitted as one group; every one gets its own slice."""
    rt = native().PodRuntime(0, 64 * 4 * MiB)
    url = f"http://127.0.0.1:{rt.serve('127.0.0.1', 0)}"
    try:
        out = _concurrent_admit(url, 16, 4 * MiB)
        assert all(v == (200, b'{"bad":0}') for v in out.values()), out
        st = json.loads(_req(url + "/v1/stats", "GET")[1])
        assert st["admitted"] == 16 and st["resident"] == 16 and st["failed"] == 0
        assert rt.stats()["resident_bytes"] == 16 * 4 * MiB
        # the arena is full now: one more fails, the others are untouched
        assert _req(url + "/v1/pods/x", "POST", {"dev": 0, "bytes": 200 * MiB})[0] == 409
    finally:
        rt.stop()


@pytest.mark.gpu
def test_pod_runtime_concurrent_admissions_on_gpu():
    """16 concurrent admissions on the MI355X: grouped into fewer GPU calls, no bad stamp, all verified."""
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.fail("gpu tests need a GPU")
    from gpushare_scheduler_extender_amd.ops import hip

    arena = 1 << 30
    buf = hip.DeviceBuffer(0, arena)
    s = hip.Stream(0)
    rt = native().PodRuntime(0, arena, buf.addr(0), s.ptr, 1 << 16, hip.lib()._name)
    url = f"http://127.0.0.1:{rt.serve('127.0.0.1', 0)}"
    try:
        out = _concurrent_admit(url, 16, 32 * MiB)
        assert all(st == 200 and json.loads(body)["bad"] == 0 for st, body in out.values()), out
        st = json.loads(_req(url + "/v1/stats", "GET")[1])
        assert st["admitted"] == 16 and st["resident"] == 16
        assert 1 <= st["batches"] <= 16
        assert rt.verify() == 0
        # damage one slice: the next group reports it
        hip.hbm_fill(s, buf.addr(0), 1 * MiB, 0)
        s.sync()
        assert rt.verify() == MiB // (1 << 16)
    finally:
        rt.stop()
        s.sync()
        s.destroy()
        buf.free()


def test_runtime_endpoint_reaps_closed_connection_threads():
    """Each connection gets a thread; once it closes, that thread is joined.  An unjoined thread keeps its stack
    mapped (8 MiB each), so 300 short-lived connections would grow the process's address space by ~2.4 GiB."""

    def vm_size_mib():
        with open("/proc/self/status") as f:
            for ln in f:
                if ln.startswith("VmSize:"):
                    return int(ln.split()[1]) / 1024
        return 0.0

    rt = native().PodRuntime(0, 64 * MiB)
    url = f"http://127.0.0.1:{rt.serve('127.0.0.1', 0)}"
    try:
        for _ in range(20):
            _req(url + "/v1/stats", "GET")
        base = vm_size_mib()
        for _ in range(300):  # urllib closes each connection after the response
            assert _req(url + "/v1/stats", "GET")[0] == 200
        grown = vm_size_mib() - base
        assert grown < 256, f"address space grew {grown:.0f} MiB over 300 connections"
    finally:
        rt.stop()
