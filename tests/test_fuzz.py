"""Property-based robustness of the extender's native edges (hypothesis).

The extender sits on hostNetwork / NodePort 32766 and its policy is ``ignorable: false``: a request that crashes
it stops GPU-share scheduling for the cluster. These tests feed the native JSON parser (the filter verb, the
bind decoder) and the HTTP front end with generated input. They check three things: every answer is
well-formed, the Go-compatible error contract holds, and the process keeps serving.
"""
import asyncio
import json
import socket

from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from gpushare_scheduler_extender_amd.core.engine import new_engine
from gpushare_scheduler_extender_amd.k8s.objects import make_node, make_pod
from gpushare_scheduler_extender_amd.models import wire

ENGINE = new_engine()
ENGINE.upsert_node_json(json.dumps(make_node("n", 4 * 64, 4)).encode())

json_leaf = st.one_of(st.none(), st.booleans(), st.integers(-2**63, 2**63 - 1), st.floats(allow_nan=False),
                      st.text(max_size=20))
json_value = st.recursive(json_leaf, lambda inner: st.one_of(st.lists(inner, max_size=5),
                                                           st.dictionaries(st.text(max_size=10), inner, max_size=5)),
                          max_leaves=30)
pod_keys = st.sampled_from(["Pod", "NodeNames", "Nodes", "metadata", "spec", "containers", "resources", "limits",
                            "aliyun.com/gpu-mem", "shared-gpu/gpu-mem", "uid", "name", "annotations"])
k8s_like = st.recursive(json_leaf, lambda inner: st.one_of(st.lists(inner, max_size=4),
                                                         st.dictionaries(pod_keys, inner, max_size=4)),
                        max_leaves=40)


def _filter_ok(out: bytes):
    r = json.loads(out)  # always valid JSON
    assert set(r) >= {"NodeNames", "FailedNodes", "Error"}
    assert isinstance(r["Error"], str)


@settings(max_examples=300, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(st.binary(max_size=512))
def test_filter_survives_arbitrary_bytes(body):
    _filter_ok(ENGINE.filter(body))


@settings(max_examples=300, deadline=None)
@given(json_value)
def test_filter_survives_arbitrary_json(v):
    _filter_ok(ENGINE.filter(json.dumps(v).encode()))


@settings(max_examples=300, deadline=None)
@given(k8s_like, st.lists(st.text(max_size=8), max_size=4))
def test_filter_survives_pod_shaped_json(pod, names):
    _filter_ok(ENGINE.filter(json.dumps({"Pod": pod, "NodeNames": names}).encode()))


@settings(max_examples=200, deadline=None)
@given(st.integers(-2**70, 2**70).map(str) | st.text(max_size=12), st.sampled_from(["n", "missing", ""]))
def test_filter_quantities(q, node):
    """gpu-mem limits of any spelling (a number beyond int64, a Kubernetes quantity, garbage): the answer is
    always a well-formed ExtenderFilterResult."""
    pod = make_pod("p", 1)
    pod["spec"]["containers"][0]["resources"]["limits"]["shared-gpu/gpu-mem"] = q
    r = json.loads(ENGINE.filter(wire.filter_args(pod, [node])))
    assert isinstance(r["Error"], str)


def test_native_front_end_survives_generated_requests():
    """Generated request heads, bodies and chunk framings against the C++ epoll front end; afterwards it still
    answers a filter request on a fresh connection."""
    from gpushare_scheduler_extender_amd.extender.server import ExtenderRunner, ExtenderServer
    from gpushare_scheduler_extender_amd.k8s.client import KubeClient
    from tests.fixtures.fakeapi import FakeApiServerRunner

    methods = st.sampled_from([b"GET", b"POST", b"PUT", b"DELETE", b"BREW", b""])
    paths = st.sampled_from([b"/gpushare-scheduler/filter", b"/gpushare-scheduler/bind", b"/version",
                             b"/gpushare-scheduler/inspect/n", b"/" + b"a" * 300, b"*", b""])
    headers = st.lists(st.sampled_from([b"Content-Length: 5", b"Content-Length: -1", b"Content-Length: 99999999999",
                                        b"Transfer-Encoding: chunked", b"Connection: close", b"Host: x",
                                        b"Expect: 100-continue", b"X: " + b"y" * 200, b": bad", b"NoColon"]),
                       max_size=4)
    bodies = st.binary(max_size=64) | st.sampled_from([b"5\r\nhello\r\n0\r\n\r\n", b"ffffffffffffffff\r\n",
                                                       b"-1\r\n", b"5\r\nhel", b"{\"Pod\":"])
    requests = st.builds(lambda m, p, h, b: m + b" " + p + b" HTTP/1.1\r\n" + b"\r\n".join(h) + b"\r\n\r\n" + b,
                         methods, paths, headers, bodies)

    async def go():
        api = await FakeApiServerRunner().start()
        c = KubeClient(api.url)
        await c.create("nodes", make_node("n", 8 * 100, 8))
        ext = await ExtenderRunner(ExtenderServer(KubeClient(api.url)), http_threads=2).start()
        try:
            def send(payload: bytes):
                s = socket.create_connection(("127.0.0.1", ext.port), timeout=2)
                try:
                    s.sendall(payload)
                    s.shutdown(socket.SHUT_WR)
                    while s.recv(65536):
                        pass
                except OSError:
                    pass
                finally:
                    s.close()

            @settings(max_examples=150, deadline=None, suppress_health_check=list(HealthCheck))
            @given(st.lists(requests, min_size=1, max_size=3))
            def storm(reqs):
                send(b"".join(reqs))

            await asyncio.get_running_loop().run_in_executor(None, storm)
            # still serving
            body = wire.filter_args(make_pod("p", 50), ["n"])
            req = (b"POST /gpushare-scheduler/filter HTTP/1.1\r\nHost: x\r\nContent-Length: %d\r\n"
                   b"Connection: close\r\n\r\n" % len(body)) + body
            s = socket.create_connection(("127.0.0.1", ext.port), timeout=5)
            s.sendall(req)
            data = b""
            while True:
                chunk = s.recv(65536)
                if not chunk:
                    break
                data += chunk
            s.close()
            assert data.startswith(b"HTTP/1.1 200") and b'"NodeNames":["n"]' in data
        finally:
            await ext.stop()
            await ext.server.client.close()
            await c.close()
            await api.stop()
    asyncio.run(go())


quantities = st.builds(
    lambda sign, whole, frac, suf: sign + whole + frac + suf,
    st.sampled_from(["", "+", "-"]),
    st.from_regex(r"\A\d{0,22}\Z"),
    st.sampled_from(["", "."]) | st.from_regex(r"\A\.\d{1,12}\Z"),
    st.sampled_from(["", "Ki", "Mi", "Gi", "Ti", "Pi", "Ei", "n", "u", "m", "k", "M", "G", "T", "P", "E", "i", "K",
                     "e", "E3", "e-3", "e+2", "e400", "e-400", "Gb", " "]) | st.from_regex(r"\A[eE][+-]?\d{1,3}\Z"))


@settings(max_examples=1000, deadline=None)
@given(quantities | st.text(max_size=10))
def test_native_quantity_parser_agrees_with_python(s):
    """native/engine/quantity.cc (filter, bind, informer) against the exact Fraction-based parser: same value
    (ceil, saturated to int64) or both reject."""
    from gpushare_scheduler_extender_amd.core.engine import parse_quantity as native_q
    from gpushare_scheduler_extender_amd.models.quantity import parse_quantity as py_q

    def run(f):
        try:
            return f(s)
        except ValueError:
            return "invalid"
    assert run(native_q) == run(py_q), s


atoi_like = st.one_of(st.from_regex(r"\A[+-]?\d{1,21}\Z"), st.sampled_from(["", "-", "+", "1.5", " 1", "1 ", "0x10",
                                                                            "٣", "9223372036854775807",
                                                                            "9223372036854775808", "-1"]),
                      st.text(max_size=6))
limit = st.one_of(st.integers(0, 2**40).map(str), st.sampled_from(["1Gi", "0.5", "1e3", "abc", "-4", "", "2k"]),
                  st.integers(0, 2**40))


@settings(max_examples=500, deadline=None)
@given(st.lists(st.one_of(st.none(), limit), min_size=0, max_size=3), atoi_like, atoi_like, atoi_like,
       st.sampled_from(["true", "false", "", "True"]), st.sampled_from(["Pending", "Running", "Succeeded", "Failed", ""]),
       st.booleans(), st.sampled_from(["", "n1"]))
def test_native_pod_view_agrees_with_python(limits, idx, mem, assume, assigned, phase, deleting, node):
    """The native pod view (what the informer, filter and bind read) against models/pod.py, the reference's
    pkg/utils/pod.go semantics, on generated annotations and limits."""
    from gpushare_scheduler_extender_amd.models import pod as podutil
    from gpushare_scheduler_extender_amd.models.profile import SHARED_GPU as P

    ann = {P.annotation_idx: idx, P.annotation_pod: mem, P.annotation_assume_time: assume,
           P.annotation_assigned: assigned}
    pod = make_pod("p", [0] * max(1, len(limits)), annotations=ann, node=node, phase=phase,
                   deletion_timestamp="2026-01-01T00:00:00Z" if deleting else None)
    for c, lim in zip(pod["spec"]["containers"], limits):
        lims = c.setdefault("resources", {}).setdefault("limits", {})
        if lim is None:
            lims.pop(P.resource, None)
        else:
            lims[P.resource] = lim
    v = ENGINE.parse_pod(json.dumps(pod).encode())
    assert v.request == podutil.gpu_mem_request(pod, P)
    assert v.dev_idx == podutil.gpu_id_from_annotation(pod, P)
    assert v.annot_mem == podutil.gpu_mem_from_annotation(pod, P)
    assert v.assume_time == podutil.assume_time(pod, P)
    assert bool(v.assigned == 1) == podutil.is_assigned(pod, P)
    assert v.complete == podutil.is_complete(pod)
    assert v.terminal == podutil.is_terminal(pod)
    assert v.assigned_non_terminated == podutil.assigned_non_terminated(pod)
