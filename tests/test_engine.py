"""Native engine: golden cases from the reference design doc, wire format, quirks, properties."""
import json
import time

import pytest
from hypothesis import given, settings, strategies as st

from gpushare_scheduler_extender_amd.core.engine import native, new_engine
from gpushare_scheduler_extender_amd.k8s.objects import make_node, make_pod
from gpushare_scheduler_extender_amd.models import wire
from gpushare_scheduler_extender_amd.models.profile import ALIYUN, SHARED_GPU
from gpushare_scheduler_extender_amd.models.quantity import parse_quantity as py_quantity

from .refmodel import RefNode

E = native()


def _annotated(name, node, dev, mem, profile=SHARED_GPU, phase="Running", **kw):
    ann = {profile.annotation_idx: str(dev), profile.annotation_pod: str(mem)}
    return make_pod(name, mem, node=node, annotations=ann, phase=phase, profile=profile, **kw)


def _load(eng, pod):
    return eng.upsert_pod(eng.parse_pod(json.dumps(pod).encode()))


def _filter(eng, pod, names):
    return json.loads(eng.filter(wire.filter_args(pod, names)))


# ---------------------------------------------------------------- quantities

@pytest.mark.parametrize("s,v", [("0", 0), ("1", 1), ("8138", 8138), ("1.5", 2), ("64Gi", 64 * 2**30),
                                 ("1k", 1000), ("1Ki", 1024), ("500m", 1), ("1e3", 1000), ("2E2", 200),
                                 ("0.1", 1), ("-1", -1), ("+3", 3), (".5", 1), ("1000m", 1), ("1001m", 2),
                                 ("16276", 16276), ("3M", 3000000), ("1n", 1)])
def test_quantity_native_matches_python(s, v):
    assert E.parse_quantity(s) == v
    assert py_quantity(s) == v


@pytest.mark.parametrize("bad", ["", "abc", "1x", "1Kib", "--1", "1e", "Gi"])
def test_quantity_rejects(bad):
    with pytest.raises(ValueError):
        E.parse_quantity(bad)
    with pytest.raises(ValueError):
        py_quantity(bad)


@settings(max_examples=300, deadline=None)
@given(st.integers(0, 10**6), st.integers(0, 999), st.sampled_from(["", "k", "M", "Ki", "Mi", "Gi", "m", "e2", "e-1"]))
def test_quantity_property(i, frac, suf):
    s = f"{i}.{frac:03d}{suf}"
    assert E.parse_quantity(s) == py_quantity(s)


# ---------------------------------------------------------------- design-doc goldens

def test_designdoc_filter_example():
    """docs/designs/designs.md:70-76: req 8138 on 3 nodes x 2 x 16276."""
    eng = new_engine()
    for n in ("n1", "n2", "n3"):
        eng.upsert_node(n, 32552, 2)
    # N1: GPU0 full, GPU1 12207 used -> 4069 free in total
    _load(eng, _annotated("a", "n1", 0, 16276))
    _load(eng, _annotated("b", "n1", 1, 12207))
    # N2: 4069 free on each device
    _load(eng, _annotated("c", "n2", 0, 12207))
    _load(eng, _annotated("d", "n2", 1, 12207))
    # N3: 8138 free on GPU0 only
    _load(eng, _annotated("e", "n3", 0, 8138))
    _load(eng, _annotated("f", "n3", 1, 16276))
    r = _filter(eng, make_pod("p", 8138), ["n1", "n2", "n3"])
    assert r["NodeNames"] == ["n3"]
    assert r["FailedNodes"] == {"n1": "Insufficient GPU Memory in one device",
                                "n2": "Insufficient GPU Memory in one device"}
    assert r["Error"] == ""


def test_designdoc_bind_example_best_fit():
    """docs/designs/designs.md:88: free {12207, 8138, 4069, 16276}, req 8138 -> GPU1."""
    eng = new_engine()
    eng.upsert_node("n1", 4 * 16276, 4)
    _load(eng, _annotated("a", "n1", 0, 16276 - 12207))
    _load(eng, _annotated("b", "n1", 1, 16276 - 8138))
    _load(eng, _annotated("c", "n1", 2, 16276 - 4069))
    dev, total = eng.assume("uid-p", "default", "p", "n1", 8138)
    assert (dev, total) == (1, 16276)


def test_best_fit_ties_lowest_index():
    eng = new_engine()
    eng.upsert_node("n", 4 * 100, 4)
    assert eng.assume("u1", "d", "a", "n", 10)[0] == 0
    assert eng.assume("u2", "d", "b", "n", 10)[0] == 0  # now dev0 is the best fit
    _load(eng, _annotated("x", "n", 2, 95))
    assert eng.assume("u3", "d", "c", "n", 5)[0] == 2  # dev2 has 5 free: exact fit


def test_binpack_samples_same_device():
    """samples/1-3.yaml: pods of gpu-mem 2 (GiB) binpack onto one device."""
    eng = new_engine()
    eng.upsert_node("n", 30, 2)
    devs = [eng.assume(f"u{i}", "d", f"binpack-{i}", "n", 2)[0] for i in range(3)]
    assert devs == [0, 0, 0]
    assert eng.node_devices("n") == [(15, 6), (15, 0)]


def test_fragmentation_guard_demo2():
    """demo2.jpg / samples/4.yaml: 16276 free on the node but 8138 per device -> refused."""
    eng = new_engine()
    eng.upsert_node("n", 32552, 2)
    _load(eng, _annotated("binpack-2", "n", 0, 8138))
    _load(eng, _annotated("binpack-3", "n", 1, 8138))
    r = _filter(eng, make_pod("big", 16276), ["n"])
    assert r["NodeNames"] == [] and r["FailedNodes"] == {"n": "Insufficient GPU Memory in one device"}
    assert eng.assume("u", "d", "big", "n", 16276)[0] == -1


# ---------------------------------------------------------------- wire format

def test_filter_response_bytes_match_go_encoding():
    eng = new_engine()
    eng.upsert_node("gpu-a", 100, 1)
    eng.upsert_node("cpu-b", 0, 0)
    out = eng.filter(wire.filter_args(make_pod("p", 10), ["gpu-a", "cpu-b", "ghost"]))
    assert out == (b'{"Nodes":null,"NodeNames":["gpu-a"],"FailedNodes":{'
                   b'"cpu-b":"The node cpu-b is not for GPU share, need skip",'
                   b'"ghost":"node \\"ghost\\" not found"},"Error":""}')


def test_filter_empty_result_shapes():
    eng = new_engine()
    out = json.loads(eng.filter(wire.filter_args(make_pod("p", 1), [])))
    assert out == {"Nodes": None, "NodeNames": [], "FailedNodes": {}, "Error": ""}


def test_filter_case_insensitive_keys():
    eng = new_engine()
    eng.upsert_node("n", 10, 1)
    body = json.dumps({"pod": make_pod("p", 5), "nodes": None, "nodenames": ["n"]}).encode()
    assert json.loads(eng.filter(body))["NodeNames"] == ["n"]
    body = json.dumps({"POD": make_pod("p", 50), "NODENAMES": ["n"]}).encode()
    assert json.loads(eng.filter(body))["FailedNodes"] == {"n": "Insufficient GPU Memory in one device"}


def test_filter_non_cache_capable_nodes_list():
    """predicate.go:17 panics without NodeNames; we accept Nodes and echo the passing items."""
    eng = new_engine()
    eng.upsert_node("a", 10, 1)
    eng.upsert_node("b", 4, 1)
    nodes = [make_node("a", 10, 1), make_node("b", 4, 1)]
    r = json.loads(eng.filter(wire.filter_args(make_pod("p", 5), nodes=nodes)))
    assert [n["metadata"]["name"] for n in r["Nodes"]["items"]] == ["a"]
    assert r["Nodes"]["items"][0] == nodes[0]
    assert r["FailedNodes"] == {"b": "Insufficient GPU Memory in one device"}


@pytest.mark.parametrize("body", [b"", b"{", b"nope", b'{"Pod": 5}', b"[]"])
def test_filter_malformed(body):
    eng = new_engine()
    r = json.loads(eng.filter(body))
    assert r["Error"] and r["NodeNames"] is None and r["FailedNodes"] is None


def test_filter_go_error_messages():
    eng = new_engine()
    assert json.loads(eng.filter(b""))["Error"] == "unexpected end of JSON input"
    assert json.loads(eng.filter(b"x"))["Error"] == "invalid character 'x' looking for beginning of value"


def test_multi_container_request_sums_and_init_ignored():
    eng = new_engine()
    eng.upsert_node("n", 100, 1)
    pod = make_pod("p", [30, 40])
    pod["spec"]["initContainers"] = [{"name": "i", "resources": {"limits": {SHARED_GPU.resource: "90"}}}]
    assert eng.parse_pod(json.dumps(pod).encode()).request == 70
    r = _filter(eng, make_pod("q", [60, 41]), ["n"])
    assert r["NodeNames"] == []


def test_aliyun_profile():
    eng = new_engine(ALIYUN)
    eng.upsert_node_json(json.dumps(make_node("n", 64, 2, profile=ALIYUN)).encode())
    pod = make_pod("p", 20, profile=ALIYUN)
    assert json.loads(eng.filter(wire.filter_args(pod, ["n"])))["NodeNames"] == ["n"]
    # shared-gpu resource names are invisible to the aliyun profile
    assert eng.parse_pod(json.dumps(make_pod("q", 20)).encode()).request == 0
    _load(eng, _annotated("x", "n", 1, 30, profile=ALIYUN))
    assert eng.node_devices("n") == [(32, 0), (32, 30)]


# ---------------------------------------------------------------- quirks fixed

def test_overcommit_does_not_underflow():
    """nodeinfo.go:260 computes free on uint -> ~4e9 on overcommit; ours stays negative."""
    eng = new_engine()
    eng.upsert_node("n", 10, 1)
    _load(eng, _annotated("a", "n", 0, 8))
    _load(eng, _annotated("b", "n", 0, 8))
    assert eng.node_devices("n") == [(10, 16)]
    assert _filter(eng, make_pod("p", 1), ["n"])["NodeNames"] == []
    assert eng.stats()["overcommit_events"] >= 1


def test_completed_not_counted_deleting_counted():
    """deviceinfo.go:46-49 skips Succeeded/Failed but counts pods being deleted."""
    eng = new_engine()
    eng.upsert_node("n", 10, 1)
    _load(eng, _annotated("a", "n", 0, 4, phase="Succeeded"))
    _load(eng, _annotated("b", "n", 0, 3, phase="Failed"))
    _load(eng, _annotated("c", "n", 0, 5, deletion_timestamp="2024-01-01T00:00:00Z"))
    assert eng.node_devices("n") == [(10, 5)]
    insp = json.loads(eng.inspect("n")[0])
    assert insp["nodes"][0]["devs"][0]["pods"] == []  # deleting pod hidden (AssignedNonTerminatedPod)


def test_capacity_change_rebuilds():
    """cache.go:144-157 never picks up capacity changes; ours rebuilds and re-accounts."""
    eng = new_engine()
    eng.upsert_node("n", 10, 1)
    _load(eng, _annotated("a", "n", 0, 4))
    assert eng.upsert_node("n", 40, 2) is True
    assert eng.node_devices("n") == [(20, 4), (20, 0)]
    assert eng.upsert_node("n", 40, 2) is False


def test_pod_before_node_is_adopted():
    eng = new_engine()
    assert _load(eng, _annotated("a", "n", 1, 7)) == 1
    eng.upsert_node("n", 20, 2)
    assert eng.node_devices("n") == [(10, 0), (10, 7)]


def test_invalid_index_not_counted():
    eng = new_engine()
    eng.upsert_node("n", 20, 2)
    pod = _annotated("a", "n", 5, 7)
    assert _load(eng, pod) == 1  # recorded, but device 5 does not exist
    assert eng.node_devices("n") == [(10, 0), (10, 0)]
    bad = make_pod("b", 3, node="n", annotations={SHARED_GPU.annotation_idx: "x1"})
    assert _load(eng, bad) == 0


def test_heterogeneous_devices_annotation():
    eng = new_engine()
    name, _ = eng.upsert_node_json(json.dumps(make_node("n", 300, 3, device_totals=[200, 50, 50])).encode())
    assert name == "n"
    assert eng.node_devices("n") == [(200, 0), (50, 0), (50, 0)]
    assert eng.assume("u", "d", "p", "n", 60)[0] == 0
    assert eng.assume("v", "d", "q", "n", 40)[0] == 1


# ---------------------------------------------------------------- bind reservations

def test_assume_reserves_and_release_on_failure():
    eng = new_engine()
    eng.upsert_node("n", 10, 1)
    assert eng.assume("u1", "d", "a", "n", 6)[0] == 0
    assert eng.assume("u2", "d", "b", "n", 6)[0] == -1  # reserved memory is visible to the next bind
    assert _filter(eng, make_pod("c", 6), ["n"])["NodeNames"] == []
    assert eng.assume("u1", "d", "a", "n", 6)[0] == -4  # bind already in flight
    eng.finish_bind("u1", False)
    assert eng.node_devices("n") == [(10, 0)]
    assert eng.assume("u2", "d", "b", "n", 6)[0] == 0


def test_assume_confirmed_by_informer_and_gc():
    eng = new_engine()
    eng.upsert_node("n", 10, 1)
    dev, _ = eng.assume("u1", "d", "a", "n", 6)
    eng.finish_bind("u1", True, 0.0)  # ttl 0: would expire immediately if unconfirmed
    pod = _annotated("a", "n", dev, 6, uid="u1")
    _load(eng, pod)  # informer observes the annotated, bound pod
    assert eng.gc() == (0, False)
    assert eng.node_devices("n") == [(10, 6)]
    eng.assume("u2", "d", "b", "n", 2)
    eng.finish_bind("u2", True, 0.0)
    # overdue, but no LIST since the binding was written: kept (the watch may be stalled), re-list asked for
    assert eng.gc() == (0, True) and eng.gc(time.monotonic() - 60) == (0, True)
    assert eng.node_devices("n") == [(10, 8)] and eng.stats()["expiry_deferred"] == 2
    # a LIST sent after the binding that did not confirm it: the apiserver has no such binding
    assert eng.gc(time.monotonic()) == (1, False)
    assert eng.node_devices("n") == [(10, 6)]


def test_assume_errors():
    eng = new_engine()
    eng.upsert_node("cpu", 0, 0)
    assert eng.assume("u", "d", "p", "ghost", 1)[0] == -2
    assert eng.assume("u", "d", "p", "cpu", 1)[0] == -3
    eng.upsert_node("n", 10, 1)
    assert eng.assume("u", "d", "p", "n", 0)[0] == -1  # no gpu-mem request: never placed


def test_annotation_race_before_binding_keeps_reservation():
    eng = new_engine()
    eng.upsert_node("n", 10, 1)
    eng.assume("u1", "d", "a", "n", 6)
    # informer sees the annotation PATCH before the Binding (nodeName still empty)
    early = make_pod("a", 6, uid="u1", annotations={SHARED_GPU.annotation_idx: "0", SHARED_GPU.annotation_pod: "6"})
    _load(eng, early)
    assert eng.node_devices("n") == [(10, 6)]


def test_remove_pod():
    eng = new_engine()
    eng.upsert_node("n", 10, 1)
    p = _annotated("a", "n", 0, 6)
    _load(eng, p)
    assert eng.known(p["metadata"]["uid"])
    assert eng.remove_pod(p["metadata"]["uid"])
    assert eng.node_devices("n") == [(10, 0)]
    assert not eng.remove_pod(p["metadata"]["uid"])


# ---------------------------------------------------------------- inspect

def test_inspect_schema():
    eng = new_engine()
    eng.upsert_node("n2", 30, 2)
    eng.upsert_node("n1", 15, 1)
    _load(eng, _annotated("b", "n2", 1, 3))
    _load(eng, _annotated("a", "n1", 0, 6))
    body, found = eng.inspect("")
    assert found
    res = wire.InspectResult.decode(body)
    assert [n.name for n in res.nodes] == ["n1", "n2"]
    assert res.nodes[1].totalGPU == 30 and res.nodes[1].usedGPU == 3
    assert res.nodes[1].devs[1].pods[0].name == "b" and res.nodes[1].devs[1].pods[0].usedGPU == 3
    assert json.loads(body)["nodes"][0]["devs"][0] == {"id": 0, "totalGPU": 15, "usedGPU": 6,
                                                       "pods": [{"name": "a", "namespace": "default", "usedGPU": 6}]}
    assert "error" not in json.loads(body)
    body, found = eng.inspect("ghost")
    assert not found and json.loads(body) == {"nodes": [], "error": 'node "ghost" not found'}


def test_json_quote_go_html_escaping():
    assert E.json_quote('<a&b>"\n') == '"\\u003ca\\u0026b\\u003e\\"\\n"'
    assert E.json_quote(" ") == '"\\u2028"'


def test_json_parser_unicode_and_escapes():
    pod = make_pod("pé", 5)
    pod["metadata"]["namespace"] = "n\\s\"x"
    raw = json.dumps(pod, ensure_ascii=True).encode()
    v = new_engine().parse_pod(raw)
    assert v.name == "pé" and v.namespace == 'n\\s"x' and v.request == 5
    assert E.json_validate(b'{"a":"\\ud83d\\ude00"}')[0]


# ---------------------------------------------------------------- property test vs reference model

@settings(max_examples=150, deadline=None)
@given(st.lists(st.integers(1, 6), min_size=1, max_size=4),
       st.lists(st.tuples(st.sampled_from(["add", "del", "bind", "term"]), st.integers(0, 40), st.integers(1, 60)),
                max_size=60))
def test_engine_matches_reference_model(counts, ops):
    eng = new_engine()
    ref = {}
    for i, c in enumerate(counts):
        ref[f"n{i}"] = RefNode(f"n{i}", 100 * c, c)
        eng.upsert_node(f"n{i}", 100 * c, c)
    live = {}
    k = 0
    for op, a, b in ops:
        node = f"n{a % len(counts)}"
        rn = ref[node]
        if op == "add":
            dev = a % rn.count
            uid = f"u{k}"
            k += 1
            _load(eng, _annotated(f"p{uid}", node, dev, b, uid=uid))
            rn.pods[uid] = (dev, b, False)
            live[uid] = node
        elif op == "bind":
            uid = f"u{k}"
            k += 1
            want = rn.best_fit(b)
            got, _ = eng.assume(uid, "d", f"p{uid}", node, b)
            assert got == (want if want >= 0 else -1)
            if got >= 0:
                eng.finish_bind(uid, True, 3600)
                rn.pods[uid] = (got, b, False)
                live[uid] = node
        elif op in ("del", "term") and live:
            uid = sorted(live)[a % len(live)]
            n2 = ref[live[uid]]
            if op == "del":
                eng.remove_pod(uid)
                del n2.pods[uid]
                del live[uid]
            else:
                dev, mem, _ = n2.pods[uid]
                _load(eng, _annotated(f"p{uid}", live[uid], dev, mem, uid=uid, phase="Succeeded"))
                n2.pods[uid] = (dev, mem, True)
        # invariants after every op
        for name, rn2 in ref.items():
            assert [u for _, u in eng.node_devices(name)] == rn2.used()
            for req in (1, 50, 100):
                ok = json.loads(eng.filter(wire.filter_args(make_pod("q", req), [name])))["NodeNames"] == [name]
                assert ok == rn2.fits(req)


# ---------------------------------------------------------------- prioritize verb (ours)

def test_prioritize_binpack_first_across_nodes():
    eng = new_engine()
    eng.upsert_node("tight", 100, 1)
    eng.upsert_node("loose", 100, 1)
    eng.upsert_node("full", 100, 1)
    eng.upsert_node("cpu", 0, 0)
    _load(eng, _annotated("a", "tight", 0, 70))
    _load(eng, _annotated("b", "full", 0, 95))
    out = json.loads(eng.prioritize(wire.filter_args(make_pod("p", 30), ["tight", "loose", "full", "cpu", "ghost"])))
    scores = {h["Host"]: h["Score"] for h in out}
    assert scores == {"tight": 10, "loose": 3, "full": 0, "cpu": 0, "ghost": 0}
    assert list(out[0]) == ["Host", "Score"]
    assert json.loads(eng.prioritize(b"junk")) == []


def test_bind_wait_returns_when_its_own_entry_is_left():
    """a cancelled Python bind calls bind_leave(seq) while its executor thread still sits in
    bind_wait(seq); the waiter must notice the entry is gone (no dangling pointer into the freed list node)."""
    import threading

    eng = new_engine()
    eng.upsert_node("n", 20, 2)
    d1, _, s1, _ = eng.assume_ordered("u1", "d", "a", "n", 10, "")
    d2, _, s2, _ = eng.assume_ordered("u2", "d", "b", "n", 10, "")
    assert d1 != d2 and eng.bind_blocked(s2)  # equal size, other GPU: ordered behind the first
    done = threading.Event()
    t = threading.Thread(target=lambda: (eng.bind_wait(s2), done.set()))
    t.start()
    time.sleep(0.05)
    assert not done.is_set()
    eng.bind_leave(s2)  # the cancelled caller's cleanup
    assert done.wait(2.0), "bind_wait did not return after its entry was removed"
    t.join()
    eng.bind_leave(s1)
    # and the normal path: a blocked bind is released by the earlier bind's completion
    _, _, s3, _ = eng.assume_ordered("u3", "d", "c", "n", 5, "")
    _, _, s4, _ = eng.assume_ordered("u4", "d", "e", "n", 5, "")
    if eng.bind_blocked(s4):
        done.clear()
        t = threading.Thread(target=lambda: (eng.bind_wait(s4), done.set()))
        t.start()
        eng.bind_leave(s3)
        assert done.wait(2.0)
        t.join()
    eng.bind_leave(s4)


def test_reconcile_hold_charges_both_devices():
    """A pod whose allocation record the device plugin is moving (hold-idx) is charged on its new and its old
    device until the hold is cleared: no device is ever under-counted mid-move (deviceplugin/reconcile.py)."""
    eng = new_engine()
    eng.upsert_node("n", 20, 2)
    a = _annotated("a", "n", 0, 8, uid="ua")
    b = _annotated("b", "n", 1, 8, uid="ub")
    _load(eng, a)
    _load(eng, b)
    assert eng.node_devices("n") == [(10, 8), (10, 8)]
    a["metadata"]["annotations"][SHARED_GPU.annotation_idx] = "1"
    a["metadata"]["annotations"]["gpushare.amd.com/hold-idx"] = "0"
    _load(eng, a)  # step 1: a moves to GPU 1, still held on GPU 0
    assert eng.node_devices("n") == [(10, 8), (10, 16)]
    b["metadata"]["annotations"][SHARED_GPU.annotation_idx] = "0"
    _load(eng, b)  # step 2: b takes GPU 0 (over-counted while the hold lasts, never under)
    assert eng.node_devices("n") == [(10, 16), (10, 8)]
    del a["metadata"]["annotations"]["gpushare.amd.com/hold-idx"]
    _load(eng, a)  # step 3: hold cleared
    assert eng.node_devices("n") == [(10, 8), (10, 8)]
    a["metadata"]["annotations"]["gpushare.amd.com/hold-idx"] = "1"  # a hold on its own device counts once
    _load(eng, a)
    assert eng.node_devices("n") == [(10, 8), (10, 8)]
    a["metadata"]["annotations"]["gpushare.amd.com/hold-idx"] = "0"
    _load(eng, a)
    eng.remove_pod("ua")  # removal drops both charges
    assert eng.node_devices("n") == [(10, 8), (10, 0)]
