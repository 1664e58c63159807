"""Test fixture: in-process fake kube-apiserver (pods, nodes, bindings, events) over real HTTP.

Not shipped: the stack, ``gsxtools/`` and ``bench.py`` run the compiled ``gsx-fakeapi`` (``native/fakeapi``), which
speaks the same REST subset.  This asyncio twin stays for tests that reach into the object store directly
(``FakeApiServer``) or run the apiserver in the test's own event loop.  The reference was only ever validated
by hand on a live cluster.  It speaks the
subset of the core/v1 REST API the scheduler extender, the controller, the
device plugin and the CLI use, with the semantics they rely on:

* LIST + chunk-streamed WATCH with ``resourceVersion`` (one global counter, as
  etcd gives kube-apiserver), ``410 Gone`` for compacted versions, field
  selectors ``spec.nodeName`` / ``metadata.name`` and equality label selectors;
* optimistic concurrency on PUT / PATCH: ``409 Conflict`` with the exact
  message client-go produces, which the reference matches by string
  (``pkg/cache/nodeinfo.go:14-16,150-168``);
* ``POST pods/{name}/binding`` sets ``spec.nodeName`` once and merges the
  Binding's ``metadata.annotations`` into the pod, as kube-apiserver's
  ``setPodHostAndAnnotations`` does (this is what lets our bind verb annotate
  and bind in one round trip instead of the reference's PUT + POST,
  ``pkg/cache/nodeinfo.go:150-189``);
* JSON merge patch and strategic-merge-patch (treated as merge patch, which is
  exact for the metadata/annotation/status patches used here);
* graceful pod deletion as kube-apiserver does it: a bound, non-terminal pod only gets ``deletionTimestamp`` (the
  grace from the request, else ``spec.terminationGracePeriodSeconds``); the object stays until the node's kubelet,
  having stopped the containers, deletes it with grace 0 (the kubelet stand-ins in ``gsxtools/agent.py`` and
  ``native/nodeagent`` do).  Unbound or terminal pods, and grace 0, are removed at once.  DELETE honours
  ``preconditions.uid`` (409 on mismatch), as kubelet's final delete relies on;
* fault injection: conflict / error / throttle (429 + ``Retry-After``) rates, latency and watch drops
  (``POST /fake/faults``), which the reference never had.

Run standalone with ``python -m tests.fixtures.fakeapi`` (or use ``gsx-fakeapi``).
"""
from __future__ import annotations

import argparse
import asyncio
import collections
import json
import logging
import random
import time
import uuid
from datetime import datetime, timezone

from gpushare_scheduler_extender_amd.k8s.fasthttp import HTTPError, Request, Response, Server, Stream

log = logging.getLogger("gsx.fakeapi")

CONFLICT_MSG = ("Operation cannot be fulfilled on {res} \"{name}\": the object has been modified; "
                "please apply your changes to the latest version and try again")


def _now_iso() -> str:
    return datetime.now(timezone.utc).strftime("%Y-%m-%dT%H:%M:%SZ")


def _obj_key(o: dict) -> tuple[str, str]:
    md = o.get("metadata") or {}
    return md.get("namespace", "") or "", md.get("name", "")


def status_body(code: int, reason: str, message: str, details: dict | None = None) -> dict:
    b = {"kind": "Status", "apiVersion": "v1", "metadata": {}, "status": "Failure", "message": message,
         "reason": reason, "code": code}
    if details:
        b["details"] = details
    return b


def merge_patch(target, patch):
    """RFC 7386 JSON merge patch."""
    if not isinstance(patch, dict):
        return patch  # values come fresh from the request body; stored objects are never mutated
    if not isinstance(target, dict):
        target = {}
    out = dict(target)
    for k, v in patch.items():
        if v is None:
            out.pop(k, None)
        else:
            out[k] = merge_patch(out.get(k), v)
    return out


def _label_match(obj: dict, selector: str) -> bool:
    if not selector:
        return True
    labels = (obj.get("metadata") or {}).get("labels") or {}
    for term in selector.split(","):
        term = term.strip()
        if not term:
            continue
        if "!=" in term:
            k, v = term.split("!=", 1)
            if labels.get(k.strip()) == v.strip():
                return False
        elif "=" in term:
            k, v = term.split("=", 1)
            k = k.strip().rstrip("=")
            if labels.get(k) != v.strip():
                return False
        elif term.startswith("!"):
            if term[1:] in labels:
                return False
        elif term not in labels:
            return False
    return True


def _field_value(obj: dict, path: str):
    cur = obj
    for p in path.split("."):
        if not isinstance(cur, dict):
            return ""
        cur = cur.get(p)
    return "" if cur is None else cur


def _field_match(obj: dict, selector: str) -> bool:
    if not selector:
        return True
    for term in selector.split(","):
        term = term.strip()
        if not term:
            continue
        if "!=" in term:
            k, v = term.split("!=", 1)
            if str(_field_value(obj, k.strip())) == v.strip():
                return False
        else:
            k, v = term.split("=", 1)
            k = k.strip().rstrip("=")
            if str(_field_value(obj, k)) != v.strip():
                return False
    return True


class _Watcher:
    """One watch stream.  Events are pushed, not pulled: ``push`` buffers the
    line and schedules one ``flush`` per event-loop iteration, so a burst of
    writes (a DeleteCollection, 32 creates) goes out as one chunk and no
    coroutine wakes per event."""

    __slots__ = ("kind", "ns", "fsel", "lsel", "closed", "pending", "scheduled", "out", "done", "sent", "drop_after",
                 "on_drop")

    def __init__(self, kind, ns, fsel, lsel):
        self.kind = kind
        self.ns = ns
        self.fsel = fsel
        self.lsel = lsel
        self.closed = False
        self.pending: list[bytes] = []
        self.scheduled = False
        self.out = None  # Stream once the backlog is written
        self.done: asyncio.Future = asyncio.get_running_loop().create_future()
        self.sent = 0
        self.drop_after = 0
        self.on_drop = None

    def push(self, line: bytes):
        self.pending.append(line)
        if not self.scheduled and self.out is not None:
            self.scheduled = True
            asyncio.get_running_loop().call_soon(self.flush)

    def go_live(self, out):
        self.out = out
        if self.pending:
            self.flush()

    def flush(self):
        self.scheduled = False
        if self.closed or self.out is None or not self.pending:
            return
        if self.out.closed:
            self.finish()
            return
        lines, self.pending = self.pending, []
        self.out.write(b"".join(lines))
        self.sent += len(lines)
        if self.drop_after and self.sent >= self.drop_after:
            if self.on_drop:
                self.on_drop()
            self.finish()

    def finish(self):
        self.closed = True
        if not self.done.done():
            self.done.set_result(None)

    def wants(self, obj: dict) -> bool:
        if self.ns and (obj.get("metadata") or {}).get("namespace") != self.ns:
            return False
        return _field_match(obj, self.fsel) and _label_match(obj, self.lsel)


class Faults:
    def __init__(self):
        self.conflict_rate = 0.0  # extra 409s on pod PUT/PATCH/binding
        self.error_rate = 0.0  # 500s on mutating pod calls
        self.latency_ms = 0.0  # added to every non-watch request
        self.drop_watch_after = 0  # close watch streams after this many events (0 = never)
        self.expire_watches = 0  # the next N watch requests get 410 Gone (history compacted)
        self.hold_watches = False  # new watch requests wait until this is cleared
        self.fail_lists = False  # LIST requests answer 503 (an apiserver that cannot serve reads)
        self.drop_binding_annotations = False  # Binding.metadata.annotations are not copied onto the pod
        self.slow_bindings: dict[str, float] = {}  # pod name -> ms a binding of it takes
        # API Priority and Fairness: this share of non-watch /api/v1 requests answers 429 Too Many Requests with
        # Retry-After: retry_after seconds (fractional in tests; kube-apiserver sends whole seconds)
        self.throttle_rate = 0.0
        self.retry_after = 1.0
        self.seed = 0
        self.rng = random.Random(0)

    def update(self, d: dict):
        for k in ("conflict_rate", "error_rate", "latency_ms", "drop_watch_after", "expire_watches", "hold_watches",
                  "fail_lists", "drop_binding_annotations", "throttle_rate", "retry_after"):
            if k in d:
                setattr(self, k, type(getattr(self, k))(d[k]))
        if "slow_bindings" in d:
            self.slow_bindings = {str(k): float(v) for k, v in (d["slow_bindings"] or {}).items()}
        if "seed" in d:
            self.seed = int(d["seed"])
            self.rng = random.Random(self.seed)

    def as_dict(self):
        return {"conflict_rate": self.conflict_rate, "error_rate": self.error_rate,
                "latency_ms": self.latency_ms, "drop_watch_after": self.drop_watch_after,
                "expire_watches": self.expire_watches, "hold_watches": self.hold_watches,
                "fail_lists": self.fail_lists, "drop_binding_annotations": self.drop_binding_annotations,
                "throttle_rate": self.throttle_rate, "retry_after": self.retry_after}


class FakeApiServer:
    """State + aiohttp application.  All mutation happens on the event loop thread."""

    KINDS = ("pods", "nodes", "events", "leases")

    def __init__(self, history: int = 200000):
        self.rv = 0
        self.store: dict[str, dict[tuple[str, str], dict]] = {k: {} for k in self.KINDS}
        self.history: collections.deque = collections.deque(maxlen=history)  # (rv, kind, type, bytes, obj)
        self.oldest_rv = 0
        self.watchers: list[_Watcher] = []
        self.faults = Faults()
        self.binding_log: list[str] = []  # pod names in binding commit order
        self.counts = collections.Counter()
        self._last: tuple | None = None
        self.app = self._make_app()

    # ------------------------------------------------------------ state
    def _bump(self) -> str:
        self.rv += 1
        return str(self.rv)

    def _emit(self, kind: str, etype: str, obj: dict):
        rv = int(obj["metadata"]["resourceVersion"])
        ob = json.dumps(obj, separators=(",", ":")).encode()
        line = b'{"type":"' + etype.encode() + b'","object":' + ob + b"}\n"
        self._last = (obj, ob)  # the write's HTTP response reuses this serialisation
        if len(self.history) == self.history.maxlen:
            self.oldest_rv = self.history[0][0]
        self.history.append((rv, kind, etype, line, obj))
        for w in self.watchers:
            if w.kind == kind and not w.closed and w.wants(obj):
                w.push(line)

    def create(self, kind: str, obj: dict, ns: str | None = None) -> dict:
        # copy-on-write: stored objects are immutable once emitted (watch history shares them)
        obj = dict(obj)
        md = obj["metadata"] = dict(obj.get("metadata") or {})
        if ns is not None and kind != "nodes":
            md["namespace"] = ns
        if kind != "nodes":
            md.setdefault("namespace", "default")
        if not md.get("name"):
            if md.get("generateName"):
                md["name"] = md["generateName"] + uuid.uuid4().hex[:5]
            else:
                raise HTTPError(422, status_body(422, "Invalid", "metadata.name: Required value"))
        key = (md.get("namespace", ""), md["name"])
        if key in self.store[kind]:
            raise HTTPError(409, status_body(409, "AlreadyExists", f'{kind} "{md["name"]}" already exists'))
        md.setdefault("uid", str(uuid.uuid4()))
        md.setdefault("creationTimestamp", _now_iso())
        if kind == "pods":
            obj["status"] = dict(obj.get("status") or {})
            obj["status"].setdefault("phase", "Pending")
            obj.setdefault("spec", {})
        md["resourceVersion"] = self._bump()
        self.store[kind][key] = obj
        self._emit(kind, "ADDED", obj)
        return obj

    def _get(self, kind: str, ns: str, name: str) -> dict:
        o = self.store[kind].get((ns if kind != "nodes" else "", name))
        if o is None:
            raise HTTPError(404, status_body(404, "NotFound", f'{kind} "{name}" not found',
                                                               {"name": name, "kind": kind}))
        return o

    def _conflict(self, kind: str, name: str):
        return HTTPError(409, status_body(409, "Conflict", CONFLICT_MSG.format(res=kind, name=name),
                                                            {"name": name, "kind": kind}))

    def replace(self, kind: str, ns: str, name: str, obj: dict, subresource: str = "") -> dict:
        cur = self._get(kind, ns, name)
        want_rv = (obj.get("metadata") or {}).get("resourceVersion")
        if want_rv and want_rv != cur["metadata"]["resourceVersion"]:
            raise self._conflict(kind, name)
        if kind == "pods" and self.faults.conflict_rate and self.faults.rng.random() < self.faults.conflict_rate:
            self.counts["injected_conflict"] += 1
            raise self._conflict(kind, name)
        new = dict(obj)
        md = new["metadata"] = dict(obj.get("metadata") or {})
        # immutable / server-owned fields
        for f in ("uid", "creationTimestamp", "namespace", "name", "deletionTimestamp"):
            if f in cur["metadata"]:
                md[f] = cur["metadata"][f]
        if subresource == "status":
            merged = dict(cur)
            merged["metadata"] = dict(cur["metadata"])
            merged["status"] = new.get("status", {})
            new = merged
        elif kind == "pods":
            # spec.nodeName is only settable through the binding subresource
            old_node = (cur.get("spec") or {}).get("nodeName")
            spec = new["spec"] = dict(new.get("spec") or {})
            if old_node:
                spec["nodeName"] = old_node
            else:
                spec.pop("nodeName", None)
            new["status"] = cur.get("status", {})
        new["metadata"]["resourceVersion"] = self._bump()
        self.store[kind][(ns if kind != "nodes" else "", name)] = new
        self._emit(kind, "MODIFIED", new)
        return new

    def patch(self, kind: str, ns: str, name: str, patch: dict, subresource: str = "") -> dict:
        cur = self._get(kind, ns, name)
        want_rv = ((patch or {}).get("metadata") or {}).get("resourceVersion")
        if want_rv and want_rv != cur["metadata"]["resourceVersion"]:
            raise self._conflict(kind, name)
        want_uid = ((patch or {}).get("metadata") or {}).get("uid")
        if want_uid and want_uid != cur["metadata"].get("uid"):
            # kube-apiserver: the patched object's metadata.uid changed, which update validation refuses (422); a
            # PATCH carries no UID precondition (a PUT's object or a Binding does: 409)
            raise HTTPError(422, status_body(
                422, "Invalid", f'Pod "{name}" is invalid: metadata.uid: Invalid value: "{want_uid}": '
                                f'field is immutable'))
        if kind == "pods" and self.faults.conflict_rate and self.faults.rng.random() < self.faults.conflict_rate:
            self.counts["injected_conflict"] += 1
            raise self._conflict(kind, name)
        if subresource == "status":
            patch = {"status": (patch or {}).get("status", {})}
        elif kind == "pods":
            patch = dict(patch or {})
            spec = patch.get("spec")
            if isinstance(spec, dict) and "nodeName" in spec:
                spec = dict(spec)
                spec.pop("nodeName")
                patch["spec"] = spec
            if subresource == "":
                patch.pop("status", None)
        new = merge_patch(cur, patch)
        new["metadata"] = dict(new["metadata"])
        for f in ("uid", "creationTimestamp", "namespace", "name", "deletionTimestamp"):
            if f in cur["metadata"]:
                new["metadata"][f] = cur["metadata"][f]
        new["metadata"]["resourceVersion"] = self._bump()
        self.store[kind][(ns if kind != "nodes" else "", name)] = new
        self._emit(kind, "MODIFIED", new)
        return new

    def bind(self, ns: str, name: str, binding: dict) -> None:
        cur = self._get("pods", ns, name)
        bmd = binding.get("metadata") or {}
        if bmd.get("uid") and bmd["uid"] != cur["metadata"]["uid"]:
            raise HTTPError(409, status_body(
                409, "Conflict", f'Precondition failed: UID in precondition: {bmd["uid"]}, '
                                 f'UID in object meta: {cur["metadata"]["uid"]}'))
        if self.faults.conflict_rate and self.faults.rng.random() < self.faults.conflict_rate:
            self.counts["injected_conflict"] += 1
            raise self._conflict("pods", name)
        if (cur.get("spec") or {}).get("nodeName"):
            raise HTTPError(409, status_body(
                409, "Conflict", f'pod {name} is already assigned to node "{cur["spec"]["nodeName"]}"'))
        if cur["metadata"].get("deletionTimestamp"):
            raise HTTPError(409, status_body(409, "Conflict", f"pod {name} is being deleted"))
        target = (binding.get("target") or {}).get("name", "")
        if not target:
            raise HTTPError(422, status_body(422, "Invalid", "target.name: Required value"))
        new = dict(cur)
        new["spec"] = dict(cur.get("spec") or {})
        new["spec"]["nodeName"] = target
        new["metadata"] = dict(cur["metadata"])
        ann = {} if self.faults.drop_binding_annotations else (bmd.get("annotations") or {})
        if ann:
            new["metadata"]["annotations"] = {**(cur["metadata"].get("annotations") or {}), **ann}
        st = new["status"] = dict(cur.get("status") or {})
        st["conditions"] = list(st.get("conditions") or []) + [
            {"type": "PodScheduled", "status": "True", "lastTransitionTime": _now_iso()}]
        new["metadata"]["resourceVersion"] = self._bump()
        self.store["pods"][(ns, name)] = new
        self._emit("pods", "MODIFIED", new)

    def delete(self, kind: str, ns: str, name: str, grace: float | None = None, uid: str = "") -> dict:
        """DELETE as kube-apiserver answers it.  A bound pod that is not terminal is deleted gracefully: it gets
        ``deletionTimestamp`` and stays until a delete with grace 0 (its kubelet's, once the containers stopped).
        ``grace`` None takes the pod's ``spec.terminationGracePeriodSeconds`` (absent: 0 -- the pods the tests build
        carry none, and a delete without a grace was immediate in every round so far)."""
        cur = self._get(kind, ns, name)
        if uid and uid != cur["metadata"].get("uid"):
            raise HTTPError(409, status_body(
                409, "Conflict", f"Precondition failed: UID in precondition: {uid}, "
                                 f"UID in object meta: {cur['metadata'].get('uid')}"))
        key = (ns if kind != "nodes" else "", name)
        if kind == "pods" and grace is None:
            grace = float((cur.get("spec") or {}).get("terminationGracePeriodSeconds") or 0)
        phase = (cur.get("status") or {}).get("phase", "")
        if (kind == "pods" and grace and grace > 0 and (cur.get("spec") or {}).get("nodeName")
                and phase not in ("Succeeded", "Failed")):
            if cur["metadata"].get("deletionTimestamp"):
                return cur
            new = dict(cur)
            new["metadata"] = dict(cur["metadata"])
            new["metadata"]["deletionTimestamp"] = _now_iso()
            new["metadata"]["deletionGracePeriodSeconds"] = int(grace)
            new["metadata"]["resourceVersion"] = self._bump()
            self.store[kind][key] = new
            self._emit(kind, "MODIFIED", new)
            return new
        del self.store[kind][key]
        gone = dict(cur)
        gone["metadata"] = dict(cur["metadata"])
        gone["metadata"]["resourceVersion"] = self._bump()
        self._emit(kind, "DELETED", gone)
        return gone

    def list(self, kind: str, ns: str = "", fsel: str = "", lsel: str = "") -> list[dict]:
        out = []
        for (ons, _), o in self.store[kind].items():
            if ns and ons != ns:
                continue
            if _field_match(o, fsel) and _label_match(o, lsel):
                out.append(o)
        return out

    # ------------------------------------------------------------ HTTP
    def _make_app(self) -> Server:
        srv = Server()
        r = srv.route
        w = self._wrap
        r("GET", "/version", w(self.h_version))
        r("GET", "/healthz", w(self.h_healthz))
        r("GET", "/api", w(self.h_api))
        for kind in ("pods", "events"):
            r("GET", f"/api/v1/{kind}", w(self._mk_list(kind)))
            r("GET", f"/api/v1/namespaces/{{ns}}/{kind}", w(self._mk_list(kind)))
            r("POST", f"/api/v1/namespaces/{{ns}}/{kind}", w(self._mk_create(kind)))
            r("DELETE", f"/api/v1/namespaces/{{ns}}/{kind}", w(self._mk_delete_collection(kind)))
            r("GET", f"/api/v1/namespaces/{{ns}}/{kind}/{{name}}", w(self._mk_get(kind)))
            r("PUT", f"/api/v1/namespaces/{{ns}}/{kind}/{{name}}", w(self._mk_put(kind, "")))
            r("PATCH", f"/api/v1/namespaces/{{ns}}/{kind}/{{name}}", w(self._mk_patch(kind, "")))
            r("DELETE", f"/api/v1/namespaces/{{ns}}/{kind}/{{name}}", w(self._mk_delete(kind)))
        r("PUT", "/api/v1/namespaces/{ns}/pods/{name}/status", w(self._mk_put("pods", "status")))
        r("PATCH", "/api/v1/namespaces/{ns}/pods/{name}/status", w(self._mk_patch("pods", "status")))
        r("POST", "/api/v1/namespaces/{ns}/pods/{name}/binding", w(self.h_binding))
        r("POST", "/api/v1/namespaces/{ns}/bindings", w(self.h_bindings))
        r("GET", "/api/v1/nodes", w(self._mk_list("nodes")))
        r("POST", "/api/v1/nodes", w(self._mk_create("nodes")))
        r("GET", "/api/v1/nodes/{name}", w(self._mk_get("nodes")))
        r("PUT", "/api/v1/nodes/{name}", w(self._mk_put("nodes", "")))
        r("PATCH", "/api/v1/nodes/{name}", w(self._mk_patch("nodes", "")))
        r("PUT", "/api/v1/nodes/{name}/status", w(self._mk_put("nodes", "status")))
        r("PATCH", "/api/v1/nodes/{name}/status", w(self._mk_patch("nodes", "status")))
        r("DELETE", "/api/v1/nodes/{name}", w(self._mk_delete("nodes")))
        lease = "/apis/coordination.k8s.io/v1/namespaces/{ns}/leases"
        r("GET", lease, w(self._mk_list("leases")))
        r("POST", lease, w(self._mk_create("leases")))
        r("GET", lease + "/{name}", w(self._mk_get("leases")))
        r("PUT", lease + "/{name}", w(self._mk_put("leases", "")))
        r("DELETE", lease + "/{name}", w(self._mk_delete("leases")))
        r("GET", "/fake/faults", w(self.h_faults_get))
        r("POST", "/fake/faults", w(self.h_faults))
        r("GET", "/fake/stats", w(self.h_stats))
        return srv

    def _wrap(self, handler):
        """Request accounting + injected latency (what an aiohttp middleware did)."""
        async def slow(request):
            await asyncio.sleep(self.faults.latency_ms / 1000.0)
            res = handler(request)
            # (a plain handler may hand back a coroutine too: the list handler's watch stream)
            return await res if asyncio.iscoroutine(res) else res

        def h(request):
            self.counts[request.method] += 1
            watch = request.query.get("watch") in ("1", "true")
            if (self.faults.throttle_rate and not watch and request.path.startswith("/api/v1/")
                    and self.faults.rng.random() < self.faults.throttle_rate):
                self.counts["injected_throttle"] += 1
                ra = self.faults.retry_after
                return Response(json.dumps(status_body(429, "TooManyRequests", "Too many requests, please try again "
                                                       "later.", {"retryAfterSeconds": int(ra)})).encode(), 429,
                                headers={"Retry-After": f"{ra:g}"})
            if self.faults.latency_ms and not watch:
                return slow(request)
            return handler(request)
        return h

    def _json(self, obj, status=200) -> Response:
        last = self._last
        if last is not None and last[0] is obj:
            return Response(last[1], status)
        return Response(json.dumps(obj, separators=(",", ":")).encode(), status)

    def h_version(self, request):
        return self._json({"major": "1", "minor": "30", "gitVersion": "v1.30.0-gsx-fake", "platform": "linux/amd64"})

    def h_healthz(self, request):
        return Response(b"ok", 200, "text/plain")

    def h_api(self, request):
        return self._json({"kind": "APIVersions", "versions": ["v1"]})

    def h_faults_get(self, request):
        return self._json(self.faults.as_dict())

    def h_faults(self, request):
        d = request.json() or {}
        self.faults.update(d)
        if d.get("drop_watches_now"):  # one-shot: end every open watch stream
            for w in list(self.watchers):
                w.finish()
        return self._json(self.faults.as_dict())

    def h_stats(self, request):
        return self._json({"rv": self.rv, "counts": dict(self.counts), "watchers": len(self.watchers),
                           **{k: len(v) for k, v in self.store.items()}})

    def _maybe_error(self):
        if self.faults.error_rate and self.faults.rng.random() < self.faults.error_rate:
            self.counts["injected_error"] += 1
            raise HTTPError(500, status_body(500, "InternalError", "injected fault"))

    def _mk_list(self, kind):
        lists = {"pods": "PodList", "nodes": "NodeList", "events": "EventList", "leases": "LeaseList"}

        def h(request: Request):
            q = request.query
            ns = request.match_info.get("ns", "")
            fsel = q.get("fieldSelector", "")
            lsel = q.get("labelSelector", "")
            if q.get("watch") in ("1", "true"):
                return self._watch(request, kind, ns, fsel, lsel, q.get("resourceVersion", ""))
            if self.faults.fail_lists:
                self.counts["list_failed"] += 1
                raise HTTPError(503, status_body(503, "ServiceUnavailable", "injected: LIST unavailable"))
            items = self.list(kind, ns, fsel, lsel)
            md = {"resourceVersion": str(self.rv)}
            # pagination (kube-apiserver limit / continue): key order, "<rv>:<ns>/<name>" resumes after an item
            cont = q.get("continue", "")
            limit = int(q.get("limit", "0") or 0)
            if cont or limit > 0:
                items.sort(key=_obj_key)
            if cont:
                rv_s, _, last = cont.partition(":")
                md["resourceVersion"] = rv_s
                items = [o for o in items if _obj_key(o) > tuple(last.split("/", 1))]
            if limit > 0 and len(items) > limit:
                items = items[:limit]
                md["continue"] = f"{md['resourceVersion']}:{'/'.join(_obj_key(items[-1]))}"
            return self._json({"kind": lists[kind], "apiVersion": "v1", "metadata": md, "items": items})
        return h

    async def _watch(self, request, kind, ns, fsel, lsel, rv_s):
        w = _Watcher(kind, ns, fsel, lsel)
        out = Stream(request.transport)
        while self.faults.hold_watches:
            await asyncio.sleep(0.005)
        if self.faults.expire_watches > 0:
            self.faults.expire_watches -= 1
            self.counts["watch_expired"] += 1
            err = {"type": "ERROR", "object": status_body(410, "Expired", "too old resource version (injected)")}
            out.write(json.dumps(err).encode() + b"\n")
            return out
        backlog = []
        if rv_s not in ("", "0"):
            try:
                rv = int(rv_s)
            except ValueError:
                rv = 0
            if self.oldest_rv and rv < self.oldest_rv:
                err = {"type": "ERROR", "object": status_body(
                    410, "Expired", f"too old resource version: {rv} ({self.oldest_rv})")}
                out.write(json.dumps(err).encode() + b"\n")
                return out
            for (erv, k, _et, line, obj) in self.history:
                if erv > rv and k == kind and w.wants(obj):
                    backlog.append(line)
        else:
            for o in self.list(kind, ns, fsel, lsel):
                backlog.append(json.dumps({"type": "ADDED", "object": o}, separators=(",", ":")).encode() + b"\n")
        self.watchers.append(w)
        try:
            out.start()
            w.drop_after = self.faults.drop_watch_after
            w.on_drop = lambda: self.counts.__setitem__("watch_dropped", self.counts["watch_dropped"] + 1)
            w.pending[:0] = backlog
            w.go_live(out)
            timeout = float(request.query.get("timeoutSeconds", "0") or 0) or None
            deadline = time.monotonic() + timeout if timeout else None
            while not w.closed:
                rem = None if deadline is None else deadline - time.monotonic()
                if rem is not None and rem <= 0:
                    break
                # events are pushed by _emit; this only watches for the end of the stream
                await asyncio.wait([w.done], timeout=1.0 if rem is None else min(rem, 1.0))
                if request.closed or out.closed:
                    break  # client went away
        finally:
            w.closed = True
            try:
                self.watchers.remove(w)
            except ValueError:
                pass
        return out

    def _mk_create(self, kind):
        def h(request):
            body = request.json()
            if kind == "pods":
                self._maybe_error()
            return self._json(self.create(kind, body, request.match_info.get("ns")), 201)
        return h

    def _mk_get(self, kind):
        def h(request):
            return self._json(self._get(kind, request.match_info.get("ns", ""), request.match_info["name"]))
        return h

    def _mk_put(self, kind, sub):
        def h(request):
            body = request.json()
            if kind == "pods":
                self._maybe_error()
            return self._json(self.replace(kind, request.match_info.get("ns", ""), request.match_info["name"], body,
                                           sub))
        return h

    def _mk_patch(self, kind, sub):
        def h(request):
            ct = request.headers.get("content-type", "")
            if "json-patch+json" in ct:
                return self._json(status_body(415, "UnsupportedMediaType", "json-patch not supported"), 415)
            body = request.json()
            if kind == "pods":
                self._maybe_error()
            return self._json(self.patch(kind, request.match_info.get("ns", ""), request.match_info["name"], body,
                                         sub))
        return h

    @staticmethod
    def _delete_options(request) -> tuple[float | None, str]:
        """(gracePeriodSeconds, preconditions.uid) from the query or the DeleteOptions body."""
        grace, uid = None, ""
        if request.body:
            try:
                b = request.json()
            except ValueError:
                b = None
            if isinstance(b, dict):
                if b.get("gracePeriodSeconds") is not None:
                    grace = float(b["gracePeriodSeconds"])
                uid = ((b.get("preconditions") or {}).get("uid")) or ""
        if "gracePeriodSeconds" in request.query:
            grace = float(request.query["gracePeriodSeconds"])
        return grace, uid

    @classmethod
    def _grace(cls, request):
        return cls._delete_options(request)[0]

    def _mk_delete(self, kind):
        def h(request):
            grace, uid = self._delete_options(request)
            obj = self.delete(kind, request.match_info.get("ns", ""), request.match_info["name"], grace, uid)
            return self._json(obj)
        return h

    def _mk_delete_collection(self, kind):
        """DELETE /api/v1/namespaces/{ns}/pods?labelSelector=... (kubectl delete pods -l ...)."""
        def h(request):
            ns = request.match_info.get("ns", "")
            q = request.query
            grace = self._grace(request)
            items = [self.delete(kind, ns, o["metadata"]["name"], grace)
                     for o in self.list(kind, ns, q.get("fieldSelector", ""), q.get("labelSelector", ""))]
            return self._json({"kind": "PodList", "apiVersion": "v1", "metadata": {}, "items": items})
        return h

    def h_binding(self, request):
        body = request.json()
        delay = self.faults.slow_bindings.get(request.match_info["name"], 0.0)
        if delay:
            async def later():
                await asyncio.sleep(delay / 1000.0)
                return self._do_binding(request, body)
            return later()
        return self._do_binding(request, body)

    def _do_binding(self, request, body):
        self._maybe_error()
        self.bind(request.match_info["ns"], request.match_info["name"], body)
        self.binding_log.append(request.match_info["name"])
        return self._json({"kind": "Status", "apiVersion": "v1", "metadata": {}, "status": "Success", "code": 201}, 201)

    def h_bindings(self, request):
        body = request.json()
        self._maybe_error()
        self.bind(request.match_info["ns"], (body.get("metadata") or {}).get("name", ""), body)
        return self._json({"kind": "Status", "apiVersion": "v1", "metadata": {}, "status": "Success", "code": 201}, 201)


class FakeApiServerRunner:
    """Start/stop helper on the current event loop (tests) or in its own process (``main``)."""

    def __init__(self, server: FakeApiServer | None = None, host: str = "127.0.0.1", port: int = 0):
        self.server = server or FakeApiServer()
        self.host = host
        self.port = port

    @property
    def url(self) -> str:
        return f"http://{self.host}:{self.port}"

    async def start(self) -> "FakeApiServerRunner":
        self.port = await self.server.app.start(self.host, self.port)
        return self

    async def stop(self):
        for w in list(self.server.watchers):
            w.finish()
        await asyncio.sleep(0)
        await self.server.app.stop()


def main(argv=None):
    ap = argparse.ArgumentParser(description="fake kube-apiserver for gpushare tests/bench")
    ap.add_argument("--host", default="127.0.0.1")
    ap.add_argument("--port", type=int, default=0)
    ap.add_argument("--port-file", default="", help="write the bound port here once listening")
    ap.add_argument("--seed-json", default="", help="JSON file with {'nodes':[...],'pods':[...]} to preload")
    a = ap.parse_args(argv)
    logging.basicConfig(level=logging.WARNING)

    async def run():
        srv = FakeApiServer()
        if a.seed_json:
            with open(a.seed_json) as f:
                seed = json.load(f)
            for n in seed.get("nodes", []):
                srv.create("nodes", n)
            for p in seed.get("pods", []):
                srv.create("pods", p)
        r = await FakeApiServerRunner(srv, a.host, a.port).start()
        if a.port_file:
            with open(a.port_file + ".tmp", "w") as f:
                f.write(str(r.port))
            import os  # noqa: PLC0415

            os.replace(a.port_file + ".tmp", a.port_file)
        print(f"fake-apiserver listening on {r.url}", flush=True)
        from ..utils.gctune import tune  # noqa: PLC0415

        tune()
        await asyncio.Event().wait()

    try:
        asyncio.run(run())
    except KeyboardInterrupt:
        pass


if __name__ == "__main__":
    main()
