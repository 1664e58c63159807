"""Minimal asynchronous Kubernetes REST + watch client.

Replaces the reference's client-go usage (``cmd/main.go:67-86``,
``pkg/gpushare/controller.go``, ``pkg/cache/nodeinfo.go:150-189``).  There is
no ``kubernetes`` Python package in this image, and the extender needs only a
handful of core/v1 verbs, so this is a small hand-written client on
:mod:`.fasthttp` (raw asyncio streams, keep-alive pool):

* config from ``KUBECONFIG`` (token / client-cert / CA / insecure), the
  in-cluster service account, or an explicit base URL (fake apiserver);
* a token-bucket rate limiter with configurable QPS / burst.  client-go's
  defaults of 5 / 10 (``vendor/k8s.io/client-go/rest/config.go:43-44``) are
  what cap the reference at ~2.5 binds/s; ours default far higher and are
  flags of the extender;
* typed errors carrying the HTTP status so conflicts are detected by ``409``
  rather than by comparing message strings (``pkg/cache/nodeinfo.go:153``);
* client-go's retry contract (``vendor/k8s.io/client-go/rest/request.go:658-734,973-995``): a ``429 Too Many
  Requests`` -- API Priority and Fairness rejected the request before it ran, so every verb is safe to repeat -- or
  a 5xx carrying ``Retry-After`` is sent again after the server's ``Retry-After``, up to 10 sends; a 429 without
  it waits a capped exponential backoff with jitter.  A 5xx without ``Retry-After`` goes to the caller (a write
  may have been applied; the caller knows whether repeating it is safe), as in client-go;
* streaming watches yielding decoded events, with ``410 Gone`` surfaced as
  :class:`ApiError` so reflectors re-list.
"""
from __future__ import annotations

import asyncio
import base64
import json
import logging
import os
import random
import ssl
import tempfile
import time
from dataclasses import dataclass, field
from typing import AsyncIterator
from urllib.parse import quote, urlencode

from .fasthttp import Client

import yaml

SA_DIR = "/var/run/secrets/kubernetes.io/serviceaccount"
log = logging.getLogger("gsx.k8s")


class ApiError(Exception):
    def __init__(self, status: int, reason: str = "", message: str = "", body=None):
        super().__init__(f"{status} {reason}: {message}")
        self.status = status
        self.reason = reason
        self.message = message
        self.body = body

    @property
    def conflict(self) -> bool:
        return self.status == 409

    @property
    def not_found(self) -> bool:
        return self.status == 404

    @property
    def gone(self) -> bool:
        return self.status == 410

    @property
    def throttled(self) -> bool:
        return self.status == 429

    @property
    def transient(self) -> bool:
        """Worth repeating later: a conflict (re-read and retry), throttling, or a server-side error."""
        return self.status in (409, 429) or self.status >= 500


def retry_wait(status: int, retry_after: str | None, attempt: int, max_attempts: int = 10,
               backoff_base: float = 0.005, backoff_max: float = 1.0, retry_after_max: float = 30.0,
               jitter: float | None = None) -> float | None:
    """Seconds to wait before sending a request again that was answered ``status`` (with header ``retry_after``) on
    send ``attempt`` (0-based); None: do not retry.  The native twin is ``ApiClient::retry_wait``
    (``native/engine/apiclient.cc``)."""
    if attempt + 1 >= max_attempts or (status != 429 and status < 500):
        return None
    if retry_after:
        try:
            s = float(retry_after)
        except ValueError:
            s = -1.0  # an HTTP-date: treated as absent
        if s >= 0:
            return min(s, retry_after_max)
    if status != 429:
        return None
    b = min(backoff_max, backoff_base * 2 ** min(attempt, 20))
    return b * (0.5 + 0.5 * (random.random() if jitter is None else jitter))


class RateLimiter:
    """Token bucket (client-go flowcontrol.NewTokenBucketRateLimiter semantics). qps<=0 disables."""

    def __init__(self, qps: float, burst: int):
        self.qps = float(qps)
        self.burst = max(1, int(burst))
        self.tokens = float(self.burst)
        self.last = time.monotonic()
        self._lock = asyncio.Lock()

    async def acquire(self):
        if self.qps <= 0:
            return
        async with self._lock:
            now = time.monotonic()
            self.tokens = min(self.burst, self.tokens + (now - self.last) * self.qps)
            self.last = now
            if self.tokens >= 1:
                self.tokens -= 1
                return
            wait = (1 - self.tokens) / self.qps
            self.tokens = 0.0
            self.last = now + wait
            await asyncio.sleep(wait)


@dataclass
class KubeConfig:
    server: str
    token: str | None = None
    ca_file: str | None = None
    cert_file: str | None = None
    key_file: str | None = None
    insecure: bool = False
    extra_headers: dict = field(default_factory=dict)
    # projected service-account tokens are rotated by kubelet: re-read this file (client-go does the same)
    token_file: str | None = None
    token_reload_s: float = 60.0
    _token_read_at: float = field(default=0.0, repr=False)

    def current_token(self) -> str | None:
        """The bearer token, re-read from ``token_file`` at most every ``token_reload_s`` (a failed read keeps
        the last one)."""
        if self.token_file and time.monotonic() - self._token_read_at >= self.token_reload_s:
            self._token_read_at = time.monotonic()
            try:
                with open(self.token_file) as f:
                    self.token = f.read().strip() or self.token
            except OSError as e:
                log.warning("re-reading token file %s: %s", self.token_file, e)
        return self.token

    @classmethod
    def from_url(cls, url: str) -> "KubeConfig":
        return cls(server=url.rstrip("/"))

    @classmethod
    def in_cluster(cls) -> "KubeConfig":
        host = os.environ.get("KUBERNETES_SERVICE_HOST")
        port = os.environ.get("KUBERNETES_SERVICE_PORT", "443")
        if not host:
            raise RuntimeError("not running in a cluster (KUBERNETES_SERVICE_HOST unset)")
        token_file = os.path.join(SA_DIR, "token")
        with open(token_file) as f:
            token = f.read().strip()
        if ":" in host:
            host = f"[{host}]"
        return cls(server=f"https://{host}:{port}", token=token, ca_file=os.path.join(SA_DIR, "ca.crt"),
                   token_file=token_file, _token_read_at=time.monotonic())

    @classmethod
    def from_kubeconfig(cls, path: str, context: str | None = None) -> "KubeConfig":
        with open(path) as f:
            kc = yaml.safe_load(f) or {}
        ctx_name = context or kc.get("current-context")
        ctxs = {c["name"]: c["context"] for c in kc.get("contexts") or []}
        if ctx_name not in ctxs:
            if len(ctxs) == 1:
                ctx_name = next(iter(ctxs))
            else:
                raise ValueError(f"kubeconfig {path}: context {ctx_name!r} not found")
        ctx = ctxs[ctx_name]
        clusters = {c["name"]: c["cluster"] for c in kc.get("clusters") or []}
        users = {u["name"]: u.get("user") or {} for u in kc.get("users") or []}
        cl = clusters[ctx["cluster"]]
        us = users.get(ctx.get("user"), {})
        base = os.path.dirname(os.path.abspath(path))

        def _file(data_key, file_key, src):
            if src.get(data_key):
                fd, p = tempfile.mkstemp(prefix="gsx-kc-")
                with os.fdopen(fd, "wb") as f:
                    f.write(base64.b64decode(src[data_key]))
                return p
            if src.get(file_key):
                p = src[file_key]
                return p if os.path.isabs(p) else os.path.join(base, p)
            return None

        token = us.get("token")
        token_file = None
        if not token and us.get("tokenFile"):
            token_file = us["tokenFile"] if os.path.isabs(us["tokenFile"]) else os.path.join(base, us["tokenFile"])
            with open(token_file) as f:
                token = f.read().strip()
        headers = {}
        if us.get("username") and us.get("password"):
            headers["Authorization"] = "Basic " + base64.b64encode(
                f"{us['username']}:{us['password']}".encode()).decode()
        return cls(server=cl["server"].rstrip("/"), token=token, token_file=token_file,
                   _token_read_at=time.monotonic(),
                   ca_file=_file("certificate-authority-data", "certificate-authority", cl),
                   cert_file=_file("client-certificate-data", "client-certificate", us),
                   key_file=_file("client-key-data", "client-key", us),
                   insecure=bool(cl.get("insecure-skip-tls-verify")), extra_headers=headers)

    @classmethod
    def auto(cls, kubeconfig: str | None = None, server: str | None = None) -> "KubeConfig":
        """cmd/main.go:67-86 order: explicit server, then $KUBECONFIG, then in-cluster."""
        if server:
            return cls.from_url(server)
        path = kubeconfig or os.environ.get("KUBECONFIG")
        if path and os.path.exists(path):
            return cls.from_kubeconfig(path)
        return cls.in_cluster()

    def ssl_context(self):
        if not self.server.startswith("https"):
            return None
        if self.insecure:
            ctx = ssl.create_default_context()
            ctx.check_hostname = False
            ctx.verify_mode = ssl.CERT_NONE
        else:
            ctx = ssl.create_default_context(cafile=self.ca_file) if self.ca_file else ssl.create_default_context()
        if self.cert_file and self.key_file:
            ctx.load_cert_chain(self.cert_file, self.key_file)
        return ctx


def _ns_path(kind: str, ns: str | None, name: str | None = None, sub: str | None = None) -> str:
    if kind == "leases":
        p = f"/apis/coordination.k8s.io/v1/namespaces/{quote(ns or 'default', safe='')}/leases"
    elif kind == "nodes":
        p = "/api/v1/nodes"
    elif ns:
        p = f"/api/v1/namespaces/{quote(ns, safe='')}/{kind}"
    else:
        p = f"/api/v1/{kind}"
    if name:
        p += "/" + quote(name, safe="")
    if sub:
        p += "/" + sub
    return p


class KubeClient:
    def __init__(self, config: KubeConfig | str, qps: float = 0.0, burst: int = 1000,
                 user_agent: str = "gpushare-schd-extender-amd/0.1.0", connector_limit: int = 256,
                 max_attempts: int = 10):
        self.config = KubeConfig.from_url(config) if isinstance(config, str) else config
        self.max_attempts = max(1, int(max_attempts))  # sends per request under 429 / Retry-After (1: no retry)
        self.throttled = 0  # responses sent again after a 429 / Retry-After
        self.throttle_wait_s = 0.0
        self.limiter = RateLimiter(qps, burst)
        self.user_agent = user_agent
        self._limit = connector_limit
        self._http: Client | None = None
        self._sent_token: str | None = None
        self.calls = 0

    def _client(self) -> Client:
        token = self.config.current_token()
        if self._http is None or self._http.closed:
            headers = {"User-Agent": self.user_agent, **self.config.extra_headers}
            if token:
                headers["Authorization"] = f"Bearer {token}"
            self._http = Client(self.config.server, ssl_context=self.config.ssl_context(), headers=headers,
                                limit=self._limit)
            self._sent_token = token
        elif token != self._sent_token:
            self._http.set_header("Authorization", f"Bearer {token}")
            self._sent_token = token
        return self._http

    async def close(self):
        if self._http is not None:
            await self._http.close()
            self._http = None

    async def __aenter__(self):
        return self

    async def __aexit__(self, *exc):
        await self.close()

    @staticmethod
    def _raise(status: int, raw: bytes):
        try:
            st = json.loads(raw)
            if not isinstance(st, dict):
                st = {"message": str(st)}
        except ValueError:
            st = {"message": raw.decode(errors="replace")}
        raise ApiError(status, st.get("reason", ""), st.get("message", ""), st)

    async def request(self, method: str, path: str, *, params: dict | None = None, body=None,
                      content_type: str = "application/json", timeout: float | None = 30.0):
        if params:
            path += "?" + urlencode(params)
        data = None
        if body is not None:
            data = body if isinstance(body, bytes) else (body.encode() if isinstance(body, str) else
                                                          json.dumps(body, separators=(",", ":")).encode())
        attempt = 0
        while True:
            if self.limiter.qps > 0:  # every send, retries too (client-go's tryThrottle)
                await self.limiter.acquire()
            self.calls += 1
            r = await self._client().request(method, path, data, content_type if data is not None else None,
                                             timeout=timeout)
            if r.status < 400:
                return json.loads(r.body) if r.body else None
            wait = retry_wait(r.status, (r.headers or {}).get("retry-after"), attempt, self.max_attempts)
            if wait is None:
                self._raise(r.status, r.body)
            self.throttled += 1
            self.throttle_wait_s += wait
            log.debug("%s %s answered %d: sending it again in %.3f s (attempt %d)", method, path, r.status, wait,
                      attempt + 1)
            await asyncio.sleep(wait)
            attempt += 1

    # ------------------------------------------------------------ verbs
    async def get(self, kind: str, name: str, ns: str | None = None) -> dict:
        return await self.request("GET", _ns_path(kind, ns, name))

    async def list(self, kind: str, ns: str | None = None, field_selector: str = "", label_selector: str = "",
                   resource_version: str = "", page_size: int = 0) -> dict:
        """One LIST; with ``page_size`` > 0 it is fetched in pages (``limit`` / ``continue``, client-go's
        pager) and returned assembled, at the first page's resourceVersion."""
        params = {}
        if field_selector:
            params["fieldSelector"] = field_selector
        if label_selector:
            params["labelSelector"] = label_selector
        if resource_version:
            params["resourceVersion"] = resource_version
        if page_size <= 0:
            return await self.request("GET", _ns_path(kind, ns), params=params, timeout=120)
        params["limit"] = str(page_size)
        out = await self.request("GET", _ns_path(kind, ns), params=params, timeout=120)
        items = list(out.get("items") or [])
        while (out.get("metadata") or {}).get("continue"):
            params["continue"] = out["metadata"]["continue"]
            out = await self.request("GET", _ns_path(kind, ns), params=params, timeout=120)
            items.extend(out.get("items") or [])
        first_md = dict(out.get("metadata") or {})
        first_md.pop("continue", None)
        return {**out, "metadata": first_md, "items": items}

    async def create(self, kind: str, obj: dict, ns: str | None = None) -> dict:
        ns = ns if ns is not None else (obj.get("metadata") or {}).get("namespace", "default")
        return await self.request("POST", _ns_path(kind, None if kind == "nodes" else ns), body=obj)

    async def replace(self, kind: str, obj: dict, sub: str | None = None) -> dict:
        md = obj["metadata"]
        return await self.request("PUT", _ns_path(kind, md.get("namespace"), md["name"], sub), body=obj)

    async def patch(self, kind: str, name: str, patch: dict, ns: str | None = None, sub: str | None = None,
                    patch_type: str = "merge") -> dict:
        ct = {"merge": "application/merge-patch+json",
              "strategic": "application/strategic-merge-patch+json"}[patch_type]
        return await self.request("PATCH", _ns_path(kind, ns, name, sub), body=patch, content_type=ct)

    async def delete(self, kind: str, name: str, ns: str | None = None, grace_seconds: float | None = None,
                     uid: str | None = None):
        """DELETE; ``uid`` adds a ``preconditions.uid`` (409 if the object under that name is another one), as
        kubelet's final grace-0 delete of a terminated pod does."""
        params = {"gracePeriodSeconds": str(int(grace_seconds))} if grace_seconds is not None else None
        body = None
        if uid:
            body = {"kind": "DeleteOptions", "apiVersion": "v1", "preconditions": {"uid": uid}}
            if grace_seconds is not None:
                body["gracePeriodSeconds"] = int(grace_seconds)
        return await self.request("DELETE", _ns_path(kind, ns, name), params=params, body=body)

    async def bind_pod(self, ns: str, name: str, node: str, uid: str | None = None,
                       annotations: dict | None = None) -> None:
        """POST pods/{name}/binding (vendor/.../typed/core/v1/pod_expansion.go:34-36).

        Binding annotations are copied onto the pod by kube-apiserver, so the
        allocation record and the node assignment land in one write.
        """
        md = {"name": name, "namespace": ns}
        if uid:
            md["uid"] = uid
        if annotations:
            md["annotations"] = annotations
        body = {"apiVersion": "v1", "kind": "Binding", "metadata": md,
                "target": {"apiVersion": "v1", "kind": "Node", "name": node}}
        await self.request("POST", _ns_path("pods", ns, name, "binding"), body=body)

    async def create_event(self, ns: str, involved: dict, reason: str, message: str, etype: str = "Normal",
                           component: str = "gpushare-schd-extender") -> dict | None:
        md = involved.get("metadata") or {}
        now = time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime())
        ev = {"apiVersion": "v1", "kind": "Event",
              "metadata": {"generateName": f"{md.get('name', 'obj')}.", "namespace": ns},
              "involvedObject": {"kind": involved.get("kind", "Pod"), "namespace": ns, "name": md.get("name"),
                                 "uid": md.get("uid"), "apiVersion": "v1",
                                 "resourceVersion": md.get("resourceVersion")},
              "reason": reason, "message": message, "type": etype, "source": {"component": component},
              "firstTimestamp": now, "lastTimestamp": now, "count": 1}
        return await self.create("events", ev, ns)

    async def watch(self, kind: str, ns: str | None = None, resource_version: str = "", field_selector: str = "",
                    label_selector: str = "", timeout_seconds: int = 0, raw: bool = False,
                    bookmarks: bool = False) -> AsyncIterator:
        """Yield watch events (dicts), or ``(event, raw_line_bytes)`` with ``raw=True``.  With ``bookmarks`` the
        apiserver may also send ``BOOKMARK`` events (metadata.resourceVersion only), which keep a re-watch after a
        timeout inside the history window instead of ending in 410 and a re-list."""
        params = {"watch": "true", "allowWatchBookmarks": "true" if bookmarks else "false"}
        if resource_version:
            params["resourceVersion"] = resource_version
        if field_selector:
            params["fieldSelector"] = field_selector
        if label_selector:
            params["labelSelector"] = label_selector
        if timeout_seconds:
            params["timeoutSeconds"] = str(timeout_seconds)
        if self.limiter.qps > 0:
            await self.limiter.acquire()
        self.calls += 1
        status, hdrs, chunks, close = await self._client().stream("GET", _ns_path(kind, ns) + "?" + urlencode(params))
        try:
            if status >= 400:
                self._raise(status, b"".join([c async for c in chunks]))
            buf = b""
            async for chunk in chunks:
                buf = buf + chunk if buf else chunk
                start = 0  # lines are cut from an offset: a chunk of many events is not re-copied once per event
                while True:
                    i = buf.find(b"\n", start)
                    if i < 0:
                        break
                    line, start = buf[start:i], i + 1
                    if not line.strip():
                        continue
                    ev = json.loads(line)
                    if ev.get("type") == "ERROR":
                        o = ev.get("object") or {}
                        raise ApiError(int(o.get("code", 500)), o.get("reason", ""), o.get("message", ""), o)
                    yield (ev, line) if raw else ev
                buf = buf[start:]
        finally:
            close()
