"""Reflector / indexer / informer on top of :class:`KubeClient` (client-go equivalent).

The reference gets pods and nodes through a ``SharedInformerFactory`` with a
30 s resync (``cmd/main.go:28,103``) and reads them through listers
(``pkg/cache/cache.go:76-78,130-133``).  This informer keeps the same model:

* LIST, then WATCH from the list's ``resourceVersion``; on a dropped stream it
  re-watches from the last seen version; on ``410 Gone`` it re-lists and
  diffs the store, emitting adds / updates / deletes (tombstones included);
* an in-memory store keyed ``namespace/name`` (``DeletionHandlingMetaNamespaceKeyFunc``,
  ``pkg/gpushare/controller.go:26-28``) that doubles as the lister;
* handlers get the decoded object and, for watch events, the raw JSON line so
  the native engine can parse pods without a Python round trip;
* optional periodic resync that re-delivers every object as an update;
* optional event filter (``FilteringResourceEventHandler``,
  ``pkg/gpushare/controller.go:77-100``).
"""
from __future__ import annotations

import asyncio
import json
import logging
import time
from typing import Callable

from .client import ApiError, KubeClient

log = logging.getLogger("gsx.informer")


def obj_key(obj: dict) -> str:
    md = obj.get("metadata") or {}
    ns = md.get("namespace")
    return f"{ns}/{md.get('name', '')}" if ns else md.get("name", "")


class Handler:
    """on_add(obj, raw), on_update(old, new, raw), on_delete(obj, raw); raw may be None."""

    def __init__(self, on_add=None, on_update=None, on_delete=None, filter_fn: Callable | None = None):
        self.on_add = on_add
        self.on_update = on_update
        self.on_delete = on_delete
        self.filter_fn = filter_fn

    def _ok(self, obj) -> bool:
        return self.filter_fn is None or self.filter_fn(obj)

    def add(self, obj, raw):
        if self.on_add and self._ok(obj):
            self.on_add(obj, raw)

    def update(self, old, new, raw):
        # FilteringResourceEventHandler semantics: transitions in/out of the
        # filter become add / delete.
        if self.filter_fn is None:
            if self.on_update:
                self.on_update(old, new, raw)
            return
        was, now = self.filter_fn(old), self.filter_fn(new)
        if was and now:
            if self.on_update:
                self.on_update(old, new, raw)
        elif now:
            if self.on_add:
                self.on_add(new, raw)
        elif was:
            if self.on_delete:
                self.on_delete(old, None)

    def delete(self, obj, raw):
        if self.on_delete and self._ok(obj):
            self.on_delete(obj, raw)


class Informer:
    def __init__(self, client: KubeClient, kind: str, namespace: str | None = None, field_selector: str = "",
                 label_selector: str = "", resync_period: float = 0.0, watch_timeout: int = 300,
                 page_size: int = 500):
        self.client = client
        self.kind = kind
        self.namespace = namespace
        self.field_selector = field_selector
        self.label_selector = label_selector
        self.resync_period = resync_period
        self.watch_timeout = watch_timeout
        self.page_size = page_size  # LIST in pages (limit / continue); 0 = one request
        self.store: dict[str, dict] = {}
        self.handlers: list[Handler] = []
        self.last_rv = ""
        self.synced = asyncio.Event()
        self._tasks: list[asyncio.Task] = []
        self._stopped = False
        self.relists = 0
        self.rewatches = 0
        self.events = 0
        self.bookmarks = 0
        self.last_list_start = 0.0  # time.monotonic() when the last applied LIST was sent
        self._relist = False
        self._watch_task: asyncio.Task | None = None

    # lister API
    def get(self, key: str) -> dict | None:
        return self.store.get(key)

    def get_by(self, name: str, namespace: str | None = None) -> dict | None:
        return self.store.get(f"{namespace}/{name}" if namespace else name)

    def list(self) -> list[dict]:
        return list(self.store.values())

    def add_handler(self, h: Handler):
        self.handlers.append(h)
        if self.synced.is_set():
            for o in list(self.store.values()):
                h.add(o, None)

    async def start(self):
        self._tasks.append(asyncio.get_running_loop().create_task(self._run(), name=f"informer-{self.kind}"))
        if self.resync_period > 0:
            self._tasks.append(asyncio.get_running_loop().create_task(self._resync_loop()))

    async def wait_synced(self, timeout: float | None = None):
        await asyncio.wait_for(self.synced.wait(), timeout)

    async def stop(self):
        self._stopped = True
        for t in self._tasks:
            t.cancel()
        for t in self._tasks:
            try:
                await t
            except (asyncio.CancelledError, Exception):  # noqa: BLE001
                pass
        self._tasks.clear()

    # internals
    def _dispatch(self, etype: str, obj: dict, raw: bytes | None):
        if etype == "BOOKMARK":  # progress marker: only the resourceVersion to resume from
            self.bookmarks += 1
            rv = (obj.get("metadata") or {}).get("resourceVersion")
            if rv:
                self.last_rv = rv
            return
        key = obj_key(obj)
        self.events += 1
        if etype == "ADDED" or etype == "MODIFIED":
            old = self.store.get(key)
            self.store[key] = obj
            for h in self.handlers:
                if old is None:
                    h.add(obj, raw)
                else:
                    h.update(old, obj, raw)
        elif etype == "DELETED":
            old = self.store.pop(key, None)
            for h in self.handlers:
                h.delete(old if old is not None else obj, raw)
        rv = (obj.get("metadata") or {}).get("resourceVersion")
        if rv:
            self.last_rv = rv

    def request_relist(self):
        """End the current watch (also one the apiserver never answered) and LIST again."""
        self._relist = True
        if self._watch_task is not None and not self._watch_task.done():
            self._watch_task.cancel()

    async def _list(self):
        started = time.monotonic()
        lst = await self.client.list(self.kind, self.namespace, self.field_selector, self.label_selector,
                                     page_size=self.page_size)
        items = lst.get("items") or []
        new = {obj_key(o): o for o in items}
        old = self.store
        self.store = {}
        # deletes for objects that disappeared while we were not watching
        for k, o in old.items():
            if k not in new:
                for h in self.handlers:
                    h.delete(o, None)
        for k, o in new.items():
            self.store[k] = o
            prev = old.get(k)
            for h in self.handlers:
                if prev is None:
                    h.add(o, None)
                elif (prev.get("metadata") or {}).get("resourceVersion") != (o.get("metadata") or {}).get(
                        "resourceVersion"):
                    h.update(prev, o, None)
        self.last_rv = (lst.get("metadata") or {}).get("resourceVersion", "")
        self.relists += 1
        self.last_list_start = started

    async def _watch_once(self):
        async for ev, raw in self.client.watch(self.kind, self.namespace, self.last_rv, self.field_selector,
                                               self.label_selector, self.watch_timeout, raw=True, bookmarks=True):
            self._dispatch(ev["type"], ev["object"], raw)

    async def _run(self):
        backoff = 0.05
        need_list = True
        while not self._stopped:
            try:
                if self._relist:
                    self._relist = False
                    need_list = True
                if need_list:
                    await self._list()
                    need_list = False
                    self.synced.set()
                # the watch runs in its own task so request_relist() can end it without ending the informer
                self._watch_task = asyncio.get_running_loop().create_task(self._watch_once())
                try:
                    await self._watch_task
                except asyncio.CancelledError:
                    if not self._relist or self._stopped:
                        raise
                    continue
                finally:
                    self._watch_task = None
                backoff = 0.05
                self.rewatches += 1
            except asyncio.CancelledError:
                raise
            except ApiError as e:
                if e.gone:
                    log.info("%s watch: resourceVersion expired, re-listing", self.kind)
                    need_list = True
                    continue
                log.warning("%s informer error: %s", self.kind, e)
                await asyncio.sleep(backoff)
                backoff = min(5.0, backoff * 2)
            except Exception as e:  # noqa: BLE001 - connection errors: retry with backoff
                if self._stopped:
                    return
                log.warning("%s informer connection error: %r", self.kind, e)
                await asyncio.sleep(backoff)
                backoff = min(5.0, backoff * 2)

    async def _resync_loop(self):
        while not self._stopped:
            await asyncio.sleep(self.resync_period)
            for o in list(self.store.values()):
                for h in self.handlers:
                    h.update(o, o, None)


def dumps(obj) -> bytes:
    return json.dumps(obj, separators=(",", ":")).encode()
