"""Event-driven view of a set of pods for load generators (the benchmark's wave driver).

An informer on pods (optionally label-selected) plus bare-future waits that
wake on every event, so "all bound", "all Running" and "all gone" are checked
when the apiserver says something changed, never by polling.
"""
from __future__ import annotations

import asyncio
import time

from ..k8s.client import KubeClient
from ..k8s.informer import Handler, Informer


class PodTracker:
    def __init__(self, client: KubeClient, namespace: str | None = None, label_selector: str = ""):
        self.pods = Informer(client, "pods", namespace=namespace, label_selector=label_selector)
        self._waiters: list[asyncio.Future] = []
        self.pods.add_handler(Handler(lambda o, r: self._notify(), lambda o, n, r: self._notify(),
                                      lambda o, r: self._notify()))

    def _notify(self):
        ws, self._waiters = self._waiters, []
        for f in ws:
            if not f.done():
                f.set_result(None)

    async def start(self):
        await self.pods.start()
        await self.pods.wait_synced(30)

    async def stop(self):
        await self.pods.stop()

    def get(self, key: str) -> dict | None:
        return self.pods.get(key)

    async def wait_for(self, cond, timeout: float = 30.0):
        loop = asyncio.get_running_loop()
        deadline = time.perf_counter() + timeout
        while not cond():
            rem = deadline - time.perf_counter()
            if rem <= 0:
                raise TimeoutError("condition not reached")
            f = loop.create_future()
            self._waiters.append(f)
            h = loop.call_later(min(rem, 0.05), lambda: f.done() or f.set_result(None))
            try:
                await f
            finally:
                h.cancel()
