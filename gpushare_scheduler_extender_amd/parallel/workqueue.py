"""Rate-limited dedup work queue for asyncio.

Same contract as client-go's ``workqueue.RateLimitingInterface`` that the
reference controller uses (``pkg/gpushare/controller.go:71,209-231``):

* an item is queued at most once ("dirty" set), and never handed to two
  workers at the same time ("processing" set); re-adds while processing are
  replayed on :meth:`done`;
* :meth:`add_rate_limited` requeues after ``max(per-item exponential backoff,
  overall token bucket)`` — ``DefaultControllerRateLimiter`` is 5 ms doubling
  to 1000 s per item and 10 qps / burst 100 overall
  (``vendor/k8s.io/client-go/util/workqueue/default_rate_limiters.go:39-45``);
* :meth:`forget` resets an item's backoff.

Unlike the reference worker loop, which returns after every *successful* item
and then sleeps 1 s in ``wait.Until`` (``controller.go:218-223``, capping sync
at ≤1 item/s), workers here loop without idling.
"""
from __future__ import annotations

import asyncio
import collections
import time


class ItemExponentialBackoff:
    def __init__(self, base: float = 0.005, cap: float = 1000.0):
        self.base = base
        self.cap = cap
        self.failures: dict = collections.defaultdict(int)

    def when(self, item) -> float:
        n = self.failures[item]
        self.failures[item] = n + 1
        return min(self.cap, self.base * (2 ** n))

    def forget(self, item):
        self.failures.pop(item, None)

    def num_requeues(self, item) -> int:
        return self.failures.get(item, 0)


class BucketLimiter:
    def __init__(self, qps: float = 10.0, burst: int = 100):
        self.qps = qps
        self.burst = burst
        self.tokens = float(burst)
        self.last = time.monotonic()

    def when(self, item) -> float:
        now = time.monotonic()
        self.tokens = min(self.burst, self.tokens + (now - self.last) * self.qps)
        self.last = now
        self.tokens -= 1
        if self.tokens >= 0:
            return 0.0
        return -self.tokens / self.qps

    def forget(self, item):
        pass

    def num_requeues(self, item) -> int:
        return 0


class MaxOfLimiter:
    def __init__(self, *limiters):
        self.limiters = limiters

    def when(self, item) -> float:
        return max(lim.when(item) for lim in self.limiters)

    def forget(self, item):
        for lim in self.limiters:
            lim.forget(item)

    def num_requeues(self, item) -> int:
        return max(lim.num_requeues(item) for lim in self.limiters)


def default_controller_rate_limiter():
    return MaxOfLimiter(ItemExponentialBackoff(0.005, 1000.0), BucketLimiter(10.0, 100))


class ShutDown(Exception):
    pass


class WorkQueue:
    def __init__(self, rate_limiter=None, name: str = ""):
        self.name = name
        self.rate_limiter = rate_limiter or default_controller_rate_limiter()
        self._queue: collections.deque = collections.deque()
        self._dirty: set = set()
        self._processing: set = set()
        self._cond = asyncio.Condition()
        self._shutdown = False
        self._delayed: set[asyncio.TimerHandle] = set()
        self.adds = 0
        self.retries = 0

    def __len__(self) -> int:
        return len(self._queue)

    def _add_nolock(self, item):
        if self._shutdown or item in self._dirty:
            return False
        self._dirty.add(item)
        self.adds += 1
        if item in self._processing:
            return False
        self._queue.append(item)
        return True

    def add(self, item):
        """Non-blocking add (callable from event handlers)."""
        if self._add_nolock(item):
            self._notify()

    def _notify(self):
        async def n():
            async with self._cond:
                self._cond.notify()
        if self._cond._waiters:  # noqa: SLF001 - avoid a task per add when nobody waits
            asyncio.get_running_loop().create_task(n())

    def add_after(self, item, delay: float):
        if self._shutdown:
            return
        if delay <= 0:
            self.add(item)
            return
        loop = asyncio.get_running_loop()
        h = None

        def fire():
            self._delayed.discard(h)
            self.add(item)
        h = loop.call_later(delay, fire)
        self._delayed.add(h)

    def add_rate_limited(self, item):
        self.retries += 1
        self.add_after(item, self.rate_limiter.when(item))

    def forget(self, item):
        self.rate_limiter.forget(item)

    def num_requeues(self, item) -> int:
        return self.rate_limiter.num_requeues(item)

    async def get(self):
        async with self._cond:
            while not self._queue and not self._shutdown:
                await self._cond.wait()
            if not self._queue:
                raise ShutDown()
            item = self._queue.popleft()
            self._processing.add(item)
            self._dirty.discard(item)
            return item

    def done(self, item):
        self._processing.discard(item)
        if item in self._dirty:
            self._queue.append(item)
            self._notify()

    async def shutdown(self):
        self._shutdown = True
        for h in list(self._delayed):
            h.cancel()
        self._delayed.clear()
        async with self._cond:
            self._cond.notify_all()

    @property
    def is_shutdown(self) -> bool:
        return self._shutdown

    def idle(self) -> bool:
        return not self._queue and not self._processing and not self._delayed
