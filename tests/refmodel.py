"""Independent pure-Python model of the reference's cache semantics.

Written directly from pkg/cache/{nodeinfo,deviceinfo}.go: used memory is
re-summed from pod annotations on every query, free = total - used (signed
here; the reference's uint underflow is a bug we do not model), filter =
any single device with free >= req, bind = best fit with lowest-index ties.
Only used by tests to cross-check the native engine.
"""
from __future__ import annotations


class RefNode:
    def __init__(self, name: str, total: int, count: int, dev_totals: list[int] | None = None):
        self.name = name
        self.total = total
        self.count = count
        if dev_totals and len(dev_totals) == count:
            self.dev_totals = list(dev_totals)
        else:
            self.dev_totals = [total // count] * count if count > 0 else []
        self.pods: dict[str, tuple[int, int, bool]] = {}  # uid -> (dev, mem, terminal)

    def used(self) -> list[int]:
        u = [0] * self.count
        for dev, mem, terminal in self.pods.values():
            if 0 <= dev < self.count and not terminal:
                u[dev] += mem
        return u

    def free(self) -> list[int]:
        return [t - u for t, u in zip(self.dev_totals, self.used())]

    def gpushare(self) -> bool:
        return self.total > 0 and self.count > 0

    def fits(self, req: int) -> bool:
        return any(f >= req for f in self.free())

    def best_fit(self, req: int) -> int:
        cand, cand_free = -1, 0
        for i, f in enumerate(self.free()):
            if f >= req and (cand < 0 or f < cand_free):
                cand, cand_free = i, f
        return cand if req > 0 else -1
