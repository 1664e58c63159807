"""The extender's cluster-state controller: the C++ pod / node reflectors of ``native/engine/controller.cc``.

Re-design of ``pkg/gpushare/controller.go`` and ``pkg/cache/cache.go:49-127`` (one controller, as the reference
has): the reference's pod filter and enqueue rules (``controller.go:77-100,257-332``), ``syncPod``
(``controller.go:174-205``) and ``BuildCache`` crash recovery (``cache.go:49-74``) are applied on the reflector
threads as events are decoded, and nodes feed the ledger directly.  This module is its Python handle.
"""
from __future__ import annotations

import asyncio
import json
import logging

from ..k8s.client import KubeClient
from ..models.profile import NamingProfile

log = logging.getLogger("gsx.controller")


def api_dict(cfg) -> dict:
    """Connection settings of a :class:`KubeConfig` for the native engine's apiserver clients."""
    return {"server": cfg.server, "token": cfg.token or "", "token_file": getattr(cfg, "token_file", None) or "",
            "token_reload_s": float(getattr(cfg, "token_reload_s", 60.0)), "ca_file": cfg.ca_file or "",
            "cert_file": cfg.cert_file or "", "key_file": cfg.key_file or "", "insecure": bool(cfg.insecure)}


class NativeController:
    """The controller in C++ (``native/engine/controller.cc``): pod and node reflectors feed the ledger directly.

    Filter transitions, enqueue rules, syncPod, BuildCache + over-commit check, applied on the reflector threads
    as events are decoded, so no pod or node event is ever turned into a Python object.  The lister keeps the
    raw JSON of gpu-share pods for binds the filter did not see (``server.cc: lookup_pod``).
    """

    def __init__(self, client: KubeClient, engine, profile: NamingProfile, resync_period: float = 30.0,
                 watch_timeout: int = 300):
        self.client = client
        self.engine = engine
        self.profile = profile
        self.resync_period = resync_period
        self.watch_timeout = watch_timeout
        self.overcommitted: list = []
        self._started = False

    async def start(self, sync_timeout: float | None = 60.0):
        loop = asyncio.get_running_loop()
        await loop.run_in_executor(None, lambda: self.engine.start_controller(
            api_dict(self.client.config), self.resync_period, float(sync_timeout or 3600.0), self.watch_timeout))
        self._started = True
        self.overcommitted = list(self.engine.controller_overcommitted())
        for node, i, used, total in self.overcommitted:
            log.warning("node %s GPU %d is over-committed after recovery: %d > %d (annotations disagree "
                        "with capacity); it accepts no new pods until it drains", node, i, used, total)

    async def stop(self):
        if self._started:
            await asyncio.get_running_loop().run_in_executor(None, self.engine.stop_controller)
            self._started = False

    def get_pod(self, name: str, ns: str | None = None) -> dict | None:
        raw = self.engine.controller_get_pod(f"{ns}/{name}" if ns else name)
        return json.loads(raw) if raw is not None else None

    def is_synced(self) -> bool:
        return self.engine.controller_synced()

    def stats(self) -> dict:
        return self.engine.controller_stats()

    def gc_reservations(self) -> tuple[int, bool]:
        return tuple(self.engine.controller_gc())

    async def wait_idle(self, timeout: float = 10.0):
        """Events are applied as they are decoded; nothing is queued."""
        await asyncio.sleep(0)
