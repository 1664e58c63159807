"""Reconcile the plugin's Allocate records with kubelet's device assignments (PodResources ``List``).

Why: kubelet never tells a device plugin which pod an Allocate is for; the reference's protocol infers it from
the request size and the earliest ``ASSUME_TIME`` (``docs/designs/designs.md:93-103``).  kubelet admits a batch
of pods (after its own restart, a re-list, pods it meets together) in creationTimestamp order, so two
equal-size pending pods for different GPUs can be served each other's Allocate: the container of P runs with
the GPU (and CU partition) the extender reserved for Q.  The pod annotations — the durable allocation record
the extender's ledger is rebuilt from (``pkg/utils/pod.go:192-206``) — then say the wrong thing, and deleting
one pod of the pair frees the wrong GPU: the next pod lands on a device that is physically full.  The
reference's node lock (``pkg/cache/nodeinfo.go:141-189``) only orders binds; it cannot prevent this.

How: every Allocate is recorded with kubelet's device IDs (:class:`.state.AllocRecord`).  A pass asks kubelet
which pod holds those IDs.  When P holds the record built for Q (same size, by construction of the match),
the allocation fields of the two pods' annotations are exchanged — ``*_IDX``, ``ASSIGNED``, the cu-mask —
so each annotation names what its container really got.  The exchange is three PATCHes, ordered so that no
device is ever under-counted by the extender in between:

1. P takes Q's fields and ``hold-idx`` = P's old device (the ledger charges P on both devices);
2. Q takes P's old fields (from the ``hold-partner`` payload on P);
3. P's hold is removed.

Every PATCH carries the pod's resourceVersion; a conflict ends the pass and the next one re-plans from fresh
state.  A plugin restarted between steps finds the hold on P and finishes steps 2-3 from ``hold-partner``.
Cycles (P holds Q's, Q holds R's, R holds P's) resolve as a chain of such exchanges.
"""
from __future__ import annotations

import asyncio
import json
import logging
import time

from ..k8s.client import ApiError
from ..models.profile import (POD_CU_MASK_ANNOTATION, POD_HOLD_IDX_ANNOTATION, POD_HOLD_PARTNER_ANNOTATION,
                              POD_RECONCILED_ANNOTATION)
from .podresources import PodResourcesClient
from .state import AllocRecord, PodRec

log = logging.getLogger("gsx.deviceplugin.reconcile")


def fields(p: PodRec) -> dict:
    return {"idx": p.dev, "assigned": p.assigned, "cu_mask": p.cu_mask}


class Reconciler:
    def __init__(self, plugin, client: PodResourcesClient, interval: float = 2.0, after_allocate: float = 0.02):
        self.plugin = plugin
        self.pr = client
        self.interval = interval
        self.after_allocate = after_allocate
        self.stats = {"passes": 0, "swaps": 0, "records_owned": 0, "unknown_ids": 0, "unreconcilable": 0,
                      "holds_finished": 0, "conflicts": 0, "errors": 0, "list_ms_max": 0.0}
        self._kick = asyncio.Event()
        self._task: asyncio.Task | None = None
        self._lock = asyncio.Lock()

    @property
    def state(self):
        return self.plugin.state

    def kick(self):
        """An Allocate returned: kubelet records its IDs right after; look soon."""
        self._kick.set()

    # ------------------------------------------------------------ one pass
    async def run_once(self) -> dict:
        async with self._lock:
            self.stats["passes"] += 1
            t0 = time.perf_counter()
            truth = await self.pr.device_ids(self.plugin.profile.resource)
            self.stats["list_ms_max"] = max(self.stats["list_ms_max"], 1e3 * (time.perf_counter() - t0))
            moves: list[tuple[str, str]] = []  # (P uid, record aid)
            for (ns, name), per_container in truth.items():
                pod = self.state.pod_by_key(f"{ns}/{name}")
                if pod is None:
                    continue
                for ids in per_container:
                    r = self.state.record_for_ids(ids)
                    if r is None:
                        self.stats["unknown_ids"] += 1
                        continue
                    if r.owner != pod.uid:
                        self.state.set_owner(r.aid, pod.uid)
                        self.stats["records_owned"] += 1
                    if r.uid != pod.uid:
                        moves.append((pod.uid, r.aid))
            done = 0
            for p_uid, aid in moves:
                r = self.state.records.get(aid)
                p = self.state.pods.get(p_uid)
                if r is None or p is None or r.uid == p_uid:
                    continue  # resolved by an earlier exchange of this pass
                if await self._exchange(p, r):
                    done += 1
            await self._finish_holds()
            if done:
                self.plugin.persist_records()
            return {"moves": done, "pods": len(truth)}

    async def _patch(self, p: PodRec, ann: dict) -> bool:
        body = {"metadata": {"resourceVersion": p.rv, "annotations": ann}}
        try:
            pod = await self.plugin.client.patch("pods", p.name, body, p.namespace)
        except ApiError as e:
            if e.conflict or e.not_found:
                self.stats["conflicts"] += 1
                return False
            raise
        self.state.observe(pod)
        return True

    def _ann(self, f: dict) -> dict:
        prof = self.plugin.profile
        return {prof.annotation_idx: str(f["idx"]), prof.annotation_assigned: f["assigned"] or "false",
                POD_CU_MASK_ANNOTATION: f["cu_mask"] or None}

    async def _exchange(self, p: PodRec, r: AllocRecord) -> bool:
        q = self.state.pods.get(r.uid)
        if q is None:
            # the pod the record was built for is gone: P simply takes the record's fields
            q_fields = None
        else:
            q_fields = fields(q)
            if q.request != p.request:
                self.stats["unreconcilable"] += 1
                log.warning("pod %s holds the allocation of %s, of another size (%d vs %d); not reconciled",
                            p.key, q.key, p.request, q.request)
                return False
        p_old = fields(p)
        new_p = {"idx": r.dev, "assigned": "true", "cu_mask": r.cu_mask}
        ann = self._ann(new_p)
        n = int((p.obj.get("metadata", {}).get("annotations") or {}).get(POD_RECONCILED_ANNOTATION, "0") or 0)
        ann[POD_RECONCILED_ANNOTATION] = str(n + 1)
        holding = q is not None and p_old["idx"] >= 0 and p_old["idx"] != r.dev
        if holding:
            ann[POD_HOLD_IDX_ANNOTATION] = str(p_old["idx"])
            ann[POD_HOLD_PARTNER_ANNOTATION] = json.dumps({"uid": q.uid, "key": q.key, **p_old}, separators=(",", ":"))
        log.warning("kubelet gave pod %s the allocation built for %s (GPU %d): exchanging their records",
                    p.key, q.key if q else r.uid, r.dev)
        if not await self._patch(p, ann):  # step 1
            return False
        self.state.move_records(p.uid, r.uid, r)
        self.stats["swaps"] += 1
        if q is not None:
            if await self._patch(self.state.pods.get(q.uid, q), self._ann(p_old)):  # step 2
                if holding:
                    await self._clear_hold(self.state.pods.get(p.uid, p))  # step 3
            # on a conflict the hold stays; _finish_holds completes the move on a later pass
        return True

    async def _clear_hold(self, p: PodRec) -> bool:
        ok = await self._patch(p, {POD_HOLD_IDX_ANNOTATION: None, POD_HOLD_PARTNER_ANNOTATION: None})
        if ok:
            self.stats["holds_finished"] += 1
        return ok

    async def _finish_holds(self):
        """Complete moves interrupted after step 1 (a conflict, or a plugin restart in between)."""
        for p in [p for p in self.state.pods.values() if p.hold_idx >= 0 or p.hold_partner]:
            try:
                want = json.loads(p.hold_partner) if p.hold_partner else {}
            except ValueError:
                want = {}
            q = self.state.pods.get(want.get("uid", ""))
            if q is not None and fields(q) != {k: want.get(k) for k in ("idx", "assigned", "cu_mask")}:
                if not await self._patch(q, self._ann(want)):
                    continue
            await self._clear_hold(self.state.pods.get(p.uid, p))

    # ------------------------------------------------------------ loop
    async def run(self):
        while True:
            try:
                await asyncio.wait_for(self._kick.wait(), self.interval)
                await asyncio.sleep(self.after_allocate)  # let kubelet record the allocation first
            except asyncio.TimeoutError:
                pass
            self._kick.clear()
            if not self.pr.available():
                continue
            try:
                await self.run_once()
            except asyncio.CancelledError:
                raise
            except Exception as e:  # noqa: BLE001 - the loop outlives a bad pass
                self.stats["errors"] += 1
                log.warning("reconcile pass failed: %r", e)

    def start(self):
        if self._task is None:
            self._task = asyncio.get_running_loop().create_task(self.run(), name="gsx-reconcile")

    async def stop(self):
        if self._task is not None:
            self._task.cancel()
            try:
                await self._task
            except (asyncio.CancelledError, Exception):  # noqa: BLE001
                pass
            self._task = None
        await self.pr.close()
