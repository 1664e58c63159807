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

Two repairs keep the records honest when a pod goes away before a pass has seen its container:

* a record whose IDs kubelet no longer reports (``stale_after`` past its Allocate) is dropped -- its container
  is gone, so its GPU share is physically free, whichever pod the record's chain of exchanges names now;
* a pod marked ``ASSIGNED=true`` that no record describes and no container of which kubelet reports
  (``stale_after`` in that state) got that mark through an exchange with an allocation nobody holds any more:
  it is reset to ``ASSIGNED=false`` so the next Allocate of its size can serve it.
"""
from __future__ import annotations

import asyncio
import json
import logging
import os
import time

from ..k8s.client import ApiError
from ..models.profile import (POD_CU_MASK_ANNOTATION, POD_HOLD_IDX_ANNOTATION, POD_HOLD_PARTNER_ANNOTATION,
                              POD_RECONCILED_ANNOTATION)
from .podresources import PodResourcesClient
from .state import AllocRecord, PodRec

log = logging.getLogger("gsx.deviceplugin.reconcile")


GONE = "~"  # owner prefix of an allocation held by a pod that is no longer on this node (ns/name follows)


def fields(p: PodRec) -> dict:
    return {"idx": p.dev, "assigned": p.assigned, "cu_mask": p.cu_mask}


def _took(q: PodRec, want: dict) -> bool:
    """Q carries the fields an exchange's step 2 gives it (``want``, the hold's partner payload), or was served an
    Allocate on them since (ASSIGNED=true where the payload said false)."""
    f = fields(q)
    if f == {k: want.get(k) for k in ("idx", "assigned", "cu_mask")}:
        return True
    return (f["idx"] == want.get("idx") and (f["cu_mask"] or "") == (want.get("cu_mask") or "")
            and f["assigned"] == "true" and want.get("assigned") == "false")


class _Held:
    """What kubelet's container of a pod physically got (the plugin's physical account, keyed by kubelet's IDs)."""

    __slots__ = ("uid", "dev", "cu_mask", "aid")

    def __init__(self, uid: str, dev: int, cu_mask: str):
        self.uid, self.dev, self.cu_mask, self.aid = uid, dev, cu_mask or "", ""


def _drifted(p: PodRec, r) -> bool:
    """P's annotation names another GPU (or CU partition) than the allocation its container holds."""
    return p.dev != r.dev or (p.cu_mask or "") != (r.cu_mask or "")


class Reconciler:
    def __init__(self, plugin, client: PodResourcesClient, interval: float = 2.0, after_allocate: float | None = None,
                 stale_after: float = 0.5, gone_after: float = 0.5):
        self.plugin = plugin
        self.pr = client
        self.interval = interval
        # a pass ~20 ms after every Allocate burst (an ambiguous one: 2 ms).  Waiting 0.25 s instead (one pass per
        # burst, less of the plugin's core) failed 3 of 90 kubelet-restart-batch chaos seeds, 0 of 90 at 20 ms: the
        # matcher's "ambiguous" flag does not catch every batch swap (the other pod may not be in its view yet)
        self.after_allocate = after_allocate if after_allocate is not None else float(
            os.environ.get("GSX_RECONCILE_AFTER_ALLOCATE", "0.02"))
        self.stale_after = stale_after
        # a record kubelet does not list whose pods (built for, and held by) are both gone: kubelet records an
        # Allocate's IDs within the admission call that made it, so past a moment nobody can hold them any more
        self.gone_after = gone_after
        self.stats = {"passes": 0, "swaps": 0, "records_owned": 0, "unknown_ids": 0, "unreconcilable": 0,
                      "holds_finished": 0, "conflicts": 0, "errors": 0, "list_ms_max": 0.0, "records_stale": 0,
                      "assigned_reset": 0, "deferred": 0,
                      "made_room": 0, "stand_in_partners": 0,
                      "drift_repaired": 0}
        self._orphan_since: dict[str, float] = {}
        # after an ambiguous Allocate (kubelet records an Allocate's IDs before it returns to its admission loop;
        # a pass skips records made after it asked, so a short delay only saves passes)
        self.after_ambiguous = 0.002
        # while a publication stands, poll kubelet this often at first, doubling (to unaccounted_poll_max) while the
        # published vector does not change: a drift with no partner can keep one standing, and kubelet's PodResources
        # budget (100 calls/s) is the node's, not ours
        self.unaccounted_poll = 0.01
        self.unaccounted_poll_max = 0.5
        self._poll = self.unaccounted_poll
        self._poll_for = None  # the publication _poll was backed off for
        # kubelet rate-limits its PodResources API (100 calls/s, burst 10, since k8s 1.27): passes stay >= 10 ms apart
        self.min_spacing = float(os.environ.get("GSX_RECONCILE_MIN_SPACING", "0.01"))
        self._last_pass = 0.0
        self._fast = False
        self._kick = asyncio.Event()
        self._task: asyncio.Task | None = None
        self._lock = asyncio.Lock()

    @property
    def state(self):
        return self.plugin.state

    def kick(self, fast: bool = False):
        """An Allocate returned: kubelet records its IDs right after; look soon.  ``fast``: the Allocate may have been
        served to another pod than the one it was matched to (``GpuSharePlugin._ambiguous``): look at once."""
        if fast:
            self._fast = True
        self._kick.set()

    # ------------------------------------------------------------ one pass
    async def run_once(self, urgent: bool = False) -> dict:
        """``urgent``: an Allocate found no candidate -- reset orphaned ``ASSIGNED`` marks without waiting."""
        async with self._lock:
            self.stats["passes"] += 1
            self._last_pass = time.monotonic()  # urgent passes (the guard's, a miss's) count against min_spacing too
            t0 = time.perf_counter()
            # kubelet's answer describes the Allocates made before it was asked: the native endpoint keeps serving
            # (and recording) while it is awaited, and kubelet re-uses the IDs of finished pods -- a record made
            # after this point must not be judged by this answer (it would pin a re-used ID set on a pod of
            # an earlier wave, or look unheld)
            t_list = time.time()
            truth = await self.pr.device_ids(self.plugin.profile.resource)
            self.state.core.set_owners_reported(True)  # from now on kubelet's report decides who holds a record
            self.stats["list_ms_max"] = max(self.stats["list_ms_max"], 1e3 * (time.perf_counter() - t0))
            moves: list[tuple[str, str]] = []  # (P uid, record aid)
            # P's annotation names another GPU (or CU partition) than its container got: (P uid, what it got)
            drifts: list[tuple[str, _Held]] = []
            seen = {tuple(ids) for per_container in truth.values() for ids in per_container}
            # the physical account (what kubelet has handed out): an allocation kubelet no longer lists is free
            # (never on a short grace: a kubelet slow to record an Allocate's IDs must not make them look free)
            self.state.core.prune_held([list(i) for i in seen], t_list, self.stale_after)
            self._drop_stale(seen, 0.1 if urgent else self.stale_after, self.gone_after, t_list)
            for (ns, name), per_container in truth.items():
                pod = self.state.pod_by_key(f"{ns}/{name}")
                if pod is None:
                    # a pod this plugin no longer knows (deleted; its container still stopping): its allocations
                    # are physically held, but by no live pod -- they describe nobody who could be served them
                    for ids in per_container:
                        r = self.state.record_for_ids(ids)
                        if r is not None and r.t <= t_list and r.owner != GONE + f"{ns}/{name}":
                            self.state.set_owner(r.aid, GONE + f"{ns}/{name}")
                    continue
                for ids in per_container:
                    r = self.state.record_for_ids(ids)
                    if r is not None and r.t > t_list:
                        continue  # made after kubelet answered: the IDs were re-used since
                    # what the container physically got: the physical account, which no exchange re-labels
                    h = self.state.core.held_for(list(ids))
                    got = _Held(pod.uid, int(h["dev"]), h["cu_mask"]) if h is not None and h["t"] <= t_list else None
                    if r is None:
                        self.stats["unknown_ids"] += 1
                        if got is not None and _drifted(pod, got):
                            drifts.append((pod.uid, got))  # its record went: the annotation is repaired all the same
                        continue
                    if r.owner != pod.uid:
                        self.state.set_owner(r.aid, pod.uid)
                        self.stats["records_owned"] += 1
                    if r.uid != pod.uid:
                        moves.append((pod.uid, r.aid))
                    elif _drifted(pod, got or r):
                        drifts.append((pod.uid, got or _Held(pod.uid, r.dev, r.cu_mask)))
            done = 0
            started = {f"{ns}/{name}" for ns, name in truth}
            # before any repair: the extender learns what the containers physically hold (a swap just found, a
            # pod deleted before its record's holder was known), so no bind lands on a GPU the annotations
            # under-count while the exchanges below are in flight
            await self.plugin.publish_physical()
            await self._finish_holds()
            for p_uid, aid in moves:
                r = self.state.records.get(aid)
                p = self.state.pods.get(p_uid)
                if r is None or p is None or r.uid == p_uid:
                    continue  # resolved by an earlier exchange of this pass
                if {p_uid, r.uid} & self.busy() or p_uid in self.state.inflight or r.uid in self.state.inflight:
                    # an interrupted exchange involves one of them, or an Allocate's ASSIGNED commit is still in
                    # flight for one of them: finish that first (next pass)
                    self.stats["deferred"] += 1
                    continue
                if await self._exchange(p, r, started):
                    done += 1
            for p_uid, r in drifts:
                p = self.state.fresh(self.state.pods.get(p_uid))
                if p is None or not _drifted(p, r) or {p_uid} & self.busy() or p_uid in self.state.inflight:
                    continue
                q = self._drift_partner(p, r, started)
                plugin = self.plugin
                if (q is None and r.dev != p.dev
                        and plugin._annotated_used(r.dev, skip=p.uid) + p.request > plugin.units.get(r.dev, 0)):
                    # no pod of P's size to trade annotations with, and P's own GPU is full by the annotations: an
                    # unstarted pod the extender has placed there, of any size with which both GPUs fit afterwards
                    # (the exchange path's stand-in partner).  Without one, a bind that landed there in the swap
                    # window -- before the pass that found the swap -- leaves P unrepairable and fails that pod's
                    # Allocate
                    q = self._stand_in_partner(r.dev, p, started)
                    if q is not None:
                        self.stats["stand_in_partners"] += 1
                log.warning("pod %s is annotated with GPU %d but its container runs on GPU %d: re-annotating%s",
                            p.key, p.dev, r.dev, f" (exchanging with {q.key})" if q else "")
                if q is None:
                    await self._make_room(r.dev, p, started)
                if await self._exchange(p, r, started, partner=q, move=False):
                    self.stats["drift_repaired"] += 1
                    done += 1
            await self._finish_holds()
            await self._reset_orphans(started, 0.0 if urgent else self.stale_after)
            await self.plugin.publish_physical()  # withdrawn once the records and the annotations agree
            if done:
                self.plugin.persist_records()
            return {"moves": done, "pods": len(truth)}

    def _drop_stale(self, seen: set, grace: float, gone_grace: float | None = None, asked: float | None = None) -> None:
        """``asked``: when kubelet's answer (``seen``) was requested; a record is judged by it only if it was made
        that long before."""
        now = time.time() if asked is None else asked
        pods = self.state.pods
        gone_grace = grace if gone_grace is None else min(grace, gone_grace)

        def stale(r) -> bool:
            if tuple(sorted(r.ids)) in seen:
                return False
            gone = r.uid not in pods and (r.owner in ("", r.uid) or r.owner.startswith(GONE) or r.owner not in pods)
            return now - r.t > (gone_grace if gone else grace)

        stale = [r for r in self.state.records.values() if stale(r)]
        for r in stale:
            log.info("allocation %s (GPU %d) is held by no container kubelet reports: dropped", r.aid, r.dev)
            self.state.drop_record(r)
            self.stats["records_stale"] += 1
        if stale:
            self.plugin.persist_records()

    async def _reset_orphans(self, started: set, grace: float) -> None:
        live = [r for r in self.state.records.values() if not r.owner.startswith(GONE)]
        described = {r.uid for r in live} | {r.holder for r in live}
        busy = self.busy()
        now = time.monotonic()
        orphans = set()
        for p in list(self.state.pods.values()):
            if (p.assigned != "true" or p.complete or p.key in started or p.uid in described
                    or p.uid in self.state.inflight or p.uid in busy):
                continue
            orphans.add(p.uid)
            since = self._orphan_since.setdefault(p.uid, now)
            if now - since < grace:
                continue
            log.warning("pod %s is ASSIGNED but holds no allocation: making it an Allocate candidate again", p.key)
            if await self._patch(p, {self.plugin.profile.annotation_assigned: "false"}):
                self.stats["assigned_reset"] += 1
                orphans.discard(p.uid)
        self._orphan_since = {u: t for u, t in self._orphan_since.items() if u in orphans}

    async def _patch(self, p: PodRec, ann: dict, partner: str = "") -> bool:
        """Write allocation fields of P, guarded by the resourceVersion this pass planned on.  Anything that touches
        ``*_IDX`` or the hold goes through the extender (``POST /gpushare-scheduler/move``, the one writer of the
        allocation record, which checks it against its ledger); ``partner``: the equal-size pod the write exchanges
        P's record with (the write is sum-neutral per GPU).  The plugin's own ``ASSIGNED`` mark is patched directly."""
        idx_key = self.plugin.profile.annotation_idx
        try:
            if idx_key in ann or POD_HOLD_IDX_ANNOTATION in ann:
                ann = dict(ann)
                to = int(ann.pop(idx_key, p.dev))
                pod = await self.plugin.move_record(p, to, ann, partner=partner)
            else:
                pod = await self.plugin.client.patch("pods", p.name, {"metadata": {"resourceVersion": p.rv,
                                                                                   "annotations": ann}}, p.namespace)
        except ApiError as e:
            if e.conflict or e.not_found:
                self.stats["conflicts"] += 1
                log.info("write of %s refused: %s", p.key, e)
                return False
            raise
        self.state.observe(pod)
        return True

    def _ann(self, f: dict) -> dict:
        prof = self.plugin.profile
        return {prof.annotation_idx: str(f["idx"]), prof.annotation_assigned: f["assigned"] or "false",
                POD_CU_MASK_ANNOTATION: f["cu_mask"] or None}

    async def _exchange(self, p: PodRec, r: AllocRecord, started: set, partner: PodRec | None = None,
                        move: bool = True) -> bool:
        """P takes ``r``'s fields, its partner Q (the pod ``r`` was built for, or ``partner``) P's old ones.
        ``move=False``: the records and CU partitions already describe who runs what; only the annotations
        are wrong (a drift repair)."""
        if partner is not None or not move:
            q = partner
        else:
            q = self.state.pods.get(r.uid)
            if q is not None and q.request != p.request:
                self.stats["unreconcilable"] += 1
                log.warning("pod %s holds the allocation of %s, of another size (%d vs %d); not reconciled",
                            p.key, q.key, p.request, q.request)
                return False
        if q is None and move:
            # its deletion freed r.dev in the extender's ledger although P's container runs there.  An unstarted
            # pod of P's size the extender has since placed on r.dev is the natural partner: exchanging with it
            # keeps the annotations' per-GPU sums exactly as they are (it starts on P's old GPU instead)
            # (P's own allocation served to another container -- a chain -- relabels that record to Q: only a Q of
            # P's size keeps every record's size its pod's, else the holder is left unreconcilable and Q, marked
            # ASSIGNED for it, never an Allocate candidate -- box chaos seed 4723)
            chain = any(o.uid == p.uid and o.aid != r.aid for o in self.state.records.values())
            q = self._stand_in_partner(r.dev, p, started, same_size=chain)
            if q is None:
                await self._make_room(r.dev, p, started)
            else:
                self.stats["stand_in_partners"] += 1
        p_old = fields(p)
        # Q takes P's old allocation fields; it is ASSIGNED only if an Allocate was served for them, i.e. a record
        # describes P now (it will describe Q after the exchange) -- in a chain (P holds Q's, Q holds R's, ...)
        # P's own allocation may have gone to nobody, and then Q must stay an Allocate candidate
        # (Q itself may already run a container -- with yet another pod's allocation -- and then stays ASSIGNED)
        recs = self.state.records.values()
        served = q is not None and (q.key in started or any(o.owner == q.uid for o in recs))
        # (a drift repair moves no record: P's records all describe P's own container, none will describe Q)
        q_new = dict(p_old, assigned="true" if served or (move and any(o.uid == p.uid and o.aid != r.aid for o in recs))
                     else "false")
        new_p = {"idx": r.dev, "assigned": "true", "cu_mask": r.cu_mask}
        ann = self._ann(new_p)
        n = int((p.obj.get("metadata", {}).get("annotations") or {}).get(POD_RECONCILED_ANNOTATION, "0") or 0)
        ann[POD_RECONCILED_ANNOTATION] = str(n + 1)
        holding = q is not None and p_old["idx"] >= 0 and p_old["idx"] != r.dev
        if holding:
            ann[POD_HOLD_IDX_ANNOTATION] = str(p_old["idx"])
            ann[POD_HOLD_PARTNER_ANNOTATION] = json.dumps({"uid": q.uid, "key": q.key, **q_new}, separators=(",", ":"))
        log.warning("kubelet gave pod %s the allocation built for %s (GPU %d): exchanging their records",
                    p.key, q.key if q else r.uid, r.dev)
        if not await self._patch(p, ann, partner=q.uid if q is not None else ""):  # step 1
            return False
        if move:
            self.state.move_records(p.uid, q.uid if q is not None else r.uid, r)
            self.stats["swaps"] += 1
        if q is not None:
            if await self._patch(self.state.pods.get(q.uid, q), self._ann(q_new), partner=p.uid):  # step 2
                if holding:
                    await self._clear_hold(self.state.pods.get(p.uid, p))  # step 3
            # on a conflict the hold stays; _finish_holds completes the move on a later pass
        return True

    def _drift_partner(self, p: PodRec, r: AllocRecord, started: set) -> PodRec | None:
        """A pod of P's size annotated with what P's container really has, whose own annotation is not what its
        container has either (or which has not started): exchanging the two annotations fixes both."""
        recs = list(self.state.records.values())
        own = {}
        for o in recs:
            if o.uid == o.holder:
                own.setdefault(o.uid, o)
        cands = []
        for q in self.state.pods.values():
            if q.uid == p.uid or q.request != p.request or q.complete or (q.dev, q.cu_mask or "") != (r.dev, r.cu_mask or ""):
                continue
            if q.uid in self.busy() or q.uid in self.state.inflight:
                continue
            o = own.get(q.uid)
            if o is not None and not _drifted(q, o):
                continue  # Q's annotation is its own container's truth
            if o is None and q.key in started:
                continue
            cands.append(q)
        return min(cands, key=lambda q: q.order) if cands else None

    def _stand_in_partner(self, dev: int, p: PodRec, started: set, same_size: bool = False) -> PodRec | None:
        """An unstarted pod Q the extender has placed on ``dev`` (where P's container runs) to exchange GPUs with P:
        Q takes P's annotated GPU, which P's container never used.  Equal-size first (the exchange keeps every
        GPU's sum); else the largest Q with which both GPUs fit after the exchange -- P's phantom share on its
        annotated GPU is exactly the room Q needs there, and the extender checks the same final state.  ``same_size``: only
        an equal-size Q."""
        recs = self.state.records.values()
        taken = {r.holder for r in recs} | {r.uid for r in recs} | self.busy()
        cands = [q for q in self.state.pods.values()
                 if q.dev == dev and q.uid != p.uid and not q.complete and q.request > 0
                 and q.key not in started and q.uid not in taken and q.uid not in self.state.inflight]
        same = [q for q in cands if q.request == p.request]
        if same:
            return min(same, key=lambda q: q.order)
        if same_size or p.dev < 0 or p.dev == dev:
            return None
        plugin = self.plugin
        cap_to, cap_from = plugin.units.get(dev, 0), plugin.units.get(p.dev, 0)
        used_to, used_from = plugin._annotated_used(dev), plugin._annotated_used(p.dev)
        fits = [q for q in cands
                if used_to - q.request + p.request <= cap_to and used_from - p.request + q.request <= cap_from
                and plugin._physical_used(p.dev) + q.request <= cap_from]
        if not fits:
            return None
        self.stats["unequal_partners"] = self.stats.get("unequal_partners", 0) + 1
        return min(fits, key=lambda q: (-q.request, q.order))

    async def _make_room(self, dev: int, p: PodRec, started: set) -> None:
        """P is about to be annotated with GPU ``dev`` alone (the pod the allocation was built for is gone -- and
        its deletion freed ``dev`` in the extender's ledger although P's container runs there).  Pods the extender
        has since placed on ``dev`` and that have not started are moved to GPUs with room first, so the
        annotations never promise ``dev`` beyond its capacity."""
        plugin = self.plugin
        need = plugin._annotated_used(dev, skip=p.uid) + p.request - plugin.units.get(dev, 0)
        if need <= 0:
            return
        owned = {r.holder for r in self.state.records.values()} | {r.uid for r in self.state.records.values()}
        busy = self.busy()
        movable = sorted((q for q in self.state.pods.values()
                          if q.dev == dev and q.uid != p.uid and not q.complete and q.key not in started
                          and q.uid not in owned and q.uid not in busy and q.uid not in self.state.inflight),
                         key=lambda q: -q.request)
        for q in movable:
            if need <= 0:
                break
            to = plugin.room_for(q, q.request)
            if to < 0:
                continue
            log.warning("GPU %d is needed back for %s: moving %s (not started) to GPU %d", dev, p.key, q.key, to)
            try:
                await plugin.move_unstarted(q, to)
            except ApiError:
                self.stats["conflicts"] += 1
                continue
            need -= q.request
            self.stats["made_room"] += 1
        if need > 0:
            log.warning("GPU %d stays over-committed by %d after the deletion of the pod %s's allocation was built "
                        "for; its unstarted pods move when they are admitted", dev, need, p.key)

    async def _clear_hold(self, p: PodRec) -> bool:
        ok = await self._patch(p, {POD_HOLD_IDX_ANNOTATION: None, POD_HOLD_PARTNER_ANNOTATION: None})
        if ok:
            self.stats["holds_finished"] += 1
        return ok

    def busy(self) -> set:
        """Pods an unfinished exchange involves: P (carrying the hold) and the partner Q named in it.  Neither
        takes part in another exchange (or a physical-guard move) until the hold is cleared, so the partner's
        fields are still what the hold's payload compares them with."""
        out = set()
        for p in self.state.pods.values():
            if p.hold_idx >= 0 or p.hold_partner:
                out.add(p.uid)
                try:
                    out.add(json.loads(p.hold_partner).get("uid", "") if p.hold_partner else "")
                except ValueError:
                    pass
        out.discard("")
        return out

    async def _finish_holds(self):
        """Complete moves interrupted after step 1 (a conflict, or a plugin restart in between)."""
        for p in [p for p in self.state.pods.values() if p.hold_idx >= 0 or p.hold_partner]:
            try:
                want = json.loads(p.hold_partner) if p.hold_partner else {}
            except ValueError:
                want = {}
            # (Q cannot have been served an Allocate with its old fields meanwhile: the matcher skips the partner of an
            # unfinished exchange, AllocState::candidates -- tests/interleave.py swap-graceful seed 25 -- and so does
            # the physical guard for a pod it matched before the exchange began.  It may have been served with the
            # fields step 2 gave it: the guard's own pass ran both steps -- batch-faults seed 1914 -- and the
            # container runs where they say)
            q = self.state.pods.get(want.get("uid", ""))
            if q is not None and not _took(q, want):
                if not await self._patch(q, self._ann(want), partner=p.uid):
                    continue
            await self._clear_hold(self.state.pods.get(p.uid, p))

    def exchange_pending(self, q: PodRec) -> bool:
        """Q is the partner of an unfinished exchange whose step 2 has not landed: its fields are about to change."""
        for p in self.state.pods.values():
            if not p.hold_partner:
                continue
            try:
                want = json.loads(p.hold_partner)
            except ValueError:
                continue
            if want.get("uid") == q.uid and not _took(q, want):
                return True
        return False

    # ------------------------------------------------------------ loop
    async def run(self):
        while True:
            # while the extender charges unaccounted use, look again soon: it is withdrawn as soon as kubelet's report
            # lets the records go (a stale publication would keep the GPU from the next pods)
            pub = self.plugin._phys_published
            if pub is None:
                wait, self._poll, self._poll_for = self.interval, self.unaccounted_poll, None
            else:
                if pub == self._poll_for:  # unchanged since the last pass: back off
                    self._poll = min(self.unaccounted_poll_max, self._poll * 2)
                else:
                    self._poll, self._poll_for = self.unaccounted_poll, list(pub)
                wait = min(self.interval, self._poll)
            try:
                await asyncio.wait_for(self._kick.wait(), wait)
                # let kubelet record the allocation first
                await asyncio.sleep(self.after_ambiguous if self._fast else self.after_allocate)
            except asyncio.TimeoutError:
                pass
            self._kick.clear()
            self._fast = False
            gap = self._last_pass + self.min_spacing - time.monotonic()
            if gap > 0:
                await asyncio.sleep(gap)
            self._last_pass = time.monotonic()
            if not self.pr.available():
                self.state.core.set_owners_reported(False)  # nobody will report owners: drop records by pod
                continue
            try:
                await self.run_once()
            except asyncio.CancelledError:
                raise
            except Exception as e:  # noqa: BLE001 - the loop outlives a bad pass
                self.stats["errors"] += 1
                log.warning("reconcile pass failed: %r", e)

    def start(self):
        # until the first report, a pod's going does not end the allocations built for it (a swapped container may
        # hold one): kubelet's report decides (AllocState::expect_owner_reports)
        self.state.core.expect_owner_reports(True)
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
