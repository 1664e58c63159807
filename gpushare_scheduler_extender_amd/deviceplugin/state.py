"""The device plugin's view of its node: Allocate candidates, CU partitions and multi-container progress.

One implementation of the Allocate matching contract (``docs/designs/designs.md:93-103``,
``docs/designs/sequence.jpg``), fed by a pod informer on ``spec.nodeName=<node>`` and used
by both the gRPC plugin (:mod:`.plugin`) and the kubelet stand-in (:mod:`.agent`):

* **candidates** — Pending gpushare pods bound to this node whose ``ASSIGNED`` annotation is
  ``false`` and whose ``*_IDX`` names one of our GPUs, ordered by ``ASSUME_TIME`` (then
  creation time and key).  An Allocate of N units takes the first whose total request is N
  (:meth:`AllocationState.match`);
* **CU partitions** (the MPS stand-in, ``README.md:77``) — owned per pod UID and released when
  the pod completes (Succeeded / Failed / deletionTimestamp) or disappears.  At start-up and on
  every re-list, ownership is rebuilt from the ``gpushare.amd.com/cu-mask`` annotation of
  ``ASSIGNED=true``, non-terminated pods, so a restarted plugin never hands out a CU that a
  running pod still holds;
* **allocation records** — every Allocate is recorded with the device IDs kubelet passed, the pod it was
  matched to and the GPU / CU partition it handed out.  kubelet's own record of which pod holds those IDs
  (PodResources API) is compared with it by :mod:`.reconcile`; a record whose *owner* (the pod kubelet gave it
  to) is not the pod it was matched to is a swap, and the annotations follow the record;
* **multi-container progress** — kubelet calls Allocate once per container.  The first
  container of a pod commits ``ASSIGNED=true``; the remaining container sizes are kept until
  they are allocated or the pod leaves Pending / goes away.  After a restart the progress of
  an ``ASSIGNED=true`` Pending pod is unknown, so all its container sizes are accepted again.

Everything here is synchronous and I/O free; the callers own the apiserver calls.
"""
from __future__ import annotations

import logging
from dataclasses import dataclass, field

from ..models import pod as podutil
from ..models.profile import (POD_CU_MASK_ANNOTATION, POD_HOLD_IDX_ANNOTATION, POD_HOLD_PARTNER_ANNOTATION,
                              NamingProfile)
from .allocator import CU_COUNT_ANNOTATION, AllocateError, CUPartitioner
from .devices import Device

log = logging.getLogger("gsx.deviceplugin.state")


def parse_cu_mask(words: str) -> list[int]:
    """``0x000000ff,0x00000000,...`` (GSX_CU_MASK / the cu-mask annotation) -> CU ids."""
    out = []
    for wi, w in enumerate(x for x in words.split(",") if x.strip()):
        v = int(w, 16)
        out.extend(32 * wi + b for b in range(32) if v >> b & 1)
    return out


@dataclass
class AllocRecord:
    """One Allocate: what the plugin handed out, for whom it built it, and (once kubelet says so) who got it."""
    aid: str
    ids: tuple  # kubelet's device IDs, sorted
    uid: str  # the pod whose annotations describe this allocation (the matched pod, until a move)
    dev: int
    units: int
    cu_mask: str  # the cu-mask annotation value of the partition handed out ("" if none)
    owner: str = ""  # the pod kubelet gave the IDs to ("" until PodResources has reported them)
    t: float = 0.0
    iso: str = ""  # isolation directory key the container's mounts point at

    @property
    def holder(self) -> str:
        return self.owner or self.uid

    def to_dict(self) -> dict:
        return {"aid": self.aid, "ids": list(self.ids), "uid": self.uid, "dev": self.dev, "units": self.units,
                "cu_mask": self.cu_mask, "owner": self.owner, "t": self.t, "iso": self.iso}

    @classmethod
    def from_dict(cls, d: dict) -> "AllocRecord":
        return cls(aid=d["aid"], ids=tuple(d.get("ids") or ()), uid=d.get("uid", ""), dev=int(d.get("dev", -1)),
                   units=int(d.get("units", 0)), cu_mask=d.get("cu_mask", ""), owner=d.get("owner", ""),
                   t=float(d.get("t", 0.0)), iso=d.get("iso", ""))


@dataclass
class PodRec:
    uid: str
    key: str
    name: str
    namespace: str
    rv: str
    phase: str
    dev: int
    request: int
    containers: list[int]
    assume_time: int
    creation: str
    assigned: str
    complete: bool
    cu_count: int
    cu_mask: str
    hold_idx: int = -1
    hold_partner: str = ""
    obj: dict = field(repr=False, default_factory=dict)

    @property
    def order(self) -> tuple:
        return self.assume_time, self.creation, self.key

    @property
    def pending(self) -> bool:
        return self.phase in ("Pending", "")


class AllocationState:
    def __init__(self, node: str, devices: dict[int, Device], profile: NamingProfile):
        self.node = node
        self.devices = devices
        self.profile = profile
        self.cus = {i: CUPartitioner(d.cu_count, d.xcc_count) for i, d in devices.items()}
        self.pods: dict[str, PodRec] = {}  # uid -> record (non-complete pods on this node)
        self.partial: dict[str, list[int]] = {}  # uid -> container sizes not yet allocated
        self.local_commits: set[str] = set()  # first container committed by this process
        self.inflight: set[str] = set()  # claimed by an Allocate whose ASSIGNED patch is in flight
        self.records: dict[str, AllocRecord] = {}  # aid -> record
        self.by_ids: dict[tuple, str] = {}  # sorted device IDs -> aid
        self.keys: dict[str, str] = {}  # ns/name -> uid of the live pod
        self.on_drop: list = []  # callbacks(record) when a record's holder is gone
        self.stats = {"cu_released": 0, "cu_adopted": 0, "cu_conflicts": 0, "partial_released": 0,
                      "pods_released": 0, "records_dropped": 0}

    # ------------------------------------------------------------ informer feed
    def _rec(self, pod: dict) -> PodRec:
        md = podutil.meta(pod)
        ann = podutil.annotations(pod)
        p = self.profile
        conts = [podutil.container_limit(c, p.resource) for c in (pod.get("spec") or {}).get("containers") or []]
        try:
            cu_count = int(ann.get(CU_COUNT_ANNOTATION, "0") or 0)
        except ValueError:
            cu_count = 0
        return PodRec(uid=md.get("uid", ""), key=podutil.pod_key(pod), name=md.get("name", ""),
                      namespace=md.get("namespace", ""), rv=md.get("resourceVersion", ""),
                      phase=podutil.phase(pod), dev=podutil.gpu_id_from_annotation(pod, p),
                      request=sum(conts), containers=[c for c in conts if c > 0],
                      assume_time=podutil.assume_time(pod, p), creation=md.get("creationTimestamp", ""),
                      assigned=ann.get(p.annotation_assigned, ""), complete=podutil.is_complete(pod),
                      cu_count=cu_count, cu_mask=ann.get(POD_CU_MASK_ANNOTATION, ""),
                      hold_idx=podutil.hold_idx(pod), hold_partner=ann.get(POD_HOLD_PARTNER_ANNOTATION, ""),
                      obj=pod)

    def observe(self, pod: dict) -> None:
        """An added / updated pod (informer event, LIST item, or our own PATCH response)."""
        rec = self._rec(pod)
        if not rec.uid:
            return
        prev = self.pods.get(rec.uid)
        if prev is not None and prev.rv and rec.rv and _older(rec.rv, prev.rv):
            return  # a stale copy (e.g. a slow LIST racing the watch): never step back
        if podutil.node_name(pod) != self.node or rec.request <= 0 or rec.complete:
            self.release(rec.uid)
            return
        self.pods[rec.uid] = rec
        self.keys[rec.key] = rec.uid
        if rec.assigned != "true":
            return
        # an assigned pod: its CU partition is owned (rebuild after restart / adopt another agent's record)
        if rec.cu_mask and rec.dev in self.cus and not self.cus[rec.dev].holds(rec.uid):
            try:
                cus = parse_cu_mask(rec.cu_mask)
            except ValueError:
                cus = []
            clash = self.cus[rec.dev].adopt(rec.uid, cus)
            self.stats["cu_adopted"] += 1
            if clash:
                self.stats["cu_conflicts"] += 1
                log.warning("pod %s: CUs %s of GPU %d already owned by another pod", rec.key, clash[:8], rec.dev)
        if not rec.pending:
            if self.partial.pop(rec.uid, None) is not None:
                self.stats["partial_released"] += 1
        elif len(rec.containers) > 1 and rec.uid not in self.local_commits and rec.uid not in self.partial:
            # restarted between containers: which ones were allocated is unknown, accept any of its sizes
            self.partial[rec.uid] = list(rec.containers)

    def forget(self, pod: dict) -> None:
        """A deleted pod (watch DELETE or gone from a re-list)."""
        self.release(podutil.meta(pod).get("uid", ""))

    def resync(self, pods: list[dict]) -> None:
        """A complete LIST of this node's pods: anything we hold that is not in it is gone."""
        seen = set()
        for p in pods:
            self.observe(p)
            seen.add(podutil.meta(p).get("uid", ""))
        for uid in [u for u in self.holders() if u not in seen]:
            self.release(uid)

    def holders(self) -> set[str]:
        out = set(self.pods) | set(self.partial) | self.local_commits
        for cp in self.cus.values():
            out |= set(cp.held())
        return out

    def release(self, uid: str) -> None:
        if not uid:
            return
        n = 0
        for cp in self.cus.values():
            n += cp.release(uid)
        if n:
            self.stats["cu_released"] += n
        if self.partial.pop(uid, None) is not None:
            self.stats["partial_released"] += 1
        gone = self.pods.pop(uid, None)
        if gone is not None:
            self.stats["pods_released"] += 1
            if self.keys.get(gone.key) == uid:
                del self.keys[gone.key]
        self.local_commits.discard(uid)
        self.inflight.discard(uid)
        for r in [r for r in self.records.values() if r.holder == uid]:
            self.drop_record(r)

    # ------------------------------------------------------------ Allocate
    def candidates(self) -> list[PodRec]:
        out = [r for r in self.pods.values()
               if r.pending and r.assigned == "false" and r.dev in self.devices and r.uid not in self.inflight]
        out.sort(key=lambda r: r.order)
        return out

    def match(self, units: int) -> tuple[PodRec | None, bool]:
        """(pod, whole_pod) for an Allocate of ``units``: a whole pod of that size (earliest ASSUME_TIME),
        else a later container of a pod whose first container was allocated, else the first container
        of a multi-container pod that has a container of that size."""
        cands = self.candidates()
        for r in cands:
            if r.request == units:
                return r, True
        for uid, left in self.partial.items():
            r = self.pods.get(uid)
            if r is not None and units in left and uid not in self.inflight:
                return r, False
        for r in cands:
            if units in r.containers:
                return r, False
        return None, False

    def unannotated(self, units: int) -> bool:
        """A pending pod of this size bound to the node without any allocation annotation (``*_IDX``)."""
        return any(r.pending and r.dev < 0 and r.assigned != "true" and r.request == units
                   and r.uid not in self.inflight for r in self.pods.values())

    def preferred_device(self, units: int) -> int:
        rec, _ = self.match(units)
        return rec.dev if rec is not None else -1

    def claim_cus(self, rec: PodRec) -> list[int] | None:
        if not rec.cu_count:
            return None
        if rec.dev not in self.cus:
            raise AllocateError(f"pod {rec.key} annotated with GPU {rec.dev}, not on this node")
        return self.cus[rec.dev].allocate(rec.uid, rec.cu_count)

    def first_container_committed(self, rec: PodRec, units: int, whole: bool) -> None:
        """The ASSIGNED=true patch of ``rec`` succeeded for a container of ``units``."""
        self.local_commits.add(rec.uid)
        if not whole:
            left = list(rec.containers)
            left.remove(units)
            if left:
                self.partial[rec.uid] = left

    def later_container_allocated(self, rec: PodRec, units: int) -> None:
        left = self.partial.get(rec.uid)
        if left is None:
            return
        left.remove(units)
        if not left:
            del self.partial[rec.uid]

    # ------------------------------------------------------------ allocation records
    def record(self, rec: PodRec, ids, units: int, cu_mask: str, aid: str, t: float = 0.0) -> AllocRecord:
        """An Allocate of ``ids`` was matched to ``rec`` (kubelet re-using the IDs of a finished pod replaces the
        older record)."""
        key = tuple(sorted(ids))
        old = self.by_ids.get(key) if key else None
        if old is not None and old in self.records:
            self.drop_record(self.records[old])
        r = AllocRecord(aid=aid, ids=key, uid=rec.uid, dev=rec.dev, units=units, cu_mask=cu_mask, t=t)
        self.records[aid] = r
        if key:
            self.by_ids[key] = aid
        return r

    def drop_record(self, r: AllocRecord) -> None:
        if self.records.pop(r.aid, None) is None:
            return
        if r.ids and self.by_ids.get(r.ids) == r.aid:
            del self.by_ids[r.ids]
        self.stats["records_dropped"] += 1
        for cb in self.on_drop:
            cb(r)

    def record_for_ids(self, ids) -> AllocRecord | None:
        aid = self.by_ids.get(tuple(sorted(ids)))
        return self.records.get(aid) if aid else None

    def pod_by_key(self, key: str) -> PodRec | None:
        uid = self.keys.get(key)
        return self.pods.get(uid) if uid else None

    def move_records(self, p_uid: str, q_uid: str, r: AllocRecord) -> None:
        """After the annotations of P and Q were exchanged because P holds ``r`` (built for Q): ``r`` now
        describes P, and whatever described P describes Q.  The CU partitions follow the same exchange."""
        for other in self.records.values():
            if other is not r and other.uid == p_uid:
                other.uid = q_uid
        r.uid = p_uid
        for cp in self.cus.values():
            cp.swap_owners(p_uid, q_uid)

    def snapshot(self) -> dict:
        """What ``/debug/state`` and the tests look at."""
        return {
            "pods": {r.key: {"uid": r.uid, "gpu": r.dev, "request": r.request, "assigned": r.assigned,
                             "phase": r.phase} for r in self.pods.values()},
            "candidates": [r.key for r in self.candidates()],
            "partial": {self.pods[u].key if u in self.pods else u: v for u, v in self.partial.items()},
            "cu_partitions": {str(i): {self.pods[u].key if u in self.pods else u: len(c) for u, c in cp.held().items()}
                              for i, cp in self.cus.items()},
            "cu_free": {str(i): cp.free_count() for i, cp in self.cus.items()},
            "records": len(self.records),
            "stats": dict(self.stats),
        }


def _older(a: str, b: str) -> bool:
    """resourceVersion a < b, when both are integers (the apiserver's are; compare nothing otherwise)."""
    try:
        return int(a) < int(b)
    except ValueError:
        return False
