"""The device plugin's view of its node: Allocate candidates, CU partitions, multi-container progress, records.

The matching contract itself (``docs/designs/designs.md:93-103``, ``docs/designs/sequence.jpg``) has ONE
implementation, in C++: ``native/engine/allocstate.{h,cc}`` (``_engine.AllocState``).  The compiled kubelet
stand-in (``native/nodeagent``) uses it directly; this module is the shipped gRPC plugin's adapter to it.  It
keeps the pod objects (the plugin answers with their annotations) and turns the native answers into
:class:`PodRec` / :class:`AllocRecord` views; every decision is the native one:

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

import json
import logging
import time
from collections.abc import Mapping
from dataclasses import dataclass, field

from ..core.engine import native
from ..models import pod as podutil
from ..models.profile import POD_CU_MASK_ANNOTATION, POD_HOLD_PARTNER_ANNOTATION, NamingProfile
from .allocator import CU_COUNT_ANNOTATION, AllocateError, CUPartitioner
from .devices import Device

log = logging.getLogger("gsx.deviceplugin.state")


def parse_cu_mask(words: str) -> list[int]:
    """``0x000000ff,0x00000000,...`` (GSX_CU_MASK / the cu-mask annotation) -> CU ids."""
    return list(native().parse_cu_words(words))


@dataclass
class AllocRecord:
    """One Allocate: what the plugin handed out, for whom it built it, and (once kubelet says so) who got it.
    A snapshot of the native record; change it through :class:`AllocationState`."""
    aid: str
    ids: tuple  # kubelet's device IDs, sorted
    uid: str  # the pod whose annotations describe this allocation (the matched pod, until a move)
    dev: int
    units: int
    cu_mask: str  # the cu-mask annotation value of the partition handed out ("" if none)
    owner: str = ""  # the pod kubelet gave the IDs to ("" until PodResources has reported them)
    t: float = 0.0
    iso: str = ""  # isolation directory key the container's mounts point at
    on_gpu: bool = False  # every ID lies on ``dev``: kubelet's per-ID accounting bounds that GPU (allocstate.h)

    @property
    def holder(self) -> str:
        return self.owner or self.uid

    def to_dict(self) -> dict:
        return {"aid": self.aid, "ids": list(self.ids), "uid": self.uid, "dev": self.dev, "units": self.units,
                "cu_mask": self.cu_mask, "owner": self.owner, "t": self.t, "iso": self.iso, "on_gpu": self.on_gpu}

    @classmethod
    def from_dict(cls, d: dict) -> "AllocRecord":
        return cls(aid=d["aid"], ids=tuple(d.get("ids") or ()), uid=d.get("uid", ""), dev=int(d.get("dev", -1)),
                   units=int(d.get("units", 0)), cu_mask=d.get("cu_mask", ""), owner=d.get("owner", ""),
                   t=float(d.get("t", 0.0)), iso=d.get("iso", ""), on_gpu=bool(d.get("on_gpu", False)))


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
    pod: dict | None = field(repr=False, default=None, compare=False)
    loader: object = field(repr=False, default=None, compare=False)  # () -> pod dict, read on first use

    @property
    def obj(self) -> dict:
        """The pod object (from the Python informer, or the raw JSON the native pod feed kept)."""
        if self.pod is None:
            self.pod = (self.loader() if self.loader is not None else None) or {}
        return self.pod

    @property
    def order(self) -> tuple:
        return self.assume_time, self.creation, self.key

    @property
    def pending(self) -> bool:
        return self.phase in ("Pending", "")


def _older_rv(a: str, b: str) -> bool:
    """resourceVersion a < b when both are integers (the native state's rule)."""
    return a.isdigit() and b.isdigit() and int(a) < int(b)


class _Inflight:
    """Pods claimed by an Allocate whose ASSIGNED patch is in flight (the native set, set-like)."""

    def __init__(self, core):
        self._core = core

    def add(self, uid: str):
        self._core.set_inflight(uid, True)

    def discard(self, uid: str):
        self._core.set_inflight(uid, False)

    def __contains__(self, uid: str) -> bool:
        return self._core.inflight(uid)


class _NativePods(Mapping):
    """uid -> :class:`PodRec` read from the native state (the shipped plugin's pod feed keeps it current): no
    Python watch decodes the node's pod events.  Views are rebuilt only for pods whose resourceVersion changed."""

    def __init__(self, core):
        self._core = core
        self._cache: dict[str, PodRec] = {}

    def _make(self, t) -> PodRec:
        uid = t[0]
        old = self._cache.get(uid)
        if old is not None and old.rv == t[4] and old.phase == t[5] and old.assigned == t[11]:
            return old
        core = self._core

        def load(uid=uid):
            raw = core.pod_json(uid)
            return json.loads(raw) if raw else None
        rec = PodRec(uid=uid, key=t[1], namespace=t[2], name=t[3], rv=t[4], phase=t[5], dev=int(t[6]),
                     request=int(t[7]), containers=list(t[8]), assume_time=int(t[9]), creation=t[10], assigned=t[11],
                     complete=bool(t[12]), cu_count=int(t[13]), cu_mask=t[14], hold_idx=int(t[15]),
                     hold_partner=t[16], loader=load)
        self._cache[uid] = rec
        return rec

    def _all(self) -> dict[str, PodRec]:
        out = {t[0]: self._make(t) for t in self._core.pod_views()}
        for uid in [u for u in self._cache if u not in out]:
            del self._cache[uid]
        return out

    def __getitem__(self, uid: str) -> PodRec:
        t = self._core.pod_full(uid)
        if t is None:
            self._cache.pop(uid, None)
            raise KeyError(uid)
        return self._make(t)

    def __contains__(self, uid) -> bool:
        return self._core.has_pod(uid)

    def __iter__(self):
        return iter(self._all())

    def __len__(self) -> int:
        return len(self._core.pod_uids())

    def values(self):
        return self._all().values()

    def items(self):
        return self._all().items()

    def keys(self):
        return self._all().keys()


class AllocationState:
    def __init__(self, node: str, devices: dict[int, Device], profile: NamingProfile):
        self.node = node
        self.devices = devices
        self.profile = profile
        self.core = native().AllocState(node, [(i, d.cu_count, d.xcc_count) for i, d in devices.items()])
        self.cus = {i: CUPartitioner(native_obj=self.core.cus(i)) for i in devices}
        self.inflight = _Inflight(self.core)
        self._recs: dict[str, PodRec] = {}  # uid -> view of every pod the native state holds (Python-fed mode)
        self._native_pods: _NativePods | None = None
        self.on_drop: list = []  # callbacks(record) when a record's holder is gone

    def use_native_views(self) -> None:
        """The native pod feed is the only feed: :attr:`pods` reads the native state (no Python mirror)."""
        self._native_pods = _NativePods(self.core)
        self._recs = {}

    @property
    def native_views(self) -> bool:
        return self._native_pods is not None

    # ------------------------------------------------------------ views
    @property
    def pods(self):
        return self._native_pods if self._native_pods is not None else self._recs

    @property
    def partial(self) -> dict[str, list[int]]:
        return self.core.partial()

    @property
    def stats(self) -> dict:
        return self.core.stats()

    @property
    def records(self) -> dict[str, AllocRecord]:
        return {d["aid"]: AllocRecord.from_dict(d) for d in self.core.records()}

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
                      pod=pod)

    def observe(self, pod: dict, mirror_only: bool = False) -> None:
        """An added / updated pod (informer event, LIST item, or our own PATCH response).

        ``mirror_only``: the native state already receives this event from its own pod feed (the plugin's native
        endpoint watches the node's pods itself): only the Python view is updated, with the native state's rule for
        which pods it holds, and the native state is left to the feed."""
        rec = self._rec(pod)
        if not rec.uid:
            return
        if self._native_pods is not None:
            if mirror_only:
                return  # the feed has it
        elif mirror_only:
            old = self._recs.get(rec.uid)
            if old is not None and _older_rv(rec.rv, old.rv):
                return  # a slow copy: never step back
            if podutil.node_name(pod) == self.node and rec.request > 0 and not rec.complete:
                self._recs[rec.uid] = rec
            else:
                self._recs.pop(rec.uid, None)
            return
        ap = native().AllocPod()
        ap.uid, ap.key, ap.namespace, ap.name, ap.rv = rec.uid, rec.key, rec.namespace, rec.name, rec.rv
        ap.phase, ap.creation, ap.node = rec.phase, rec.creation, podutil.node_name(pod)
        ap.dev, ap.request, ap.containers, ap.assume_time = rec.dev, rec.request, rec.containers, rec.assume_time
        ap.assigned, ap.complete, ap.cu_count, ap.cu_mask = rec.assigned, rec.complete, rec.cu_count, rec.cu_mask
        ap.hold_idx, ap.hold_partner = rec.hold_idx, rec.hold_partner
        ap.terminating = bool(podutil.meta(pod).get("deletionTimestamp")) and not podutil.is_terminal(pod)
        tg = (pod.get("spec") or {}).get("terminationGracePeriodSeconds")
        ap.term_grace_s = float(tg) if isinstance(tg, (int, float)) and tg >= 0 else 0.0
        try:
            ap.dev_total = int(podutil.annotations(pod).get(self.profile.annotation_dev, "-1") or -1)
        except ValueError:
            ap.dev_total = -1
        if self._native_pods is not None:
            ap.raw = json.dumps(pod, separators=(",", ":"))
        if not self.core.observe(ap):
            return  # a stale copy (e.g. a slow LIST racing the watch): never step back
        if self._native_pods is not None:
            self._flush()
            return
        if self.core.has_pod(rec.uid):
            self._recs[rec.uid] = rec
        else:
            self._recs.pop(rec.uid, None)
        self._flush()

    def forget(self, pod: dict) -> None:
        """A deleted pod (watch DELETE or gone from a re-list): released and remembered (AllocState::deleted), so a
        copy of it another feed still delivers cannot bring it back.  Deleted while live here (a force delete), what
        its containers hold lingers on their GPUs for their termination grace."""
        uid = podutil.meta(pod).get("uid", "")
        if not uid:
            return
        self.core.deleted(uid, time.time())
        self._recs.pop(uid, None)
        self._flush()

    def resync(self, pods: list[dict]) -> None:
        """A complete LIST of this node's pods: anything we hold that is not in it is gone."""
        seen = []
        for p in pods:
            self.observe(p)
            seen.append(podutil.meta(p).get("uid", ""))
        self.core.resync(seen, time.time())
        self._prune()

    def holders(self) -> set[str]:
        return set(self.core.holders())

    def release(self, uid: str) -> None:
        if not uid:
            return
        self.core.release(uid)
        self._recs.pop(uid, None)
        self._flush()

    def _prune(self):
        live = set(self.core.pod_uids())
        for uid in [u for u in self._recs if u not in live]:
            del self._recs[uid]
        self._flush()

    def flush_dropped(self) -> None:
        """Run the drop callbacks for records the native side dropped on its own (the plugin's pod feed)."""
        self._flush()

    def _flush(self):
        for d in self.core.take_dropped():
            r = AllocRecord.from_dict(d)
            for cb in self.on_drop:
                cb(r)

    # ------------------------------------------------------------ Allocate
    def candidates(self) -> list[PodRec]:
        pods = self.pods
        return [pods[u] for u in self.core.candidates() if u in pods]

    def match(self, units: int) -> tuple[PodRec | None, bool]:
        """(pod, whole_pod) for an Allocate of ``units``: a whole pod of that size (earliest ASSUME_TIME),
        else a later container of a pod whose first container was allocated, else the first container
        of a multi-container pod that has a container of that size."""
        uid, whole = self.core.match(int(units))
        return (self.fresh(self.pods.get(uid)), whole) if uid else (None, False)

    def fresh(self, rec: PodRec | None) -> PodRec | None:
        """``rec`` with the allocation fields the native state holds for it: the native pod feed may be ahead of the
        Python informer's copy, and the matcher decided on the native one (an Allocate acting on a stale ASSIGNED
        or GPU would take the wrong branch)."""
        if rec is None:
            return None
        if self._native_pods is not None:
            return self._native_pods.get(rec.uid, rec)  # the native state is the one view
        v = self.core.pod_view(rec.uid)
        if v is None or not _older_rv(rec.rv, v["rv"]):
            return rec
        rec.rv, rec.phase, rec.dev, rec.assigned = v["rv"], v["phase"], int(v["dev"]), v["assigned"]
        rec.cu_mask, rec.hold_idx, rec.hold_partner = v["cu_mask"], int(v["hold_idx"]), v["hold_partner"]
        return rec

    def unannotated(self, units: int) -> bool:
        """A pending pod of this size bound to the node without any allocation annotation (``*_IDX``)."""
        return self.core.unannotated(int(units))

    def preferred_device(self, units: int) -> int:
        return self.core.preferred_device(int(units))

    def claim_cus(self, rec: PodRec) -> list[int] | None:
        if not rec.cu_count:
            return None
        try:
            return list(self.core.claim_cus(rec.uid))
        except ValueError as e:
            raise AllocateError(str(e)) from e

    def first_container_committed(self, rec: PodRec, units: int, whole: bool) -> None:
        """The ASSIGNED=true patch of ``rec`` succeeded for a container of ``units``."""
        self.core.first_container_committed(rec.uid, int(units), whole)

    def later_container_allocated(self, rec: PodRec, units: int) -> None:
        self.core.later_container_allocated(rec.uid, int(units))

    # ------------------------------------------------------------ allocation records
    def record(self, rec: PodRec, ids, units: int, cu_mask: str, aid: str, t: float = 0.0,
               iso: str = "", on_gpu: bool = False) -> AllocRecord:
        """An Allocate of ``ids`` was matched to ``rec`` (kubelet re-using the IDs of a finished pod replaces the
        older record).  ``on_gpu``: every ID lies on the pod's GPU."""
        d = self.core.record(rec.uid, list(ids), int(units), cu_mask or "", aid, t, iso)
        if on_gpu:
            self.core.mark_on_gpu(aid, True)
            d["on_gpu"] = True
        self._flush()
        return AllocRecord.from_dict(d)

    def restore_record(self, r: AllocRecord) -> None:
        self.core.add_record(r.to_dict())

    def drop_record(self, r: AllocRecord) -> None:
        self.core.drop_record(r.aid)
        self._flush()

    def record_for_ids(self, ids) -> AllocRecord | None:
        d = self.core.record_for_ids(list(ids))
        return AllocRecord.from_dict(d) if d else None

    def set_owner(self, aid: str, uid: str) -> None:
        self.core.set_owner(aid, uid)

    def pod_by_key(self, key: str) -> PodRec | None:
        """ns/name -> pod: one lookup in the native key index (the reconciliation asks for every pod kubelet
        reports; walking every pod's view per question made a pass O(P^2) copies under the state lock)."""
        if self._native_pods is not None:
            uid = self.core.uid_for_key(key)
            return self._native_pods.get(uid) if uid else None
        for r in self._recs.values():
            if r.key == key:
                return r
        return None

    def move_records(self, p_uid: str, q_uid: str, r) -> None:
        """After the annotations of P and Q were exchanged because P holds ``r`` (built for Q): ``r`` now
        describes P, and whatever described P describes Q.  The CU partitions follow the same exchange."""
        self.core.move_records(p_uid, q_uid, r.aid if isinstance(r, AllocRecord) else str(r))

    def snapshot(self) -> dict:
        """What ``/debug/state`` and the tests look at."""
        pods = dict(self.pods.items())
        return {
            "pods": {r.key: {"uid": r.uid, "gpu": r.dev, "request": r.request, "assigned": r.assigned,
                             "phase": r.phase} for r in pods.values()},
            "candidates": [r.key for r in self.candidates()],
            "partial": {pods[u].key if u in pods else u: v for u, v in self.partial.items()},
            "cu_partitions": {str(i): {pods[u].key if u in pods else u: len(c) for u, c in cp.held().items()}
                              for i, cp in self.cus.items()},
            "cu_free": {str(i): cp.free_count() for i, cp in self.cus.items()},
            "records": self.core.record_count(),
            # the physical account (units kubelet has handed out per GPU, by Allocate IDs) the Allocate guard reads
            "physical": {str(i): self.core.physical_used(i) for i in self.cus},
            "held": self.core.held_count(),
            "native": True,
        }
