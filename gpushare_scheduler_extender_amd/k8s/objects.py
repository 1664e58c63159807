"""Factories for synthetic v1.Pod / v1.Node objects (tests, simulator, bench)."""
from __future__ import annotations

import uuid as _uuid

from ..models.profile import NamingProfile, SHARED_GPU, NODE_DEVICE_MEMORY_ANNOTATION


def make_pod(name: str, mem: int | str | list = 0, *, namespace: str = "default", profile: NamingProfile = SHARED_GPU,
             node: str = "", uid: str | None = None, annotations: dict | None = None, phase: str = "Pending",
             scheduler_name: str = "default-scheduler", labels: dict | None = None,
             image: str = "rocm/pytorch:latest", deletion_timestamp: str | None = None) -> dict:
    """A pod whose containers request ``mem`` units of gpu-mem (a list = one container each)."""
    mems = mem if isinstance(mem, list) else [mem]
    containers = []
    for i, m in enumerate(mems):
        c = {"name": f"{name}-{i}" if len(mems) > 1 else name, "image": image, "resources": {}}
        if m not in (0, "0", None):
            c["resources"] = {"limits": {profile.resource: str(m)}}
        containers.append(c)
    md = {"name": name, "namespace": namespace, "uid": uid or str(_uuid.uuid4())}
    if annotations:
        md["annotations"] = dict(annotations)
    if labels:
        md["labels"] = dict(labels)
    if deletion_timestamp:
        md["deletionTimestamp"] = deletion_timestamp
    spec = {"containers": containers, "schedulerName": scheduler_name}
    if node:
        spec["nodeName"] = node
    return {"apiVersion": "v1", "kind": "Pod", "metadata": md, "spec": spec, "status": {"phase": phase}}


def make_node(name: str, total: int = 0, count: int = 0, *, profile: NamingProfile = SHARED_GPU,
              address: str = "10.0.0.1", device_totals: list[int] | None = None, labels: dict | None = None,
              annotations: dict | None = None, extra_capacity: dict | None = None) -> dict:
    cap = {"cpu": "192", "memory": "2113645384Ki", "pods": "110"}
    if total:
        cap[profile.resource] = str(total)
    if count:
        cap[profile.count] = str(count)
    if extra_capacity:
        cap.update(extra_capacity)
    ann = dict(annotations or {})
    if device_totals is not None:
        ann[NODE_DEVICE_MEMORY_ANNOTATION] = ",".join(str(x) for x in device_totals)
    md = {"name": name, "uid": str(_uuid.uuid4()), "labels": dict(labels or {"kubernetes.io/hostname": name})}
    if ann:
        md["annotations"] = ann
    return {
        "apiVersion": "v1",
        "kind": "Node",
        "metadata": md,
        "spec": {},
        "status": {
            "capacity": cap,
            "allocatable": dict(cap),
            "addresses": [{"type": "InternalIP", "address": address}, {"type": "Hostname", "address": name}],
            "conditions": [{"type": "Ready", "status": "True"}],
        },
    }
