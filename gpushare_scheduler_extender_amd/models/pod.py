"""Pod / node accessors on plain JSON dicts.

Python counterparts of the reference's ``pkg/utils/pod.go`` and
``pkg/utils/node.go`` used by the device plugin, the scheduler simulator, the
fake apiserver and the CLI.  (The extender itself uses the native engine's
C++ extraction, native/engine/model.cc.)
"""
from __future__ import annotations

import copy
import time

from .profile import NamingProfile, NODE_DEVICE_MEMORY_ANNOTATION
from .quantity import parse_quantity


def meta(obj: dict) -> dict:
    return obj.get("metadata") or {}


def annotations(obj: dict) -> dict:
    return meta(obj).get("annotations") or {}


def pod_key(pod: dict) -> str:
    m = meta(pod)
    return f"{m.get('namespace', '')}/{m.get('name', '')}"


def phase(pod: dict) -> str:
    return (pod.get("status") or {}).get("phase", "")


def node_name(pod: dict) -> str:
    return (pod.get("spec") or {}).get("nodeName", "") or ""


def is_terminal(pod: dict) -> bool:
    return phase(pod) in ("Succeeded", "Failed")


def is_complete(pod: dict) -> bool:
    """pkg/utils/pod.go:28-37 IsCompletePod."""
    return bool(meta(pod).get("deletionTimestamp")) or is_terminal(pod)


def assigned_non_terminated(pod: dict) -> bool:
    """pkg/utils/pod.go:13-25 AssignedNonTerminatedPod."""
    return not meta(pod).get("deletionTimestamp") and bool(node_name(pod)) and not is_terminal(pod)


def container_limit(container: dict, resource: str) -> int:
    lim = ((container.get("resources") or {}).get("limits") or {}).get(resource)
    if lim is None:
        return 0
    try:
        return parse_quantity(lim)
    except ValueError:
        return 0


def gpu_mem_request(pod: dict, profile: NamingProfile) -> int:
    """Sum of container limits (pkg/utils/pod.go:146-155); init containers ignored."""
    return sum(container_limit(c, profile.resource) for c in (pod.get("spec") or {}).get("containers") or [])


def is_gpushare_pod(pod: dict, profile: NamingProfile) -> bool:
    """pkg/utils/pod.go:40-42."""
    return gpu_mem_request(pod, profile) > 0


def _atoi(v) -> int | None:
    """Go's strconv.Atoi on a 64-bit platform: ASCII digits with an optional sign, within int64, else None."""
    if not isinstance(v, str) or not v:
        return None
    s = v[1:] if v[0] in "+-" else v
    if not s.isdigit() or not s.isascii():
        return None
    n = int(v)
    return n if -(2**63) <= n < 2**63 else None


def gpu_id_from_annotation(pod: dict, profile: NamingProfile) -> int:
    """pkg/utils/pod.go:45-60: -1 if absent or invalid."""
    v = _atoi(annotations(pod).get(profile.annotation_idx))
    return -1 if v is None or v < 0 else v


def hold_idx(pod: dict) -> int:
    """``gpushare.amd.com/hold-idx``: the second device a pod is charged on during a reconciliation, else -1."""
    from .profile import POD_HOLD_IDX_ANNOTATION  # noqa: PLC0415

    v = _atoi(annotations(pod).get(POD_HOLD_IDX_ANNOTATION))
    return -1 if v is None or v < 0 else v


def gpu_mem_from_annotation(pod: dict, profile: NamingProfile) -> int:
    """pkg/utils/pod.go:94-113: parse errors / negatives -> 0."""
    v = _atoi(annotations(pod).get(profile.annotation_pod))
    return 0 if v is None or v < 0 else v


def assume_time(pod: dict, profile: NamingProfile) -> int:
    v = _atoi(annotations(pod).get(profile.annotation_assume_time))
    return -1 if v is None else v


def is_assigned(pod: dict, profile: NamingProfile) -> bool:
    return annotations(pod).get(profile.annotation_assigned) == "true"


def bind_annotations(profile: NamingProfile, dev_id: int, dev_total: int, pod_mem: int,
                     now_ns: int | None = None) -> dict[str, str]:
    """The allocation record written at bind (pkg/utils/pod.go:192-206)."""
    return {
        profile.annotation_idx: str(dev_id),
        profile.annotation_dev: str(dev_total),
        profile.annotation_pod: str(pod_mem),
        profile.annotation_assigned: "false",
        profile.annotation_assume_time: str(time.time_ns() if now_ns is None else now_ns),
    }


def with_annotations(pod: dict, ann: dict[str, str]) -> dict:
    p = copy.deepcopy(pod)
    p.setdefault("metadata", {}).setdefault("annotations", {}).update(ann)
    return p


# ---------------------------------------------------------------- nodes (node.go)

def node_capacity(node: dict, resource: str) -> int:
    v = ((node.get("status") or {}).get("capacity") or {}).get(resource)
    if v is None:
        return 0
    try:
        return parse_quantity(v)
    except ValueError:
        return 0


def node_allocatable(node: dict, resource: str) -> int:
    st = node.get("status") or {}
    v = (st.get("allocatable") or {}).get(resource)
    if v is None:
        v = (st.get("capacity") or {}).get(resource)
    if v is None:
        return 0
    try:
        return parse_quantity(v)
    except ValueError:
        return 0


def is_gpushare_node(node: dict, profile: NamingProfile) -> bool:
    """pkg/utils/node.go:6-12."""
    return node_capacity(node, profile.resource) > 0


def node_device_totals(node: dict, profile: NamingProfile) -> list[int]:
    total = node_capacity(node, profile.resource)
    count = node_capacity(node, profile.count)
    ann = annotations(node).get(NODE_DEVICE_MEMORY_ANNOTATION)
    if ann:
        try:
            vals = [int(x) for x in ann.split(",")]
            if len(vals) == count:
                return vals
        except ValueError:
            pass
    if count <= 0:
        return []
    return [total // count] * count


def node_address(node: dict) -> str:
    for a in (node.get("status") or {}).get("addresses") or []:
        if a.get("type") == "InternalIP":
            return a.get("address", "")
    return ""
