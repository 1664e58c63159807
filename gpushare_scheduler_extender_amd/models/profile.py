"""Resource / annotation naming profiles.

The reference hard-codes its names in ``pkg/utils/const.go:4-12``
(``shared-gpu/gpu-mem``, ``SHARED_GPU_MEM_IDX`` ...).  Upstream Aliyun naming
(``aliyun.com/gpu-mem``, ``ALIYUN_COM_GPU_MEM_*``) appears in
``docs/designs/bind.jpg`` and is what BASELINE.json's pod specs request, so the
domain is a switchable profile here.  Both profiles share one wire format.
"""
from __future__ import annotations

from dataclasses import asdict, dataclass, replace

# Annotations that are ours (not in the reference) and profile-independent.
NODE_DEVICE_MEMORY_ANNOTATION = "gpushare.amd.com/device-memory"  # "268,268,..." per-device totals
NODE_DEVICE_INFO_ANNOTATION = "gpushare.amd.com/devices"  # JSON device inventory from the plugin
# "landing": the node's device plugin matches an Allocate to the earliest pod *landed* on the node (kubelet's
# admission order, native/engine/allocstate.h); the extender then needs no ASSUME_TIME order of binds there
NODE_ALLOCATE_ORDER_ANNOTATION = "gpushare.amd.com/allocate-order"
# "true": the node's device plugin publishes its unaccounted GPU use to the extender (POST .../physical); after an
# extender restart or leader change binds to the node wait for its first publication (native/engine/ledger.h)
NODE_PHYSICAL_PUBLICATION_ANNOTATION = "gpushare.amd.com/physical-publication"
POD_CU_MASK_ANNOTATION = "gpushare.amd.com/cu-mask"  # per-pod CU partition (isolation)
POD_CU_COUNT_ANNOTATION = "gpushare.amd.com/cu-count"  # the pod asks for a CU partition of this size
POD_ASSIGN_TIME_ANNOTATION = "gpushare.amd.com/assign-time"
# reconciliation with kubelet's device assignments (deviceplugin/reconcile.py): while the plugin moves a pod's
# allocation record to the GPU kubelet really gave it, the pod is charged on its old device too (hold-idx);
# hold-partner keeps what the partner pod must receive, so a plugin restart can finish the move
POD_HOLD_IDX_ANNOTATION = "gpushare.amd.com/hold-idx"
POD_HOLD_PARTNER_ANNOTATION = "gpushare.amd.com/hold-partner"
POD_RECONCILED_ANNOTATION = "gpushare.amd.com/reconciled"  # count of record moves applied to this pod
NODE_RUNTIME_ENDPOINTS_ANNOTATION = "gpushare.amd.com/runtime-endpoints"  # JSON {gpu index: runtime shim URL}


@dataclass(frozen=True)
class NamingProfile:
    name: str
    resource: str  # gpu memory extended resource (node capacity, pod limits)
    count: str  # gpu count extended resource (node capacity)
    annotation_idx: str
    annotation_pod: str
    annotation_dev: str
    annotation_assigned: str
    annotation_assume_time: str
    env_container: str  # container env var with the pod's memory (run.sh / userguide.md:58-64)
    annotation_node_devices: str = NODE_DEVICE_MEMORY_ANNOTATION

    def engine_dict(self) -> dict:
        d = asdict(self)
        d.pop("name")
        d.pop("env_container")
        return d

    def with_(self, **kw) -> "NamingProfile":
        return replace(self, **kw)


SHARED_GPU = NamingProfile(
    name="shared-gpu",
    resource="shared-gpu/gpu-mem",
    count="shared-gpu/gpu-count",
    annotation_idx="SHARED_GPU_MEM_IDX",
    annotation_pod="SHARED_GPU_MEM_POD",
    annotation_dev="SHARED_GPU_MEM_DEV",
    annotation_assigned="SHARED_GPU_MEM_ASSIGNED",
    annotation_assume_time="SHARED_GPU_MEM_ASSUME_TIME",
    env_container="SHARED_GPU_MEM_CONTAINER",
)

ALIYUN = NamingProfile(
    name="aliyun",
    resource="aliyun.com/gpu-mem",
    count="aliyun.com/gpu-count",
    annotation_idx="ALIYUN_COM_GPU_MEM_IDX",
    annotation_pod="ALIYUN_COM_GPU_MEM_POD",
    annotation_dev="ALIYUN_COM_GPU_MEM_DEV",
    annotation_assigned="ALIYUN_COM_GPU_MEM_ASSIGNED",
    annotation_assume_time="ALIYUN_COM_GPU_MEM_ASSUME_TIME",
    env_container="ALIYUN_COM_GPU_MEM_CONTAINER",
)

PROFILES = {p.name: p for p in (SHARED_GPU, ALIYUN)}


def get_profile(name: str | None) -> NamingProfile:
    if not name:
        return SHARED_GPU
    try:
        return PROFILES[name]
    except KeyError as e:
        raise ValueError(f"unknown naming profile {name!r}; choose one of {sorted(PROFILES)}") from e
