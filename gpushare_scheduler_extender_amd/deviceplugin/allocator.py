"""Device-plugin Allocate building blocks: the container response, the ASSIGNED patch, CU partitions.

Which pod an Allocate belongs to is decided by :mod:`.state` (one implementation, used by the
gRPC plugin and the kubelet stand-in alike).

Behaviour reconstructed from ``docs/designs/designs.md:93-103`` and
``docs/designs/sequence.jpg`` (the plugin itself is not in the reference tree,
SURVEY.md §2.8):

1. kubelet asks for N fake device IDs (N = gpu-mem units of the container);
2. the plugin lists this node's Pending gpushare pods whose ``ASSIGNED``
   annotation is ``false``, ordered by ``ASSUME_TIME`` (earliest first), and
   takes the first whose request equals N;
3. it flips ``ASSIGNED`` to ``true`` (with a resourceVersion precondition, so
   two Allocates can never claim the same pod) — the commit point;
4. it returns the container's environment and device nodes.

MI355X-specific response: ``/dev/kfd`` + the chosen GPU's
``/dev/dri/renderD*`` / ``card*`` nodes, ``HIP_VISIBLE_DEVICES`` /
``ROCR_VISIBLE_DEVICES`` (0 inside the container when only that GPU's nodes
are mounted, the host index otherwise), the ``*_IDX/_DEV/_POD/_CONTAINER``
variables the sample workload reads (``samples/docker/run.sh:3-6``), a memory
fraction for ``torch.cuda.set_per_process_memory_fraction``, and — optional —
a per-pod CU partition (``HSA_CU_MASK`` + ``GSX_CU_MASK``), the stand-in for
the reference's "integrate Nvidia MPS" roadmap item (``README.md:77``).
"""
from __future__ import annotations

import time
from dataclasses import dataclass, field

from ..core.engine import native as _native
from ..models import pod as podutil
from ..models.profile import POD_ASSIGN_TIME_ANNOTATION, POD_CU_COUNT_ANNOTATION, NamingProfile
from .devices import Device

CU_COUNT_ANNOTATION = POD_CU_COUNT_ANNOTATION  # pod asks for a CU partition of this size


@dataclass
class ContainerAllocation:
    envs: dict[str, str]
    devices: list[dict]  # {container_path, host_path, permissions}
    annotations: dict[str, str] = field(default_factory=dict)
    mounts: list[dict] = field(default_factory=list)  # {container_path, host_path, read_only}
    iso: str = ""  # the isolation directory key (pod UID) its mounts point at


class AllocateError(Exception):
    pass


class CUPartitioner:
    """Per-device ledger of compute units handed to pods as CU masks (the native ``_engine.CuPartitioner``,
    ``native/engine/allocstate.cc``: the same code the compiled node agent runs).

    A partition is spread evenly over the XCDs (CU ``c`` of a 256-CU MI355X is
    logical CU ``c``; ROCr stripes logical CUs over XCDs/SEs, so contiguous
    ranges in *per-XCD* order keep each pod's work on every L2 slice).  The
    bitmap words are what ``hipExtStreamCreateWithCUMask`` and ``HSA_CU_MASK``
    take.
    """

    def __init__(self, cu_count: int = 256, xcc_count: int = 8, native_obj=None):
        from ..core.engine import native  # noqa: PLC0415

        self._p = native_obj if native_obj is not None else native().CuPartitioner(cu_count, xcc_count)
        self.cu_count = self._p.cu_count
        self.xcc_count = self._p.xcc_count

    def allocate(self, uid: str, n: int) -> list[int]:
        try:
            return list(self._p.allocate(uid, int(n)))
        except ValueError as e:
            raise AllocateError(str(e)) from e

    def release(self, uid: str) -> int:
        return self._p.release(uid)

    def adopt(self, uid: str, cus: list[int]) -> list[int]:
        """Record an existing partition (rebuilt from a pod's cu-mask annotation); returns the CUs that
        another pod already owned (left with their owner)."""
        return list(self._p.adopt(uid, list(cus)))

    def swap_owners(self, a: str, b: str) -> None:
        """Exchange the partitions of pods ``a`` and ``b`` (either may hold none)."""
        self._p.swap_owners(a, b)

    def holds(self, uid: str) -> bool:
        return self._p.holds(uid)

    def held(self) -> dict[str, list[int]]:
        return {u: list(c) for u, c in self._p.held().items()}

    def free_count(self) -> int:
        return self._p.free_count()

    @staticmethod
    def words(cus: list[int], cu_count: int = 256) -> list[int]:
        w = [0] * ((cu_count + 31) // 32)
        for c in cus:
            w[c // 32] |= 1 << (c % 32)
        return w

    @staticmethod
    def ranges(cus: list[int]) -> str:
        """``0-7,32-39`` — the list syntax of ROCr's HSA_CU_MASK."""
        from ..core.engine import native  # noqa: PLC0415

        return native().cu_ranges(sorted(cus))


def build_response(pod: dict, device: Device, container_units: int, profile: NamingProfile, *,
                   mount_mode: str = "isolated", cus: list[int] | None = None) -> ContainerAllocation:
    """Env + device nodes for one container of ``pod`` on ``device``: the reference's env contract
    (``*_IDX``, ``*_DEV``, ``*_POD``, the container's share), ``HIP/ROCR_VISIBLE_DEVICES``, the memory fraction
    (scaled to the HBM pool of a partition that shares one), the CU partition (``GSX_CU_MASK`` bitmap words,
    ``HSA_CU_MASK`` ranges, the ``cu-mask`` pod annotation) and, in ``isolated`` mount mode, the GPU's device
    nodes.  One implementation: ``native/engine/dpcore.cc`` build_response, which the native Allocate path uses."""
    E = _native()
    ap = E.AllocPod()
    try:
        ap.dev_total = int(podutil.annotations(pod).get(profile.annotation_dev, "0") or 0)
    except ValueError:
        ap.dev_total = 0
    ap.request = podutil.gpu_mem_request(pod, profile)
    dev = {"index": device.index, "bdf": device.bdf, "cu_count": device.cu_count, "total_bytes": device.total_bytes,
           "share_bytes": device.share_bytes, "nodes": device.device_nodes()}
    r = E.build_response(ap, dev, int(container_units), list(cus or []), mount_mode,
                         {**profile.engine_dict(), "env_container": profile.env_container})
    return ContainerAllocation(envs=dict(r["envs"]), devices=list(r["devices"]), annotations=dict(r["annotations"]))


def assigned_patch(pod: dict, profile: NamingProfile, extra: dict | None = None) -> dict:
    """Merge patch flipping ASSIGNED to true, guarded by the pod's resourceVersion."""
    ann = {profile.annotation_assigned: "true", POD_ASSIGN_TIME_ANNOTATION: str(time.time_ns())}
    if extra:
        ann.update(extra)
    return {"metadata": {"resourceVersion": podutil.meta(pod).get("resourceVersion"), "annotations": ann}}
