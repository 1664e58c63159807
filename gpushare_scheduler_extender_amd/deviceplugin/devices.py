"""GPU inventory for the device plugin: what each MI355X offers to gpu-mem sharing.

Upstream's device plugin reads NVML through cgo (``docs/designs/designs.md:59``).
Here the inventory comes from, in order of preference:

* ``amdsmi``  — the native C++ ``_mxdev`` module over libamd_smi (BDF, UUID,
  VRAM total, render / card minor, KFD id, partition, xGMI links, health);
* ``hip``     — ``libgsx_kernels.so`` (hipGetDeviceProperties + hipMemGetInfo),
  used where amdsmi has no access (containers without /sys/class/drm);
* ``fake``    — a JSON topology (``GSX_FAKE_DEVICES``: a file path or a spec
  like ``8x288GB``) for CPU-only tests and the simulator.

Compute / memory partitions.  An MI355X in DPX / QPX / CPX mode appears as
2 / 4 / 8 logical devices (one PCI function each), and in NPS1 they all sit in
one 288 GB HBM pool; KFD reports that pool's VRAM to every partition.  Summing
the raw totals would advertise 8 x 288 GB per GPU in CPX/NPS1, so
``apply_memory_pools`` gives each logical device its share of the pool
(``share_bytes``) and ``units()`` advertises that.  ``GSX_MEMORY_POOLS=off``
advertises the raw totals (for a driver that already reports per-partition
VRAM).  The CU count and XCD count follow the partition (CPX: 32 CUs on 1 XCD),
so per-pod CU masks stay inside the logical device.

Memory is advertised in a configurable unit.  GiB is the default on MI355X:
kubelet's device-plugin API needs one fake device ID per unit, and MiB would
mean 8 x ~274k IDs per node.
"""
from __future__ import annotations

import json
import os
import re
from dataclasses import asdict, dataclass, field

UNITS = {"B": 1, "KiB": 1 << 10, "MiB": 1 << 20, "GiB": 1 << 30, "GB": 10**9, "MB": 10**6}


@dataclass
class Device:
    index: int
    name: str = "AMD Instinct MI355X"
    arch: str = "gfx950"
    bdf: str = ""
    uuid: str = ""
    total_bytes: int = 288 * 10**9
    cu_count: int = 256
    xcc_count: int = 8
    render_minor: int = -1  # /dev/dri/renderD<minor>
    card_minor: int = -1  # /dev/dri/card<minor>
    kfd_id: int = -1
    partition: str = "SPX"
    memory_partition: str = ""  # NPS1 / NPS2 / NPS4 / NPS8
    partition_id: int = 0  # compute-partition index on its physical GPU
    pool: str = ""  # physical GPU key (BDF without the function): partitions of one GPU share it
    share_bytes: int = 0  # this device's share of its HBM pool (0: the whole total_bytes)
    healthy: bool = True
    numa_node: int = -1
    links: dict = field(default_factory=dict)  # peer index -> link type ("XGMI", "PCIE")

    @property
    def usable_bytes(self) -> int:
        return self.share_bytes or self.total_bytes

    def units(self, unit: str, reserve_bytes: int = 0) -> int:
        return max(0, (self.usable_bytes - reserve_bytes) // UNITS[unit])

    def device_nodes(self) -> list[str]:
        out = ["/dev/kfd"]
        if self.render_minor >= 0:
            out.append(f"/dev/dri/renderD{self.render_minor}")
        if self.card_minor >= 0:
            out.append(f"/dev/dri/card{self.card_minor}")
        return out

    def to_dict(self) -> dict:
        return asdict(self)


_SPEC = re.compile(r"^(\d+)x(\d+(?:\.\d+)?)(GB|GiB|MiB|MB)(?::(SPX|DPX|QPX|CPX))?(?::NPS(1|2|4|8))?$")
PARTITIONS = {"SPX": 1, "DPX": 2, "QPX": 4, "CPX": 8}
XCDS_PER_GPU = 8
CUS_PER_GPU = 256


def fake_devices(spec: str) -> list[Device]:
    """``8x288GB``, ``8x288GB:CPX:NPS1`` (8 GPUs x 8 partitions) or a JSON file ``[{"total_bytes":...}, ...]``.

    Same layout as the native fake backend (``native/mxdev/mxdev.cc: fake_spec``): partition ``p`` of GPU ``g``
    is PCI function ``p`` and reports the VRAM of its memory pool.
    """
    m = _SPEC.match(spec.strip())
    if m:
        n, size, unit = int(m.group(1)), float(m.group(2)), m.group(3)
        mode, nps = m.group(4) or "SPX", int(m.group(5) or 1)
        parts = PARTITIONS[mode]
        if nps > parts:
            raise ValueError(f"NPS{nps} needs at least as many compute partitions ({mode})")
        pool = int(size * UNITS[unit]) // nps
        out = []
        for g in range(n):
            for p in range(parts):
                i = g * parts + p
                bdf = f"0000:{0x05 + 0x10 * g:02x}:00.{p}"
                out.append(Device(index=i, bdf=bdf, uuid=f"fake-{i:04d}", total_bytes=pool,
                                  cu_count=CUS_PER_GPU // parts, xcc_count=XCDS_PER_GPU // parts,
                                  render_minor=128 + 8 * i if parts == 1 else 128 + i, card_minor=i + 1, kfd_id=i,
                                  partition=mode, memory_partition=f"NPS{nps}" if m.group(4) else "",
                                  partition_id=p, pool=bdf[:-2]))
        return out
    with open(spec) as f:
        items = json.load(f)
    out = []
    for i, d in enumerate(items):
        d = dict(d)
        d.setdefault("index", i)
        out.append(Device(**d))
    return out


def apply_memory_pools(devs: list[Device], mode: str | None = None) -> list[Device]:
    """Set ``share_bytes`` so that logical devices sharing one HBM pool advertise it once in total.

    A physical GPU (devices with the same ``pool`` key) in compute mode ``c`` (1/2/4/8 partitions) and memory
    mode NPS``k`` has ``k`` pools, each shared by ``c / k`` partitions; a partition's share is its reported
    (pool) VRAM divided by that, the remainder going to the lowest partition ids.  Unknown NPS is taken as
    NPS1, which never over-advertises.  ``mode`` (default ``GSX_MEMORY_POOLS``): ``auto`` or ``off``.
    """
    mode = mode or os.environ.get("GSX_MEMORY_POOLS", "auto")
    for d in devs:
        d.share_bytes = 0
    if mode == "off":
        return devs
    if mode != "auto":
        raise ValueError(f"GSX_MEMORY_POOLS must be auto or off, got {mode!r}")
    groups: dict[str, list[Device]] = {}
    for d in devs:
        if d.pool:
            groups.setdefault(d.pool, []).append(d)
    for members in groups.values():
        if len(members) < 2:
            continue
        nps_s = (members[0].memory_partition or "").upper()
        nps = int(nps_s[3:]) if nps_s.startswith("NPS") and nps_s[3:].isdigit() else 1
        per_pool = max(1, len(members) // max(1, nps))
        if per_pool == 1:
            continue
        members.sort(key=lambda d: d.partition_id)
        for k, d in enumerate(members):
            # partitions p, p+nps, p+2*nps ... share pool p % nps (interleaved like KFD's NUMA-node order)
            rank_in_pool = k // nps
            base, rem = divmod(d.total_bytes, per_pool)
            d.share_bytes = base + (1 if rank_in_pool < rem else 0)
    return devs


def hip_devices() -> list[Device]:
    from ..ops import hip  # noqa: PLC0415

    out = []
    for i in range(hip.device_count()):
        info = hip.device_info(i)
        _free, total = hip.mem_info(i)
        out.append(Device(index=i, name=info["name"] or "AMD Instinct MI355X", arch=info["arch"].split(":")[0],
                          bdf=info["pci_bus_id"].lower(), total_bytes=total, cu_count=info["cu_count"],
                          render_minor=_render_minor_for_bdf(info["pci_bus_id"].lower())))
    return out


def _render_minor_for_bdf(bdf: str) -> int:
    base = "/sys/class/drm"
    try:
        for e in os.listdir(base):
            if not e.startswith("renderD"):
                continue
            dev = os.path.realpath(os.path.join(base, e, "device"))
            if dev.rsplit("/", 1)[-1].lower() == bdf:
                return int(e[len("renderD"):])
    except OSError:
        pass
    return -1


def amdsmi_devices() -> list[Device]:
    from ..ops import mxdev  # noqa: PLC0415

    return [Device(**d) for d in mxdev.enumerate_devices()]


def discover(backend: str = "auto") -> tuple[str, list[Device]]:
    """Return (backend_used, devices)."""
    fake = os.environ.get("GSX_FAKE_DEVICES")
    if backend == "fake" or (backend == "auto" and fake):
        return "fake", apply_memory_pools(fake_devices(fake or "8x288GB"))
    errors = []
    if backend in ("auto", "amdsmi"):
        try:
            devs = amdsmi_devices()
            if devs:
                return "amdsmi", apply_memory_pools(devs)
        except Exception as e:  # noqa: BLE001
            errors.append(f"amdsmi: {e}")
        if backend == "amdsmi":
            raise RuntimeError("; ".join(errors))
    if backend in ("auto", "hip"):
        try:
            devs = hip_devices()
            if devs:
                return "hip", devs
        except Exception as e:  # noqa: BLE001
            errors.append(f"hip: {e}")
    raise RuntimeError("no GPU devices found (" + "; ".join(errors) + "); set GSX_FAKE_DEVICES for simulation")
