"""GPU inventory for the device plugin: what each MI355X offers to gpu-mem sharing.

Upstream's device plugin reads NVML through cgo (``docs/designs/designs.md:59``).
Here the inventory comes from, in order of preference:

* ``amdsmi``  — the native C++ ``_mxdev`` module over libamd_smi (BDF, UUID,
  VRAM total, render / card minor, KFD id, partition, xGMI links, health);
* ``hip``     — ``libgsx_kernels.so`` (hipGetDeviceProperties + hipMemGetInfo),
  used where amdsmi has no access (containers without /sys/class/drm);
* ``fake``    — a JSON topology (``GSX_FAKE_DEVICES``: a file path or a spec
  like ``8x288GB``) for CPU-only tests and the simulator.

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
    healthy: bool = True
    numa_node: int = -1
    links: dict = field(default_factory=dict)  # peer index -> link type ("XGMI", "PCIE")

    def units(self, unit: str, reserve_bytes: int = 0) -> int:
        return max(0, (self.total_bytes - reserve_bytes) // UNITS[unit])

    def device_nodes(self) -> list[str]:
        out = ["/dev/kfd"]
        if self.render_minor >= 0:
            out.append(f"/dev/dri/renderD{self.render_minor}")
        if self.card_minor >= 0:
            out.append(f"/dev/dri/card{self.card_minor}")
        return out

    def to_dict(self) -> dict:
        return asdict(self)


_SPEC = re.compile(r"^(\d+)x(\d+(?:\.\d+)?)(GB|GiB|MiB|MB)$")


def fake_devices(spec: str) -> list[Device]:
    """``8x288GB`` or a JSON file ``[{"total_bytes":...}, ...]``."""
    m = _SPEC.match(spec.strip())
    if m:
        n, size, unit = int(m.group(1)), float(m.group(2)), m.group(3)
        total = int(size * UNITS[unit])
        return [Device(index=i, bdf=f"0000:{0x05 + 0x10 * i:02x}:00.0", uuid=f"fake-{i:04d}", total_bytes=total,
                       render_minor=128 + 8 * i, card_minor=i + 1, kfd_id=i)
                for i in range(n)]
    with open(spec) as f:
        items = json.load(f)
    out = []
    for i, d in enumerate(items):
        d = dict(d)
        d.setdefault("index", i)
        out.append(Device(**d))
    return out


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
        return "fake", fake_devices(fake or "8x288GB")
    errors = []
    if backend in ("auto", "amdsmi"):
        try:
            devs = amdsmi_devices()
            if devs:
                return "amdsmi", devs
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
