"""The native amdsmi layer (``native/mxdev``) on a real MI355X.

amdsmi enumeration, VRAM totals, BDF and render node, health counters and link
types are checked against what HIP reports for the same GPU — the inventory the
device plugin advertises to kubelet and publishes on the node.  HIP is queried in
a child process so this process only ever talks to amdsmi.
"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _hip_view() -> list[dict]:
    code = ("import json;from gpushare_scheduler_extender_amd.ops import hip;"
            "out=[];"
            "[out.append(dict(hip.device_info(i), total=hip.mem_info(i)[1])) for i in range(hip.device_count())];"
            "print(json.dumps(out))")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=180, cwd=ROOT,
                       env=dict(os.environ, PYTHONPATH=ROOT))
    assert r.returncode == 0, r.stderr[-2000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


def test_amdsmi_inventory_matches_hip():
    from gpushare_scheduler_extender_amd.ops import mxdev

    s = mxdev.session("amdsmi")
    assert s.backend == "amdsmi"
    devs = s.devices()
    hip = _hip_view()
    assert len(devs) >= 1 and len(devs) == len(hip), (devs, hip)
    by_bdf = {h["pci_bus_id"].lower(): h for h in hip}
    for d in devs:
        print(json.dumps({k: v for k, v in d.items() if k != "links"}))
        assert d["arch"].startswith("gfx950"), d
        assert d["cu_count"] == 256 and d["xcc_count"] == 8, d
        h = by_bdf.get(d["bdf"].lower())
        assert h is not None, (d["bdf"], list(by_bdf))
        # amdsmi VRAM total vs hipMemGetInfo total: same device memory (hip may hold back a little)
        assert abs(d["total_bytes"] - h["total"]) <= 0.02 * d["total_bytes"], (d["total_bytes"], h["total"])
        assert d["total_bytes"] > 250 * 10**9
        assert d["render_minor"] >= 128 and os.path.exists(f"/dev/dri/renderD{d['render_minor']}"), d
        assert d["partition"] in ("SPX", "DPX", "QPX", "CPX", "UNKNOWN", ""), d
        assert d["links"].get(d["index"]) in ("SELF", None), d["links"]
        assert d["pool"] and d["bdf"].startswith(d["pool"]), d
        print("memory partition:", d["memory_partition"], "partition id:", d["partition_id"])


def test_amdsmi_discover_memory_pools():
    """Logical devices of one physical GPU advertise its HBM once (SPX on the box: one device per pool)."""
    from gpushare_scheduler_extender_amd.deviceplugin.devices import discover

    backend, devs = discover("amdsmi")
    assert backend == "amdsmi"
    pools = {}
    for d in devs:
        pools.setdefault(d.pool, []).append(d)
    for members in pools.values():
        if len(members) == 1:
            assert members[0].share_bytes == 0 and members[0].usable_bytes == members[0].total_bytes
        else:  # a partitioned GPU: the shares never add up to more than the GPU's memory
            nps = members[0].memory_partition
            n_pools = int(nps[3:]) if nps.startswith("NPS") else 1
            assert sum(d.usable_bytes for d in members) <= n_pools * max(d.total_bytes for d in members)


def test_amdsmi_health_counters_readable():
    from gpushare_scheduler_extender_amd.ops import mxdev

    s = mxdev.session("amdsmi")
    for d in s.devices():
        h = s.health(d["index"])
        print(d["index"], h)
        assert h["healthy"] is True and h["reason"] == ""
        assert h["ecc_uncorrectable"] >= 0 and h["ecc_correctable"] >= 0
        # RAS per block (HBM / GFX / SDMA / xGMI), the xGMI link status, throttle state and the partition modes
        # the plugin polls (a partition change re-shapes the advertised devices)
        for k in ("ras_umc_uncorrectable", "ras_gfx_uncorrectable", "ras_sdma_uncorrectable",
                  "ras_xgmi_uncorrectable", "ras_xgmi_correctable"):
            assert h[k] >= 0, (k, h)
        assert h["xgmi_error"] == 0, h
        assert isinstance(h["thermal_throttle"], bool) and isinstance(h["power_throttle"], bool)
        assert h["partition"] == d["partition"] and h["memory_partition"] == d["memory_partition"], (h, d)


def test_device_plugin_advertises_real_inventory():
    """What ListAndWatch would advertise for this node: gpu-mem in GiB, one fake ID per GiB per GPU."""
    from gpushare_scheduler_extender_amd.deviceplugin.devices import discover
    from gpushare_scheduler_extender_amd.deviceplugin.plugin import fake_ids

    backend, devs = discover("amdsmi")
    assert backend == "amdsmi"
    per_dev = {d.index: fake_ids(d, d.units("GiB")) for d in devs}
    ids = [i for v in per_dev.values() for i in v]
    assert len(set(ids)) == len(ids)  # kubelet needs unique device IDs across the node
    assert all(len(v) >= 256 for v in per_dev.values()), {k: len(v) for k, v in per_dev.items()}
