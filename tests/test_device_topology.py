""""GPU i" must mean one physical device everywhere -- the HIP ordinal a bench rank's HBM arena lives
on, the device plugin's inventory entry, the render node a container of that GPU gets -- also on platforms whose
amdsmi enumeration (PCI order) differs from the HIP ordinals.  ``native/mxdev/fake_amdsmi.cc`` stands in for
libamd_smi.so with such a shuffled 8-GPU topology (amdsmi device k: BDF bus 0x11 + 0x10 k, renderD128+k, HIP ordinal
perm[k]); libmxdev loads it through ``GSX_AMDSMI_LIB``."""
import os
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
FAKE = ROOT / "build" / "libfake_amdsmi.so"
PERM = [3, 1, 0, 2, 7, 5, 4, 6]  # hip_id of amdsmi device k


@pytest.fixture(scope="module")
def shuffled(tmp_path_factory):
    if not FAKE.exists():
        subprocess.run([sys.executable, str(ROOT / "native" / "build.py"), "mxdev"], check=True)
    return {"GSX_AMDSMI_LIB": str(FAKE), "GSX_FAKE_AMDSMI": ",".join(map(str, PERM))}


PROBE = r"""
import json, sys
sys.path.insert(0, %r)
import bench
from gpushare_scheduler_extender_amd.deviceplugin.allocator import build_response
from gpushare_scheduler_extender_amd.deviceplugin.devices import discover
from gpushare_scheduler_extender_amd.deviceplugin.plugin import device_tags
from gpushare_scheduler_extender_amd.k8s.objects import make_pod
from gpushare_scheduler_extender_amd.models.profile import ALIYUN
backend, devs = discover("amdsmi")
out = {"backend": backend, "devices": [(d.index, d.bdf, d.render_minor, d.uuid) for d in devs], "ranks": [],
       "tags": sorted(device_tags(devs).items())}
for r in range(8):  # bench.py, 8 ranks: rank r's arena on HIP device r (torch.cuda.set_device(r))
    _, fresh = discover("amdsmi")
    d = bench.rank_device(fresh, r, r, True)
    inv = bench.node_inventory([d])[0]
    alloc = build_response(make_pod("p", 8, profile=ALIYUN), d, 8, ALIYUN)
    host = build_response(make_pod("p", 8, profile=ALIYUN), d, 8, ALIYUN, mount_mode="all")
    out["ranks"].append({"rank": r, "bdf": d.bdf, "inventory": inv, "envs": alloc.envs, "nodes": alloc.devices,
                         "host_envs": host.envs})
print(json.dumps(out))
"""


def test_hip_ordinal_is_the_device_index_everywhere(shuffled):
    env = {**os.environ, **shuffled}
    env.pop("GSX_FAKE_DEVICES", None)
    r = subprocess.run([sys.executable, "-c", PROBE % str(ROOT)], capture_output=True, text=True, env=env,
                       timeout=300, cwd=str(ROOT))
    assert r.returncode == 0, r.stderr[-3000:]
    import json
    got = json.loads(r.stdout.strip().splitlines()[-1])
    assert got["backend"] == "amdsmi"
    hip_to_k = {h: k for k, h in enumerate(PERM)}
    # libmxdev orders devices by HIP ordinal, each keeping its own BDF / render node / UUID
    assert [i for i, *_ in got["devices"]] == list(range(8))
    for i, bdf, render, uuid in got["devices"]:
        k = hip_to_k[i]
        assert bdf == f"0000:{0x11 + 0x10 * k:02x}:00.0" and render == 128 + k and uuid == f"fake-smi-{k}", (i, k)
    assert [b for _i, b, *_ in got["devices"]] != sorted(b for _i, b, *_ in got["devices"])  # really shuffled
    for row in got["ranks"]:
        rank = row["rank"]
        k = hip_to_k[rank]
        want_bdf = f"0000:{0x11 + 0x10 * k:02x}:00.0"
        # the device a rank advertises is the one its arena lives on (HIP ordinal == rank)
        assert row["bdf"] == want_bdf and row["inventory"]["bdf"] == want_bdf and row["inventory"]["index"] == rank
        assert row["inventory"]["render"] == 128 + k
        # and a container given GPU `rank` sees that device: in isolated mount mode only its render node is mounted
        # (so it is the container's GPU 0); a host process (mount mode "all") is pointed at host ordinal `rank`
        envs = row["envs"]
        assert envs["HIP_VISIBLE_DEVICES"] == "0", envs
        paths = [n.get("host_path") or n.get("hostPath") or n.get("container_path") for n in row["nodes"]]
        renders = [p for p in paths if p and "renderD" in p]
        assert renders == [f"/dev/dri/renderD{128 + k}"] and "/dev/kfd" in paths, row["nodes"]
        assert row["host_envs"]["HIP_VISIBLE_DEVICES"] == str(rank), row["host_envs"]
    # the plugin's fake-ID tags are per device (UUID-derived): eight distinct ones, stable across re-enumeration
    assert len({t for _i, t in got["tags"]}) == 8
