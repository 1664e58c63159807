"""End-to-end slice B on a real MI355X.

One pod requesting 64 GiB of ``gpu-mem`` goes through the whole stack —
fake kube-apiserver, the extender (native front end), the kube-scheduler
simulator's filter and bind, the device plugin's Allocate (``ASSIGNED=true``)
— and is then started by :class:`ProcessRuntime` with exactly the container
environment Allocate returned.  The container is the sample workload
(``samples/workload``: its ``run.sh`` entry and standalone ``main.py``, bf16 MFMA GEMM loop) which must run on the assigned
GPU inside its memory share: ``set_per_process_memory_fraction`` =
share / device total, and a second share-sized allocation is refused.

The workload runs in a child process (fork+exec in the child); this process
only discovers the device (amdsmi, or HIP as the fallback).
"""
import asyncio
import json
import sys
from pathlib import Path

import pytest

from gsxtools.agent import NodeAgent
from gpushare_scheduler_extender_amd.deviceplugin.devices import discover
from gpushare_scheduler_extender_amd.deviceplugin.runtime import ProcessRuntime
from gpushare_scheduler_extender_amd.extender.server import ExtenderRunner, ExtenderServer
from gpushare_scheduler_extender_amd.k8s.client import KubeClient
from tests.fixtures.fakeapi import FakeApiServerRunner
from gpushare_scheduler_extender_amd.k8s.objects import make_node, make_pod
from gpushare_scheduler_extender_amd.models import pod as podutil
from gpushare_scheduler_extender_amd.models.profile import SHARED_GPU
from tests.fixtures.schedsim import SchedulerSim

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parents[1]


def test_slice_b_pod_runs_inside_its_share_on_mi355x():
    backend, devs = discover("auto")
    assert backend in ("amdsmi", "hip"), backend
    dev = devs[0]
    gib = dev.units("GiB")
    assert gib >= 256, (backend, dev)

    async def go():
        api = await FakeApiServerRunner().start()
        client = KubeClient(api.url)
        ext = await ExtenderRunner(ExtenderServer(KubeClient(api.url), SHARED_GPU)).start()
        # the sample image's entry (samples/workload/run.sh -> main.py, standalone), with the MFMA kernel library
        # the image builds -- here the repository's build of it, as if mounted; nothing else of the repo is visible
        app = ROOT / "samples" / "workload"
        cmd = ["bash", str(app / "run.sh"), "--iters", "40", "--size", "4096", "--touch", "--probe-limit", "--json",
               "--kernel", "gsx"]
        lib = ROOT / "gpushare_scheduler_extender_amd" / "_native" / "libgsx_kernels.so"
        rt = ProcessRuntime(cmd, extra_env={"GSX_APP_DIR": str(app), "GSX_KERNELS_LIB": str(lib), "PYTHONPATH": ""},
                            cwd="/tmp")
        agent = NodeAgent(KubeClient(api.url), "mi355x-0", [dev], SHARED_GPU, rt, unit="GiB")
        sim = SchedulerSim(KubeClient(api.url), ext.url, SHARED_GPU)
        try:
            await client.create("nodes", make_node("mi355x-0", gib, 1, device_totals=[gib]))
            await agent.start()
            await sim.start()
            await client.create("pods", make_pod("slice-b", 64))
            await sim.wait_bound(["default/slice-b"], 30)
            for _ in range(3000):
                if rt.procs:
                    break
                await asyncio.sleep(0.01)
            (uid,) = rt.procs
            rc, so, se = await rt.wait(uid, 300)
            assert rc == 0, se[-3000:]
            res = json.loads(so.strip().splitlines()[-1])
            pod = await client.get("pods", "slice-b", "default")
            return res, rt.envs[uid], pod
        finally:
            await sim.stop()
            await sim.client.close()
            await agent.stop()
            await agent.client.close()
            rt.close()
            await ext.stop()
            await ext.server.client.close()
            await client.close()
            await api.stop()

    res, env, pod = asyncio.run(go())
    ann = podutil.annotations(pod)
    assert ann[SHARED_GPU.annotation_idx] == "0"
    assert ann[SHARED_GPU.annotation_assigned] == "true"
    assert ann[SHARED_GPU.annotation_pod] == "64"
    assert env["HIP_VISIBLE_DEVICES"] == "0" and env["SHARED_GPU_MEM_CONTAINER"] == "64"
    assert res["visible_devices"] == "0"
    assert abs(res["fraction"] - 64 / gib) < 1e-6
    assert res["limit_enforced"] is True
    assert res["kernel"] == "gsx" and res["kernels_lib"].endswith("_native/libgsx_kernels.so"), res
    assert res["tflops"] > 100, res  # bf16 MFMA GEMM at 4096^3 on MI355X runs at ~1 PFLOP/s
    print("slice B:", json.dumps(res))
