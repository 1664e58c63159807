"""BASELINE.json configurations 1-5 and the hardware-partition scenario (6) through the whole stack (gsxtools/configs.py):
CPU plumbing and, on MI355X, real device sizes, the HBM arena and hardware-verified CU partitions.

The default kubelet + device-plugin path is the shipped gRPC plugin driven over its unix socket
(``--agent plugin``); the in-process plugin and the compiled node agent must agree with it."""
import json

import pytest

from gsxtools import configs


@pytest.mark.parametrize("k", sorted(configs.CONFIGS))
def test_baseline_config_cpu(k, tmp_path):
    assert configs.main(["--only", str(k), "--json-out", str(tmp_path / "r.json")]) == 0


@pytest.mark.parametrize("agent", ["inproc", "native", "native-serial", "native-plugin"])
def test_configs_agree_across_agents(agent, tmp_path):
    """Same placements and partitions whichever agent plays kubelet + plugin (one Allocate contract)."""
    outs = {}
    for a in ("plugin", agent):
        out = tmp_path / f"{a}.json"
        assert configs.main(["--only", "3,5", "--agent", a, "--json-out", str(out)]) == 0
        outs[a] = json.loads(out.read_text())
    for k in ("per_device_gib", "resident_slices"):
        assert outs["plugin"]["3"][k] == outs[agent]["3"][k]
    # the same four partitions (which pod gets which depends on the order the binds land in)
    masks = {a: sorted(p["HSA_CU_MASK"] for p in o["5"]["partitions"]) for a, o in outs.items()}
    assert masks["plugin"] == masks[agent]


@pytest.mark.parametrize("latency_ms", [0, 5])
def test_config3_through_a_faithful_kubelet(latency_ms, tmp_path):
    """32 x 64 GiB on 8 devices with kubelet as it is (no re-routing, one admission per watch event,
    PodResources reconciliation) at 0 and 5 ms apiserver latency: binpack 4 per device and every container runs on
    the GPU its annotation names.  The node advertises landing-order matching, so the extender binds the 32 pods
    concurrently, in no particular order, and still no Allocate is matched to another pod than the one kubelet
    admits: nothing is left for reconciliation to repair."""
    out = tmp_path / "r.json"
    rc = configs.main(["--only", "3", "--faithful", "--api-latency-ms", str(latency_ms), "--json-out", str(out)])
    rep = json.loads(out.read_text())["3"]
    assert rc == 0, rep
    assert rep["faithful_kubelet"] and rep["per_device_gib"] == [256] * 8 and rep["physical_drift"] == 0
    assert rep["allocate_mismatch"] == 0 and rep["reconcile"]["swaps"] == 0, rep


@pytest.mark.gpu
def test_baseline_configs_on_mi355x(tmp_path):
    out = tmp_path / "r.json"
    rc = configs.main(["--gpu", "--json-out", str(out)])
    rep = json.loads(out.read_text())
    assert rc == 0, rep
    assert rep["2"]["hbm_arena"] and rep["2"]["bad_stamps"] == 0
    # config 5 through the gRPC device plugin: hardware-verified disjoint 64-CU partitions
    assert rep["5"]["agent"] == "plugin"
    assert rep["5"]["probe_cus_per_pod"] == [64] * 4 and rep["5"]["probe_disjoint"]
    # ... and enforced: a plain probe process per pod, HSA_CU_MASK unset, confined by libgsx_isolate.so with the
    # isolation config the plugin's Allocate wrote for that pod
    assert rep["5"]["enforced_cus_per_pod"] == [64] * 4 and rep["5"]["enforced_disjoint"]


@pytest.mark.gpu
def test_config3_32_pods_in_8_real_hbm_arenas(tmp_path):
    """8 x MI355X: 32 x 64 GiB co-resident in 8 real HBM arenas (skipped on a box with fewer GPUs)."""
    import torch

    if torch.cuda.device_count() < 8:
        pytest.skip(f"{torch.cuda.device_count()} GPU(s) visible; needs an 8 x MI355X node")
    out = tmp_path / "r.json"
    rc = configs.main(["--gpu", "--only", "3,4", "--json-out", str(out)])
    rep = json.loads(out.read_text())
    assert rc == 0, rep
    assert rep["3"]["real_gpus"] == 8 and rep["3"]["resident_slices"] == [4] * 8 and rep["3"]["bad_stamps"] == 0
    assert rep["4"]["real_gpus"] == 8


@pytest.mark.gpu
def test_config3_32_pods_in_8_hbm_arenas_on_one_gpu(tmp_path):
    """The 8-device config on a one-GPU box: eight HBM arenas carved out of GPU 0 (4 GiB pods on 18 GiB devices,
    the same 4-per-device fill), every slice stamped and verified by the HIP kernels."""
    out = tmp_path / "r.json"
    rc = configs.main(["--gpu", "--share-gpu", "--only", "3", "--json-out", str(out)])
    rep = json.loads(out.read_text())
    assert rc == 0, rep
    r3 = rep["3"]
    assert r3["shared_gpu"] and r3["real_gpus"] == 8 and r3["per_device_gib"] == [16] * 8
    assert r3["resident_slices"] == [4] * 8 and r3["bad_stamps"] == 0 and r3["physical_drift"] == 0


@pytest.mark.parametrize("agent", ["plugin", "native"])
def test_node_agent_restart_keeps_cu_partitions_disjoint(agent):
    """Kill the device plugin / node agent while 3 CU-partitioned pods run; the restarted one rebuilds ownership
    from the pods' cu-mask annotations, so a new pod's partition is disjoint from every running pod's."""
    import asyncio

    from gpushare_scheduler_extender_amd.deviceplugin.state import parse_cu_mask
    from gpushare_scheduler_extender_amd.models.profile import ALIYUN, POD_CU_MASK_ANNOTATION
    from gsxtools.cluster import start_node_agent

    async def go():
        cl = configs.Cluster(ALIYUN, [268], gpu=False, agent=agent)
        try:
            await cl.start()
            cu = {configs.CU_COUNT_ANNOTATION: "64"}
            for i in range(3):
                await cl.create(f"r{i}", 16, annotations=cu)
            pods = await cl.wait([f"r{i}" for i in range(3)])
            running = [set(parse_cu_mask(p["metadata"]["annotations"][POD_CU_MASK_ANNOTATION])) for p in pods.values()]
            old = next(c for c in cl.children if c.name == "node-agent")
            old.proc.kill()
            old.proc.wait(5)
            old.stop()
            new_agent = start_node_agent(cl.api.url, configs.NODE, profile=ALIYUN.name, native=agent == "native",
                                         extender=cl.ext.url)
            cl.children[cl.children.index(old)] = new_agent
            await cl.agent_http.close()
            from gpushare_scheduler_extender_amd.k8s.fasthttp import Client as HttpClient
            cl.agent_http = HttpClient(new_agent.url)
            await cl.create("new", 16, annotations=cu)
            new = (await cl.wait(["new"]))["new"]
            got = set(parse_cu_mask(new["metadata"]["annotations"][POD_CU_MASK_ANNOTATION]))
            assert len(got) == 64 and all(not got & r for r in running)
        finally:
            await cl.close()
    asyncio.run(go())
