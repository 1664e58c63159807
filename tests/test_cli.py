"""kubectl-inspect-gpushare output (docs/userguide.md:9-19 golden) from objects, apiserver and extender."""
import asyncio

from gpushare_scheduler_extender_amd.cli import inspect as cli
from gpushare_scheduler_extender_amd.k8s.objects import make_node, make_pod
from gpushare_scheduler_extender_amd.models.profile import SHARED_GPU as P


def placed(name, node, dev, mem, phase="Running"):
    return make_pod(name, mem, node=node, phase=phase,
                    annotations={P.annotation_idx: str(dev), P.annotation_pod: str(mem)})


def userguide_cluster():
    n1 = make_node("cn-shanghai.i-uf61h64dz1tmlob9hmtb", 15, 1, address="192.168.0.71")
    n2 = make_node("cn-shanghai.i-uf61h64dz1tmlob9hmtc", 15, 1, address="192.168.0.70")
    pods = [placed("binpack-1-0", n1["metadata"]["name"], 0, 2), placed("binpack-1-1", n1["metadata"]["name"], 0, 2),
            placed("binpack-1-2", n1["metadata"]["name"], 0, 2), placed("binpack-2-0", n2["metadata"]["name"], 0, 3),
            placed("done", n2["metadata"]["name"], 0, 5, phase="Succeeded")]
    return [n1, n2], pods


def test_summary_matches_userguide():
    nodes, pods = userguide_cluster()
    out = cli.render_summary(cli.views_from_objects(nodes, pods, P))
    assert out == (
        "NAME                                IPADDRESS     GPU0(Allocated/Total)  GPU Memory(GiB)\n"
        "cn-shanghai.i-uf61h64dz1tmlob9hmtb  192.168.0.71  6/15                   6/15\n"
        "cn-shanghai.i-uf61h64dz1tmlob9hmtc  192.168.0.70  3/15                   3/15\n"
        "------------------------------------------------------------------------------\n"
        "Allocated/Total GPU Memory In Cluster:\n"
        "9/30 (30%)\n")


def test_details_block():
    nodes, pods = userguide_cluster()
    out = cli.render_details(cli.views_from_objects(nodes, pods, P))
    assert "NAME:       cn-shanghai.i-uf61h64dz1tmlob9hmtb" in out
    assert "Allocated GPU Memory In Node cn-shanghai.i-uf61h64dz1tmlob9hmtb:  6 (40%)" in out
    assert "Total GPU Memory In Node cn-shanghai.i-uf61h64dz1tmlob9hmtb:      15" in out
    assert out.rstrip().endswith("Allocated/Total GPU Memory In Cluster:  9/30 (30%)")
    assert "done" not in out  # terminated pods are not listed (AssignedNonTerminatedPod)


DEMO_NODE = "cn-shanghai.i-uf63li6prnicrvggce0x"


def demo_cluster(with_pods=True):
    n = make_node(DEMO_NODE, 32552, 2, address="192.168.168.133")
    pods = [placed("binpack-2-65df4b8b9b-rwxx9", DEMO_NODE, 0, 8138),
            placed("binpack-3-594f6bcb46-8wc7w", DEMO_NODE, 1, 8138)] if with_pods else []
    return [n], pods


def test_details_match_demo2_screenshot():
    """demo2.jpg, byte for byte: node header block, one table whose first column is as wide as the node lines,
    the rule, two blank lines, the cluster line."""
    nodes, pods = demo_cluster()
    out = cli.render_details(cli.views_from_objects(nodes, pods, P), unit="MiB")
    assert out == (
        "\n"
        "NAME:       cn-shanghai.i-uf63li6prnicrvggce0x\n"
        "IPADDRESS:  192.168.168.133\n"
        "\n"
        "NAME                                                              NAMESPACE    GPU0(Request MiB)  GPU1(Request MiB)\n"
        "binpack-2-65df4b8b9b-rwxx9                                        default      8138               0\n"
        "binpack-3-594f6bcb46-8wc7w                                        default      0                  8138\n"
        "Allocated GPU Memory In Node cn-shanghai.i-uf63li6prnicrvggce0x:  16276 (50%)\n"
        "Total GPU Memory In Node cn-shanghai.i-uf63li6prnicrvggce0x:      32552\n"
        + "-" * 95 + "\n"
        "\n"
        "\n"
        "Allocated/Total GPU Memory In Cluster:  16276/32552 (50%)\n")


def test_summary_matches_demo1_screenshot():
    """demo1.jpg: the MiB summary header ``GPU<i>(Request MiB/Total MiB)`` and ``GPU Memory``."""
    nodes, _ = demo_cluster(with_pods=False)
    out = cli.render_summary(cli.views_from_objects(nodes, [], P), unit="MiB")
    assert out == (
        "NAME                                IPADDRESS        GPU0(Request MiB/Total MiB)  GPU1(Request MiB/Total MiB)"
        "  GPU Memory\n"
        "cn-shanghai.i-uf63li6prnicrvggce0x  192.168.168.133  0/16276                      0/16276"
        "                      0/32552\n"
        + "-" * 95 + "\n"
        "Allocated/Total GPU Memory In Cluster:\n"
        "0/32552 (0%)\n")
    # the GiB (userguide) header is one flag away
    assert "GPU0(Allocated/Total)" in cli.render_summary(cli.views_from_objects(nodes, [], P), unit="MiB",
                                                        style="userguide")


def test_demo2_two_gpus_half_allocated():
    """demo2.jpg: 2 x 16276 per node, one 8138 pod on each GPU -> 16276/32552 (50%)."""
    nodes, pods = demo_cluster()
    out = cli.render_summary(cli.views_from_objects(nodes, pods, P), unit="MiB")
    assert "8138/16276                   8138/16276                   16276/32552" in out
    assert out.endswith("16276/32552 (50%)\n")


def test_cli_against_live_extender_and_apiserver(capsys):
    from .test_e2e import Cluster

    async def go():
        async with Cluster() as c:
            await c.client.create("nodes", make_node("n1", 30, 2, address="10.1.1.1"))
            await c.start_sim()
            for i in range(3):
                await c.client.create("pods", make_pod(f"p{i}", 5))
            await c.sim.wait_bound([f"default/p{i}" for i in range(3)], 10)
            await c.settle(lambda: sum(u for _, u in c.ext.server.engine.node_devices("n1")) == 15)
            loop = asyncio.get_running_loop()
            rc = await loop.run_in_executor(None, cli.main, ["--apiserver", c.api.url])
            assert rc == 0
            rc = await loop.run_in_executor(None, cli.main, ["--extender", c.ext.url, "--apiserver", c.api.url])
            assert rc == 0
    asyncio.run(go())
    out = capsys.readouterr().out
    blocks = out.split("Allocated/Total GPU Memory In Cluster:\n")
    assert "n1    10.1.1.1   15/15" in out
    assert out.count("15/30 (50%)") == 2 and len(blocks) == 3
