"""``kubectl inspect gpushare`` equivalent (the upstream CLI ships with the device plugin, not the reference).

Output format from ``docs/userguide.md:9-19`` and ``demo1.jpg`` / ``demo2.jpg``:

    NAME     IPADDRESS     GPU0(Allocated/Total)  GPU Memory(GiB)
    node-a   192.168.0.71  6/15                   6/15
    ------------------------------------------------------------------------------
    Allocated/Total GPU Memory In Cluster:
    9/30 (30%)

``-d`` prints one block per node with a row per pod and a column per GPU.
Data comes from the apiserver (nodes + pods, like the upstream plugin) or,
with ``--extender URL``, from the extender's ``/gpushare-scheduler/inspect``.
Install as ``kubectl-inspect-gpushare`` on PATH to get the kubectl plugin
form (``deploy/kubectl-inspect-gpushare``).
"""
from __future__ import annotations

import argparse
import asyncio
import json
import sys
from dataclasses import dataclass, field

from ..models import pod as podutil
from ..models.profile import NamingProfile, get_profile

DASH = "-" * 78


@dataclass
class NodeView:
    name: str
    address: str
    totals: list[int]
    used: list[int]
    pods: list[tuple[str, str, int, int]] = field(default_factory=list)  # (name, ns, dev, mem)

    @property
    def total(self) -> int:
        return sum(self.totals)

    @property
    def allocated(self) -> int:
        return sum(self.used)


def tabwrite(rows: list[list[str]], pad: int = 2) -> str:
    """Go text/tabwriter with minwidth 0, padding ``pad``: every column as wide as its widest cell."""
    if not rows:
        return ""
    ncol = max(len(r) for r in rows)
    width = [0] * ncol
    for r in rows:
        for i, c in enumerate(r[:-1]):
            width[i] = max(width[i], len(c))
    out = []
    for r in rows:
        cells = [c.ljust(width[i] + pad) if i < len(r) - 1 else c for i, c in enumerate(r)]
        out.append("".join(cells).rstrip())
    return "\n".join(out)


def pct(a: int, t: int) -> int:
    return int(a * 100 / t) if t else 0


def views_from_objects(nodes: list[dict], pods: list[dict], profile: NamingProfile) -> list[NodeView]:
    out = []
    for n in sorted(nodes, key=lambda x: x["metadata"]["name"]):
        if not podutil.is_gpushare_node(n, profile):
            continue
        totals = podutil.node_device_totals(n, profile)
        if not totals:
            continue
        v = NodeView(n["metadata"]["name"], podutil.node_address(n), totals, [0] * len(totals))
        out.append(v)
    by = {v.name: v for v in out}
    for p in pods:
        v = by.get(podutil.node_name(p))
        if v is None or not podutil.assigned_non_terminated(p):
            continue
        dev = podutil.gpu_id_from_annotation(p, profile)
        mem = podutil.gpu_mem_from_annotation(p, profile) or podutil.gpu_mem_request(p, profile)
        if 0 <= dev < len(v.used):
            v.used[dev] += mem
            v.pods.append((podutil.meta(p).get("name", ""), podutil.meta(p).get("namespace", ""), dev, mem))
    return out


def views_from_inspect(doc: dict, addresses: dict[str, str] | None = None) -> list[NodeView]:
    out = []
    for n in doc.get("nodes") or []:
        devs = n.get("devs") or []
        v = NodeView(n["name"], (addresses or {}).get(n["name"], ""), [d["totalGPU"] for d in devs],
                     [d["usedGPU"] for d in devs])
        for d in devs:
            for p in d.get("pods") or []:
                v.pods.append((p["name"], p["namespace"], d["id"], p["usedGPU"]))
        out.append(v)
    return out


def render_summary(views: list[NodeView], unit: str = "GiB") -> str:
    ndev = max((len(v.totals) for v in views), default=0)
    header = ["NAME", "IPADDRESS"] + [f"GPU{i}(Allocated/Total)" for i in range(ndev)] + [f"GPU Memory({unit})"]
    rows = [header]
    for v in views:
        cells = [v.name, v.address]
        for i in range(ndev):
            cells.append(f"{v.used[i]}/{v.totals[i]}" if i < len(v.totals) else "")
        cells.append(f"{v.allocated}/{v.total}")
        rows.append(cells)
    a = sum(v.allocated for v in views)
    t = sum(v.total for v in views)
    return "\n".join([tabwrite(rows), DASH, "Allocated/Total GPU Memory In Cluster:", f"{a}/{t} ({pct(a, t)}%)"]) + "\n"


def render_details(views: list[NodeView], unit: str = "GiB") -> str:
    blocks = []
    for v in views:
        lines = [tabwrite([["NAME:", v.name], ["IPADDRESS:", v.address]]), ""]
        rows = [["NAME", "NAMESPACE"] + [f"GPU{i}(Allocated)" for i in range(len(v.totals))]]
        for name, ns, dev, mem in sorted(v.pods, key=lambda x: (x[1], x[0])):
            rows.append([name, ns] + [str(mem) if i == dev else "0" for i in range(len(v.totals))])
        lines.append(tabwrite(rows))
        lines.append(tabwrite([["Allocated :", f"{v.allocated} ({pct(v.allocated, v.total)}%)"],
                               ["Total :", f"{v.total}"]]))
        lines.append(DASH)
        blocks.append("\n".join(lines))
    a = sum(v.allocated for v in views)
    t = sum(v.total for v in views)
    blocks.append(f"\nAllocated/Total GPU Memory In Cluster:  {a}/{t} ({pct(a, t)}%)")
    return "\n".join(blocks) + "\n"


async def collect(args) -> list[NodeView]:
    from ..k8s.client import KubeClient, KubeConfig  # noqa: PLC0415

    profile = get_profile(args.profile)
    if args.extender:
        import aiohttp  # noqa: PLC0415

        url = args.extender.rstrip("/") + "/gpushare-scheduler/inspect" + (f"/{args.node}" if args.node else "")
        async with aiohttp.ClientSession() as s:
            async with s.get(url) as r:
                doc = json.loads(await r.read())
        addrs = {}
        if args.apiserver or args.kubeconfig:
            async with KubeClient(KubeConfig.auto(args.kubeconfig, args.apiserver)) as c:
                for n in (await c.list("nodes")).get("items") or []:
                    addrs[n["metadata"]["name"]] = podutil.node_address(n)
        return views_from_inspect(doc, addrs)
    async with KubeClient(KubeConfig.auto(args.kubeconfig, args.apiserver)) as c:
        nodes = (await c.list("nodes")).get("items") or []
        if args.node:
            nodes = [n for n in nodes if n["metadata"]["name"] == args.node]
        pods = (await c.list("pods")).get("items") or []
    return views_from_objects(nodes, pods, profile)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="kubectl inspect gpushare")
    ap.add_argument("node", nargs="?", default="")
    ap.add_argument("-d", "--details", action="store_true")
    ap.add_argument("--profile", default="shared-gpu")
    ap.add_argument("--unit", default="GiB")
    ap.add_argument("--kubeconfig", default=None)
    ap.add_argument("--apiserver", default=None)
    ap.add_argument("--extender", default=None, help="read the extender's /gpushare-scheduler/inspect instead")
    ap.add_argument("-o", "--output", default="table", choices=["table", "json"])
    a = ap.parse_args(argv)
    views = asyncio.run(collect(a))
    if a.output == "json":
        print(json.dumps([v.__dict__ for v in views], indent=2))
    elif a.details:
        sys.stdout.write(render_details(views, a.unit))
    else:
        sys.stdout.write(render_summary(views, a.unit))
    return 0


if __name__ == "__main__":
    sys.exit(main())
