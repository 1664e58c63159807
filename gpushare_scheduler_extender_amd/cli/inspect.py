"""``kubectl inspect gpushare`` equivalent (the upstream CLI ships with the device plugin, not the reference).

Two output styles, both reproduced byte for byte (Go ``text/tabwriter``, padding 2):

* ``userguide`` (``docs/userguide.md:9-19``; default for GiB)::

    NAME     IPADDRESS     GPU0(Allocated/Total)  GPU Memory(GiB)
    node-a   192.168.0.71  6/15                   6/15
    ------------------------------------------------------------------------------
    Allocated/Total GPU Memory In Cluster:
    9/30 (30%)

* ``demo`` (``demo1.jpg``; default for MiB)::

    NAME  IPADDRESS  GPU0(Request MiB/Total MiB)  GPU1(Request MiB/Total MiB)  GPU Memory
    ...

``-d`` prints the ``demo2.jpg`` layout: a ``NAME:`` / ``IPADDRESS:`` block per
node, then one table holding ``NAME NAMESPACE GPU<i>(Request <unit>)``, a row
per pod, ``Allocated GPU Memory In Node <n>:  x (p%)`` and ``Total GPU Memory
In Node <n>:  y`` (one tabwriter block, so the node lines set the first
column's width, as in the screenshot), the dashed rule, and after all nodes
``Allocated/Total GPU Memory In Cluster:  a/t (p%)``.

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

DASH = "-" * 78  # docs/userguide.md:14
DEMO_DASH = "-" * 95  # demo1.jpg / demo2.jpg rule


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


def default_style(unit: str) -> str:
    return "demo" if unit == "MiB" else "userguide"


def render_summary(views: list[NodeView], unit: str = "GiB", style: str | None = None) -> str:
    style = style or default_style(unit)
    ndev = max((len(v.totals) for v in views), default=0)
    if style == "demo":  # demo1.jpg
        header = (["NAME", "IPADDRESS"] + [f"GPU{i}(Request {unit}/Total {unit})" for i in range(ndev)]
                  + ["GPU Memory"])
        dash = DEMO_DASH
    else:  # docs/userguide.md:11
        header = ["NAME", "IPADDRESS"] + [f"GPU{i}(Allocated/Total)" for i in range(ndev)] + [f"GPU Memory({unit})"]
        dash = DASH
    rows = [header]
    for v in views:
        cells = [v.name, v.address]
        for i in range(ndev):
            cells.append(f"{v.used[i]}/{v.totals[i]}" if i < len(v.totals) else "")
        cells.append(f"{v.allocated}/{v.total}")
        rows.append(cells)
    a = sum(v.allocated for v in views)
    t = sum(v.total for v in views)
    return "\n".join([tabwrite(rows), dash, "Allocated/Total GPU Memory In Cluster:", f"{a}/{t} ({pct(a, t)}%)"]) + "\n"


def render_details(views: list[NodeView], unit: str = "GiB") -> str:
    """``demo2.jpg``: per-node block, then the cluster line two blank lines below the last rule."""
    out = []
    for v in views:
        out.append("")
        out.append(tabwrite([["NAME:", v.name], ["IPADDRESS:", v.address]]))
        out.append("")
        ndev = len(v.totals)
        # one tabwriter block: pod rows and the two node lines share column widths (tab-terminated cells)
        rows = [["NAME", "NAMESPACE"] + [f"GPU{i}(Request {unit})" for i in range(ndev)] + [""]]
        for name, ns, dev, mem in sorted(v.pods, key=lambda x: (x[1], x[0])):
            rows.append([name, ns] + [str(mem) if i == dev else "0" for i in range(ndev)] + [""])
        rows.append([f"Allocated GPU Memory In Node {v.name}:", f"{v.allocated} ({pct(v.allocated, v.total)}%)", ""])
        rows.append([f"Total GPU Memory In Node {v.name}:", f"{v.total}", ""])
        out.append(tabwrite(rows))
        out.append(DEMO_DASH)
    a = sum(v.allocated for v in views)
    t = sum(v.total for v in views)
    out += ["", "", tabwrite([["Allocated/Total GPU Memory In Cluster:", f"{a}/{t} ({pct(a, t)}%)", ""]])]
    return "\n".join(out) + "\n"


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
    ap.add_argument("--style", default=None, choices=["userguide", "demo"],
                    help="summary header: docs/userguide.md (default for GiB) or demo1.jpg (default for MiB)")
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
        sys.stdout.write(render_summary(views, a.unit, a.style))
    return 0


if __name__ == "__main__":
    sys.exit(main())
