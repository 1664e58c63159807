"""Cluster scale: the extender against 100 / 1,000 / 5,000 GPU nodes (8 x MI355X each) with pod churn.

    python -m gsxtools.scale [--nodes 100,1000,5000] [--pods-per-node 2]
                                                       [--churn-batches 8] [--batch 250] [--json-out F]

The reference's filter walks every NodeName under a global write lock and re-sums every pod annotation
of every device on every call (``pkg/cache/cache.go:130-162``, ``pkg/cache/deviceinfo.go:41-54``): its
cost grows with nodes x devices x pods.  Per node count this harness measures, on the real processes
(compiled fake kube-apiserver, the extender, the compiled kube-scheduler stand-in, each pinned to its own
core):

* **initial sync** — the apiserver already holds N nodes and ``pods-per-node`` x N bound, annotated pods
  (the BuildCache path, ``pkg/cache/cache.go:49-74``); time from starting the extender process to
  ``/healthz`` ready with every node in its ledger, the number of LIST pages its reflectors read
  (``limit=500`` / ``continue``), and the same for an empty cluster (process start-up alone);
* **extender memory** — VmRSS after the sync and after the churn;
* **filter latency at full NodeNames** — ``POST /filter`` with all N node names (what kube-scheduler
  sends when every node passes its own predicates and ``percentageOfNodesToScore`` is 100), sequential,
  p50 / p99 / max, client-observed;
* **bind throughput under churn** — batches of pods are created while the previous batch is deleted; the
  scheduler stand-in samples feasible nodes like kube-scheduler (``numFeasibleNodesToFind``, adaptive
  percentage) and binds through the extender.  pods bound per second and p50 / p99 bind latency.
"""
from __future__ import annotations

import argparse
import json
import sys
import time

from gpushare_scheduler_extender_amd.k8s.objects import make_node, make_pod
from gpushare_scheduler_extender_amd.models.profile import ALIYUN
from gpushare_scheduler_extender_amd.utils.cpuset import plan
from gsxtools.cluster import start_apiserver, start_extender, start_scheduler

GIB_PER_DEV = 268  # a 288 GB MI355X in GiB units
DEVS = 8


def _pct(xs, q):
    if not xs:
        return None
    xs = sorted(xs)
    return xs[min(len(xs) - 1, max(0, int(round(q / 100.0 * (len(xs) - 1)))))]


def _rss_mib(pid: int) -> float:
    try:
        with open(f"/proc/{pid}/status") as f:
            for ln in f:
                if ln.startswith("VmRSS:"):
                    return round(int(ln.split()[1]) / 1024.0, 1)
    except OSError:
        pass
    return 0.0


def node_name(i: int) -> str:
    return f"gpu-node-{i:05d}"


def populate(E, api_url: str, n_nodes: int, pods_per_node: int) -> float:
    """N gpushare nodes (8 x 268 GiB) and pods_per_node bound, annotated, Running 64 GiB pods per node."""
    b = E.BatchClient({"server": api_url})
    t0 = time.perf_counter()
    reqs = []
    for i in range(n_nodes):
        node = make_node(node_name(i), DEVS * GIB_PER_DEV, DEVS, profile=ALIYUN, device_totals=[GIB_PER_DEV] * DEVS,
                         labels={"gpushare": "true"}, address=f"10.{i // 65536}.{i // 256 % 256}.{i % 256}")
        reqs.append(("POST", "/api/v1/nodes", json.dumps(node, separators=(",", ":")).encode()))
    for st, body in b.run(reqs, 32):
        if st != 201:
            raise RuntimeError(f"node create failed: {st} {body[:200]!r}")
    reqs = []
    for i in range(n_nodes):
        for k in range(pods_per_node):
            ann = {ALIYUN.annotation_idx: str(k % DEVS), ALIYUN.annotation_pod: "64",
                   ALIYUN.annotation_dev: str(GIB_PER_DEV), ALIYUN.annotation_assigned: "true",
                   ALIYUN.annotation_assume_time: str(time.time_ns())}
            pod = make_pod(f"resident-{i:05d}-{k}", 64, profile=ALIYUN, node=node_name(i), annotations=ann,
                           phase="Running")
            del pod["metadata"]["uid"]
            reqs.append(("POST", "/api/v1/namespaces/default/pods", json.dumps(pod, separators=(",", ":")).encode()))
    for st, body in b.run(reqs, 32):
        if st != 201:
            raise RuntimeError(f"pod create failed: {st} {body[:200]!r}")
    return time.perf_counter() - t0


def wait_ready(E, ext_url: str, n_nodes: int, timeout: float = 600.0) -> None:
    b = E.BatchClient({"server": ext_url})
    deadline = time.perf_counter() + timeout
    while time.perf_counter() < deadline:
        try:
            st, _ = b.run([("GET", "/healthz", b"")], 1)[0]
            if st == 200:
                st, body = b.run([("GET", "/gpushare-scheduler/inspect", b"")], 1)[0]
                if st == 200 and len(json.loads(body).get("nodes") or []) == n_nodes:
                    return
        except Exception:  # noqa: BLE001 - not listening yet
            pass
        time.sleep(0.01)
    raise TimeoutError(f"extender not ready with {n_nodes} nodes after {timeout}s")


def extender_stats(E, ext_url: str) -> dict:
    st, body = E.BatchClient({"server": ext_url}).run([("GET", "/debug/engine", b"")], 1)[0]
    return json.loads(body) if st == 200 else {}


def filter_latency(E, ext_url: str, n_nodes: int, reps: int) -> dict:
    pod = make_pod("probe", 64, profile=ALIYUN)
    body = json.dumps({"Pod": pod, "Nodes": None, "NodeNames": [node_name(i) for i in range(n_nodes)]},
                      separators=(",", ":")).encode()
    b = E.BatchClient({"server": ext_url})
    lat = []
    for _ in range(reps):
        t0 = time.perf_counter()
        st, resp = b.run([("POST", "/gpushare-scheduler/filter", body)], 1)[0]
        lat.append(time.perf_counter() - t0)
        if st != 200:
            raise RuntimeError(f"filter failed: {st}")
    ok = len(json.loads(resp)["NodeNames"])
    return {"request_kib": round(len(body) / 1024, 1), "nodes_passed": ok, "reps": reps,
            "p50_ms": round(1e3 * _pct(lat, 50), 3), "p99_ms": round(1e3 * _pct(lat, 99), 3),
            "max_ms": round(1e3 * max(lat), 3), "per_node_us_p50": round(1e6 * _pct(lat, 50) / n_nodes, 3)}


def churn(E, api_url: str, sched_url: str, batches: int, batch: int) -> dict:
    """Create batch k while deleting batch k-1; all of batch k must bind."""
    api = E.BatchClient({"server": api_url})
    sched = E.BatchClient({"server": sched_url})
    tracker = E.PodTracker({"server": api_url}, "default", "gsx-churn")
    tracker.start(60)
    tmpl = make_pod("__NAME__", 64, profile=ALIYUN, labels={"gsx-churn": "__B__"})
    del tmpl["metadata"]["uid"]
    tmpl = json.dumps(tmpl, separators=(",", ":"))
    lat, per_batch = [], []
    t_all = time.perf_counter()
    prev = None
    try:
        for k in range(batches):
            names = [f"churn-{k}-{i}" for i in range(batch)]
            keys = [f"default/{n}" for n in names]
            body = tmpl.replace("__B__", str(k))
            t0 = time.perf_counter()
            reqs = [("POST", "/api/v1/namespaces/default/pods", body.replace("__NAME__", n).encode()) for n in names]
            if prev is not None:  # churn: the previous batch goes away while this one schedules
                reqs.append(("DELETE", f"/api/v1/namespaces/default/pods?labelSelector=gsx-churn%3D{prev}", b""))
            for st, b in api.run(reqs, 32):
                if st not in (200, 201):
                    raise RuntimeError(f"churn request failed: {st} {b[:200]!r}")
            err = tracker.wait(keys, E.TRACK_BOUND, 300)
            if err:
                raise RuntimeError(err)
            per_batch.append(batch / (time.perf_counter() - t0))
            st, tb = sched.run([("POST", "/v1/timings", json.dumps(keys).encode())], 1)[0]
            for t in json.loads(tb).values():
                lat.append(t["bound"] - t["seen"])
            sched.run([("POST", "/v1/forget", json.dumps(keys).encode())], 1)
            prev = k
        dt = time.perf_counter() - t_all
    finally:
        tracker.stop()
    return {"batches": batches, "batch": batch, "pods_per_s": round(batches * batch / dt, 1),
            "batch_pods_per_s_p50": round(_pct(per_batch, 50), 1),
            "p50_bind_latency_ms": round(1e3 * _pct(lat, 50), 3), "p99_bind_latency_ms": round(1e3 * _pct(lat, 99), 3)}


def run_one(n_nodes: int, pods_per_node: int, churn_batches: int, batch: int, filter_reps: int) -> dict:
    from gpushare_scheduler_extender_amd.core.engine import native

    E = native()
    cpus = plan(["apiserver", "extender", "scheduler"], {"extender": 2}, "spread")
    api = start_apiserver(cpus=cpus.get("apiserver"), history=max(200000, 4 * n_nodes * (pods_per_node + 2)))
    children = [api]
    try:
        t_pop = populate(E, api.url, n_nodes, pods_per_node)
        t0 = time.perf_counter()
        ext = start_extender(api.url, profile=ALIYUN.name, cpus=cpus.get("extender"))
        children.append(ext)
        wait_ready(E, ext.url, n_nodes)
        ready = time.perf_counter() - t0
        rss_sync = _rss_mib(ext.proc.pid)
        ctl = extender_stats(E, ext.url).get("controller", {})
        flt = filter_latency(E, ext.url, n_nodes, filter_reps)
        sched = start_scheduler(api.url, ext.url, profile=ALIYUN.name, max_inflight_binds=16,
                                cpus=cpus.get("scheduler"), nodes_to_score="adaptive")
        children.append(sched)
        ch = churn(E, api.url, sched.url, churn_batches, batch)
        return {"nodes": n_nodes, "devices": n_nodes * DEVS, "resident_pods": n_nodes * pods_per_node,
                "populate_s": round(t_pop, 2), "extender_ready_s": round(ready, 3),
                "pod_list_pages": ctl.get("pod_list_pages"), "node_list_pages": ctl.get("node_list_pages"),
                "extender_rss_mib_after_sync": rss_sync, "extender_rss_mib_after_churn": _rss_mib(ext.proc.pid),
                "filter_full_nodenames": flt, "churn": ch, "cpu_pinning": cpus or "none"}
    finally:
        for c in reversed(children):
            c.stop()


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--nodes", default="100,1000,5000")
    ap.add_argument("--pods-per-node", type=int, default=2)
    ap.add_argument("--churn-batches", type=int, default=8)
    ap.add_argument("--batch", type=int, default=250)
    ap.add_argument("--filter-reps", type=int, default=200)
    ap.add_argument("--json-out", default="")
    a = ap.parse_args(argv)
    out = {}
    # process start-up alone (empty cluster): what extender_ready_s includes besides LIST + BuildCache
    from gpushare_scheduler_extender_amd.core.engine import native

    E = native()
    api = start_apiserver()
    try:
        t0 = time.perf_counter()
        ext = start_extender(api.url, profile=ALIYUN.name)
        try:
            wait_ready(E, ext.url, 0)
            out["empty_cluster_ready_s"] = round(time.perf_counter() - t0, 3)
            out["empty_cluster_rss_mib"] = _rss_mib(ext.proc.pid)
        finally:
            ext.stop()
    finally:
        api.stop()
    for n in [int(x) for x in a.nodes.split(",") if x]:
        r = run_one(n, a.pods_per_node, a.churn_batches, a.batch, a.filter_reps)
        out[str(n)] = r
        print(json.dumps(r), flush=True)
    if a.json_out:
        with open(a.json_out, "w") as f:
            json.dump(out, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
