"""The five BASELINE.json configurations (plus hardware partitions), end to end through the whole stack.

    python -m gsxtools.configs [--gpu] [--json-out F] [--only 1,4]

Every configuration starts the same processes as ``bench.py`` (fake kube-apiserver, the extender, the
kube-scheduler stand-in and the node agent as child processes; a pod runtime endpoint per GPU in this
process), registers one node, creates pods and checks where they land:

1. kind-style plumbing: one fake 16 GiB device, 2 pods x 2 GiB (reference ``shared-gpu`` naming) ->
   both bound to device 0 and admitted (``samples/1.yaml``, ``docs/designs/designs.md:88``);
2. 1 x MI355X: 4 pods x 64 GiB (``aliyun.com/gpu-mem``) on the single 288 GB device -> 4 co-resident;
3. 8 x MI355X: 32 pods x 64 GiB on 8 devices -> binpack-first, 4 per device;
4. fragmentation guard: 8 devices each holding a 200 GiB pod (68 GiB free each, 544 GiB free on the
   node), then 100 / 200 / 50 GiB requests: the 100 and 200 GiB pods pass kube-scheduler's aggregate
   fit but the extender filters the node ("Insufficient GPU Memory in one device",
   ``pkg/scheduler/gpushare-predicate.go:29``) and they stay Pending; the 50 GiB pod is placed;
5. CU-mask isolation (MPS stand-in): 4 pods x 64 GiB with ``gpushare.amd.com/cu-count: 64`` on one
   device -> disjoint 64-CU partitions, 8 CUs on each of the 8 XCDs.  With ``--gpu`` each pod's
   partition is also checked on the MI355X: a CU-masked stream runs the CU probe kernel and the
   hardware CU ids it records must be 64 per pod and disjoint across pods;
6. hardware partitions (CPX / NPS1): one MI355X as 8 logical devices sharing one HBM pool.  Each
   advertises its share of the pool (``deviceplugin/devices.py: apply_memory_pools``), not the whole
   pool 8 times; a 64 GiB request that fits the node but no partition is filtered; 8 x 32 GiB pods
   land one per partition.

``--gpu``: device sizes come from the real MI355X and configs 2 and 5 use a real HBM arena on GPU 0
(each pod's slice stamped and every resident slice verified by the admission kernel).  Configs 3 and
4 use one real HBM arena per GPU when 8 GPUs are visible (an 8 x MI355X node); with fewer, the
devices beyond the box's GPUs are fakes of the same size.  Without ``--gpu`` everything is CPU-only.

``--agent``: who plays kubelet + device plugin.  ``plugin`` (default): the kubelet stand-in
(``gsxtools/agent.py``) drives the shipped gRPC :class:`GpuSharePlugin` over its unix socket;
``inproc``: the same plugin called in-process; ``native``: the compiled ``gsx-nodeagent``.
"""
from __future__ import annotations

import argparse
import asyncio
import json
import sys
import time

from gpushare_scheduler_extender_amd.k8s.client import KubeClient
from gpushare_scheduler_extender_amd.k8s.fasthttp import Client as HttpClient
from gpushare_scheduler_extender_amd.k8s.objects import make_node, make_pod
from gpushare_scheduler_extender_amd.models.profile import (ALIYUN, NODE_ALLOCATE_ORDER_ANNOTATION, NODE_DEVICE_INFO_ANNOTATION, NODE_RUNTIME_ENDPOINTS_ANNOTATION,
                              POD_CU_MASK_ANNOTATION, POD_HOLD_IDX_ANNOTATION, SHARED_GPU, NamingProfile)
from gsxtools.cluster import start_apiserver, start_extender, start_node_agent, start_scheduler

GIB = 1 << 30
NODE = "mi355x-node-0"
CU_COUNT_ANNOTATION = "gpushare.amd.com/cu-count"
AGENT = {"kind": "plugin", "args": [], "api_latency_ms": 0.0}  # --agent, --faithful, --api-latency-ms


class Runtimes:
    """One pod runtime endpoint per device (native ``_engine.PodRuntime``): accounting only, or GPU 0's HBM arena."""

    def __init__(self, n: int, unit_bytes: int, gib_per_dev: int, gpu: bool | int, share_gpu: bool = False):
        """``gpu``: False, True (GPU 0 backs device 0) or the number of leading devices backed by real GPUs.
        ``share_gpu``: every real-backed device is an arena on physical GPU 0 (one-GPU rehearsal of an N-GPU node)."""
        from gpushare_scheduler_extender_amd.core.engine import native

        E = native()
        n_real = int(gpu)
        self.rts, self.urls, self.bufs, self.streams = [], [], [], []
        self.real = n_real
        for i in range(n):
            arena = gib_per_dev * unit_bytes
            if i < n_real:
                from gpushare_scheduler_extender_amd.ops import hip

                phys = 0 if share_gpu else i
                buf = hip.DeviceBuffer(phys, arena)
                st = hip.Stream(phys)
                rt = E.PodRuntime(phys, arena, buf.addr(0), st.ptr, 1 << 20, hip.lib()._name)
                self.bufs.append(buf)
                self.streams.append(st)
            else:
                rt = E.PodRuntime(i, arena)
            self.rts.append(rt)
            self.urls.append(f"http://127.0.0.1:{rt.serve('127.0.0.1', 0)}")

    def stats(self) -> list[dict]:
        return [rt.stats() for rt in self.rts]

    def verify(self) -> int:
        return sum(rt.verify() for rt in self.rts)

    def close(self):
        for rt in self.rts:
            rt.stop()
        for s in self.streams:
            s.sync()
            s.destroy()
        for b in self.bufs:
            b.free()


class Cluster:
    """apiserver + extender + scheduler + node agent (child processes) and one node with ``len(totals)`` devices."""

    def __init__(self, profile: NamingProfile, totals: list[int], gpu: bool | int, cu_count: int = 256,
                 partition: str = "SPX", xcc_count: int = 8, agent: str | None = None,
                 pool_gib: int = 0, bind_mode: str = "binding", agent_args: list[str] | None = None,
                 share_gpu: bool = False):
        self.profile = profile
        self.totals = totals
        self.children = []
        self.api = start_apiserver()
        self.children.append(self.api)
        self.ext = start_extender(self.api.url, profile=profile.name, bind_mode=bind_mode)
        self.children.append(self.ext)
        # the compiled kube-scheduler stand-in, its own process like the real one
        self.children.append(start_scheduler(self.api.url, self.ext.url, profile=profile.name))
        self.agent_kind = agent or AGENT["kind"]
        self.agent_args = list(agent_args if agent_args is not None else AGENT["args"])
        self.api_latency_ms = AGENT["api_latency_ms"]
        self.children.append(self._agent())
        self.rt = Runtimes(len(totals), GIB, max(totals), gpu, share_gpu=share_gpu)
        self.cu_count = cu_count
        self.xcc_count = xcc_count
        self.partition = partition
        self.pool_gib = pool_gib  # partitions sharing one HBM pool: each reports the pool, owns a share

    async def start(self):
        self.c = KubeClient(self.api.url)
        inv = [{"index": i, "bdf": f"0000:{0x10 + i:02x}:00.0", "uuid": f"gpu-{i}", "units": t,
                "total_bytes": (self.pool_gib or t) * GIB, "share_bytes": t * GIB if self.pool_gib else 0,
                "cu": self.cu_count, "xcc": self.xcc_count, "render": 128 + i, "card": i, "partition": self.partition}
               for i, t in enumerate(self.totals)]
        node = make_node(NODE, sum(self.totals), len(self.totals), profile=self.profile, device_totals=self.totals,
                         annotations={NODE_DEVICE_INFO_ANNOTATION: json.dumps(inv),
                                      # what the device plugin publishes: its matcher is landing-ordered
                                      NODE_ALLOCATE_ORDER_ANNOTATION: "landing",
                                      NODE_RUNTIME_ENDPOINTS_ANNOTATION: json.dumps(
                                          {str(i): u for i, u in enumerate(self.rt.urls)})},
                         labels={"gpushare": "true"})
        await self.c.create("nodes", node)
        self.ext_http = HttpClient(self.ext.url)
        if self.api_latency_ms:
            api = HttpClient(self.api.url)
            await api.request("POST", "/fake/faults", json.dumps({"latency_ms": self.api_latency_ms}).encode())
            await api.close()
        self.agent_http = HttpClient(next(ch.url for ch in self.children if ch.name == "node-agent"))
        for _ in range(2000):  # the extender has seen the node
            if (await self.inspect()).get("nodes"):
                break
            await asyncio.sleep(0.005)
        else:
            raise TimeoutError("extender never saw the node")
        # the node agent (kubelet stand-in) watches the node's pods before any is bound: pods it first met in one
        # LIST would be admitted in name order rather than in the order their bindings landed
        for _ in range(6000):
            if (await self.agent_http.request("GET", "/v1/stats")).status == 200:
                return
            await asyncio.sleep(0.005)
        raise TimeoutError("node agent never became ready")

    def _agent(self):
        kind = self.agent_kind
        plugin = {"inproc": "inproc", "native-plugin": "spawn"}.get(kind, "grpc")
        native = kind.startswith("native")
        # the compiled stand-in is kubelet-faithful in plugin mode by construction: it takes no --faithful
        extra = [x for x in self.agent_args if x != "--faithful"] if native else self.agent_args
        return start_node_agent(self.api.url, NODE, profile=self.profile.name, native=native,
                                plugin=plugin, extra=extra, serial_admission=kind == "native-serial",
                                extender=self.ext.url)

    def agent_child(self):
        return next(ch for ch in self.children if ch.name == "node-agent")

    def stop_agent(self):
        """kubelet (and the plugin beside it) goes down; pods bound meanwhile are admitted as one batch later."""
        self.agent_child().stop()

    async def start_agent(self):
        old = self.agent_child()
        new = self._agent()
        self.children[self.children.index(old)] = new
        await self.agent_http.close()
        self.agent_http = HttpClient(new.url)
        for _ in range(6000):
            if (await self.agent_http.request("GET", "/v1/stats")).status == 200:
                return
            await asyncio.sleep(0.005)
        raise TimeoutError("node agent never became ready")

    async def bind(self, pod: dict) -> int:
        """kube-scheduler's filter + bind for one pod (tests that choose the binding order themselves)."""
        from gpushare_scheduler_extender_amd.models import wire

        f = await self.filter(pod)
        if NODE not in (f.get("NodeNames") or []):
            return 0
        md = pod["metadata"]
        args = wire.ExtenderBindingArgs(md["name"], md.get("namespace", "default"), md["uid"], NODE)
        r = await self.ext_http.request("POST", "/gpushare-scheduler/bind", args.encode())
        return r.status

    async def inspect(self) -> dict:
        r = await self.ext_http.request("GET", "/gpushare-scheduler/inspect")
        return json.loads(r.body)

    async def filter(self, pod: dict) -> dict:
        body = json.dumps({"Pod": pod, "Nodes": None, "NodeNames": [NODE]}).encode()
        r = await self.ext_http.request("POST", "/gpushare-scheduler/filter", body)
        return json.loads(r.body)

    async def agent_stats(self) -> dict:
        r = await self.agent_http.request("GET", "/v1/stats")
        return json.loads(r.body) if r.status == 200 else {}

    async def allocation(self, uid: str) -> dict:
        r = await self.agent_http.request("GET", f"/v1/allocations/{uid}")
        return json.loads(r.body) if r.status == 200 else {}

    async def create(self, name: str, gib: int, annotations: dict | None = None) -> dict:
        pod = make_pod(name, gib, profile=self.profile, annotations=annotations)
        del pod["metadata"]["uid"]
        return await self.c.create("pods", pod)

    async def wait(self, names: list[str], phase: str = "Running", timeout: float = 30.0) -> dict[str, dict]:
        deadline = time.monotonic() + timeout
        while True:
            pods = {p["metadata"]["name"]: p for p in (await self.c.list("pods", "default"))["items"]}
            got = {n: pods[n] for n in names if n in pods and pods[n].get("status", {}).get("phase") == phase}
            if len(got) == len(names):
                return got
            failed = [n for n in names if n in pods and pods[n].get("status", {}).get("phase") == "Failed"]
            if failed or time.monotonic() > deadline:
                raise RuntimeError(f"pods not {phase}: {sorted(set(names) - set(got))}; failed: {failed}")
            await asyncio.sleep(0.01)

    async def pending_after(self, names: list[str], seconds: float) -> list[str]:
        """Names still unbound after ``seconds`` (the scheduler keeps retrying them)."""
        await asyncio.sleep(seconds)
        pods = {p["metadata"]["name"]: p for p in (await self.c.list("pods", "default"))["items"]}
        return [n for n in names if not pods[n].get("spec", {}).get("nodeName")]

    def kill_extender(self):
        """SIGKILL the extender: no graceful shutdown, its in-memory ledger is gone."""
        self.ext.proc.kill()
        self.ext.proc.wait(5)

    def restart_extender(self):
        """A new extender process on the same port (kube-scheduler keeps its urlPrefix); it rebuilds its
        ledger from the pod annotations before serving (BuildCache, pkg/cache/cache.go:49-74)."""
        old = self.ext
        old.stop()
        self.ext = start_extender(self.api.url, profile=self.profile.name, port=old.port)
        self.children[self.children.index(old)] = self.ext

    def device_of(self, pod: dict) -> int:
        return int(pod["metadata"]["annotations"][self.profile.annotation_idx])

    async def physical_drift(self, names: list[str], timeout: float = 10.0) -> tuple[int, dict]:
        """Pods whose container runs on another GPU than their ``*_IDX`` annotation says (the env kubelet gave
        the container, from the kubelet stand-in), after waiting up to ``timeout`` for reconciliation."""
        deadline = time.monotonic() + timeout
        while True:
            pods = {p["metadata"]["name"]: p for p in (await self.c.list("pods", "default"))["items"]}
            drift = {}
            for n in names:
                p = pods.get(n)
                if p is None or p.get("status", {}).get("phase") != "Running":
                    continue
                if POD_HOLD_IDX_ANNOTATION in (p["metadata"].get("annotations") or {}):
                    drift[n] = "reconciliation in progress"
                    continue
                env = (await self.allocation(p["metadata"]["uid"])).get("envs", {})
                if env and int(env.get(self.profile.annotation_idx, -1)) != self.device_of(p):
                    drift[n] = (self.device_of(p), int(env[self.profile.annotation_idx]))  # (annotated, physical)
            if not drift or time.monotonic() > deadline:
                return len(drift), drift
            await asyncio.sleep(0.05)

    async def close(self):
        await self.c.close()
        await self.ext_http.close()
        await self.agent_http.close()
        self.rt.close()
        for ch in reversed(self.children):
            ch.stop()


def _gpu_gib() -> int:
    from gpushare_scheduler_extender_amd.ops import hip

    return hip.mem_info(0)[1] // GIB


SHARE = {"on": False}  # --share-gpu: the 8-device configs carve their devices out of GPU 0


def _real_gpus(gpu: bool, want: int) -> int:
    """How many of ``want`` devices real GPUs back: all of them on a node with that many (or, with --share-gpu, all
    of them as arenas on GPU 0), else none."""
    if not gpu:
        return 0
    if SHARE["on"]:
        return want
    import torch

    return want if torch.cuda.device_count() >= want else 0


async def config1(gpu: bool) -> dict:
    cl = Cluster(SHARED_GPU, [16], gpu=False)
    try:
        await cl.start()
        for i in range(2):
            await cl.create(f"binpack-{i}", 2)
        pods = await cl.wait([f"binpack-{i}" for i in range(2)])
        devs = sorted(cl.device_of(p) for p in pods.values())
        insp = await cl.inspect()
        ok = devs == [0, 0] and insp["nodes"][0]["usedGPU"] == 4
        return {"ok": ok, "devices": devs, "inspect_used": insp["nodes"][0]["usedGPU"],
                "inspect_total": insp["nodes"][0]["totalGPU"]}
    finally:
        await cl.close()


async def config2(gpu: bool) -> dict:
    total = _gpu_gib() if gpu else 268
    cl = Cluster(ALIYUN, [total], gpu=gpu)
    try:
        await cl.start()
        t0 = time.perf_counter()
        for i in range(4):
            await cl.create(f"p64-{i}", 64)
        pods = await cl.wait([f"p64-{i}" for i in range(4)])
        dt = time.perf_counter() - t0
        insp = await cl.inspect()
        used = insp["nodes"][0]["usedGPU"]
        bad = cl.rt.verify() if gpu else 0
        st = cl.rt.stats()[0]
        ok = sorted(cl.device_of(p) for p in pods.values()) == [0] * 4 and used == 256 and bad == 0
        return {"ok": ok, "device_gib": total, "used_gib": used, "util_pct": round(100 * used / total, 2),
                "resident_slices": st.get("resident"), "bad_stamps": bad, "hbm_arena": gpu, "seconds": round(dt, 4)}
    finally:
        await cl.close()


async def config3(gpu: bool) -> dict:
    per = _gpu_gib() if gpu else 268
    real = _real_gpus(gpu, 8)
    share = bool(gpu and SHARE["on"])
    # with --share-gpu the eight devices are arenas on GPU 0: scaled down 16x (18 GiB devices, 4 GiB pods), the
    # same 4-per-device fill as 64 GiB pods on a 287 GiB MI355X
    pod = 4 if share else 64
    if share:
        per = 18
    cl = Cluster(ALIYUN, [per] * 8, gpu=real, share_gpu=share)
    try:
        await cl.start()
        t0 = time.perf_counter()
        await asyncio.gather(*(cl.create(f"p64-{i}", pod) for i in range(32)))
        pods = await cl.wait([f"p64-{i}" for i in range(32)])
        dt = time.perf_counter() - t0
        # physical placement (the env each container got) == the annotation the extender accounts (a faithful
        # kubelet may start a container with another pod's Allocate; reconciliation must then fix the record)
        drift, drifted = await cl.physical_drift(list(pods))
        pods = {p["metadata"]["name"]: p for p in (await cl.c.list("pods", "default"))["items"] if p["metadata"]["name"] in pods}
        per_dev = [0] * 8
        for p in pods.values():
            per_dev[cl.device_of(p)] += pod
        insp = await cl.inspect()
        used = insp["nodes"][0]["usedGPU"]
        bad = cl.rt.verify() if real else 0
        resident = [st.get("resident") for st in cl.rt.stats()]
        # 32 equal-size pods for 8 GPUs of one node: kubelet's Allocate must never be matched to a pod with another
        # allocation (the plugin matches in landing order, the order kubelet admits in; the extender binds them
        # concurrently because the node advertises it)
        ast = await cl.agent_stats()
        mismatch = ast.get("mismatch", 0)
        faithful = "--faithful" in cl.agent_args
        ok = per_dev == [4 * pod] * 8 and used == 4 * pod * 8 and bad == 0 and drift == 0 and (faithful or mismatch == 0)
        if real:  # 32 x 64 GiB co-resident in 8 real HBM arenas, 4 slices each
            ok = ok and resident == [4] * 8
        return {"ok": ok, "per_device_gib": per_dev, "device_gib": per, "util_pct": round(100 * used / (8 * per), 2),
                "real_gpus": real, "shared_gpu": share, "pod_gib": pod, "resident_slices": resident, "bad_stamps": bad,
                "seconds": round(dt, 4), "allocate_mismatch": mismatch, "allocate_swapped_equivalent": ast.get("swapped_equivalent", 0),
                "physical_drift": drift, "drifted": drifted, "faithful_kubelet": faithful,
                "api_latency_ms": cl.api_latency_ms, "reconcile": ast.get("reconcile")}
    finally:
        await cl.close()


async def config4(gpu: bool) -> dict:
    per = _gpu_gib() if gpu else 268
    real = 0 if SHARE["on"] else _real_gpus(gpu, 8)  # 8 x 287 GiB arenas never fit one GPU: accounting only
    cl = Cluster(ALIYUN, [per] * 8, gpu=real)
    try:
        await cl.start()
        for i in range(8):
            await cl.create(f"big-{i}", 200)
        big = await cl.wait([f"big-{i}" for i in range(8)])
        placed = sorted(cl.device_of(p) for p in big.values())
        free_dev = per - 200
        free_node = 8 * free_dev
        out = {"device_gib": per, "fill": "8 x 200 GiB", "placed_devices": placed, "free_per_device_gib": free_dev,
               "free_on_node_gib": free_node, "real_gpus": real, "requests": []}
        ok = placed == list(range(8))
        for name, gib in (("req-100", 100), ("req-200", 200), ("req-50", 50)):
            pod = make_pod(name, gib, profile=ALIYUN)
            f = await cl.filter(pod)
            await cl.create(name, gib)
            fits_aggregate = gib <= free_node
            rec = {"request_gib": gib, "fits_node_aggregate": fits_aggregate, "extender_nodes": f["NodeNames"],
                   "failed_reason": (f.get("FailedNodes") or {}).get(NODE, "")}
            if gib <= free_dev:
                p = (await cl.wait([name]))[name]
                rec["placed_device"] = cl.device_of(p)
                ok = ok and f["NodeNames"] == [NODE]
            else:
                rec["pending_after_0.5s"] = bool(await cl.pending_after([name], 0.5))
                ok = ok and fits_aggregate and f["NodeNames"] == [] and \
                    rec["failed_reason"] == "Insufficient GPU Memory in one device" and rec["pending_after_0.5s"]
            out["requests"].append(rec)
        if real:
            out["bad_stamps"] = cl.rt.verify()
            ok = ok and out["bad_stamps"] == 0
        out["ok"] = ok
        return out
    finally:
        await cl.close()


async def config5(gpu: bool) -> dict:
    import tempfile

    total = _gpu_gib() if gpu else 268
    iso_dir = tempfile.mkdtemp(prefix="gsx-iso-")
    # the shipped plugin with enforced isolation: every Allocate writes the pod's isolation config (the files the
    # container would get mounted); with --gpu a probe process per pod runs under libgsx_isolate.so with it
    args = ["--isolation-dir", iso_dir] if AGENT["kind"] == "plugin" else []
    cl = Cluster(ALIYUN, [total], gpu=gpu, agent_args=AGENT["args"] + args)
    try:
        await cl.start()
        for i in range(4):
            await cl.create(f"cu-{i}", 64, annotations={CU_COUNT_ANNOTATION: "64"})
        pods = await cl.wait([f"cu-{i}" for i in range(4)])
        from gpushare_scheduler_extender_amd.deviceplugin.allocator import CUPartitioner
        from gpushare_scheduler_extender_amd.deviceplugin.state import parse_cu_mask

        parts = []
        for name in sorted(pods):
            # the partition the device plugin committed with ASSIGNED=true (and handed to the container)
            cus = parse_cu_mask(pods[name]["metadata"]["annotations"].get(POD_CU_MASK_ANNOTATION, ""))
            parts.append({"pod": name, "HSA_CU_MASK": f"0:{CUPartitioner.ranges(cus)}", "cus": cus})
        sets = [set(p["cus"]) for p in parts]
        disjoint = all(not (sets[i] & sets[j]) for i in range(4) for j in range(i + 1, 4))
        per_xcd = [sorted({c // 32 for c in s}) for s in sets]
        ok = disjoint and all(len(s) == 64 for s in sets) and all(x == list(range(8)) for x in per_xcd)
        if args:
            from pathlib import Path

            from gpushare_scheduler_extender_amd.deviceplugin.isolation import CONF
            confs = [Path(iso_dir) / "pods" / p["metadata"]["uid"] / CONF for p in pods.values()]
            n_conf = sum(1 for c in confs if c.exists() and "cu_mask=" in c.read_text())
            ok = ok and n_conf == 4
        out = {"device_gib": total, "agent": cl.agent_kind, "isolation_configs": n_conf if args else None,
               "partitions": [{"pod": p["pod"], "HSA_CU_MASK": p["HSA_CU_MASK"], "n_cus": len(p["cus"])} for p in parts],
               "disjoint": disjoint, "xcds_per_pod": [len(x) for x in per_xcd]}
        if gpu:
            from gpushare_scheduler_extender_amd.ops import hip

            hw = []
            for p in parts:
                s = hip.Stream(0, hip.mask_words(p["cus"]))
                hw.append(hip.physical_cus(hip.cuprobe(s, 8192, 20000)))
                s.destroy()
            hw_disjoint = all(not (hw[i] & hw[j]) for i in range(4) for j in range(i + 1, 4))
            out["probe_cus_per_pod"] = [len(h) for h in hw]
            out["probe_disjoint"] = hw_disjoint
            # physical XCDs each partition landed on (the partitioner intends 8 CUs on each of the 8)
            out["probe_xcds_per_pod"] = [len({t[0] for t in h}) for h in hw]
            out["probe_cus_per_xcd"] = [sorted(sum(1 for t in h if t[0] == x) for x in {t[0] for t in h}) for h in hw]
            ok = ok and hw_disjoint and all(len(h) == 64 for h in hw)
            if args:
                enforced = _enforced_probe(iso_dir, [p["metadata"]["uid"] for _, p in sorted(pods.items())])
                out["enforced_cus_per_pod"] = [len(e) for e in enforced]
                out["enforced_disjoint"] = all(not (enforced[i] & enforced[j]) for i in range(4) for j in range(i + 1, 4))
                ok = ok and out["enforced_disjoint"] and all(len(e) == 64 for e in enforced)
        out["ok"] = ok
        return out
    finally:
        await cl.close()
        import shutil

        shutil.rmtree(iso_dir, ignore_errors=True)


def _enforced_probe(iso_dir: str, uids: list[str]) -> list[set]:
    """Run the CU probe once per pod as a plain HIP process with HSA_CU_MASK unset, confined only by
    libgsx_isolate.so and the isolation config the device plugin wrote for that pod at Allocate."""
    import os
    import subprocess
    from pathlib import Path

    from gpushare_scheduler_extender_amd.deviceplugin.isolation import CONF, LIB

    native = Path(__file__).resolve().parents[1] / "gpushare_scheduler_extender_amd" / "_native"
    out = []
    for uid in uids:
        env = {k: v for k, v in os.environ.items() if k not in ("HSA_CU_MASK", "GSX_CU_MASK", "HSA_TOOLS_LIB")}
        env.update({"HSA_TOOLS_LIB": str(Path(iso_dir) / LIB), "GSX_ISOLATION_CONFIG": str(Path(iso_dir) / "pods" / uid / CONF)})
        r = subprocess.run([str(native / "gsx-cuprobe"), "--list"], env=env, capture_output=True, text=True, timeout=120)
        if r.returncode != 0:
            raise RuntimeError(f"cuprobe under isolation failed: {r.stderr[-500:]}")
        out.append({tuple(c) for c in json.loads(r.stdout.strip().splitlines()[-1])["cus"]})
    return out


async def config6(gpu: bool) -> dict:
    from gpushare_scheduler_extender_amd.deviceplugin.devices import apply_memory_pools, fake_devices

    total = _gpu_gib() if gpu else 268
    devs = apply_memory_pools(fake_devices(f"1x{total}GiB:CPX:NPS1"), "auto")
    shares = [d.units("GiB") for d in devs]
    raw = [d.total_bytes // GIB for d in devs]
    cl = Cluster(ALIYUN, shares, gpu=False, cu_count=devs[0].cu_count, xcc_count=devs[0].xcc_count, partition="CPX",
                 pool_gib=total)
    try:
        await cl.start()
        f = await cl.filter(make_pod("req-64", 64, profile=ALIYUN))
        reason = (f.get("FailedNodes") or {}).get(NODE, "")
        names = [f"cpx-{i}" for i in range(8)]
        await asyncio.gather(*(cl.create(n, 32) for n in names))
        pods = await cl.wait(names)
        placed = sorted(cl.device_of(p) for p in pods.values())
        insp = await cl.inspect()
        used, node_total = insp["nodes"][0]["usedGPU"], insp["nodes"][0]["totalGPU"]
        # the container's memory fraction is of the pool its partition sees, not of the partition
        env = (await cl.allocation(pods[names[0]]["metadata"]["uid"])).get("envs", {})
        frac = float(env.get("GSX_GPU_MEM_FRACTION", "nan"))
        want = 32 / shares[0] * (shares[0] / total)
        ok = (len(devs) == 8 and sum(shares) <= total and f["NodeNames"] == []
              and reason == "Insufficient GPU Memory in one device" and placed == list(range(8)) and used == 256
              and abs(frac - want) < 1e-4)
        return {"ok": ok, "gpu_gib": total, "logical_devices": len(devs), "reported_gib_per_partition": raw[0],
                "advertised_gib_per_partition": shares, "node_gpu_mem": node_total, "cus_per_partition": devs[0].cu_count,
                "req64_filtered": reason, "placed_devices": placed, "used_gib": used, "mem_fraction": frac,
                "mem_fraction_expected": round(want, 6)}
    finally:
        await cl.close()


CONFIGS = {
    1: ("kind cluster + fake device plugin: 2 pods binpack onto one fake device", config1),
    2: ("1xMI355X: 4 pods x 64 GiB binpacked onto the single 288 GB device", config2),
    3: ("8xMI355X: 32 pods x 64 GiB, binpack-first across all 8 devices", config3),
    4: ("fragmentation guard: 200/100/50 GiB requests that fit the node total but no single device", config4),
    5: ("CU-mask isolation: 4 pods co-resident on one MI355X with per-pod CU partitions", config5),
    6: ("hardware partitions: one MI355X in CPX/NPS1 as 8 logical devices sharing one HBM pool", config6),
}


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--gpu", action="store_true", help="real MI355X sizes, HBM arena and CU probe (needs a GPU)")
    ap.add_argument("--only", default="", help="comma-separated config numbers")
    ap.add_argument("--agent", default="plugin", choices=["plugin", "inproc", "native", "native-serial", "native-plugin"],
                    help="kubelet + device plugin: the shipped gRPC plugin driven over its socket (default), "
                         "the same in-process, the compiled gsx-nodeagent (its in-process matcher admitting on all "
                         "workers, or serially as kubelet: native-serial), or gsx-nodeagent calling the shipped "
                         "plugin process over gRPC (native-plugin)")
    ap.add_argument("--faithful", action="store_true",
                    help="the kubelet stand-in behaves like kubelet (no re-routing, sorted batches, PodResources); "
                         "the plugin reconciles against it")
    ap.add_argument("--api-latency-ms", type=float, default=0.0, help="fake apiserver latency per request")
    ap.add_argument("--share-gpu", action="store_true",
                    help="with --gpu: config 3's eight devices are HBM arenas on GPU 0 (one-GPU rehearsal)")
    ap.add_argument("--json-out", default="")
    a = ap.parse_args(argv)
    SHARE["on"] = a.share_gpu
    AGENT["kind"] = a.agent
    AGENT["args"] = ["--faithful"] if a.faithful else []
    AGENT["api_latency_ms"] = a.api_latency_ms
    which = [int(x) for x in a.only.split(",") if x] or sorted(CONFIGS)
    report = {}
    for k in which:
        desc, fn = CONFIGS[k]
        t0 = time.perf_counter()
        try:
            res = asyncio.run(fn(a.gpu))
        except Exception as e:  # noqa: BLE001 - reported per config
            res = {"ok": False, "error": f"{type(e).__name__}: {e}"}
        res["wall_s"] = round(time.perf_counter() - t0, 3)
        report[str(k)] = {"config": desc, **res}
        print(f"[{'PASS' if res['ok'] else 'FAIL'}] {k}. {desc}: "
              f"{json.dumps({x: y for x, y in res.items() if x not in ('ok', 'requests', 'partitions')})}", flush=True)
    if a.json_out:
        with open(a.json_out, "w") as f:
            json.dump(report, f, indent=1)
    return 0 if all(v["ok"] for v in report.values()) else 1


if __name__ == "__main__":
    sys.exit(main())
