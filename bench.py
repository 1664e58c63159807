#!/usr/bin/env python3
"""Headline benchmark: pods bound/s, p50/p99 bind latency and gpu-mem binpack utilisation on N x MI355X.

BASELINE.json metric/config: "8xMI355X: 32 pods x 64 GiB, binpack-first
placement across all 8 devices" (1 GPU: 4 pods x 64 GiB on the single 288 GB
device).  One rank per GPU (torchrun); per-GPU work is fixed (weak scaling):
every step is one *wave* of ``pods_per_gpu x N`` pods of ``pod_gib`` GiB
(``aliyun.com/gpu-mem``, the BASELINE naming) through the whole stack:

  rank 0 (before touching the GPU) starts the fake kube-apiserver and the
  scheduler extender as child processes, registers one node whose
  ``gpu-mem``/``gpu-count`` come from the ranks' real MI355X HBM sizes, and
  runs the kube-scheduler simulator (aggregate fit -> extender filter ->
  async extender bind);  every rank runs a node agent for its own GPU:
  Allocate (ASSIGNED=true, env, /dev nodes) -> the pod's slice of a real HBM
  arena is stamped by a HIP kernel and every co-resident pod's stamps are
  verified -> pod Running.  When all pods of the wave run, utilisation is
  read from the extender's /inspect and from bytes resident in HBM; then the
  wave is deleted and the step ends when the extender's ledger is empty.

Timed region: exactly K steps bracketed by barrier + torch.cuda.synchronize()
on both sides; the max over ranks is reported.  Every collective is gloo (control traffic only: barriers, small
objects, one float MAX on a CPU tensor); the scheduling data path has none, so RCCL is never initialised.
``--share-gpu`` runs N ranks on physical GPU 0 (one logical device per rank), the one-box rehearsal of the
N-GPU launch.  ``value`` = pods bound per
second over the whole job (all GPUs).  Synthetic pods; no cluster, no real
kubelet (there is none in this environment) — see SURVEY.md §4.  ``dtype`` is
"n/a": the timed region does no floating-point work (the GPU work is the HIP
stamp / verify of each pod's HBM slice).

Stability: every control-plane process is pinned to its own physical core, the idlest ones of the
(shared) host as sampled at start (``--pin``, utils/cpuset.py), and the per-wave distribution is reported next to
``value`` (``wave_pods_per_s``: p50 and IQR).

After the timed region rank 0 runs, as extra keys outside ``value``:
``device_plugin_path``: the same waves with kubelet + device plugin played by the shipped gRPC
``GpuSharePlugin`` over its unix socket (the kubelet stand-in in gsxtools/agent.py) instead of the
compiled node agent; ``device_plugin_path_native_kubelet``: the compiled kubelet stand-in calling the shipped
plugin process over gRPC; and ``latency_sweep`` (extra keys, not part of
``value``): the same waves with the fake kube-apiserver answering every
non-watch request after 0 / 1 / 2 / 5 ms, for ``--bind-mode binding`` (one
``pods/binding`` POST per pod) and ``update`` (the reference's PUT + POST), and
``reference_client``: ``update`` mode behind client-go's default token bucket
(QPS 5, burst 10 — what the reference runs with, ``cmd/main.go:76-82``) next to
``binding`` mode behind the same bucket: the same-condition comparison.
"""
from __future__ import annotations

import argparse
import asyncio
import gc
import json
import os
import statistics
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# the load generator's pod creates in flight at once (keep-alive connections of its batch client)
CREATE_CONCURRENCY = int(os.environ.get("GSX_CREATE_CONCURRENCY", "16"))
BASELINE_BINDS_PER_S = 2.5  # derived reference ceiling (client-go QPS 5 / 2 calls per bind)
NODE = "mi355x-node-0"


class LoopThread:
    """An asyncio loop in a daemon thread; the main thread keeps torch.distributed."""

    def __init__(self):
        self.loop = asyncio.new_event_loop()
        self.t = threading.Thread(target=self.loop.run_forever, daemon=True, name="gsx-loop")
        self.t.start()

    def run(self, coro, timeout: float | None = None):
        return asyncio.run_coroutine_threadsafe(coro, self.loop).result(timeout)

    def stop(self):
        self.loop.call_soon_threadsafe(self.loop.stop)
        self.t.join(5)


def _task_cpu_s(pid: int, field: int = 0) -> float | None:
    """On-CPU seconds of every thread of `pid` (/proc/<pid>/task/*/schedstat, nanosecond resolution: the
    timed region is milliseconds, far below the 10 ms ticks of /proc/<pid>/stat).  ``field=1``: the seconds its
    threads waited runnable for a CPU (scheduler run-delay) instead."""
    try:
        tids = os.listdir(f"/proc/{pid}/task")
    except OSError:
        return None
    ns = 0
    for t in tids:
        try:
            with open(f"/proc/{pid}/task/{t}/schedstat") as f:
                ns += int(f.read().split()[field])
        except (OSError, ValueError, IndexError):
            pass
    return ns / 1e9


def _psi_us() -> dict:
    """The host's pressure stall totals (/proc/pressure/{cpu,io,memory} "some total=", microseconds), {} without PSI."""
    out = {}
    for k in ("cpu", "io", "memory"):
        try:
            with open(f"/proc/pressure/{k}") as f:
                for ln in f:
                    if ln.startswith("some"):
                        out[k] = int(ln.rsplit("total=", 1)[1])
        except (OSError, ValueError, IndexError):
            pass
    return out


def _thread_cpu_s(pid: int) -> dict:
    """On-CPU seconds of `pid`'s threads summed per thread name (/proc/<pid>/task/*/comm + schedstat)."""
    out: dict = {}
    try:
        tids = os.listdir(f"/proc/{pid}/task")
    except OSError:
        return out
    for t in tids:
        try:
            with open(f"/proc/{pid}/task/{t}/comm") as f:
                name = f.read().strip()
            with open(f"/proc/{pid}/task/{t}/schedstat") as f:
                out[name] = out.get(name, 0.0) + int(f.read().split()[0]) / 1e9
        except (OSError, ValueError, IndexError):
            pass
    return out


def _threads_of_node(children) -> dict:
    """Per-thread-name on-CPU seconds of the node agent (kubelet stand-in) and the plugin process it spawned: which
    thread of the node's serial admission path is busy."""
    out = {}
    for c in children:
        pid = getattr(getattr(c, "proc", None), "pid", None)
        if pid is None or c.name != "node-agent":
            continue
        out["node-agent"] = _thread_cpu_s(pid)
        for k in _child_pids(pid):
            out["plugin"] = _thread_cpu_s(k)
    return out


def _child_pids(pid: int) -> list[int]:
    out = []
    try:
        for t in os.listdir(f"/proc/{pid}/task"):
            with open(f"/proc/{pid}/task/{t}/children") as f:
                out += [int(x) for x in f.read().split()]
    except (OSError, ValueError):
        pass
    return out


def _cpu_times(children, field: int = 0) -> dict:
    """On-CPU seconds (``field=1``: run-delay seconds) of this process (rank 0), the child servers and the
    device-plugin process the node agent spawned (the shipped plugin, the node's DaemonSet pod)."""
    out = {}
    me = _task_cpu_s(os.getpid(), field)
    if me is not None:
        out["rank0"] = me
    for c in children:
        pid = getattr(getattr(c, "proc", None), "pid", None)
        if pid is None:
            continue
        v = _task_cpu_s(pid, field)
        if v is not None:
            out[c.name] = v
        if c.name == "node-agent":
            for k in _child_pids(pid):
                pv = _task_cpu_s(k, field)
                if pv is not None:
                    out["plugin"] = out.get("plugin", 0.0) + pv
    return out


def _rss_mib(children) -> dict:
    """Resident set of this process and the child servers (a long run shows whether any of them grows)."""
    out = {}
    procs = [("rank0", os.getpid())] + [(c.name, getattr(getattr(c, "proc", None), "pid", None)) for c in children]
    for c in children:  # the device-plugin process the node agent spawned (the product's node-side process)
        pid = getattr(getattr(c, "proc", None), "pid", None)
        if c.name == "node-agent" and pid is not None:
            procs += [("plugin", k) for k in _child_pids(pid)]
    for name, pid in procs:
        try:
            with open(f"/proc/{pid}/status") as f:
                for ln in f:
                    if ln.startswith("VmRSS:"):
                        out[name] = round(int(ln.split()[1]) / 1024, 1)
                        break
        except (OSError, TypeError, ValueError):
            pass
    return out


class NativeRuntime:
    """One GPU's pod runtime endpoint served from C++ (``_engine.PodRuntime``) with the rank's HBM arena."""

    def __init__(self, dev: int, arena_bytes: int, use_gpu: bool, stride: int, cpus: list[int] | None = None):
        from gpushare_scheduler_extender_amd.core.engine import native

        self.buf = self.stream = None
        if use_gpu:
            from gpushare_scheduler_extender_amd.ops import hip

            self.buf = hip.DeviceBuffer(dev, arena_bytes)
            self.stream = hip.Stream(dev)
            self.rt = native().PodRuntime(dev, arena_bytes, self.buf.addr(0), self.stream.ptr, stride,
                                          hip.lib()._name)
        else:
            self.rt = native().PodRuntime(dev, arena_bytes)
        self.url = f"http://127.0.0.1:{self.rt.serve('127.0.0.1', 0, list(cpus or []))}"

    @property
    def admitted(self):
        return self.rt.stats()["admitted"]

    @property
    def failed(self):
        return self.rt.stats()["failed"]

    @property
    def bad(self):
        return self.rt.stats()["bad"]

    @property
    def batches(self):
        return self.rt.stats()["batches"]

    def verify(self) -> int:
        return self.rt.verify()

    def stop(self):
        self.rt.stop()

    def close(self):
        self.rt.stop()
        if self.stream is not None:
            self.stream.sync()
            self.stream.destroy()
        if self.buf is not None:
            self.buf.free()


def _cgroup_cpu() -> dict:
    """cgroup v2 cpu.stat (usage / throttling) of this container, {} where unavailable."""
    try:
        with open("/sys/fs/cgroup/cpu.stat") as f:
            return {k: int(v) for k, v in (ln.split() for ln in f if ln.strip())}
    except (OSError, ValueError):
        return {}


def pct(xs, q):
    if not xs:
        return None
    xs = sorted(xs)
    k = min(len(xs) - 1, max(0, int(round(q / 100.0 * (len(xs) - 1)))))
    return xs[k]


def wave_dist(xs) -> dict:
    if not xs:
        return {}
    p25, p50, p75 = pct(xs, 25), pct(xs, 50), pct(xs, 75)
    return {"p50": round(p50, 1), "p25": round(p25, 1), "p75": round(p75, 1),
            "iqr_pct": round(100 * (p75 - p25) / p50, 1) if p50 else None, "n": len(xs)}


def set_latency(api_batch, ms: float):
    st, b = api_batch.run([("POST", "/fake/faults", json.dumps({"latency_ms": ms}).encode())], 1)[0]
    if st != 200:
        raise RuntimeError(f"setting apiserver latency failed: {st} {b[:200]!r}")


SWEEP_LATENCIES_MS = (0, 1, 2, 5)
APISERVER_THREADS_MULTI = 1


class WaveRunner:
    """Untimed waves after the headline (same wave shape), with per-pod bind latency from the scheduler."""

    def __init__(self, wave, fetch_timings, lt, n_pods, first_step, counters=None):
        self.wave, self.fetch_timings, self.lt, self.n_pods = wave, fetch_timings, lt, n_pods
        self.step = first_step
        self.counters = counters  # the extender's bind counters (bind-order waits), diffed around the waves

    def measure(self, warm: int, steps: int) -> dict:
        for _ in range(warm):
            self.wave(self.step)
            self.step += 1
        rs = []
        c0 = self.counters() if self.counters else None
        t0 = time.perf_counter()
        for _ in range(steps):
            rs.append(self.wave(self.step))
            self.step += 1
        dt = time.perf_counter() - t0
        order = {}
        if c0 is not None:
            c1 = self.counters()
            n_binds = c1["binds"] - c0["binds"]
            order = {"bind_order_waits": c1["bind_order_waits"] - c0["bind_order_waits"], "binds": n_binds,
                     "bind_order_wait_ms_per_wave": round(1e3 * (c1["bind_order_wait_s"] - c0["bind_order_wait_s"])
                                                          / max(1, steps), 3)}
        lat, rtt = [], []
        for r in rs:
            for t in self.lt.run(self.fetch_timings(r["keys"]), 60):
                lat.append(t["bound"] - t["seen"])
                rtt.append(t["bind_rtt"])
        p50 = pct([r["t_total"] for r in rs], 50)
        return {"pods_per_s": round(self.n_pods * steps / dt, 1),
                # the median wave's rate next to the mean: one slow wave of a short row moves only the mean
                "pods_per_s_p50_wave": round(self.n_pods / p50, 1) if p50 > 0 else None,
                "wave_ms_p50": round(1e3 * p50, 3),
                "wave_ms_p50_running": round(1e3 * pct([r["t_run"] for r in rs], 50), 3),
                "p50_bind_latency_ms": round(1e3 * pct(lat, 50), 3), "p99_bind_latency_ms": round(1e3 * pct(lat, 99), 3),
                "p50_bind_rtt_ms": round(1e3 * pct(rtt, 50), 3), "pods": self.n_pods * steps, **order}


def restart_child(children, name: str, start):
    old = next(c for c in children if c.name == name)
    old.stop()
    new = start(old)
    children[children.index(old)] = new
    return new


def wait_until(fn, timeout: float, what: str):
    deadline = time.perf_counter() + timeout
    while True:
        try:
            if fn():
                return
        except Exception:  # noqa: BLE001 - not up yet
            pass
        if time.perf_counter() > deadline:
            raise TimeoutError(what)
        time.sleep(0.01)


def latency_sweep(a, children, api_url, api_batch, runner: WaveRunner, inspect_used):
    """Waves of the headline shape with the apiserver answering after L ms, for both bind modes, and behind
    client-go's default token bucket (QPS 5 / burst 10, the reference's client).  Rank 0 only; untimed by the
    driver's headline.  Returns (sweep rows, reference_client rows)."""
    from gsxtools.cluster import start_extender

    def restart_extender(mode: str, qps: float = 0.0, burst: int = 1000, order: str | None = None):
        restart_child(children, "extender", lambda old: start_extender(
            api_url, profile=a.profile, bind_mode=mode, port=old.port, cpus=old.cpus, kube_qps=qps, kube_burst=burst,
            bind_order=order or a.bind_order))
        # serving and synced: the node is in its ledger
        wait_until(lambda: bool(inspect_used().get("nodes")), 60, "restarted extender never saw the node")

    rows, cur = [], (a.bind_mode, a.bind_order)
    orders = [o for o in a.sweep_orders.split(",") if o]
    for order in orders:
        for m in ("binding", "update"):
            if (m, order) != cur:
                restart_extender(m, order=order)
                cur = (m, order)
            for ms in SWEEP_LATENCIES_MS:
                set_latency(api_batch, ms)
                rows.append({"bind_mode": m, "bind_order": order, "api_latency_ms": ms,
                             **runner.measure(1, a.sweep_steps)})
    set_latency(api_batch, 0)
    # the reference's client: client-go defaults QPS 5 / burst 10 (cmd/main.go:76-82 never overrides them).
    # The warm-up waves drain the burst, so the timed waves see the sustained rate.
    ref = []
    for m, calls in (("update", 2), ("binding", 1)):
        restart_extender(m, qps=5.0, burst=10)
        row = runner.measure(3, 3)
        ref.append({"bind_mode": m, "kube_qps": 5, "kube_burst": 10, "apiserver_calls_per_bind": calls,
                    "derived_ceiling_pods_per_s": round(5.0 / calls, 2), **row})
    restart_extender(a.bind_mode)
    return rows, ref


OPEN_LOOP_LATENCIES_MS = (1, 2, 5)
OPEN_LOOP_RATES = (500, 1000, 2000, 4000, 8000, 16000, 32000)


def _grpc_delta(p0, p1) -> dict | None:
    g0, g1 = (p0 or {}).get("grpc") or {}, (p1 or {}).get("grpc") or {}
    if not g1:
        return None
    out = {k: g1.get(k, 0) - g0.get(k, 0) for k in ("fast_allocate", "slow_allocate", "waited", "guard_by_ids",
                                                      "patch_failures")}
    out["wait_ms_total"] = round((g1.get("wait_ms") or {}).get("total", 0.0) - (g0.get("wait_ms") or {}).get("total", 0.0), 3)
    out["handler_us_allocate"] = (g1.get("handler_us") or {}).get("allocate")
    out["early_answer_backlog"] = g1.get("early_answer_backlog")
    out["allocate_phases_us"] = g1.get("allocate_phases_us")  # cumulative means
    out["last_slow_reason"] = g1.get("last_slow_reason")
    return out


def _allowed_cpus() -> list[int]:
    """The CPUs this container may use (its cgroup cpuset), whatever this process is pinned to now."""
    for path in ("/sys/fs/cgroup/cpuset.cpus.effective", "/sys/fs/cgroup/cpuset/cpuset.effective_cpus"):
        try:
            with open(path) as f:
                txt = f.read().strip()
        except OSError:
            continue
        out = []
        for part in txt.split(","):
            if "-" in part:
                lo, hi = part.split("-")
                out.extend(range(int(lo), int(hi) + 1))
            elif part:
                out.append(int(part))
        if out:
            return out
    return list(range(os.cpu_count() or 1))


def _agent_delta(s0, s1) -> dict | None:
    """Per-admission means (ms) of the node agent's steps between two /v1/stats reads."""
    if not s0 or not s1 or "mean_ms" not in s1:
        return None
    n0, n1 = s0.get("admitted", 0), s1.get("admitted", 0)
    c0, c1 = (s0.get("plugin_calls_mean_ms") or {}).get("n", 0), (s1.get("plugin_calls_mean_ms") or {}).get("n", 0)
    out = {}
    if n1 > n0:
        for k in ("queue", "runtime", "running_patch"):
            out[k] = round((s1["mean_ms"][k] * n1 - s0["mean_ms"][k] * n0) / (n1 - n0), 4)
    if c1 > c0:
        for k in ("slot_wait", "get_preferred", "allocate"):
            out["plugin_" + k] = round((s1["plugin_calls_mean_ms"][k] * c1 - s0["plugin_calls_mean_ms"][k] * c0)
                                       / (c1 - c0), 4)
    out["admitted"] = n1 - n0
    return out


def open_loop(a, api_url, api_batch, E, profile, inspect_used, sched_stats, agent_stats=None) -> dict:
    """Open-loop throughput under apiserver latency: pods arrive at a constant rate with many in
    flight -- no waves in lock-step -- and each is deleted as soon as it runs, so the node's room turns over.  Per
    apiserver latency the offered rate steps up until the stack stops keeping up (bound rate < 90 % of offered, or
    p99 arrival-to-bound over 100 ms): the knee.  Every pod's stages are timed by the native driver
    (native/engine/tracker.cc OpenLoop): create (the client's POST), bind (created -> bound: scheduler + extender),
    admit (bound -> Running: kubelet + device plugin + runtime + Running patch), free (DELETE -> gone).  At the first
    rate that failed the bound is named: when the scheduler found no room meanwhile (``room_waits``: its filter
    found the node full and it retried), pods held their room too long -- the one of admit / free that grew most;
    otherwise the one of create / bind / admit that grew most.  Pods of ``--open-loop-gib`` (1 GiB: 287 on one
    MI355X), so that room binds only a stack whose pods sit in admission.  Rank 0 only, untimed by the headline."""
    from gpushare_scheduler_extender_amd.k8s.objects import make_pod

    rates = OPEN_LOOP_RATES if a.open_loop == "auto" else tuple(int(x) for x in a.open_loop.split(",") if x)
    out = {"pod_gib": a.open_loop_gib, "duration_s": a.open_loop_s, "warm_s": 0.3, "hold_s": 0.0,
           "creators": a.open_loop_creators, "rows": [],
           "knee_pods_per_s": {}, "max_sustained_pods_per_s": {}, "bound_stage": {}}

    def pctl(xs, q):
        return round(1e3 * pct(xs, q), 3) if xs else None

    def cleanup(run):
        api_batch.run([("DELETE", f"/api/v1/namespaces/default/pods?labelSelector=gsx-ol%3D{run}", b"")], 1)
        deadline = time.perf_counter() + 60
        while sum(n["usedGPU"] for n in inspect_used()["nodes"]) != 0:
            if time.perf_counter() > deadline:
                # what the ledger still charges (pods, and the unaccounted use the plugin published), and what the
                # node agent and the plugin hold
                na = agent_stats() if agent_stats else {}
                pg = _plugin_debug(E, (na or {}).get("plugin_debug"))
                raise TimeoutError("open loop: ledger did not drain: " + json.dumps(
                    {"inspect": inspect_used(), "node_agent": na, "plugin": pg}, default=str)[:6000])
            time.sleep(0.005)

    k = 0
    for ms in OPEN_LOOP_LATENCIES_MS:
        set_latency(api_batch, ms)
        first = None
        for rate in rates:
            k += 1
            run = f"r{k}"
            tmpl = make_pod("__NAME__", a.open_loop_gib, profile=profile, labels={"gsx-ol": run})
            del tmpl["metadata"]["uid"]
            if a.term_grace >= 0:
                tmpl["spec"]["terminationGracePeriodSeconds"] = a.term_grace
            u0 = sched_stats().get("unschedulable", 0)
            na0 = agent_stats() if agent_stats else None
            pg0 = _plugin_debug(E, (na0 or {}).get("plugin_debug"))
            res = E.open_loop_run({"server": api_url}, run, json.dumps(tmpl, separators=(",", ":")), float(rate),
                                  duration_s=a.open_loop_s, warm_s=0.3, drain_s=10.0,
                                  creators=a.open_loop_creators, deleters=a.open_loop_creators,
                                  grace=-1 if a.term_grace >= 0 else 0)
            room_waits = sched_stats().get("unschedulable", 0) - u0
            na1 = agent_stats() if agent_stats else None
            pg1 = _plugin_debug(E, (na1 or {}).get("plugin_debug"))
            cleanup(run)
            pods = res["pods"]
            t0 = min(p[0] for p in pods if p[0] > 0)
            lo, hi = t0 + 0.3, t0 + a.open_loop_s
            win = [p for p in pods if lo <= p[0] < hi]
            bound_in = sum(1 for p in pods if lo <= p[2] < hi and p[2] > 0)
            run_in = sum(1 for p in pods if lo <= p[3] < hi and p[3] > 0)
            st = {"create": [p[1] - p[0] for p in win if p[1] > 0],
                  "bind": [p[2] - p[1] for p in win if p[2] > 0 and p[1] > 0],
                  "admit": [p[3] - p[2] for p in win if p[3] > 0 and p[2] > 0],
                  "free": [p[5] - p[4] for p in win if p[5] > 0 and p[4] > 0]}
            arr_bound = [p[2] - p[0] for p in win if p[2] > 0]
            row = {"api_latency_ms": ms, "offered_pods_per_s": rate,
                   "bound_pods_per_s": round(bound_in / (hi - lo), 1),
                   "running_pods_per_s": round(run_in / (hi - lo), 1),
                   "p50_bind_latency_ms": pctl(arr_bound, 50), "p99_bind_latency_ms": pctl(arr_bound, 99),
                   "p50_admit_latency_ms": pctl(st["admit"], 50), "p99_admit_latency_ms": pctl(st["admit"], 99),
                   "p50_e2e_ms": pctl([p[3] - p[0] for p in win if p[3] > 0], 50),
                   "stage_p50_ms": {k2: pctl(v, 50) for k2, v in st.items()},
                   "stage_p99_ms": {k2: pctl(v, 99) for k2, v in st.items()},
                   "not_bound": sum(1 for p in pods if p[2] == 0), "failed": sum(1 for p in pods if p[6]),
                   "room_waits": room_waits,
                   # kubelet stand-in over the row: mean ms per admission of its serial steps (the queue wait, the
                   # plugin's Allocate as kubelet sees it) and of the pod workers' (runtime, Running patch)
                   "kubelet_mean_ms": _agent_delta(na0, na1),
                   # the plugin's gRPC endpoint over the row: Allocates on its native fast path / handed to Python,
                   # calls that waited for their pod's event, and how long in all
                   "plugin_grpc": _grpc_delta(pg0, pg1),
                   "create_errors": res["create_errors"], "delete_errors": res["delete_errors"]}
            ok = (row["bound_pods_per_s"] >= 0.9 * rate and (row["p99_bind_latency_ms"] or 1e9) <= 100.0
                  and row["not_bound"] == 0 and row["failed"] == 0)
            row["kept_up"] = ok
            out["rows"].append(row)
            key = str(ms)
            out["max_sustained_pods_per_s"][key] = max(out["max_sustained_pods_per_s"].get(key, 0.0),
                                                       row["bound_pods_per_s"])
            if first is None:
                first = row
            if ok:
                out["knee_pods_per_s"][key] = rate
                continue
            # the stage whose median grew most against the lowest rate of this latency: the serial stage that binds
            # (the bound rate kept up but its p99 did not: the stage whose p99 grew most -- a tail, not a queue)
            q = "stage_p50_ms" if row["bound_pods_per_s"] < 0.9 * rate else "stage_p99_ms"
            growth = {s2: (row[q][s2] or 0.0) - (first[q][s2] or 0.0) for s2 in st}
            cands = ("admit", "free") if room_waits > 0 else ("create", "bind", "admit")
            stage = max(cands, key=growth.get)
            km, k0 = row.get("kubelet_mean_ms") or {}, first.get("kubelet_mean_ms") or {}
            if stage == "admit" and km:
                # which step of an admission grew: the serial queue, the plugin's Allocate (kubelet's serial call),
                # the runtime (the container start, here the HBM stand-in) or the Running status patch
                sub = {k2: km.get(k2, 0.0) - k0.get(k2, 0.0) for k2 in ("queue", "plugin_allocate", "runtime",
                                                                       "running_patch")}
                stage += "/" + max(sub, key=sub.get)
            if stage == "create" and rate >= 0.8 * a.open_loop_creators * 1e3 / ms:
                # the driver's own creators (each a POST at the injected latency): not the product's bound
                stage += f" (driver: {a.open_loop_creators} creators at {ms} ms)"
            elif q == "stage_p99_ms":
                stage += " (p99)"
            out["bound_stage"][key] = stage + (" (room held)" if room_waits > 0 else "")
            break
    set_latency(api_batch, 0)
    return out


def plugin_path(a, children, api_url, runner: WaveRunner, E) -> dict:
    """The same waves with kubelet + device plugin = the shipped gRPC GpuSharePlugin, driven over its unix socket
    by the kubelet stand-in (serial admission, GetPreferredAllocation + Allocate per pod) instead of the
    compiled node agent.  The plugin's own pod informer and allocation state decide every Allocate.  With
    ``--plugin-proc process`` (default) the plugin is its own process (``python -m ...deviceplugin``) that
    registers with the stand-in's Registration service, as under a real kubelet."""
    from gsxtools.cluster import start_node_agent

    ext_url = next(c.url for c in children if c.name == "extender")
    na = restart_child(children, "node-agent", lambda old: start_node_agent(
        api_url, NODE, profile=a.profile, native=False, plugin=a.plugin_proc, cpus=old.cpus,
        extra=["--faithful"] if a.kubelet == "faithful" else [], plugin_cpus=a.plugin_cpus, extender=ext_url))
    client = E.BatchClient({"server": na.url})
    wait_until(lambda: client.run([("GET", "/v1/stats", b"")], 1)[0][0] == 200, 120, "plugin agent never ready")
    row = runner.measure(3, max(a.sweep_steps, 40))  # ~2 ms waves: 40 of them cost little and steady the row
    st, body = client.run([("GET", "/v1/stats", b"")], 1)[0]
    stats = json.loads(body) if st == 200 else {}
    return {**row, "admit_p50_ms": stats.get("admit_p50_ms"), "breakdown_ms": stats.get("breakdown_ms"),
            "plugin_breakdown_ms": stats.get("plugin_breakdown_ms"), "allocate_calls": stats.get("allocate_calls"),
            "allocate_errors": stats.get("allocate_errors"), "mismatch": stats.get("mismatch"),
            "swapped_equivalent": stats.get("swapped_equivalent"),
            "plugin_stats": stats.get("plugin_stats"), "plugin": stats.get("plugin")}


def inprocess_matcher_path(a, children, api_url, runner: WaveRunner, E) -> dict:
    """The same waves with the compiled kubelet stand-in deciding every Allocate with the plugin's matcher linked
    in-process (allocstate.h) and committing ASSIGNED itself -- no gRPC hop to a plugin process, no PodResources
    reconciliation.  The rounds-1..3 headline path, kept as a comparison row."""
    from gsxtools.cluster import start_node_agent

    ext_url = next(c.url for c in children if c.name == "extender")
    na = restart_child(children, "node-agent", lambda old: start_node_agent(
        api_url, NODE, profile=a.profile, native=True, plugin="grpc", cpus=old.cpus, serial_admission=True,
        extender=ext_url))
    client = E.BatchClient({"server": na.url})
    wait_until(lambda: client.run([("GET", "/v1/stats", b"")], 1)[0][0] == 200, 120, "node agent never ready")
    row = runner.measure(3, max(a.sweep_steps, 40))
    st, body = client.run([("GET", "/v1/stats", b"")], 1)[0]
    stats = json.loads(body) if st == 200 else {}
    return {**row, "admit_p50_ms": stats.get("admit_p50_ms"), "failed": stats.get("failed"),
            "kubelet_mean_ms": stats.get("mean_ms")}


def _plugin_debug(E, url: str | None) -> dict | None:
    """The shipped plugin process's own counters (its /debug/state): Allocates answered on the native fast path,
    early-answer commits, kubelet-PodResources reconciliation (swaps repaired, moves through the extender)."""
    if not url:
        return None
    try:
        st, body = E.BatchClient({"server": url}).run([("GET", "/debug/state", b"")], 1)[0]
        d = json.loads(body) if st == 200 else {}
    except Exception as e:  # noqa: BLE001 - a missing row never costs the headline line
        return {"error": repr(e)}
    g = d.get("grpc") or {}
    return {"grpc": {k: g.get(k) for k in ("impl", "fast_allocate", "slow_allocate", "fast_preferred",
                                           "slow_preferred", "patch_failures", "guard_by_ids", "journaling",
                                           "early_answer_backlog", "waited", "feed_events", "passes",
                                           "last_slow_reason", "handler_us", "allocate_phases_us", "lock_wait",
                                           "wait_ms", "commits_gone")},
            "stats": d.get("stats"), "reconcile": d.get("reconcile"),
            "physical": d.get("physical"), "held": d.get("held"), "records": d.get("records"),
            # mean seconds per native fast-path Allocate: match, isolation files, record + answer (handler)
            "timing": {k: (v / max(1, (d.get("timing") or {}).get("n", 0)) if k != "n" else v)
                       for k, v in (d.get("timing") or {}).items() if not k.startswith("preferred")}}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=int(os.environ.get("WORLD_SIZE", "1")))
    # a 1-GPU wave takes ~0.6 ms: 300 steps keep the timed region >= ~0.2 s (at 50 steps the same binaries
    # read 5.0k-7.0k pods/s run to run on one box, scripts/experiments/gpu_ab.sh)
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--warmup", type=int, default=30)
    ap.add_argument("--pods-per-gpu", type=int, default=4)
    ap.add_argument("--pod-gib", type=int, default=64)
    ap.add_argument("--profile", default="aliyun")
    ap.add_argument("--bind-mode", default="binding", choices=["binding", "update"])
    ap.add_argument("--devices", default="auto", help="auto|hip|amdsmi|fake (fake: no GPU, CPU plumbing only)")
    # one stamp per 2 MiB carve unit: slices are carved in 2 MiB units, so any overlap of two slices hits a stamp
    # (1 MiB put two in each unit: verify 11.9 -> 7.2 us per admission on MI355X, profiles/r02_stride_ab/)
    ap.add_argument("--stamp-stride", type=int, default=2 << 20)
    ap.add_argument("--json-out", default="")
    ap.add_argument("--dump-timings", default="",
                    help="write every timed pod's scheduler timeline (CLOCK_MONOTONIC, like the wave's t0) here")
    ap.add_argument("--agent", default="node", choices=["node", "rank"],
                    help="node: one node-agent process (the node's device plugin) driving a runtime shim per GPU rank (default); rank: one agent per GPU rank")
    ap.add_argument("--node-agent", default="native-plugin", choices=["native", "native-plugin", "plugin", "inproc"],
                    help="kubelet + device plugin: the compiled kubelet stand-in (gsx-nodeagent: faithful serial "
                         "admission, never re-routes, serves PodResources) calling the shipped plugin process over "
                         "the device-plugin gRPC API (native-plugin, default: the product path), gsx-nodeagent with "
                         "the plugin's matcher linked in-process (native), or the Python kubelet stand-in driving the "
                         "shipped plugin over its socket (plugin) / in-process (inproc)")
    ap.add_argument("--pin", default="auto", choices=["auto", "spread", "static", "compact", "none"],
                    help="CPU placement of the control-plane processes (auto = spread: the idlest physical cores, "
                         "sampled at start; static: topology order without the load sample)")
    ap.add_argument("--pin-widths", default="", help='JSON {"process": n_cpus} overriding the CPU slot widths')
    ap.add_argument("--runtime-cpu", default="shared", choices=["split", "shared"],
                    help="split: GPU 0's runtime endpoint threads get their own CPU (rank 0's SMT sibling); "
                         "shared: they share rank 0's CPU with the wave driver")
    ap.add_argument("--gpu-warm-ms", type=float, default=300.0,
                    help="run GEMMs on each rank's GPU for this long before the warmup waves (clock ramp; "
                         "interleaved A/B after 20 s idle: 10.5-11.0k vs 8.9-10.8k pods/s, profiles/r02_pinload)")
    ap.add_argument("--pin-smt", type=int, default=1,
                    help="1: a 2-CPU slot is one physical core with both SMT threads, so the N=1 plan fits one "
                         "L3 domain (6 cores with the plugin; 7 at N > 1); 0: two physical cores")
    ap.add_argument("--api-latency-ms", type=float, default=0.0,
                    help="fake kube-apiserver answers every non-watch request after this delay (timed region)")
    ap.add_argument("--bind-order", default="auto", choices=["auto", "strict", "relaxed"],
                    help="extender --bind-order: auto (default; no order on this node, whose plugin matches in landing "
                         "order), strict ASSUME_TIME order of equal-size cross-GPU binds (the reference plugin's "
                         "contract) or relaxed (all concurrent; swaps repaired by the plugin's PodResources "
                         "reconciliation)")
    ap.add_argument("--sweep-orders", default="auto", help="bind orders the latency sweep covers (comma list)")
    # serial by default: kubelet admits a node's pods one at a time.  Measured on MI355X boxes: N = 1 unchanged
    # (wave p50 10.2-11.1k vs 10.1-11.6k parallel), N = 8 -10 % (16.9-17.6k vs 18.7-19.8k), profiles/r03_admission/
    ap.add_argument("--admission", default="serial", choices=["parallel", "serial"],
                    help="compiled node agent with its in-process matcher: admit (Allocate + ASSIGNED commit) one pod "
                         "at a time in arrival order as kubelet does (serial, default), or on all workers at once "
                         "(parallel); containers start in parallel either way")
    ap.add_argument("--kubelet", default="faithful", choices=["standin", "faithful"],
                    help="with --node-agent plugin (the Python kubelet stand-in): it behaves like kubelet and lets the "
                         "plugin reconcile from its PodResources record (faithful, default), or re-routes a "
                         "mismatched Allocate (standin)")
    ap.add_argument("--plugin-proc", default="process", choices=["process", "grpc"],
                    help="device-plugin path row: the plugin as its own process registered with the kubelet "
                         "stand-in, as the DaemonSet runs it (process), or served from the stand-in's process (grpc)")
    ap.add_argument("--sweep", type=int, default=1, help="1: run the latency sweep after the timed region")
    # 20 waves a latency point (~0.4 s at 5 ms): with 8, single points read 20-45 % below their neighbours
    ap.add_argument("--sweep-steps", type=int, default=20)
    ap.add_argument("--open-loop", default="auto",
                    help="open-loop throughput rows after the timed region: 'auto' (the rate ladder "
                         f"{OPEN_LOOP_RATES} at {OPEN_LOOP_LATENCIES_MS} ms apiserver latency), a comma list of "
                         "rates, or 0 (off)")
    ap.add_argument("--open-loop-gib", type=int, default=1, help="pod size of the open-loop rows")
    ap.add_argument("--open-loop-s", type=float, default=1.5, help="seconds of arrivals per open-loop rate")
    ap.add_argument("--term-grace", type=int, default=-1,
                    help="the pods' spec.terminationGracePeriodSeconds: >= 0 makes every deletion graceful (the node "
                         "agent stops the containers, reports the terminal phase, then deletes the object, as kubelet "
                         "does); -1 (default) leaves it unset, and the fake apiserver deletes at once (a force delete: "
                         "the node agent's PodResources lists a container until its runtime slice is released, and "
                         "the plugin runs GSX_PLUGIN_FORCE_DELETE=report)")
    ap.add_argument("--open-loop-creators", type=int, default=64,
                    help="open-loop driver threads creating (and as many deleting) pods: at apiserver latency L they "
                         "offer at most creators / L pods/s (16 made the 2 ms row's knee the driver's own)")
    ap.add_argument("--share-gpu", action="store_true",
                    help="every rank uses physical GPU 0 (a one-box rehearsal of the N-GPU launch): each rank advertises "
                         "a logical device sized for its wave (pods-per-gpu x pod-gib plus half a pod) and carves its "
                         "own HBM arena out of GPU 0, so N processes run their stamp / verify kernels on one card")
    ap.add_argument("--wave-sampler", type=int, default=0,
                    help="1: a sampler process on a spare CPU records every pipeline process's scheduler run-delay and "
                         "the host's pressure counters, so each timed wave (and any slow one) is attributed "
                         "(gsxtools/wavesampler.py; the JSON line's wave_attribution).  Off by default: reading the "
                         "threads' /proc stats every 2 ms slows the pipeline (N = 8: 11.0-11.2k -> 6.0-8.3k pods/s, "
                         "profiles/r05_session5/).  The region-level run_delay_pct and psi_timed_ms are always there")
    ap.add_argument("--apiserver-threads", type=int, default=0,
                    help="event loops of the fake apiserver (0: auto; GSX_FAKEAPI_THREADS overrides)")
    return ap.parse_args()


def rank_device(devs, phys: int, local_rank: int, use_gpu: bool, who: str = "rank"):
    """The device a rank advertises: the one whose HIP ordinal is ``phys`` -- the GPU its HBM arena and kernels live on
    (``torch.cuda.set_device(phys)``).  Device indices are HIP ordinals (libmxdev orders amdsmi's devices by their
    hip_id), so this holds on platforms whose amdsmi order is not the HIP order (tests/test_device_topology.py).
    Without a GPU: the fake inventory's entry.  The advertised index is the rank's (one GPU per rank)."""
    if use_gpu:
        mine = [d for d in devs if d.index == phys]
        if not mine:
            raise SystemExit(f"{who}: GPU {phys} not found")
        dev = mine[0]
    else:
        dev = devs[local_rank % len(devs)]
    dev.index = local_rank
    return dev


def node_inventory(devs, unit: str = "GiB") -> list[dict]:
    """The node's device inventory annotation (what the device plugin publishes, plugin.py publish_node)."""
    return [{"index": d.index, "bdf": d.bdf, "uuid": d.uuid, "units": d.units(unit), "total_bytes": d.total_bytes,
             "share_bytes": d.share_bytes, "cu": d.cu_count, "xcc": d.xcc_count, "render": d.render_minor,
             "card": d.card_minor, "partition": d.partition} for d in devs]


def cpu_slots(world: int, runtime_cpu: str = "shared", apiserver_threads: int = 0) -> tuple[list[str], dict, int]:
    """The processes of a bench run on ``world`` GPUs and the CPUs each asks for (utils/cpuset.py plans them; with
    fewer CPUs than asked the plan is empty and nothing is pinned).  Returns (names, widths, apiserver threads)."""
    # "plugin": the shipped device-plugin process when an agent starts one (its own CPUs, as a DaemonSet pod)
    names = ["rank0", "apiserver", "extender", "scheduler", "node-agent", "plugin"] + [f"rank{r}" for r in range(1, world)]
    # CPUs per process: the extender (2 loops + bind pool + reflectors), schedsim (cycle + bind threads) and the
    # node agent (reflector + workers) get two; rank 0 stays on one core (a second one let its driver, tracker
    # and runtime threads migrate: 7.5-9.4k vs 10.1k pods/s, interleaved A/B in profiles/r02_bench_stability.md)
    # The plugin gets one core (2 CPUs) on a one-GPU node, what its DaemonSet requests.  Round 4 gave it two: its
    # serving thread then busy-looped on a stuck deferred wake-up between bursts (fixed in round 5, bindings.cc
    # DpServer::serve), and on one core its pod feed queued behind it (profiles/r04_pinw/).  An 8-GPU node admits 8x
    # the pods through it: two cores there (run-delay of its threads 214 ms per 170 ms region on one core,
    # profiles/r05_session4/)
    widths = {"extender": 2, "scheduler": 2, "node-agent": 2, "plugin": 2 if world == 1 else 4}
    if runtime_cpu == "split":
        # rank 0 = the wave driver + GPU 0's runtime endpoint (the CRI-runtime role): one core, the driver on
        # one SMT thread and the endpoint's threads on the other, instead of both time-sharing one thread
        widths["rank0"] = 2
    # the kubelet stand-in on a multi-GPU node admits N x 4 pods a wave with its pod workers starting the previous
    # ones: two cores there (N = 8: 15.2-15.9k pods/s vs 13.2-14.3k on one core, where its threads waited for a CPU
    # 150-190 % of the region; profiles/r05_session26/).  A real kubelet has the node's cores.
    if world > 1:
        widths["node-agent"] = 4
    # ranks > 0 idle in a gloo barrier during the timed waves while their runtime endpoint admits pods: on a
    # single CPU the endpoint thread waited behind gloo's threads for up to 9 ms (N=4/8 rehearsal, 2 CPUs fix it)
    widths.update({f"rank{r}": 2 for r in range(1, world)})
    if world > 1:
        # with N GPUs rank 0's wave driver creates and tracks N x 4 pods per wave: on one CPU the creates trickled
        # out (scheduler saw the 32nd pod of an N = 8 wave 0.96 ms in, 0.53 ms with a second CPU; per-wave p50
        # 13.0k -> 19.2k pods/s at N = 8, 10.6k -> 15.7k at N = 4; N = 1 unchanged, profiles/r03_ab/)
        widths["rank0"] = 2
    # the fake apiserver's event loops (a shared store): GSX_FAKEAPI_THREADS, else --apiserver-threads, else one loop
    # at N = 1 and APISERVER_THREADS_MULTI at N > 1, each on its own CPU
    api_threads = int(os.environ.get("GSX_FAKEAPI_THREADS", "0")) or apiserver_threads or (
        1 if world == 1 else APISERVER_THREADS_MULTI)
    widths["apiserver"] = api_threads
    return names, widths, api_threads


def _same_condition(ref_client) -> float | None:
    rows = {r.get("bind_mode"): r for r in ref_client or [] if isinstance(r, dict)}
    b = rows.get("binding", {}).get("pods_per_s")
    return round(b / BASELINE_BINDS_PER_S, 2) if b else None


def launch_ranks(n: int) -> int:
    """One rank per GPU over torch.distributed.run (rendezvous on 127.0.0.1), as a child process."""
    import socket
    import subprocess

    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__), *sys.argv[1:]]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    p = subprocess.Popen(cmd, env=env)
    try:
        return p.wait()
    except KeyboardInterrupt:
        p.terminate()
        return p.wait()


def main():
    import signal

    # torchrun stops the other ranks with SIGTERM when one fails: exit through atexit so child servers stop too
    signal.signal(signal.SIGTERM, lambda *_: sys.exit(143))
    a = parse()
    # pods deleted outright (no --term-grace): the node agent's PodResources lists a container until its runtime slice
    # is released, so the plugin may take that report as the truth instead of waiting out a kill deadline
    os.environ.setdefault("GSX_PLUGIN_FORCE_DELETE", "report" if a.term_grace < 0 else "grace")
    if "WORLD_SIZE" not in os.environ and a.gpus > 1:
        # `python bench.py --gpus N` without a launcher: start torchrun as a CHILD process (this process has not
        # touched the GPU, and is never replaced by exec) and exit with its code
        sys.exit(launch_ranks(a.gpus))
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", str(rank)))
    if world != a.gpus:
        a.gpus = world

    # ---- CPU placement (the same plan on every rank: each takes its own slot)
    from gpushare_scheduler_extender_amd.utils.cpuset import forget_shared_plan, pin_self, plan, shared_plan

    names, widths, api_threads = cpu_slots(world, a.runtime_cpu, a.apiserver_threads)
    if a.pin_widths:
        widths.update(json.loads(a.pin_widths))
    mode = a.pin if a.pin != "auto" else "spread"
    # the chain of round trips shares one L3 domain: rank 0, apiserver, extender, scheduler, node agent AND the
    # plugin (kubelet's two calls per admission).  With the plugin left out (round 5 until session 17) it landed in
    # another CCD whenever the first one was full: N = 8 read 12.1-13.1k pods/s with node agent and plugin in one
    # L3 domain, 9.8-11.8k across two (profiles/r05_session18/)
    local = int(os.environ.get("GSX_PIN_LOCAL", "0")) or names.index("plugin") + 1  # (env: A/B only)
    if world > 1 and mode != "none":
        # one plan for the whole job (the ranks' load samples would differ): keyed by the torchrun agent
        key = f"{os.getppid()}-{os.environ.get('MASTER_PORT', '0')}"
        cpu_plan = shared_plan(names, widths, mode, key, smt=bool(a.pin_smt), local=local)
        if rank == 0:
            import atexit

            atexit.register(forget_shared_plan, key)
    else:
        cpu_plan = plan(names, widths, mode, smt=bool(a.pin_smt), local=local)
    mine_cpus = cpu_plan.get(f"rank{rank}")
    a.plugin_cpus = cpu_plan.get("plugin")
    runtime_cpus = None
    if rank == 0 and a.runtime_cpu == "split" and mine_cpus and len(mine_cpus) >= 2:
        mine_cpus, runtime_cpus = mine_cpus[:1], mine_cpus[1:]
    pin_self(mine_cpus)

    # ---- rank 0 starts its child processes BEFORE anything initialises the GPU
    children = []
    api_url = ext_url = ""
    lt = LoopThread()
    if rank == 0:
        from gsxtools.cluster import (start_apiserver, start_extender, start_node_agent,
                                                                 start_scheduler)

        api = start_apiserver(cpus=cpu_plan.get("apiserver"), threads=api_threads)
        children.append(api)
        ext = start_extender(api.url, profile=a.profile, bind_mode=a.bind_mode, cpus=cpu_plan.get("extender"),
                             bind_order=a.bind_order)
        children.append(ext)
        # kube-scheduler stand-in: its own process, like the real one (serial scheduling cycle)
        children.append(start_scheduler(api.url, ext.url, profile=a.profile,
                                        cpus=cpu_plan.get("scheduler")))
        if a.agent == "node":
            # the node's device plugin / kubelet stand-in: one process for all GPUs of the node, like a DaemonSet
            def start_agent(cpus, api_url=api.url, ext_url=ext.url):
                return start_node_agent(api_url, NODE, profile=a.profile,
                                        native=a.node_agent in ("native", "native-plugin"),
                                        plugin={"inproc": "inproc", "native-plugin": "spawn"}.get(a.node_agent, "grpc"),
                                        workers=min(16, max(8, 2 * a.pods_per_gpu * world)), cpus=cpus,
                                        # the compiled stand-in is kubelet-faithful in plugin mode already
                                        extra=["--faithful"] if a.kubelet == "faithful" and a.node_agent in (
                                            "plugin", "inproc") else [],
                                        plugin_cpus=a.plugin_cpus, serial_admission=a.admission == "serial",
                                        extender=ext_url)

            def restore_node_agent():
                na = restart_child(children, "node-agent", lambda old: start_agent(old.cpus))
                client = E.BatchClient({"server": na.url})
                wait_until(lambda: client.run([("GET", "/v1/stats", b"")], 1)[0][0] == 200, 120,
                           "node agent never ready")
                wait_until(lambda: bool(json.loads(client.run([("GET", "/v1/stats", b"")], 1)[0][1]).get(
                    "plugin_debug")), 30, "plugin debug endpoint")

            children.append(start_agent(cpu_plan.get("node-agent")))
        api_url, ext_url = api.url, ext.url

    import torch
    import torch.distributed as dist

    from gsxtools.agent import NodeAgent
    from gpushare_scheduler_extender_amd.deviceplugin.devices import UNITS, discover
    from gpushare_scheduler_extender_amd.deviceplugin.runtime import HbmArenaRuntime, LedgerRuntime, RuntimeShim
    from gpushare_scheduler_extender_amd.k8s.client import KubeClient
    from gpushare_scheduler_extender_amd.k8s.objects import make_node, make_pod
    from gpushare_scheduler_extender_amd.models.profile import get_profile

    # ranks do no CPU tensor work: one intra-op thread each, so 8 ranks never burst past a container's CPU quota
    torch.set_num_threads(1)
    profile = get_profile(a.profile)
    use_gpu = a.devices != "fake" and torch.cuda.is_available()
    # the physical GPU this rank's HBM arena and kernels live on (all ranks on GPU 0 with --share-gpu)
    phys = 0 if a.share_gpu else local_rank
    if use_gpu:
        torch.cuda.set_device(phys)
    if world > 1:
        # every collective of the bench is control traffic (barriers, a few small objects, one float MAX): gloo over
        # loopback TCP.  The scheduling data path has no collectives, so RCCL is never initialised here.
        dist.init_process_group("gloo")
    ctl = None  # the default (gloo) group

    def barrier():
        if world > 1:
            dist.barrier()
        if use_gpu:
            torch.cuda.synchronize()

    def bcast(obj):
        if world == 1:
            return obj
        box = [obj]
        dist.broadcast_object_list(box, src=0, group=ctl)
        return box[0]

    def gather(obj):
        if world == 1:
            return [obj]
        out = [None] * world
        dist.all_gather_object(out, obj, group=ctl)
        return out

    api_url, ext_url = bcast((api_url, ext_url))

    # ---- this rank's GPU
    backend, devs = discover("fake" if not use_gpu else a.devices)
    dev = rank_device(devs, phys, local_rank, use_gpu, f"rank {rank} ({backend})")
    unit = "GiB"
    pod_bytes = a.pod_gib * UNITS[unit]
    arena = a.pods_per_gpu * pod_bytes
    if a.share_gpu:
        # one logical device per rank, carved out of GPU 0: room for the wave's pods plus half a pod, so best fit
        # puts exactly pods_per_gpu pods on each (as 4 x 64 GiB fill one 287 GiB MI355X)
        if world * arena > 0.85 * dev.total_bytes:
            raise SystemExit(f"--share-gpu: {world} arenas of {arena >> 30} GiB do not fit GPU 0 "
                             f"({dev.total_bytes >> 30} GiB); lower --pod-gib")
        dev.share_bytes = arena + (pod_bytes // 2 // UNITS[unit]) * UNITS[unit]
    # this GPU's runtime endpoint (CRI-runtime role): the node agent starts pods on it over HTTP
    if a.agent == "node":
        # native (native/engine/podruntime.cc): request threads carve the slice and run the HIP admission
        runtime = shim = NativeRuntime(phys, arena, use_gpu, a.stamp_stride, runtime_cpus)
        shim_url = shim.url
    else:
        if a.share_gpu:
            raise SystemExit("--share-gpu needs --agent node (the per-rank agent keys its arena by the logical index)")
        runtime = (HbmArenaRuntime({local_rank: arena}, stamp_stride=a.stamp_stride) if use_gpu
                   else LedgerRuntime({local_rank: arena}))
        shim = RuntimeShim(runtime)
        shim_url = lt.run(shim.start("127.0.0.1", 0))
    all_devs = gather((dev.to_dict(), shim_url))
    from gpushare_scheduler_extender_amd.deviceplugin.devices import Device
    from gpushare_scheduler_extender_amd.models.profile import (NODE_ALLOCATE_ORDER_ANNOTATION,
                                                                NODE_DEVICE_INFO_ANNOTATION,
                                                                NODE_RUNTIME_ENDPOINTS_ANNOTATION)

    agent_client = KubeClient(api_url)

    async def setup_node():
        c = KubeClient(api_url)
        devs_ = [Device(**d) for d, _ in all_devs]
        totals = [d.units(unit) for d in devs_]
        inv = node_inventory(devs_, unit)
        node = make_node(NODE, sum(totals), len(totals), profile=profile, device_totals=totals,
                         annotations={NODE_DEVICE_INFO_ANNOTATION: json.dumps(inv),
                                      # as the device plugin publishes it: its matcher is landing-ordered
                                      NODE_ALLOCATE_ORDER_ANNOTATION: "landing",
                                      NODE_RUNTIME_ENDPOINTS_ANNOTATION: json.dumps(
                                          {str(d.index): u for d, (_, u) in zip(devs_, all_devs)})})
        node["metadata"].setdefault("labels", {})["gpushare"] = "true"
        await c.create("nodes", node)
        await c.close()
        return totals

    totals = lt.run(setup_node()) if rank == 0 else None
    totals = bcast(totals)
    agent = None
    if a.agent == "rank":
        # one agent per GPU rank (each watches the node's pods; heavier on the apiserver)
        agent = NodeAgent(agent_client, NODE, [dev], profile, runtime, unit=unit, verify_each=True,
                          mount_mode="isolated")
        lt.run(agent.start())

    client = tracker = sched_http = None
    if rank == 0:
        from gpushare_scheduler_extender_amd.core.engine import native as _native_engine
        from gpushare_scheduler_extender_amd.k8s.fasthttp import Client as _HttpClient

        E = _native_engine()
        client = KubeClient(api_url)
        sched_http = _HttpClient(next(c.url for c in children if c.name == "scheduler"))
        # the wave driver (load generator) is native: a reflector over the wave's pods that answers
        # "all bound / Running / gone?" and a keep-alive batch client for the creates (native/engine/tracker.cc)
        tracker = E.PodTracker({"server": api_url}, "default", "gsx-wave")
        tracker.start(60)
        api_batch = E.BatchClient({"server": api_url})
        ext_batch = E.BatchClient({"server": ext_url})
        # wait until the extender has seen the node
        for _ in range(2000):
            st, body = ext_batch.run([("GET", "/gpushare-scheduler/inspect", b"")], 1)[0]
            if st == 200 and json.loads(body).get("nodes"):
                break
            time.sleep(0.005)
        if a.agent == "node":
            # kubelet (the node agent) watches the node's pods before the first wave is bound, as on a live node:
            # pods it first met in one LIST would be admitted as one batch in name order, not as they landed
            na_batch = E.BatchClient({"server": next(c.url for c in children if c.name == "node-agent")})
            wait_until(lambda: na_batch.run([("GET", "/v1/stats", b"")], 1)[0][0] == 200, 300, "node agent never ready")
            if a.node_agent == "native-plugin":
                # the spawned plugin serves kubelet before its debug endpoint is up: wait for it (bounded), so that
                # its counters reach the JSON line even on a slow host
                def _debug_up():
                    st, body = na_batch.run([("GET", "/v1/stats", b"")], 1)[0]
                    return st == 200 and bool(json.loads(body).get("plugin_debug"))
                try:
                    wait_until(_debug_up, 20, "plugin debug endpoint")
                except TimeoutError:
                    pass
        pod_tmpl = make_pod("__NAME__", a.pod_gib, profile=profile, labels={"gsx-wave": "__STEP__"})
        if a.term_grace >= 0:
            pod_tmpl["spec"]["terminationGracePeriodSeconds"] = a.term_grace
        del pod_tmpl["metadata"]["uid"]  # the apiserver assigns one per pod
        pod_tmpl = json.dumps(pod_tmpl, separators=(",", ":"))
    from gpushare_scheduler_extender_amd.utils.gctune import tune

    rank_pids = gather(os.getpid())
    sampler = None
    if rank == 0 and a.wave_sampler:
        # per-wave attribution (run-delay of every pipeline process, host pressure) from a process of its own, on a
        # CPU outside the plan when there is one
        from gsxtools.wavesampler import Sampler

        pids = {"rank0": os.getpid(), **{f"rank{r}": p for r, p in enumerate(rank_pids) if r > 0}}
        for c in children:
            pid = getattr(getattr(c, "proc", None), "pid", None)
            if pid:
                pids[c.name] = pid
                if c.name == "node-agent":
                    for k in _child_pids(pid):
                        pids["plugin"] = k
        planned = {x for v in cpu_plan.values() for x in (v or [])}
        spare = sorted(set(os.sched_getaffinity(0)) - planned) if planned else []
        import tempfile

        sampler = Sampler(pids, os.path.join(tempfile.gettempdir(), f"gsx-waves-{os.getpid()}.json"),
                          cpu=spare[-1] if spare else None)
        if not sampler.wait_ready():
            sampler = None  # diagnosis only: the headline runs without it
    if rank == 0 and a.api_latency_ms:
        set_latency(api_batch, a.api_latency_ms)
    tune()
    if use_gpu and a.gpu_warm_ms > 0:
        # bring this GPU out of its idle power state before the warmup waves: the admissions are ~10 us kernels,
        # too short and too sparse to ramp the clocks themselves (a first bench on an idle box admitted at half
        # speed: node agent p50 0.19 vs 0.10 ms)
        x = torch.randn(4096, 4096, device="cuda", dtype=torch.bfloat16)
        t_warm = time.perf_counter() + a.gpu_warm_ms / 1e3
        while time.perf_counter() < t_warm:
            for _ in range(8):
                x = (x @ x).clamp_(-1, 1)
            torch.cuda.synchronize()
        del x
    barrier()

    n_pods = a.pods_per_gpu * world
    step_stats = []

    def inspect_used():
        st, body = ext_batch.run([("GET", "/gpushare-scheduler/inspect", b"")], 1)[0]
        if st != 200:
            raise RuntimeError(f"inspect failed: {st} {body[:200]!r}")
        return json.loads(body)

    prepared = {}

    def wave_requests(step: int):
        # the load generator's create requests, built ahead of the timed region (pure client-side formatting)
        if step not in prepared:
            names = [f"w{step}-p{i}" for i in range(n_pods)]
            body = pod_tmpl.replace("__STEP__", str(step))
            prepared[step] = (names, [f"default/{nm}" for nm in names],
                              [("POST", "/api/v1/namespaces/default/pods", body.replace("__NAME__", nm).encode())
                               for nm in names])
        return prepared[step]

    def wave(step: int):
        try:
            return wave_once(step)
        except Exception:
            # a failed wave leaves none of its pods behind: the rows after it re-use the step's names and need the
            # room (one comparison row's failed admission failed the next row and the open loop's drain)
            try:
                api_batch.run([("DELETE", f"/api/v1/namespaces/default/pods?labelSelector=gsx-wave%3D{step}", b"")], 1)
            except Exception:  # noqa: BLE001 - the wave's own error is the one to report
                pass
            raise

    def wave_once(step: int):
        names, keys, reqs = wave_requests(step)
        t0 = time.perf_counter()
        res = api_batch.run(reqs, min(CREATE_CONCURRENCY, n_pods))
        t_created = time.perf_counter()
        bad = [(st, b[:200]) for st, b in res if st != 201]
        if bad:
            raise RuntimeError(f"pod create failed: {bad[:3]}")
        err = tracker.wait(keys, E.TRACK_BOUND, 120)
        if err:
            raise RuntimeError(err)
        t_bound = time.perf_counter()
        # every pod admitted on its GPU and Running (a Failed admission aborts the run)
        err = tracker.wait(keys, E.TRACK_RUNNING, 120)
        if err:
            raise RuntimeError(f"pod admission failed: {err}")
        t_run = time.perf_counter()
        insp = inspect_used()
        t_insp = time.perf_counter()
        used = sum(n["usedGPU"] for n in insp["nodes"])
        total = sum(n["totalGPU"] for n in insp["nodes"])
        per_dev = [d["usedGPU"] for n in insp["nodes"] for d in n["devs"]]
        # teardown: one DeleteCollection for the wave; the step ends when the extender's ledger is empty.
        # The wait is event-driven first (the wave driver's informer sees the deletions about when the
        # extender's does); polling /inspect straight away would pay a sleep quantum per poll instead.
        st, b = api_batch.run([("DELETE", f"/api/v1/namespaces/default/pods?labelSelector=gsx-wave%3D{step}", b"")],
                              1)[0]
        if st != 200:
            raise RuntimeError(f"delete collection failed: {st} {b[:200]!r}")
        t_del = time.perf_counter()
        # the wave's pods are deleted gracefully (TERM_GRACE_S): the node agent stops each pod's containers, reports
        # the terminal phase -- which frees its share in the extender -- and then deletes the object.  The next wave
        # needs the room, not the old objects gone
        err = tracker.wait(keys, E.TRACK_STOPPED, 120)
        if err:
            raise RuntimeError(err)
        t_gone = time.perf_counter()
        while sum(n["usedGPU"] for n in inspect_used()["nodes"]) != 0:
            if time.perf_counter() - t0 > 120:
                raise TimeoutError("ledger did not drain")
            time.sleep(0.0002)
        t_end = time.perf_counter()
        # per-pod scheduler timings are collected after the timed region (fetch_timings)
        return {"keys": keys, "used": used, "total": total, "per_dev": per_dev,
                "t_bound": t_bound - t0, "t_run": t_run - t0, "t_total": t_end - t0, "t0": t0,
                "teardown": (t_insp - t_run, t_del - t_insp, t_gone - t_del, t_end - t_gone), "t_created": t_created - t0}

    async def fetch_timings(keys):
        # the scheduler process's per-pod timings (its own clock; only differences are used)
        body = json.dumps(keys).encode()
        got = json.loads((await sched_http.request("POST", "/v1/timings", body)).body)
        await sched_http.request("POST", "/v1/forget", body)
        return [got[k] for k in keys]

    prof = None
    if rank == 0 and os.environ.get("GSX_CPROFILE_DIR"):
        import cProfile  # the scheduler simulator + load generator run on the loop thread

        prof = cProfile.Profile()
        lt.loop.call_soon_threadsafe(prof.enable)
    def extender_counters():
        # the native front end's bind counters (GET /debug/engine); diffed around the timed region
        st, body = ext_batch.run([("GET", "/debug/engine", b"")], 1)[0]
        srv = json.loads(body).get("server", {}) if st == 200 else {}
        out = {k: srv.get(k, 0) for k in ("binds", "bind_ok", "bind_fail", "bind_order_waits", "bind_order_wait_s",
                                           "api_calls", "conflicts_retried")}
        for h in ("filter_latency", "bind_latency", "api_latency"):
            out[h + "_n"] = (srv.get(h) or {}).get("n", 0)
            out[h + "_s"] = (srv.get(h) or {}).get("sum", 0.0)
        out["bind_order_wait_max_s"] = srv.get("bind_order_wait_max_s", 0.0)
        return out

    def bracket():
        # both ends of the timed region: this rank's GPU work drained, one barrier over the gloo control group
        # (ranks > 0 block in it -- no CPU or GPU-sync spinning -- while rank 0 drives the timed waves), then
        # drained again.  A second, default-group barrier behind it cost 6-10 ms per run on its own (gloo,
        # N=4/8 rehearsal), a third of the 20-wave region.
        if use_gpu:
            torch.cuda.synchronize()
        if world > 1:
            dist.barrier(group=ctl)
        if use_gpu:
            torch.cuda.synchronize()

    if rank == 0:
        for step in range(a.warmup + a.steps):
            wave_requests(step)
    ext0 = None
    t_start = None
    for step in range(a.warmup + a.steps):
        if step == max(0, a.warmup - 1):
            # the wave driver's objects are long-lived: a cyclic-GC pass inside a 0.3 ms wave is pure noise.  Done
            # before the last warmup wave, so the pipeline's processes are busy again, not idle, when the timed
            # region starts (an idle gap of a few ms let their threads sleep and the first timed wave pay every
            # wake-up)
            gc.collect()
            gc.freeze()
            gc.disable()
            # dirty page cache left by what ran before (a test session, the build) is written back now, not by the
            # flusher inside the ~10 ms region: a first bench on a fresh box read 3.8 ms of IO pressure and one
            # 10 ms wave there (profiles/r05_final/bench.1.json)
            os.sync()
        if step == a.warmup:
            if rank == 0:
                ext0 = extender_counters()
            # the CPU-time counters are read before the bracket: reading /proc for every child took ~0.5 ms, which
            # sat inside the timed region (rank 0's span exceeded the sum of its waves by that much)
            cpu0 = _cpu_times(children)
            rd0 = _cpu_times(children, 1)
            psi0 = _psi_us()
            thr0 = _threads_of_node(children)
            rss0 = _rss_mib(children)
            cg0 = _cgroup_cpu()
            bracket()
            if world > 1:
                # rank 0 leaves the barrier up to ~1.5 ms after the others (its one core also runs the wave
                # driver's threads), and the max over ranks would count that skew: the other ranks start their
                # clock when rank 0's start signal arrives, so every rank's region begins at or after rank 0's
                go = torch.zeros(1)
                if rank == 0:
                    t_start = time.perf_counter()
                    dist.broadcast(go, src=0, group=ctl)
                else:
                    dist.broadcast(go, src=0, group=ctl)
                    t_start = time.perf_counter()
            else:
                t_start = time.perf_counter()
        if rank == 0:
            r = wave(step)
            if step >= a.warmup:
                step_stats.append(r)
        elif step < a.warmup:
            dist.barrier(group=ctl)  # warmup waves in lockstep; timed waves are driven by rank 0 alone
        if rank == 0 and world > 1 and step < a.warmup:
            dist.barrier(group=ctl)
    t_waves_end = time.perf_counter()
    bracket()
    elapsed = time.perf_counter() - t_start
    gc.enable()
    own_elapsed = elapsed
    cpu1 = _cpu_times(children)
    rd1 = _cpu_times(children, 1)
    psi1 = _psi_us()
    thr1 = _threads_of_node(children)
    rss1 = _rss_mib(children)
    cg1 = _cgroup_cpu()
    wave_attr = None
    if sampler is not None:
        from gsxtools.wavesampler import attribute

        data = sampler.stop()
        try:
            wave_attr = attribute(data, [(s["t0"], s["t_total"]) for s in step_stats]) if data else None
        except Exception as e:  # noqa: BLE001 - diagnosis never costs the headline line
            wave_attr = {"error": repr(e)}
    if prof is not None:
        lt.run(asyncio.sleep(0))
        lt.loop.call_soon_threadsafe(prof.disable)
        lt.run(asyncio.sleep(0))
        prof.dump_stats(os.path.join(os.environ["GSX_CPROFILE_DIR"], "rank0-loop.prof"))
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64)  # gloo: a CPU tensor
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    bad = runtime.verify() if use_gpu else 0
    if agent is not None:
        mine = {"admitted": agent.admitted, "failed": agent.failed, "bad_stamps": agent.bad_stamps + bad,
                "admit_p50_ms": round((pct(agent.latency, 50) or 0) * 1e3, 3)}
    else:
        mine = {"admitted": shim.admitted, "failed": shim.failed, "bad_stamps": shim.bad + bad}
        if isinstance(shim, NativeRuntime):
            mine["gpu_admission_calls"] = shim.batches  # concurrent admissions share one stamp+verify+sync
    mine.update({"gpu": local_rank, "physical_gpu": phys if use_gpu else None, "hbm_total": dev.usable_bytes,
                 "arena": arena})
    agent_stats = gather(mine)
    node_agent_stats = plugin_stats = None
    if rank == 0 and a.agent == "node":
        na = next(c for c in children if c.name == "node-agent")
        st, body = E.BatchClient({"server": na.url}).run([("GET", "/v1/stats", b"")], 1)[0]
        node_agent_stats = json.loads(body) if st == 200 else {"error": st}
        plugin_stats = _plugin_debug(E, (node_agent_stats or {}).get("plugin_debug"))
    extender_stats = None
    if rank == 0:
        ext1 = extender_counters()
        d = {k: ext1[k] - ext0.get(k, 0) for k in ext1 if k != "bind_order_wait_max_s"}
        extender_stats = {k: d[k] for k in ("binds", "bind_ok", "bind_fail", "bind_order_waits", "api_calls",
                                            "conflicts_retried")}
        extender_stats["bind_order_wait_ms"] = round(1e3 * d["bind_order_wait_s"], 3)
        extender_stats["bind_order_wait_max_ms_run"] = round(1e3 * ext1["bind_order_wait_max_s"], 3)
        for h in ("filter_latency", "bind_latency", "api_latency"):
            n = d[h + "_n"]
            extender_stats[h + "_mean_ms"] = round(1e3 * d[h + "_s"] / n, 4) if n else None
    apiserver_stats = None
    if rank == 0:
        st, body = api_batch.run([("GET", "/fake/stats", b"")], 1)[0]
        apiserver_stats = json.loads(body) if st == 200 else {"error": st}
        apiserver_stats.pop("counts", None)

    sweep = ref_client = plugin_row = plugin_row_native = None
    if rank == 0 and a.sweep:
        runner = WaveRunner(wave, fetch_timings, lt, n_pods, a.warmup + a.steps, extender_counters)
        try:
            sweep, ref_client = latency_sweep(a, children, api_url, api_batch, runner, inspect_used)
        except Exception as e:  # noqa: BLE001 - the sweep never costs the headline line
            sweep = {"error": f"{type(e).__name__}: {e}"}
        if a.agent == "node" and a.node_agent == "native-plugin":
            try:
                plugin_row = plugin_path(a, children, api_url, runner, E)
            except Exception as e:  # noqa: BLE001
                plugin_row = {"error": f"{type(e).__name__}: {e}"}
            try:
                plugin_row_native = inprocess_matcher_path(a, children, api_url, runner, E)
            except Exception as e:  # noqa: BLE001
                plugin_row_native = {"error": f"{type(e).__name__}: {e}"}
    # the open-loop rows run on the shipped plugin path the timed region ran on: the sweep's comparison rows above
    # restarted the node agent with other kubelet / plugin set-ups, so it is started again as the timed region had it
    # (after the sweep: open-loop churn left behind slowed the sweep's waves 2-4x, profiles/r06_final/README.md)
    ol = None
    if rank == 0 and a.open_loop not in ("", "0"):
        try:
            if a.sweep and a.agent == "node" and a.node_agent == "native-plugin":
                restore_node_agent()
            def sched_stats():
                return json.loads(lt.run(sched_http.request("GET", "/v1/stats"), 30).body)

            na_client = None
            if a.agent == "node":
                na_client = E.BatchClient({"server": next(c.url for c in children if c.name == "node-agent")})

            def na_stats():
                st_, body_ = na_client.run([("GET", "/v1/stats", b"")], 1)[0]
                return json.loads(body_) if st_ == 200 else None

            na_workers = []

            def na_verify(on: bool):
                if na_client is not None:
                    # and 64 pod workers for the open loop: each blocks on the runtime call and the Running patch
                    # (one apiserver round trip), and kubelet's status manager does not hold a pod worker for it;
                    # the agent's own number again afterwards (the sweep's wave rows below)
                    st_, body_ = na_client.run([("POST", "/v1/config", json.dumps({"verify": on}).encode())], 1)[0]
                    if not on and st_ == 200:
                        na_workers.append(json.loads(body_).get("workers", 16))
                    n = 64 if not on else (na_workers[0] if na_workers else None)
                    if n:
                        na_client.run([("POST", "/v1/config", json.dumps({"workers": n}).encode())], 1)

            # the open-loop driver (its creators, deleters and watch are threads of this process) is a load
            # generator, not the cluster: it gets every allowed CPU no other process of the run is pinned to, not
            # rank 0's one (on one CPU its 32 threads throttled the arrivals, profiles/r06_first/)
            own = set(os.sched_getaffinity(0))
            others = {c for k, v in cpu_plan.items() if k != f"rank{rank}" for c in (v or [])}
            try:
                spare = set(_allowed_cpus()) - others
                if len(spare) > len(own):
                    os.sched_setaffinity(0, spare)
                # each admission stamps and verifies its own HBM slice only: with hundreds of pods resident the
                # stand-in runtime's check of every resident slice per admission bounded the rows (runtime 60-150 ms
                # per admission at the knee, profiles/r06_ol/), and it is the harness, not the stack under test
                na_verify(False)
                ol = open_loop(a, api_url, api_batch, E, profile, inspect_used, sched_stats,
                               na_stats if na_client is not None else None)
                if isinstance(ol, dict):
                    ol["driver_cpus"] = len(os.sched_getaffinity(0))
                    ol["runtime_verify"] = "own slice"
            finally:
                na_verify(True)
                os.sched_setaffinity(0, own)
        except Exception as e:  # noqa: BLE001 - never costs the headline line
            ol = {"error": f"{type(e).__name__}: {e}"}
    if world > 1:
        dist.barrier(group=ctl)  # every rank's runtime endpoint stays up until rank 0's sweep is done

    if rank == 0:
        for s in step_stats:
            tm = lt.run(fetch_timings(s["keys"]), 60)
            s["timings"] = tm
            s.update({"bind_latency": [t["bound"] - t["seen"] for t in tm], "bind_rtt": [t["bind_rtt"] for t in tm],
                      "filter_rtt": [t["filter_rtt"] for t in tm], "attempts": [t["attempts"] for t in tm]})
        if a.dump_timings:
            with open(a.dump_timings, "w") as f:
                json.dump([{"t0": s["t0"], "t_bound": s["t_bound"], "t_run": s["t_run"], "t_total": s["t_total"],
                            "pods": s["timings"]} for s in step_stats], f)
        pods_total = n_pods * a.steps
        value = pods_total / elapsed
        lat = [x for s in step_stats for x in s["bind_latency"]]
        rtt = [x for s in step_stats for x in s["bind_rtt"]]
        frtt = [x for s in step_stats for x in s["filter_rtt"]]
        util = statistics.mean(s["used"] / s["total"] for s in step_stats) if step_stats else 0.0
        hbm_total = sum(x["hbm_total"] for x in agent_stats)
        hbm_resident = n_pods * pod_bytes
        out = {
            "metric": "pods bound/sec",
            "value": round(value, 3),
            "unit": "pods/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(1e3 * elapsed / a.steps, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": round(value / BASELINE_BINDS_PER_S, 2),
            # the same condition as the reference's derived ceiling: our extender (one annotated Binding per pod)
            # behind client-go's default QPS 5 / burst 10 bucket, over the 2.5 binds/s the reference gets there
            "vs_baseline_same_condition": _same_condition(ref_client),
            "dtype": "n/a",
            "data": "synthetic pods (random-init ledger, fake kube-apiserver); HBM slices on real MI355X" if use_gpu
                    else "synthetic pods; fake devices (no GPU)",
            "config": {"model": f"gpushare extender+device plugin: {a.pods_per_gpu} pods/GPU x {a.pod_gib} GiB "
                                f"({profile.resource}), binpack", "global_batch": n_pods, "seq_len": 0,
                       "parallelism": f"{world} GPU(s) advertised on 1 node; 1 rank (HBM runtime) per GPU; "
                                      f"agent={a.agent}" + ("; all ranks share physical GPU 0" if a.share_gpu else ""),
                       "collectives": "gloo (control only)" if world > 1 else "none",
                       "bind_mode": a.bind_mode, "bind_order": a.bind_order, "admission": a.admission,
                       "node_agent": a.node_agent, "device_backend": backend},
            "p50_bind_latency_ms": round(1e3 * pct(lat, 50), 3),
            "p99_bind_latency_ms": round(1e3 * pct(lat, 99), 3),
            "p50_bind_rtt_ms": round(1e3 * pct(rtt, 50), 3),
            "p50_filter_rtt_ms": round(1e3 * pct(frtt, 50), 3),
            "binpack_util_pct": round(100 * util, 2),
            "per_device_used_gib": step_stats[-1]["per_dev"] if step_stats else [],
            "device_gpu_mem_gib": totals,
            "hbm_resident_pct": round(100 * hbm_resident / hbm_total, 2) if hbm_total else None,
            "wave_ms": {"bound": round(1e3 * statistics.mean(s["t_bound"] for s in step_stats), 3),
                        "running": round(1e3 * statistics.mean(s["t_run"] for s in step_stats), 3),
                        "total": round(1e3 * statistics.mean(s["t_total"] for s in step_stats), 3)},
            "wave_ms_p50": {k: round(1e3 * pct([s[t] for s in step_stats], 50), 3)
                            for k, t in (("bound", "t_bound"), ("running", "t_run"), ("total", "t_total"))},
            # after Running: the /inspect read (binpack check), the DeleteCollection call, the wave driver's informer
            # seeing every pod gone, the extender's ledger reading empty
            # the load generator's creates of one wave (every POST answered)
            "create_ms_mean": round(1e3 * statistics.mean(s["t_created"] for s in step_stats), 3),
            "teardown_ms_mean": {k: round(1e3 * statistics.mean(s["teardown"][i] for s in step_stats), 3)
                                 for i, k in enumerate(("inspect", "delete_call", "stopped_seen", "ledger_empty"))},
            "wave_ms_max": {k: round(1e3 * max(s[t] for s in step_stats), 3)
                            for k, t in (("bound", "t_bound"), ("running", "t_run"), ("total", "t_total"))},
            # every timed wave: [bound, running, total] ms (where a slow wave lost its time)
            "wave_ms_each": [[round(1e3 * s["t_bound"], 3), round(1e3 * s["t_run"], 3), round(1e3 * s["t_total"], 3)]
                             for s in step_stats] if len(step_stats) <= 400 else None,
            # per-wave throughput distribution: p50 and IQR next to `value` (one number from ~20 short waves is
            # sensitive to single slow waves)
            "wave_pods_per_s": wave_dist([n_pods / s["t_total"] for s in step_stats]),
            # where the timed region lost time to the host: each process's threads' scheduler run-delay (waiting
            # runnable for a CPU) over the region, in % of its wall time, and the host's pressure-stall deltas (ms).
            # Read at the bracket, outside the waves.  Per wave (--wave-sampler 1): wave_attribution
            "run_delay_pct": {k: round(100.0 * (rd1[k] - rd0.get(k, 0.0)) / max(elapsed, 1e-9), 1) for k in rd1},
            "psi_timed_ms": {k: round((psi1[k] - psi0.get(k, 0)) / 1e3, 3) for k in psi1},
            # why a wave was slow (opt-in, --wave-sampler 1: the sampler's /proc reads slow the pipeline down, up to
            # 45 % at N = 8, profiles/r05_session5/): per-wave run-delay of every process and the host's pressure
            # counters, and for each wave over 5 x the p50 the process (or the host) that waited longest for a CPU
            "wave_attribution": wave_attr,
            # rank 0's view of the timed region: the waves back to back, then the closing barriers
            "timed_region_ms": {"waves": round(1e3 * sum(s["t_total"] for s in step_stats), 3),
                                "rank0_waves_span": round(1e3 * (t_waves_end - t_start), 3),
                                "closing_bracket": round(1e3 * (t_start + own_elapsed - t_waves_end), 3),
                                "max_over_ranks": round(1e3 * elapsed, 3)},
            "cpu_pinning": {k: v for k, v in cpu_plan.items()} or "none",
            "api_latency_ms": a.api_latency_ms,
            "latency_sweep": sweep,
            # the headline path (node agent + plugin as above, bind mode binding, default bind order) per apiserver
            # latency: kubelet admits serially, so each ms of apiserver latency the Allocate waits costs throughput
            "latency_sweep_pods_per_s": {str(r["api_latency_ms"]): r["pods_per_s"] for r in (sweep or [])
                                         if r.get("bind_mode") == "binding" and r.get("bind_order") == a.bind_order},
            "reference_client": ref_client,
            # open-loop arrivals with many pods in flight (untimed by the headline): the knee per apiserver latency,
            # and the stage that bounds it (open_loop)
            "open_loop": ol,
            "open_loop_knee_pods_per_s": (ol or {}).get("knee_pods_per_s"),
            # the shipped gRPC device plugin on the kubelet path (untimed by the headline, same waves)
            # extra rows (untimed by the headline, same waves): the Python kubelet stand-in driving the shipped plugin
            # process, and the compiled stand-in with the plugin's matcher linked in-process (no gRPC hop)
            "device_plugin_path_python_kubelet": plugin_row,
            "inprocess_matcher_path": plugin_row_native,
            "bind_retries": sum(sum(s["attempts"]) - len(s["attempts"]) for s in step_stats),
            "agents": agent_stats,
            "node_agent": node_agent_stats,
            # the shipped plugin process behind the headline (native-plugin): fast-path share, early-answer commits,
            # PodResources reconciliation (swaps) and moves through the extender
            "plugin": plugin_stats,
            # the extender's native front end over the timed waves (bind-order waits, apiserver round trips)
            "extender": extender_stats,
            "apiserver": apiserver_stats,
            "cpu_s": {k: round(cpu1[k] - cpu0.get(k, 0.0), 4) for k in cpu1},
            # on-CPU time of each process over the timed region's wall time (all its threads; 100 = one CPU busy):
            # which process the wave pipeline waits on
            "busy_pct": {k: round(100.0 * (cpu1[k] - cpu0.get(k, 0.0)) / max(elapsed, 1e-9), 1) for k in cpu1},
            # the same per thread name inside the node agent and the plugin (threads under 1 % left out)
            "busy_threads_pct": {p: {t: v for t, v in ((t, round(100.0 * (s1 - thr0.get(p, {}).get(t, 0.0))
                                                                  / max(elapsed, 1e-9), 1)) for t, s1 in th.items())
                                     if v >= 1.0} for p, th in thr1.items()},
            # resident memory of each process at the start and the end of the timed region
            "rss_mib": {k: [rss0.get(k), rss1[k]] for k in rss1},
            # CPU-quota throttling of the container during the timed region (cgroup v2), if any
            "cgroup_timed": {"usage_ms": round((cg1.get("usage_usec", 0) - cg0.get("usage_usec", 0)) / 1e3, 1),
                             "nr_throttled": cg1.get("nr_throttled", 0) - cg0.get("nr_throttled", 0),
                             "throttled_ms": round((cg1.get("throttled_usec", 0) - cg0.get("throttled_usec", 0)) / 1e3,
                                                   1)} if cg1 else None,
        }
        line = json.dumps(out)
        print(line, flush=True)
        if a.json_out:
            with open(a.json_out, "w") as f:
                f.write(line + "\n")

    # ---- teardown
    try:
        if agent is not None:
            lt.run(agent.stop(), 30)
        lt.run(agent_client.close(), 30)
        if isinstance(shim, NativeRuntime):
            shim.stop()
        else:
            lt.run(shim.stop(), 30)
        if rank == 0:
            tracker.stop()
            if sched_http is not None:
                lt.run(sched_http.close(), 30)
            lt.run(client.close(), 30)
    finally:
        runtime.close()
        lt.stop()
        for c in children:
            c.stop()
        if world > 1:
            dist.barrier(group=ctl)
            dist.destroy_process_group()


if __name__ == "__main__":
    main()
