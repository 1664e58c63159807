"""CPU cost of the shipped device-plugin process on a quiet node.

    python -m gsxtools.plugincpu [--gpus 8] [--idle 60] [--trickle 60] [--rate 1] [--json-out F]

Starts the stack (fake apiserver, extender, scheduler simulator, the compiled kubelet stand-in calling the shipped
plugin process over the device-plugin gRPC API) on one node with ``--gpus`` fake MI355X, then measures the plugin
process's on-CPU time (every thread, /proc/<pid>/task/*/schedstat):

* ``idle``: ``--idle`` seconds with no pod activity;
* ``trickle``: ``--trickle`` seconds in which one 8 GiB pod per ``1 / --rate`` seconds is created, admitted and deleted.

Reports percent of one CPU per phase and per thread name.  The budget the DaemonSet is sized for
(``deploy/device-plugin-ds.yaml``): idle < 1 %, trickle < 5 %.
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import sys
import time

from gpushare_scheduler_extender_amd.models.profile import ALIYUN
from gsxtools.configs import AGENT, Cluster


def _child_pids(pid: int) -> list[int]:
    out = []
    try:
        for t in os.listdir(f"/proc/{pid}/task"):
            with open(f"/proc/{pid}/task/{t}/children") as f:
                out += [int(x) for x in f.read().split()]
    except (OSError, ValueError):
        pass
    return out


def thread_cpu(pid: int) -> dict[str, float]:
    out: dict[str, float] = {}
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


def _pct(t0: dict, t1: dict, secs: float) -> dict:
    per = {k: round(100.0 * (v - t0.get(k, 0.0)) / secs, 3) for k, v in t1.items()}
    return {"total_pct": round(sum(per.values()), 3), "threads_pct": {k: v for k, v in per.items() if v >= 0.01}}


async def run(gpus: int, idle: float, trickle: float, rate: float) -> dict:
    AGENT["kind"] = "native-plugin"
    cl = Cluster(ALIYUN, [287] * gpus, gpu=False, agent="native-plugin")
    try:
        await cl.start()
        agent_pid = cl.agent_child().proc.pid
        plugin_pid = None
        for _ in range(600):
            kids = _child_pids(agent_pid)
            if kids:
                plugin_pid = kids[0]
                break
            await asyncio.sleep(0.05)
        if plugin_pid is None:
            raise RuntimeError("the node agent spawned no plugin process")
        # one pod through first: every lazy path (imports, connections) taken before the measurement
        await cl.create("warm", 8)
        await cl.wait(["warm"])
        await cl.c.delete("pods", "warm", "default")
        await asyncio.sleep(2.0)
        out = {"gpus": gpus, "plugin_pid": plugin_pid}
        t0, w0 = thread_cpu(plugin_pid), time.monotonic()
        await asyncio.sleep(idle)
        t1, w1 = thread_cpu(plugin_pid), time.monotonic()
        out["idle"] = {"seconds": round(w1 - w0, 2), **_pct(t0, t1, w1 - w0)}
        n = 0
        t0, w0 = thread_cpu(plugin_pid), time.monotonic()
        period = 1.0 / rate
        nxt = w0
        while time.monotonic() - w0 < trickle:
            name = f"t{n}"
            await cl.create(name, 8)
            await cl.wait([name])
            await cl.c.delete("pods", name, "default")
            n += 1
            nxt += period
            await asyncio.sleep(max(0.0, nxt - time.monotonic()))
        t1, w1 = thread_cpu(plugin_pid), time.monotonic()
        out["trickle"] = {"seconds": round(w1 - w0, 2), "pods": n, "rate_per_s": round(n / (w1 - w0), 3),
                          **_pct(t0, t1, w1 - w0)}
        return out
    finally:
        await cl.close()


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--gpus", type=int, default=8)
    ap.add_argument("--idle", type=float, default=60.0)
    ap.add_argument("--trickle", type=float, default=60.0)
    ap.add_argument("--rate", type=float, default=1.0)
    ap.add_argument("--json-out", default="")
    a = ap.parse_args(argv)
    res = asyncio.run(run(a.gpus, a.idle, a.trickle, a.rate))
    line = json.dumps(res)
    print(line, flush=True)
    if a.json_out:
        with open(a.json_out, "w") as f:
            f.write(line + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
