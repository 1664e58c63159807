"""kube-scheduler simulator as its own process (kube-scheduler is one in a real cluster).

    python -m gpushare_scheduler_extender_amd.sim --apiserver URL --extender URL [--port-file F]

Runs :class:`SchedulerSim` and serves its per-pod timings for the benchmark:

* ``POST /v1/timings``  body ``["ns/name", ...]`` -> ``{"ns/name": {seen, filtered, bound,
  filter_rtt, bind_rtt, attempts, node, error}, ...}`` (``bound`` = 0 while unbound);
* ``POST /v1/forget``   body ``["ns/name", ...]`` -> drops those timings;
* ``GET  /v1/stats``    scheduled / bound / bind_errors / unschedulable / filter_calls.

Timestamps are ``time.perf_counter()`` of this process; only differences are meaningful.
"""
from __future__ import annotations

import argparse
import asyncio
import json
import logging
import os
import signal

from ..k8s.client import KubeClient
from ..k8s.fasthttp import Response, Server
from ..models.profile import get_profile
from .scheduler import SchedulerSim


def _timing(t) -> dict:
    return {"seen": t.seen, "filtered": t.filtered, "bound": t.bound, "filter_rtt": t.filter_rtt,
            "bind_rtt": t.bind_rtt, "attempts": t.attempts, "node": t.node, "error": t.error}


def serve_stats(sim: SchedulerSim) -> Server:
    srv = Server()

    def h_timings(request):
        keys = request.json() or []
        tm = sim.stats.timings
        return Response.json({k: _timing(tm[k]) for k in keys if k in tm})

    def h_forget(request):
        sim.forget(request.json() or [])
        return Response.json({"ok": True})

    def h_stats(_request):
        s = sim.stats
        return Response.json({"scheduled": s.scheduled, "bound": s.bound, "bind_errors": s.bind_errors,
                              "unschedulable": s.unschedulable, "filter_calls": s.filter_calls,
                              "pending": sim.queue.qsize()})

    srv.route("POST", "/v1/timings", h_timings)
    srv.route("POST", "/v1/forget", h_forget)
    srv.route("GET", "/v1/stats", h_stats)
    return srv


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description="kube-scheduler simulator (extender protocol)")
    ap.add_argument("--apiserver", required=True)
    ap.add_argument("--extender", required=True, help="extender base URL (urlPrefix without /gpushare-scheduler)")
    ap.add_argument("--profile", default="shared-gpu")
    ap.add_argument("--max-inflight-binds", type=int, default=256)
    ap.add_argument("--node-policy", default="binpack", choices=["binpack", "spread", "first"])
    ap.add_argument("--prioritize", action="store_true", help="call the extender's prioritize verb")
    ap.add_argument("--host", default="127.0.0.1")
    ap.add_argument("--port", type=int, default=0)
    ap.add_argument("--port-file", default="")
    a = ap.parse_args(argv)
    logging.basicConfig(level=logging.WARNING)

    async def run():
        sim = SchedulerSim(KubeClient(a.apiserver), a.extender, get_profile(a.profile),
                           max_inflight_binds=a.max_inflight_binds, node_policy=a.node_policy,
                           use_prioritize=a.prioritize)
        await sim.start()
        srv = serve_stats(sim)
        port = await srv.start(a.host, a.port)
        if a.port_file:
            with open(a.port_file + ".tmp", "w") as f:
                f.write(str(port))
            os.replace(a.port_file + ".tmp", a.port_file)
        from ..utils.gctune import tune  # noqa: PLC0415

        tune()
        stop = asyncio.Event()
        loop = asyncio.get_running_loop()
        for s in (signal.SIGINT, signal.SIGTERM):
            loop.add_signal_handler(s, stop.set)
        await stop.wait()
        await srv.stop()
        await sim.stop()
        await sim.client.close()

    asyncio.run(run())
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
