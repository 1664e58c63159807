"""Process entry for the scheduler extender (``cmd/main.go`` equivalent).

Environment (same names as the reference, ``cmd/main.go:23,92-98`` and
``config/gpushare-schd-extender.yaml:93-98``):

* ``PORT``        listen port (default 39999)
* ``KUBECONFIG``  kubeconfig path; in-cluster service account otherwise
* ``THREADNESS``  bind threads (a floor under ``--bind-threads``; the reference ignored it)
* ``LOG_LEVEL``   debug|info|warning|error (set by the reference's yaml, never read)

Ours: ``GSX_PROFILE`` (shared-gpu|aliyun), ``GSX_BIND_MODE`` (binding|update),
``GSX_KUBE_QPS`` / ``GSX_KUBE_BURST`` (client-go defaults 5/10 cap the
reference at ~2.5 binds/s), ``GSX_APISERVER`` (explicit apiserver URL).
Every variable has a flag of the same meaning.  SIGINT/SIGTERM shut down
gracefully; a second signal exits at once (``pkg/utils/signals/signal.go``).
"""
from __future__ import annotations

import argparse
import asyncio
import logging
import os
import signal
import sys

from ..k8s.client import KubeClient, KubeConfig
from ..models.profile import get_profile
from ..utils.logsetup import setup_logging
from .server import ExtenderRunner, ExtenderServer


def parse_args(argv=None):
    env = os.environ
    ap = argparse.ArgumentParser(prog="gpushare-schd-extender", description=__doc__,
                                 formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--host", default=env.get("HOST", "0.0.0.0"))
    ap.add_argument("--port", type=int, default=int(env.get("PORT", "39999")))
    ap.add_argument("--kubeconfig", default=env.get("KUBECONFIG"))
    ap.add_argument("--apiserver", default=env.get("GSX_APISERVER"))
    ap.add_argument("--threadness", type=int, default=int(env.get("THREADNESS", "1") or 1))
    ap.add_argument("--log-level", default=env.get("LOG_LEVEL", "info"))
    ap.add_argument("--log-dir", default=env.get("GSX_LOG_DIR", ""),
                    help="also write per-level rotating log files here (the reference used /var/log/device-plugin)")
    ap.add_argument("--profile", default=env.get("GSX_PROFILE", "shared-gpu"))
    ap.add_argument("--bind-mode", default=env.get("GSX_BIND_MODE", "binding"), choices=["binding", "update"])
    ap.add_argument("--bind-order", default=env.get("GSX_BIND_ORDER", "auto"), choices=["auto", "strict", "relaxed"],
                    help="auto (default): equal-size binds of one node for different GPUs land in ASSUME_TIME order, "
                         "except on nodes whose device plugin advertises landing-order matching "
                         "(gpushare.amd.com/allocate-order=landing); strict: ASSUME_TIME order on every node; "
                         "relaxed: all binds concurrent, swaps repaired by the device plugin's PodResources "
                         "reconciliation")
    ap.add_argument("--kube-qps", type=float, default=float(env.get("GSX_KUBE_QPS", "0")))
    ap.add_argument("--kube-burst", type=int, default=int(env.get("GSX_KUBE_BURST", "1000")))
    ap.add_argument("--resync", type=float, default=float(env.get("GSX_RESYNC", "30")))
    ap.add_argument("--reservation-ttl", type=float, default=float(env.get("GSX_RESERVATION_TTL", "60")))
    ap.add_argument("--http-threads", type=int, default=int(env.get("GSX_HTTP_THREADS", "2")))
    ap.add_argument("--bind-threads", type=int, default=int(env.get("GSX_BIND_THREADS", "16")))
    ap.add_argument("--leader-elect", type=int, default=int(env.get("GSX_LEADER_ELECT", "0")),
                    help="1: run as an HA replica; only the holder of the Lease binds (reference: single replica)")
    ap.add_argument("--lease-name", default=env.get("GSX_LEASE_NAME", "gpushare-schd-extender"))
    ap.add_argument("--lease-namespace", default=env.get("POD_NAMESPACE", "kube-system"))
    ap.add_argument("--pprof", type=int, default=int(env.get("GSX_PPROF", "1")),
                    help="1: serve /debug/pprof/* on the API port, as the reference (default); 0: off (the port is "
                         "hostNetwork / NodePort, and profiles cost CPU)")
    ap.add_argument("--port-file", default="", help="write the bound port to this file once serving")
    ap.add_argument("--plugin-auth", default=env.get("GSX_PLUGIN_AUTH", "none"), choices=["none", "tokenreview"],
                    help="who may call the device plugin's endpoints (POST /gpushare-scheduler/move, /physical): "
                         "anyone who reaches the port (none), or a bearer token the apiserver's TokenReview "
                         "authenticates as one of --plugin-users (tokenreview; the shipped manifests)")
    ap.add_argument("--plugin-users", default=env.get(
        "GSX_PLUGIN_USERS", "system:serviceaccount:kube-system:gpushare-device-plugin"),
                    help="comma-separated usernames allowed with --plugin-auth tokenreview")
    return ap.parse_args(argv)


def main(argv=None) -> int:
    a = parse_args(argv)
    setup_logging(a.log_level, a.log_dir or None, "gpushare-schd-extender")
    log = logging.getLogger("gsx.main")

    async def run():
        cfg = KubeConfig.auto(a.kubeconfig, a.apiserver)
        client = KubeClient(cfg, qps=a.kube_qps, burst=a.kube_burst)
        srv = ExtenderServer(client, get_profile(a.profile), bind_mode=a.bind_mode,
                             reservation_ttl=a.reservation_ttl, resync_period=a.resync,
                             leader_elect=bool(a.leader_elect), lease_name=a.lease_name,
                             lease_namespace=a.lease_namespace, pprof=bool(a.pprof), bind_order=a.bind_order)
        runner = await ExtenderRunner(srv, a.host, a.port, http_threads=a.http_threads,
                                      pool_threads=max(a.bind_threads, a.threadness), plugin_auth=a.plugin_auth,
                                      plugin_users=[u for u in a.plugin_users.split(",") if u]).start()
        if a.port_file:
            with open(a.port_file + ".tmp", "w") as f:
                f.write(str(runner.port))
            os.replace(a.port_file + ".tmp", a.port_file)
        log.info("gpushare extender %s listening on %s:%d (profile=%s bind=%s)", "0.1.0", a.host, runner.port,
                 a.profile, a.bind_mode)
        from ..utils.gctune import tune  # noqa: PLC0415

        tune()
        stop = asyncio.Event()
        loop = asyncio.get_running_loop()
        hits = {"n": 0}

        def on_sig():
            hits["n"] += 1
            if hits["n"] > 1:
                os._exit(1)
            stop.set()
        for s in (signal.SIGINT, signal.SIGTERM):
            loop.add_signal_handler(s, on_sig)
        await stop.wait()
        await runner.stop()
        await client.close()

    asyncio.run(run())
    return 0


if __name__ == "__main__":
    sys.exit(main())
