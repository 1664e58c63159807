"""``python -m gpushare_scheduler_extender_amd.deviceplugin`` — the node DaemonSet process.

Deployed on nodes labelled ``gpushare=true`` (``docs/install.md:69-79``; see
``deploy/device-plugin-ds.yaml``).  ``NODE_NAME`` comes from the downward API.
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
from . import api
from .devices import discover
from .plugin import GpuSharePlugin


def _pin_from_env() -> None:
    """``GSX_PLUGIN_CPUS=a,b``: run on these CPUs (the benchmark gives the plugin process its own, as a DaemonSet pod
    has, instead of the CPUs of the kubelet stand-in that started it)."""
    cpus = os.environ.get("GSX_PLUGIN_CPUS", "")
    if cpus:
        try:
            os.sched_setaffinity(0, {int(c) for c in cpus.split(",") if c.strip()})
        except (OSError, ValueError):
            pass


def main(argv=None) -> int:
    _pin_from_env()
    env = os.environ
    ap = argparse.ArgumentParser(prog="gpushare-device-plugin-amd")
    ap.add_argument("--node", default=env.get("NODE_NAME", ""))
    ap.add_argument("--kubeconfig", default=env.get("KUBECONFIG"))
    ap.add_argument("--apiserver", default=env.get("GSX_APISERVER"))
    ap.add_argument("--profile", default=env.get("GSX_PROFILE", "shared-gpu"))
    ap.add_argument("--unit", default=env.get("GSX_MEMORY_UNIT", "GiB"), choices=["GiB", "MiB", "GB"])
    ap.add_argument("--backend", default=env.get("GSX_DEVICE_BACKEND", "auto"), choices=["auto", "amdsmi", "hip", "fake"])
    ap.add_argument("--socket-dir", default=env.get("GSX_SOCKET_DIR", api.DEVICE_PLUGIN_PATH))
    ap.add_argument("--mount-mode", default=env.get("GSX_MOUNT_MODE", "isolated"), choices=["isolated", "all"])
    ap.add_argument("--reserve-gib", type=float, default=float(env.get("GSX_RESERVE_GIB", "0")),
                    help="HBM per GPU withheld from sharing (driver / runtime overhead)")
    ap.add_argument("--health-interval", type=float, default=float(env.get("GSX_HEALTH_INTERVAL", "10")))
    ap.add_argument("--debug-port", type=int, default=int(env.get("GSX_DEBUG_PORT", "0")),
                    help="serve /healthz, /metrics and /debug/state on this port (0: off)")
    ap.add_argument("--debug-host", default=env.get("GSX_DEBUG_HOST", "127.0.0.1"))
    ap.add_argument("--debug-port-file", default="", help="write the debug port here once it listens (port 0)")
    ap.add_argument("--no-register", action="store_true",
                    help="do not register with kubelet (a stand-in that connects to the endpoint directly)")
    ap.add_argument("--no-publish", action="store_true",
                    help="do not publish the node's capacity / device inventory (a harness already did)")
    ap.add_argument("--isolation", default=env.get("GSX_ISOLATION", "enforce"), choices=["enforce", "advisory"],
                    help="enforce: Allocate mounts the pod's CU partition / HBM share config and libgsx_isolate.so "
                         "(via /etc/ld.so.preload); advisory: env hints only (HSA_CU_MASK, GSX_GPU_MEM_FRACTION)")
    ap.add_argument("--isolation-dir", default=env.get("GSX_ISOLATION_DIR", "/var/lib/gsx/isolation"))
    ap.add_argument("--podresources-socket", default=env.get("GSX_PODRESOURCES_SOCKET",
                                                              "/var/lib/kubelet/pod-resources/kubelet.sock"),
                    help="kubelet's PodResources API; '' disables the reconciliation of Allocates")
    ap.add_argument("--extender", default=env.get("GSX_EXTENDER_URL", ""),
                    help="the scheduler extender's URL (its POST /gpushare-scheduler/move): reconciliation moves of "
                         "allocation records go through it, the one writer of *_IDX; '' leaves records as they are")
    ap.add_argument("--no-extender", action="store_true", default=env.get("GSX_NO_EXTENDER") == "1",
                    help="run the PodResources reconciliation without a scheduler extender: swaps are detected and "
                         "the physical guard holds, but no allocation record can be repaired (tests / diagnosis)")
    ap.add_argument("--reconcile-interval", type=float, default=float(env.get("GSX_RECONCILE_INTERVAL", "2")))
    ap.add_argument("--log-level", default=env.get("LOG_LEVEL", "info"))
    ap.add_argument("--log-dir", default=env.get("GSX_LOG_DIR", ""))
    a = ap.parse_args(argv)
    setup_logging(a.log_level, a.log_dir or None, "gpushare-device-plugin")
    if not a.node:
        ap.error("--node / NODE_NAME is required")
    if a.podresources_socket and not a.extender and not a.no_extender:
        # every repair of an allocation record goes through the extender (the one writer of *_IDX): without it the
        # reconciliation could only watch swaps it cannot fix, and the physical guard would fail the pods they hit
        ap.error("the PodResources reconciliation (--podresources-socket) needs the scheduler extender's URL "
                 "(--extender / GSX_EXTENDER_URL, e.g. http://gpushare-schd-extender.kube-system.svc:12345); "
                 "pass --podresources-socket '' to run without reconciliation, or --no-extender to run it unrepaired")

    async def run():
        backend, devs = discover(a.backend)
        logging.getLogger("gsx.main").info("%d GPU(s) via %s: %s", len(devs), backend,
                                           ", ".join(f"{d.index}:{d.bdf}:{d.total_bytes >> 30}GiB" for d in devs))
        client = KubeClient(KubeConfig.auto(a.kubeconfig, a.apiserver))
        from .isolation import IsolationManager  # noqa: PLC0415

        iso = IsolationManager(a.isolation_dir) if a.isolation == "enforce" else None
        plugin = GpuSharePlugin(client, a.node, devs, get_profile(a.profile), unit=a.unit, socket_dir=a.socket_dir,
                                mount_mode=a.mount_mode, health_backend="amdsmi" if backend == "amdsmi" else None,
                                health_interval=a.health_interval, reserve_bytes=int(a.reserve_gib * (1 << 30)),
                                podresources_socket=a.podresources_socket or None,
                                reconcile_interval=a.reconcile_interval, isolation=iso, extender=a.extender or None)
        # the debug endpoint first: its setup (importing aiohttp) blocks the loop for a few hundred ms, and once the
        # plugin serves, kubelet's Allocates must find the reconciliation (this loop) running
        if a.debug_port or a.debug_port_file:
            port = await plugin.serve_debug(a.debug_host, a.debug_port)
            if a.debug_port_file:
                with open(a.debug_port_file + ".tmp", "w") as f:
                    f.write(str(port))
                os.replace(a.debug_port_file + ".tmp", a.debug_port_file)
            logging.getLogger("gsx.main").info("debug endpoints on %s:%d", a.debug_host, port)
        await plugin.start(publish=not a.no_publish, register=not a.no_register)
        stop = asyncio.Event()
        loop = asyncio.get_running_loop()
        for s in (signal.SIGINT, signal.SIGTERM):
            loop.add_signal_handler(s, stop.set)
        await stop.wait()
        n = max(1, plugin.timing["n"])
        logging.getLogger("gsx.main").warning(
            "stopping: %s; grpc %s; per Allocate ms: %s", plugin.stats, plugin.debug_state().get("grpc"),
            {k: round(1e3 * v / n, 4) for k, v in plugin.timing.items() if isinstance(v, float)})
        stats_dir = os.environ.get("GSX_PLUGIN_STATS_DIR") or os.environ.get("GSX_PLUGIN_CPROFILE_DIR")
        if stats_dir:  # diagnosis: the plugin's counters and timings at exit
            import json  # noqa: PLC0415

            with open(os.path.join(stats_dir, f"plugin-{os.getpid()}.json"), "w") as f:
                import resource  # noqa: PLC0415

                json.dump({"stats": plugin.stats, "debug": plugin.debug_state(), "timing": plugin.timing,
                           "max_rss_mib": round(resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 1024, 1)}, f,
                          default=str)
        await plugin.stop()
        await client.close()

    prof_dir = os.environ.get("GSX_PLUGIN_CPROFILE_DIR")  # diagnosis: where the plugin process spends its time
    if prof_dir:
        import cProfile  # noqa: PLC0415

        prof = cProfile.Profile()
        prof.runcall(asyncio.run, run())
        prof.dump_stats(os.path.join(prof_dir, f"plugin-{os.getpid()}.prof"))
        return 0
    asyncio.run(run())
    return 0


if __name__ == "__main__":
    sys.exit(main())
