"""Process-level harness: run the fake apiserver and the extender as child processes.

kube-apiserver and the extender are separate processes in a real cluster
(``config/gpushare-schd-extender.yaml``); the benchmark keeps them separate
too, so the extender's event loop is not shared with the load generator.
Children are started with ``subprocess.Popen`` (fork+exec happens in the
child; callers start them before touching the GPU).
"""
from __future__ import annotations

import atexit
import os
import subprocess
import sys
import tempfile
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def _wait_port(path: str, proc: subprocess.Popen, timeout: float = 60.0) -> int:
    deadline = time.monotonic() + timeout
    while time.monotonic() < deadline:
        if os.path.exists(path):
            with open(path) as f:
                s = f.read().strip()
            if s:
                return int(s)
        if proc.poll() is not None:
            raise RuntimeError(f"child exited with {proc.returncode} before listening")
        time.sleep(0.02)
    raise TimeoutError(f"child did not publish a port in {path}")


_LIVE: set = set()


@atexit.register
def _stop_all():
    """Children never outlive their parent, also when it fails before its own teardown."""
    for c in list(_LIVE):
        try:
            c.stop()
        except Exception:  # noqa: BLE001 - best effort at exit
            pass


class ChildProc:
    def __init__(self, args: list[str], name: str, env: dict | None = None, cpus: list[int] | None = None):
        self.name = name
        self.cpus = list(cpus or [])
        self.tmp = tempfile.mkdtemp(prefix=f"gsx-{name}-")
        self.port_file = os.path.join(self.tmp, "port")
        self.log_path = os.path.join(self.tmp, "log")
        e = dict(os.environ)
        e["PYTHONPATH"] = str(ROOT) + os.pathsep + e.get("PYTHONPATH", "")
        e.setdefault("GSX_AUTOBUILD", "0")
        if env:
            e.update(env)
        self.log = open(self.log_path, "w")
        prof = os.environ.get("GSX_CPROFILE_DIR")
        if prof and args[0] == "-m":  # profile the child (see utils/profrun.py)
            os.makedirs(prof, exist_ok=True)
            args = ["-m", "gpushare_scheduler_extender_amd.utils.profrun", os.path.join(prof, f"{name}.prof"), *args[1:]]
        # "-m module ..." runs under this interpreter; anything else is a native executable
        argv = [sys.executable, *args] if args[0] == "-m" else list(args)
        pin = None
        if self.cpus:
            mask = set(self.cpus)

            def pin():  # in the child between fork and exec: the whole program starts pinned
                os.sched_setaffinity(0, mask)
        self.proc = subprocess.Popen([*argv, "--port-file", self.port_file], stdout=self.log,
                                     stderr=subprocess.STDOUT, env=e, cwd=str(ROOT), preexec_fn=pin)
        _LIVE.add(self)
        self.port = _wait_port(self.port_file, self.proc)
        self.url = f"http://127.0.0.1:{self.port}"

    def tail(self, n: int = 40) -> str:
        try:
            with open(self.log_path) as f:
                return "".join(f.readlines()[-n:])
        except OSError:
            return ""

    def stop(self):
        import shutil  # noqa: PLC0415

        _LIVE.discard(self)
        if self.proc.poll() is None:
            self.proc.terminate()
            try:
                self.proc.wait(5)
            except subprocess.TimeoutExpired:
                self.proc.kill()
                self.proc.wait(5)
        self.log.close()
        keep = os.environ.get("GSX_LOG_DIR")  # a copy of the child's log (stdout + stderr) survives the run
        if keep:
            os.makedirs(keep, exist_ok=True)
            shutil.copyfile(self.log_path, os.path.join(keep, f"{self.name}.{self.proc.pid}.log"))
        if os.environ.get("GSX_KEEP_LOGS") != "1":
            shutil.rmtree(self.tmp, ignore_errors=True)


def tool_path(name: str) -> Path:
    """A compiled stand-in: ``_native/<name>``, or ``build/<name><suffix>`` when ``GSX_NATIVE_TOOLS_SUFFIX`` is set
    (e.g. ``_tsan``: the ThreadSanitizer builds of ``native/build.py tools_tsan``, used by tests/test_sanitizers.py)."""
    suffix = os.environ.get("GSX_NATIVE_TOOLS_SUFFIX", "")
    if suffix:
        return ROOT / "build" / f"{name}{suffix}"
    return ROOT / "gpushare_scheduler_extender_amd" / "_native" / name


FAKEAPI = ROOT / "gpushare_scheduler_extender_amd" / "_native" / "gsx-fakeapi"


def start_apiserver(history: int = 200000, threads: int | None = None, cpus: list[int] | None = None,
                    watch_loop: bool | None = None) -> ChildProc:
    """Fake kube-apiserver: the compiled ``gsx-fakeapi`` (native/fakeapi).  (``tests/fixtures/fakeapi.py`` is its
    in-process test-only twin.)

    ``threads``: event loops of the native server (default ``GSX_FAKEAPI_THREADS`` or 1).
    ``GSX_FAKEAPI_WATCH_FLUSH``: ``iteration`` (default) or ``request`` -- when watch events are pushed.
    ``GSX_FAKEAPI_WATCH_LOOP=1``: with 2+ threads, loop 0 serves only the watch streams (``--watch-loop``).
    """
    exe = tool_path("gsx-fakeapi")
    if not exe.exists():
        raise FileNotFoundError(f"{exe} missing; run `python native/build.py fakeapi`")
    threads = threads or int(os.environ.get("GSX_FAKEAPI_THREADS", "1"))
    flush = os.environ.get("GSX_FAKEAPI_WATCH_FLUSH", "iteration")
    if watch_loop is None:
        watch_loop = os.environ.get("GSX_FAKEAPI_WATCH_LOOP", "0") == "1"
    extra = ["--watch-loop"] if watch_loop else []
    return ChildProc([str(exe), "--port", "0", "--history", str(history), "--threads", str(threads),
                      "--watch-flush", flush, *extra], "apiserver", cpus=cpus)


def start_extender(apiserver: str, profile: str = "shared-gpu", bind_mode: str = "binding", threadness: int = 1,
                   log_level: str = "warning", port: int = 0, cpus: list[int] | None = None,
                   kube_qps: float = 0.0, kube_burst: int = 1000, bind_order: str = "auto") -> ChildProc:
    return ChildProc(["-m", "gpushare_scheduler_extender_amd.extender", "--host", "127.0.0.1", "--port", str(port),
                      "--apiserver", apiserver, "--profile", profile, "--bind-mode", bind_mode,
                      "--bind-order", bind_order,
                      "--threadness", str(threadness), "--log-level", log_level, "--kube-qps", str(kube_qps),
                      "--kube-burst", str(kube_burst)], "extender", cpus=cpus)


NODEAGENT = ROOT / "gpushare_scheduler_extender_amd" / "_native" / "gsx-nodeagent"


def start_node_agent(apiserver: str, node: str, profile: str = "shared-gpu", workers: int = 32,
                     native: bool = True, plugin: str = "grpc", cpus: list[int] | None = None,
                     extra: list[str] | None = None, plugin_cpus: list[int] | None = None,
                     serial_admission: bool = False, extender: str | None = None) -> ChildProc:
    """kubelet + device-plugin Allocate + runtime stand-in for ``node``.

    ``native=True``: the compiled ``gsx-nodeagent`` (native/nodeagent, the plugin's native matcher in-process, or
    with ``plugin="spawn"`` the shipped plugin as its child process, called over the device-plugin gRPC API);
    otherwise ``python -m gsxtools.agent``: a kubelet stand-in driving
    the shipped device plugin, over its unix socket (``plugin="grpc"``) or in-process (``"inproc"``).
    ``serial_admission``: the compiled agent admits one pod at a time with its in-process matcher too, as kubelet
    does (with ``plugin="spawn"`` it always does).
    ``plugin_cpus``: CPUs of the plugin process the agent starts (as a DaemonSet pod has its own, instead of
    sharing the kubelet stand-in's), through ``GSX_PLUGIN_CPUS``.
    ``extender``: the scheduler extender's URL, handed to the device plugin (``GSX_EXTENDER_URL``): its
    reconciliation moves allocation records through the extender, the one writer of ``*_IDX``.
    """
    env = {"GSX_PLUGIN_CPUS": ",".join(map(str, plugin_cpus))} if plugin_cpus else {}
    if extender:
        env["GSX_EXTENDER_URL"] = extender
    # both stand-ins list a container in PodResources, and keep its device IDs taken, until it has stopped: the
    # plugin may take their report as the truth about force-deleted pods' containers (deviceplugin/plugin.py
    # FORCE_DELETE; a real kubelet drops them at once, and the default "grace" policy is for that)
    env["GSX_PLUGIN_FORCE_DELETE"] = os.environ.get("GSX_PLUGIN_FORCE_DELETE", "report")
    env = env or None
    if native:
        exe = Path(os.environ.get("GSX_NODEAGENT_BIN") or tool_path("gsx-nodeagent"))  # an A/B build of the stand-in
        if not exe.exists():
            raise FileNotFoundError(f"{exe} missing; run `python native/build.py nodeagent`")
        spawn = ["--plugin-spawn", sys.executable] if plugin == "spawn" else []
        if serial_admission:
            spawn.append("--serial-admission")
        return ChildProc([str(exe), "--node", node, "--apiserver", apiserver, "--profile", profile,
                          "--workers", str(min(workers, 16)), *spawn, *(extra or [])], "node-agent", cpus=cpus,
                         env=env)
    return ChildProc(["-m", "gsxtools.agent", "--node", node, "--apiserver",
                      apiserver, "--profile", profile, "--workers", str(workers), "--plugin", plugin,
                      *(extra or [])], "node-agent", cpus=cpus, env=env)


SCHEDSIM = ROOT / "gpushare_scheduler_extender_amd" / "_native" / "gsx-schedsim"


def start_scheduler(apiserver: str, extender: str, profile: str = "shared-gpu", max_inflight_binds: int = 256,
                    cpus: list[int] | None = None, nodes_to_score: str = "") -> ChildProc:
    """kube-scheduler stand-in: the compiled ``gsx-schedsim`` (native/schedsim, built by ``native/build.py``) with a
    timings endpoint (``/v1/timings``, ``/v1/forget``, ``/v1/stats``).  (``tests/fixtures/schedsim.py`` is its
    in-process test-only twin.)"""
    exe = tool_path("gsx-schedsim")
    if not exe.exists():
        raise FileNotFoundError(f"{exe} missing; run `python native/build.py schedsim`")
    extra = ["--nodes-to-score", nodes_to_score] if nodes_to_score else []
    return ChildProc([str(exe), "--apiserver", apiserver, "--extender", extender, "--profile", profile,
                      "--bind-threads", str(min(16, max_inflight_binds)), *extra], "scheduler", cpus=cpus)
