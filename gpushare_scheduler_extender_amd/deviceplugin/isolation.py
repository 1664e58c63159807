"""Enforced per-pod isolation: what the device plugin mounts so that a pod cannot leave its CU partition or HBM share.

The reference leaves isolation to the application (``docs/designs/designs.md:25-28``; the sample caps itself
with a TF memory fraction, ``samples/docker/main.py:37``) and lists "integrate Nvidia MPS" as a roadmap item
(``README.md:77``).  Advice in the container env (``HSA_CU_MASK``, ``GSX_GPU_MEM_FRACTION``) is dropped by
any process that clears its environment, so the plugin also hands every container, through the Allocate
response's ``mounts`` (kubelet passes them to the container runtime):

========================================  ========  ==========================================================
container path                            mode      content
========================================  ========  ==========================================================
``/run/gsx/isolation.conf``               ro        the pod's ``cu_mask`` words and ``hbm_limit_bytes``
``/run/gsx/hbm.ledger``                   rw        the pod's shared HBM account (one slot per live process)
``/run/gsx/libgsx_isolate.so``            ro        ``native/isolate/gsx_isolate.cc``
``/etc/ld.so.preload``                    ro        ``/run/gsx/libgsx_isolate.so``
========================================  ========  ==========================================================

The preload entry loads the library into every dynamically linked process of the container; its constructor
adds itself to ``HSA_TOOLS_LIB`` before the process's first HIP call, and ROCr then hands it the HSA API table:
every queue gets the pod's CU mask, every device allocation is charged to the pod's share (see the library's
header for the exact hooks).  Files live under a host directory per pod UID, written before Allocate returns
and removed when the plugin's informer sees the pod complete or go away.

A host-process launcher (``mount_mode="all"``, :class:`~.runtime.ProcessRuntime`) has no mount namespace: it
gets ``HSA_TOOLS_LIB`` / ``GSX_ISOLATION_CONFIG`` naming the host files instead.
"""
from __future__ import annotations

import logging
import os
import shutil
from pathlib import Path

from ..core.engine import native

log = logging.getLogger("gsx.deviceplugin.isolation")

CONTAINER_DIR = "/run/gsx"
CONF = "isolation.conf"
LEDGER = "hbm.ledger"
LIB = "libgsx_isolate.so"
PRELOAD = "ld.so.preload"
DEFAULT_HOST_DIR = "/var/lib/gsx/isolation"


def shipped_library() -> Path:
    return Path(__file__).resolve().parents[1] / "_native" / LIB


def config_text(cus: list[int] | None, cu_count: int, limit_bytes: int) -> str:
    """The library's config file (one implementation: ``native/engine/dpcore.cc``, shared with the native
    Allocate path)."""
    return native().isolation_config_text(list(cus or []), cu_count, int(limit_bytes))


class IsolationManager:
    """Host side of enforced isolation: per-pod config + ledger files, the mounts and env for Allocate."""

    def __init__(self, host_dir: str = DEFAULT_HOST_DIR, library: str | None = None):
        self.host_dir = Path(host_dir)
        self.library = Path(library) if library else shipped_library()
        self.prepared: set[str] = set()
        self.stats = {"prepared": 0, "released": 0}
        self._installed = False

    def install(self):
        """The library and the preload list, once per host directory (kubelet's runtime mounts them from here)."""
        if self._installed:
            return
        self.host_dir.mkdir(parents=True, exist_ok=True)
        if not self.library.exists():
            raise FileNotFoundError(f"{self.library} not built (python native/build.py isolate)")
        dst = self.host_dir / LIB
        tmp = self.host_dir / (LIB + ".tmp")
        shutil.copyfile(self.library, tmp)
        os.chmod(tmp, 0o755)
        os.replace(tmp, dst)
        _write_atomic(self.host_dir / PRELOAD, f"{CONTAINER_DIR}/{LIB}\n", 0o644)
        self._installed = True

    def pod_dir(self, uid: str) -> Path:
        return self.host_dir / "pods" / uid

    def prepare(self, uid: str, cus: list[int] | None, cu_count: int, limit_bytes: int,
                host_process: bool = False) -> tuple[list[dict], dict[str, str]]:
        """Write the pod's files (idempotent: every container of a pod shares them) and return
        (Allocate ``mounts``, Allocate ``envs``)."""
        self.install()
        try:  # one implementation (native/engine/dpcore.cc isolation_prepare), shared with the native Allocate path
            mounts, envs = native().isolation_prepare(str(self.host_dir), uid, list(cus or []), cu_count,
                                                      int(limit_bytes), host_process)
        except RuntimeError as e:
            raise OSError(str(e)) from e
        self.note_prepared(uid)
        return list(mounts), dict(envs)

    def note_prepared(self, uid: str) -> None:
        if uid not in self.prepared:
            self.prepared.add(uid)
            self.stats["prepared"] += 1

    def release(self, uid: str) -> None:
        if not uid:
            return
        d = self.pod_dir(uid)
        if uid in self.prepared or d.exists():
            shutil.rmtree(d, ignore_errors=True)
            self.prepared.discard(uid)
            self.stats["released"] += 1

    def gc(self, live: set[str]) -> int:
        """Remove the files of pods that are gone (after a plugin restart, from the informer's first sync)."""
        root = self.host_dir / "pods"
        n = 0
        if root.is_dir():
            for d in root.iterdir():
                if d.name not in live:
                    shutil.rmtree(d, ignore_errors=True)
                    self.prepared.discard(d.name)
                    n += 1
        return n


def _write_atomic(path: Path, text: str, mode: int) -> None:
    tmp = path.with_name(path.name + ".tmp")
    try:
        os.chmod(tmp, 0o644)
    except FileNotFoundError:
        pass
    with open(tmp, "w") as f:
        f.write(text)
    os.chmod(tmp, mode)
    os.replace(tmp, path)
