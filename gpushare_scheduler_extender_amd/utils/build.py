"""Programmatic access to ``native/build.py`` (used by __graft_entry__.build and autobuild)."""
from __future__ import annotations

import importlib.util
from pathlib import Path

REPO = Path(__file__).resolve().parents[2]


def _build_module():
    spec = importlib.util.spec_from_file_location("gsx_native_build", REPO / "native" / "build.py")
    mod = importlib.util.module_from_spec(spec)
    assert spec.loader is not None
    spec.loader.exec_module(mod)
    return mod


def build_native(targets=None, force: bool = False, verbose: bool = False) -> None:
    """One build at a time per tree: parallel test workers (pytest -n) each build on start, and one worker's
    half-written object must not be another's input."""
    import fcntl  # noqa: PLC0415

    mod = _build_module()
    lock = REPO / "build" / ".native-build.lock"
    lock.parent.mkdir(parents=True, exist_ok=True)
    with open(lock, "w") as f:
        fcntl.flock(f, fcntl.LOCK_EX)
        for t in targets or mod.DEFAULT:
            mod.TARGETS[t](force=force, verbose=verbose)
