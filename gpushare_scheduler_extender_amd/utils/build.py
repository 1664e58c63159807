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
    mod = _build_module()
    for t in targets or mod.DEFAULT:
        mod.TARGETS[t](force=force, verbose=verbose)
