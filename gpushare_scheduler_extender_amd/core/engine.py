"""Loader for the native ledger engine (``_native/_engine*.so``).

There is deliberately no pure-Python fallback: the engine owns every
scheduling decision, and a silently different implementation would make
results depend on the build.  If the extension is missing we fail loudly with
the command that builds it.  (``tests/refmodel.py`` holds an independent
Python model used only to cross-check the engine in property tests.)
"""
from __future__ import annotations

import importlib
import os

from ..models.profile import NamingProfile, SHARED_GPU

_mod = None

CHECK_OK, CHECK_NODE_NOT_FOUND, CHECK_NOT_GPUSHARE, CHECK_INSUFFICIENT = 0, 1, 2, 3
ASSUME_INSUFFICIENT, ASSUME_NO_NODE, ASSUME_NOT_GPUSHARE, ASSUME_IN_FLIGHT = -1, -2, -3, -4


def native():
    """Return the ``_engine`` extension module, building it in-tree if allowed."""
    global _mod
    if _mod is not None:
        return _mod
    try:
        _mod = importlib.import_module("gpushare_scheduler_extender_amd._native._engine")
    except ImportError as e:
        if os.environ.get("GSX_AUTOBUILD", "1") == "1":
            from ..utils.build import build_native  # noqa: PLC0415

            build_native(["engine"])
            _mod = importlib.import_module("gpushare_scheduler_extender_amd._native._engine")
        else:
            raise ImportError(
                "native engine extension missing; run `python native/build.py engine`"
            ) from e
    return _mod


def new_engine(profile: NamingProfile = SHARED_GPU):
    return native().Engine(profile.engine_dict())


def parse_quantity(s: str) -> int:
    return native().parse_quantity(s)
