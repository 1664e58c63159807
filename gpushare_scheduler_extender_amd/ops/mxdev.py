"""Python face of the native amdsmi device library (``native/mxdev`` -> ``_native/_mxdev*.so``)."""
from __future__ import annotations

import importlib
import os

_mod = None
_sessions: dict[str, object] = {}


def native():
    global _mod
    if _mod is None:
        try:
            _mod = importlib.import_module("gpushare_scheduler_extender_amd._native._mxdev")
        except ImportError:
            if os.environ.get("GSX_AUTOBUILD", "1") != "1":
                raise
            from ..utils.build import build_native  # noqa: PLC0415

            build_native(["mxdev"])
            _mod = importlib.import_module("gpushare_scheduler_extender_amd._native._mxdev")
    return _mod


def session(backend: str = "amdsmi"):
    s = _sessions.get(backend)
    if s is None:
        s = native().Session(backend)
        _sessions[backend] = s
    return s


def enumerate_devices(backend: str = "amdsmi") -> list[dict]:
    return session(backend).devices()


def health(index: int, backend: str = "amdsmi") -> dict:
    """ECC / RAS (HBM, GFX, SDMA, xGMI) counters, xGMI link status, thermal / power throttle, partition modes."""
    return session(backend).health(index)


def inject(index: int, what: str, backend: str) -> None:
    """Fake backend only: ``ecc_uncorrectable=1``, ``xgmi_error=1``, ``thermal_throttle=1``, ``partition=CPX``,
    ``memory_partition=NPS2``, ``event=GPU_PRE_RESET`` ..."""
    session(backend).inject(index, what)
