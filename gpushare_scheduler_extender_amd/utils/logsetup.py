"""Logging setup shared by the extender, device plugin and node agent.

The reference logged through beego's multi-file adapter: one file per level
under ``/var/log/device-plugin`` plus the console at level 6
(``cmd/main.go:32-54``), and never read the ``LOG_LEVEL`` its own Deployment
sets.  Here ``LOG_LEVEL`` (or ``--log-level``) drives the console, and an
optional ``--log-dir`` adds rotating per-level files (``<name>.error.log``,
``<name>.warning.log``, ``<name>.info.log``, ``<name>.debug.log``), each holding
records of that level and above.
"""
from __future__ import annotations

import logging
import logging.handlers
import os

FORMAT = "%(asctime)s %(levelname)s %(name)s: %(message)s"


def setup_logging(level: str = "info", log_dir: str | None = None, name: str = "gpushare",
                  max_bytes: int = 64 << 20, backups: int = 3) -> logging.Logger:
    root = logging.getLogger()
    lvl = getattr(logging, str(level).upper(), logging.INFO)
    root.setLevel(logging.DEBUG if log_dir else lvl)
    for h in list(root.handlers):
        root.removeHandler(h)
    console = logging.StreamHandler()
    console.setLevel(lvl)
    console.setFormatter(logging.Formatter(FORMAT))
    root.addHandler(console)
    if log_dir:
        os.makedirs(log_dir, mode=0o711, exist_ok=True)
        for lname in ("error", "warning", "info", "debug"):
            fh = logging.handlers.RotatingFileHandler(os.path.join(log_dir, f"{name}.{lname}.log"),
                                                      maxBytes=max_bytes, backupCount=backups)
            fh.setLevel(getattr(logging, lname.upper()))
            fh.setFormatter(logging.Formatter(FORMAT))
            root.addHandler(fh)
    return logging.getLogger(name)
