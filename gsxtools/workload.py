"""The pod workload: ``samples/workload/main.py``, the file the sample image ships, loaded from there.

The harness (``python -m gsxtools.workload``, the isolation bench, ``ProcessRuntime`` pods) runs the very code the
container runs; ``libgsx_kernels.so`` is found in the repository's build tree (the image builds its own copy).
"""
from __future__ import annotations

import importlib.util
import sys
from pathlib import Path

_MAIN = Path(__file__).resolve().parents[1] / "samples" / "workload" / "main.py"
_spec = importlib.util.spec_from_file_location("gsx_sample_workload", _MAIN)
_mod = importlib.util.module_from_spec(_spec)
sys.modules.setdefault("gsx_sample_workload", _mod)
_spec.loader.exec_module(_mod)

run = _mod.run
main = _mod.main
parse_mask = _mod.parse_mask
kernels_lib_path = _mod.kernels_lib_path

if __name__ == "__main__":
    sys.exit(main())
