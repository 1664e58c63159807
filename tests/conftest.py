import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))
os.environ.setdefault("GSX_LOG_LEVEL", "warning")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run with -m gpu on the GPU box)")
    config.addinivalue_line("markers", "slow: long-running test")


@pytest.fixture(scope="session", autouse=True)
def _native_built():
    """Build the native extensions in-tree once per session (no-op when up to date)."""
    from gpushare_scheduler_extender_amd.utils.build import build_native

    build_native(["engine", "mxdev"])
    yield
