"""Native engine under AddressSanitizer+UBSan and ThreadSanitizer (host code only)."""
import subprocess

import pytest

from gpushare_scheduler_extender_amd.utils.build import build_native, REPO


@pytest.mark.slow
@pytest.mark.parametrize("target", ["asan", "tsan"])
def test_engine_under_sanitizer(target):
    build_native([target])
    exe = REPO / "build" / f"engine_test_{target}"
    env = {"TSAN_OPTIONS": "halt_on_error=1 second_deadlock_stack=1", "ASAN_OPTIONS": "detect_leaks=1",
           "UBSAN_OPTIONS": "halt_on_error=1 print_stacktrace=1", "PATH": "/usr/bin:/bin"}
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "all checks passed" in r.stdout
    assert "WARNING: ThreadSanitizer" not in r.stderr and "runtime error" not in r.stderr
