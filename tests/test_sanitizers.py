"""Native code under AddressSanitizer+UBSan and ThreadSanitizer (host code only).

* ``engine_test``: JSON / quantity / ledger / HTTP units and a filter+bind storm on the epoll front end;
* ``controller_test``: the concurrent extender stack against a real gsx-fakeapi -- Controller with its pod
  and node reflectors, resync thread, forced re-lists and reservation GC, the NativeServer's loops and bind
  pool under filter/bind storms with pod churn and injected watch drops, PodTracker and PodRuntime threads;
* the compiled stand-ins (gsx-fakeapi, gsx-schedsim, gsx-nodeagent) built with TSan and driven through
  BASELINE configurations and a chaos run; any report fails the test.
"""
import glob
import os
import subprocess
import sys

import pytest

from gpushare_scheduler_extender_amd.utils.build import REPO, build_native

ENV = {"TSAN_OPTIONS": "halt_on_error=1 second_deadlock_stack=1", "ASAN_OPTIONS": "detect_leaks=1",
       "UBSAN_OPTIONS": "halt_on_error=1 print_stacktrace=1", "PATH": "/usr/bin:/bin"}


def _clean(r, name):
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "all checks passed" in r.stdout
    assert "WARNING: ThreadSanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr[-4000:]
    assert "ERROR: AddressSanitizer" not in r.stderr and "ERROR: LeakSanitizer" not in r.stderr, name


@pytest.mark.slow
@pytest.mark.parametrize("target", ["asan", "tsan"])
def test_engine_under_sanitizer(target):
    build_native([target])
    r = subprocess.run([str(REPO / "build" / f"engine_test_{target}")], capture_output=True, text=True, timeout=240,
                       env=ENV)
    _clean(r, "engine_test")


@pytest.mark.slow
@pytest.mark.parametrize("target", ["asan", "tsan"])
def test_controller_stack_under_sanitizer(target):
    from gsxtools.cluster import start_apiserver

    build_native([target, "fakeapi"])
    api = start_apiserver()
    try:
        r = subprocess.run([str(REPO / "build" / f"controller_test_{target}"), "--apiserver", api.url,
                            "--seconds", "3"], capture_output=True, text=True, timeout=240, env=ENV)
    finally:
        api.stop()
    _clean(r, "controller_test")


@pytest.mark.slow
def test_standins_under_tsan(tmp_path):
    """gsx-fakeapi / gsx-schedsim / gsx-nodeagent under TSan: BASELINE configs 2, 3, 5 and a chaos seed."""
    build_native(["tools_tsan"])
    logs = tmp_path / "tsan"
    env = dict(os.environ, GSX_NATIVE_TOOLS_SUFFIX="_tsan", PYTHONPATH=str(REPO),
               TSAN_OPTIONS=f"halt_on_error=0 second_deadlock_stack=1 log_path={logs}")
    r = subprocess.run([sys.executable, "-m", "gsxtools.configs", "--agent", "native",
                        "--only", "2,3,5"], capture_output=True, text=True, timeout=600, env=env, cwd=REPO)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    # the compiled stand-in with its in-process matcher, and calling the shipped plugin process (PodResources server
    # thread, serial admission slot)
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-p", "no:cacheprovider",
                        "tests/test_chaos.py::test_chaos_whole_stack_converges_without_overcommit[23-native-binding-True]",
                        "tests/test_chaos.py::test_chaos_whole_stack_converges_without_overcommit"
                        "[17-native-plugin-binding-True]"],
                       capture_output=True, text=True, timeout=600, env=env, cwd=REPO)
    assert r.returncode == 0, r.stdout[-3000:]
    reports = sorted(glob.glob(str(logs) + "*"))
    assert not reports, open(reports[0]).read()[-4000:]
