"""bench.py contract on CPU: single process and a 2-rank torch.distributed (gloo) run with fake devices."""
import json
import os
import socket
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _json_line(out: str) -> dict:
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out[-3000:]
    return json.loads(lines[0])


KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config"}


def _env():
    e = dict(os.environ)
    e["PYTHONPATH"] = str(ROOT)
    e.setdefault("OMP_NUM_THREADS", "1")
    return e


@pytest.mark.slow
def test_bench_single_process_fake_devices():
    r = subprocess.run([sys.executable, "bench.py", "--steps", "3", "--warmup", "1", "--devices", "fake"],
                       cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _json_line(r.stdout)
    assert KEYS <= set(d)
    assert d["n_gpus"] == 1 and d["steps"] == 3 and d["scaling"] == "weak" and d["higher_is_better"] is True
    assert d["config"]["global_batch"] == 4 and d["value"] > 0
    assert d["per_device_used_gib"] == [256] and d["binpack_util_pct"] > 90
    assert all(a["bad_stamps"] == 0 and a["failed"] == 0 for a in d["agents"])


@pytest.mark.slow
@pytest.mark.parametrize("agent", ["rank", "node"])
def test_bench_two_ranks_gloo(agent):
    port = _free_port()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port), "bench.py", "--gpus", "2", "--steps", "3",
           "--warmup", "1", "--devices", "fake", "--agent", agent]
    r = subprocess.run(cmd, cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    d = _json_line(r.stdout)
    assert d["n_gpus"] == 2 and d["config"]["global_batch"] == 8
    # 4 x 64 GiB on each of the two devices: binpack fills GPU0 before GPU1 ... and both end full
    assert d["per_device_used_gib"] == [256, 256]
    assert sum(a["admitted"] for a in d["agents"]) == 8 * 4  # (warmup + steps) waves x 8 pods
    assert all(a["bad_stamps"] == 0 for a in d["agents"])
