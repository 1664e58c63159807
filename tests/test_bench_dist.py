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
    assert d["dtype"] == "n/a" and d["wave_pods_per_s"]["n"] == 3
    # latency sweep (extra keys): both bind modes at 0/1/2/5 ms; bind latency tracks the injected RTT
    rows = {(r["bind_mode"], r["api_latency_ms"]): r for r in d["latency_sweep"]}
    assert set(rows) == {(m, ms) for m in ("binding", "update") for ms in (0, 1, 2, 5)}
    assert rows[("binding", 5)]["p50_bind_latency_ms"] >= 5.0
    assert rows[("update", 5)]["p50_bind_latency_ms"] >= 10.0  # PUT + POST: two round trips
    # the reference's client (QPS 5 / burst 10, PUT + POST) reproduces the derived 2.5 binds/s on this stack
    ref = {r["bind_mode"]: r for r in d["reference_client"]}
    assert 2.0 <= ref["update"]["pods_per_s"] <= 3.0
    assert ref["binding"]["pods_per_s"] > ref["update"]["pods_per_s"]
    assert d["vs_baseline_same_condition"] == round(ref["binding"]["pods_per_s"] / 2.5, 2)
    assert "bind_order_waits" in rows[("binding", 0)]


@pytest.mark.slow
@pytest.mark.parametrize("agent,extra", [("rank", []), ("node", []), ("node", ["--node-agent", "plugin"])])
def test_bench_two_ranks_gloo(agent, extra):
    port = _free_port()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port), "bench.py", "--gpus", "2", "--steps", "3",
           "--warmup", "1", "--devices", "fake", "--agent", agent, "--sweep", "0", *extra]
    r = subprocess.run(cmd, cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=300)
    # (the ranks' own errors come before torchrun's summary at the end of stderr)
    assert r.returncode == 0, (r.stdout[-2000:], [ln for ln in r.stderr.splitlines() if "rror" in ln][-30:],
                               r.stderr[-3000:])
    d = _json_line(r.stdout)
    assert d["n_gpus"] == 2 and d["config"]["global_batch"] == 8
    # 4 x 64 GiB on each of the two devices: binpack fills GPU0 before GPU1 ... and both end full
    assert d["per_device_used_gib"] == [256, 256]
    assert sum(a["admitted"] for a in d["agents"]) == 8 * 4  # (warmup + steps) waves x 8 pods
    assert all(a["bad_stamps"] == 0 for a in d["agents"])


@pytest.mark.slow
def test_bench_eight_ranks_gloo():
    """The N=8 run of an 8 x MI355X node, rehearsed with 8 gloo ranks on fake devices -- started as
    ``python bench.py --gpus 8`` with no launcher: bench.py starts torch.distributed.run as a child itself."""
    cmd = [sys.executable, "bench.py", "--gpus", "8", "--steps", "2",
           "--warmup", "1", "--devices", "fake", "--agent", "node", "--sweep", "0"]
    r = subprocess.run(cmd, cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    d = _json_line(r.stdout)
    assert d["n_gpus"] == 8 and d["config"]["global_batch"] == 32
    assert d["per_device_used_gib"] == [256] * 8  # 32 x 64 GiB: 4 per device, binpack-first
    assert sum(a["admitted"] for a in d["agents"]) == 3 * 32 or d["node_agent"]["admitted"] == 3 * 32
    assert all(a["bad_stamps"] == 0 for a in d["agents"])


@pytest.mark.gpu
def test_bench_four_ranks_share_one_gpu():
    """The driver's N-GPU launch on a one-GPU box: 4 ranks (torch.distributed.run, gloo only) each carve an HBM
    arena out of GPU 0 and run their own pod runtime endpoint with the stamp / verify kernels."""
    cmd = [sys.executable, "bench.py", "--gpus", "4", "--share-gpu", "--pod-gib", "8", "--steps", "5", "--warmup", "2",
           "--sweep", "0", "--gpu-warm-ms", "50"]
    r = subprocess.run(cmd, cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    d = _json_line(r.stdout)
    assert d["n_gpus"] == 4 and d["config"]["global_batch"] == 16 and d["value"] > 0
    assert d["config"]["collectives"] == "gloo (control only)"
    assert d["per_device_used_gib"] == [32] * 4  # 4 x 8 GiB per logical device, binpack-first
    agents = d["agents"]
    assert len(agents) == 4 and all(a["physical_gpu"] == 0 and a["hbm_total"] > 0 for a in agents)
    assert all(a["bad_stamps"] == 0 and a["failed"] == 0 for a in agents)
    assert sum(a["admitted"] for a in agents) == 7 * 16
    # no rank brought up RCCL: the bench's collectives are gloo
    assert "NCCL INFO" not in r.stderr and "RCCL" not in r.stderr
