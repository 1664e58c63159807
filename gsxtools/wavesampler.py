"""Per-wave attribution for ``bench.py``: why was a wave slow?

A sampler process, pinned to a CPU of its own (outside the bench's CPU plan when the host has one to spare), reads
every ``--interval`` seconds:

* the scheduler run-delay of each pipeline process -- ``/proc/<pid>/task/*/schedstat`` field 2, the nanoseconds its
  threads spent runnable but waiting for a CPU, summed over the threads (the plugin's threads included);
* the host's pressure stall information -- ``/proc/pressure/{cpu,io,memory}`` ``some total=`` (microseconds in which
  at least one task stalled on that resource), when the kernel exposes it.

Each sample carries ``time.perf_counter()`` (CLOCK_MONOTONIC, the clock ``bench.py`` stamps its waves with).  On
SIGTERM the samples go to ``--out`` as JSON; :func:`attribute` turns them and the waves' [t0, t0 + total] spans into
per-wave deltas and names, for a wave slower than 5 x the p50, the process whose threads waited longest for a CPU --
or the host, when its pressure counters say every process stalled.

Reference: the reference's own diagnosis surface is net/http/pprof (``/root/reference/pkg/routes/pprof.go:10-64``);
this is the benchmark-side counterpart for stalls no single process can see.
"""
from __future__ import annotations

import argparse
import json
import os
import signal
import sys
import time

PSI = ("cpu", "io", "memory")


def _run_delay_ns(pid: int, tids: list[str]) -> int:
    ns = 0
    for t in tids:
        try:
            with open(f"/proc/{pid}/task/{t}/schedstat", "rb") as f:
                ns += int(f.read().split()[1])
        except (OSError, ValueError, IndexError):
            pass
    return ns


def _psi_some_us(kind: str) -> int | None:
    try:
        with open(f"/proc/pressure/{kind}") as f:
            for ln in f:
                if ln.startswith("some"):
                    return int(ln.rsplit("total=", 1)[1])
    except (OSError, ValueError, IndexError):
        return None
    return None


def sample_loop(pids: dict[str, int], interval: float, out: str) -> None:
    names = list(pids)
    samples: list[list] = []
    stop = {"now": False}
    signal.signal(signal.SIGTERM, lambda *_: stop.__setitem__("now", True))
    with open(out + ".ready", "w"):  # the bench waits for this before its warmup waves
        pass
    tids: dict[str, list[str]] = {}
    t_tids = 0.0
    while not stop["now"]:
        now = time.perf_counter()
        if now - t_tids > 0.05:  # thread lists change rarely: refresh them every 50 ms
            for n in names:
                try:
                    tids[n] = os.listdir(f"/proc/{pids[n]}/task")
                except OSError:
                    tids[n] = []
            t_tids = now
        row = [now] + [_run_delay_ns(pids[n], tids.get(n, [])) for n in names] + [_psi_some_us(k) for k in PSI]
        samples.append(row)
        left = interval - (time.perf_counter() - now)
        if left > 0:
            time.sleep(left)
    with open(out + ".tmp", "w") as f:
        json.dump({"names": names, "interval": interval, "samples": samples}, f)
    os.replace(out + ".tmp", out)


def _at_or_before(ts: list[float], t: float) -> int:
    lo, hi = 0, len(ts) - 1
    if hi < 0 or ts[0] > t:
        return 0
    while lo < hi:
        mid = (lo + hi + 1) // 2
        if ts[mid] <= t:
            lo = mid
        else:
            hi = mid - 1
    return lo


def attribute(data: dict, waves: list[tuple[float, float]], slow_factor: float = 5.0, cap: int = 400) -> dict:
    """``waves``: (t0, seconds) per timed wave.  Per-wave run-delay (ms) per process and host pressure deltas, plus
    the slow waves (over ``slow_factor`` x the p50) with the process (or the host) to blame."""
    names, rows = data["names"], data["samples"]
    if not rows or not waves:
        return {"samples": len(rows)}
    ts = [r[0] for r in rows]
    k = len(names)
    per_proc = {n: [] for n in names}
    psi = {p: [] for p in PSI}
    for t0, dur in waves:
        a = _at_or_before(ts, t0)
        b = min(len(rows) - 1, _at_or_before(ts, t0 + dur) + 1)
        ra, rb = rows[a], rows[b]
        for i, n in enumerate(names):
            per_proc[n].append(round((rb[1 + i] - ra[1 + i]) / 1e6, 3))
        for j, p in enumerate(PSI):
            x, y = ra[1 + k + j], rb[1 + k + j]
            psi[p].append(round((y - x) / 1e3, 3) if x is not None and y is not None else None)
    durs = sorted(d for _, d in waves)
    p50 = durs[len(durs) // 2]
    slow = []
    for w, (_, dur) in enumerate(waves):
        if p50 <= 0 or dur < slow_factor * p50:
            continue
        delays = {n: per_proc[n][w] for n in names}
        worst = max(delays, key=delays.get)
        cpu = psi["cpu"][w]
        wave_ms = dur * 1e3
        if delays[worst] >= 0.25 * wave_ms:
            blame = worst
        elif cpu is not None and cpu >= 0.25 * wave_ms:
            blame = "host (cpu pressure)"
        elif psi["io"][w] is not None and psi["io"][w] >= 0.25 * wave_ms:
            blame = "host (io pressure)"
        elif psi["memory"][w] is not None and psi["memory"][w] >= 0.25 * wave_ms:
            blame = "host (memory pressure)"
        else:
            blame = "unattributed (no process waited for a CPU: off-CPU wait)"
        slow.append({"wave": w, "ms": round(wave_ms, 3), "x_p50": round(dur / p50, 1), "blame": blame,
                     "run_delay_ms": delays, "psi_ms": {p: psi[p][w] for p in PSI}})
    n = len(waves)
    return {"interval_ms": round(1e3 * data["interval"], 3), "samples": len(rows),
            "run_delay_ms_each": {p: v for p, v in per_proc.items()} if n <= cap else None,
            "psi_ms_each": psi if n <= cap else None,
            "run_delay_ms_total": {p: round(sum(v), 3) for p, v in per_proc.items()},
            "slow_waves": slow}


class Sampler:
    """The sampler as a child process of the bench (started before the timed region, stopped after it)."""

    def __init__(self, pids: dict[str, int], out: str, interval: float = 0.002, cpu: int | None = None):
        import subprocess  # noqa: PLC0415

        self.out = out
        for f in (out, out + ".ready"):
            try:
                os.unlink(f)
            except OSError:
                pass
        spec = ",".join(f"{n}={p}" for n, p in pids.items() if p)
        pre = None
        if cpu is not None:
            def pre():
                os.sched_setaffinity(0, {cpu})
        self.proc = subprocess.Popen([sys.executable, "-m", "gsxtools.wavesampler", "--pids", spec, "--interval",
                                      str(interval), "--out", out], preexec_fn=pre)

    def wait_ready(self, timeout: float = 30.0) -> bool:
        """The sampler runs (its SIGTERM handler is in place): it must not start up inside a timed region."""
        deadline = time.monotonic() + timeout
        while time.monotonic() < deadline:
            if os.path.exists(self.out + ".ready"):
                return True
            if self.proc.poll() is not None:
                return False
            time.sleep(0.005)
        return False

    def stop(self) -> dict | None:
        self.proc.terminate()
        try:
            self.proc.wait(10)
        except Exception:  # noqa: BLE001
            self.proc.kill()
            return None
        try:
            with open(self.out) as f:
                return json.load(f)
        except (OSError, ValueError):
            return None
        finally:
            for f in (self.out, self.out + ".ready"):
                try:
                    os.unlink(f)
                except OSError:
                    pass


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description="per-wave run-delay / pressure sampler (bench.py)")
    ap.add_argument("--pids", required=True, help="name=pid,name=pid,...")
    ap.add_argument("--interval", type=float, default=0.002)
    ap.add_argument("--out", required=True)
    a = ap.parse_args(argv)
    pids = {}
    for kv in a.pids.split(","):
        if "=" in kv:
            n, p = kv.split("=", 1)
            pids[n] = int(p)
    sample_loop(pids, a.interval, a.out)
    return 0


if __name__ == "__main__":
    sys.exit(main())
