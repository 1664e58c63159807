"""CPU placement for the benchmark's control-plane processes (fake apiserver, extender, scheduler, node agent).

Every step of ``bench.py`` is a chain of dependent loopback round trips between those
processes, so its time is mostly wake-up latency: a process woken on an idle core pays
the core's C-state exit and a cold cache, and the scheduler may move it between runs.
Pinning each process to its own physical core, all inside one L3 domain, keeps the
chain on warm cores and makes run-to-run spread small (``profiles/r02_bench_stability.md``).

Only CPUs in this process's affinity mask are used; SMT siblings are skipped while
physical cores remain.
"""
from __future__ import annotations

import os


def _read_list(path: str) -> list[int]:
    """``0-3,8,10-11`` -> [0, 1, 2, 3, 8, 10, 11]."""
    try:
        with open(path) as f:
            txt = f.read().strip()
    except OSError:
        return []
    out = []
    for part in txt.split(","):
        if not part:
            continue
        if "-" in part:
            a, b = part.split("-")
            out.extend(range(int(a), int(b) + 1))
        else:
            out.append(int(part))
    return out


def _group_key(cpu: int) -> tuple:
    base = f"/sys/devices/system/cpu/cpu{cpu}"
    l3 = _read_list(f"{base}/cache/index3/shared_cpu_list")
    return (min(l3) if l3 else 0,)


def physical_cpus(allowed: list[int] | None = None) -> list[int]:
    """Allowed CPUs ordered so that the first ones are distinct physical cores of the largest L3 domain."""
    allowed = sorted(allowed if allowed is not None else os.sched_getaffinity(0))
    allowed_set = set(allowed)
    seen_cores, primary, siblings = set(), [], []
    for c in allowed:
        sib = tuple(_read_list(f"/sys/devices/system/cpu/cpu{c}/topology/thread_siblings_list") or [c])
        if sib in seen_cores:
            siblings.append(c)
            continue
        seen_cores.add(sib)
        primary.append(c)
    groups: dict[tuple, list[int]] = {}
    for c in primary:
        groups.setdefault(_group_key(c), []).append(c)
    ordered = []
    for _, cs in sorted(groups.items(), key=lambda kv: -len(kv[1])):
        ordered.extend(cs)
    return ordered + [c for c in siblings if c in allowed_set]


def plan(names: list[str], widths: dict[str, int] | None = None, mode: str = "spread") -> dict[str, list[int]]:
    """CPU list per process name.

    ``spread``: each process gets ``widths[name]`` (default 1) CPUs of its own, physical cores first;
    ``compact``: all processes share the first ``max(widths)`` cores;
    ``none``: {} (no pinning).  Falls back to {} when there are not enough CPUs for ``spread``.
    """
    if mode == "none":
        return {}
    widths = widths or {}
    cpus = physical_cpus()
    need = sum(widths.get(n, 1) for n in names)
    if mode == "compact":
        w = max((widths.get(n, 1) for n in names), default=1)
        return {n: cpus[:w] for n in names}
    if len(cpus) < need:
        return {}
    out, i = {}, 0
    for n in names:
        w = widths.get(n, 1)
        out[n] = cpus[i:i + w]
        i += w
    return out


def pin_self(cpus: list[int] | None) -> None:
    """Pin the calling process (all threads created afterwards inherit it)."""
    if cpus:
        os.sched_setaffinity(0, set(cpus))
