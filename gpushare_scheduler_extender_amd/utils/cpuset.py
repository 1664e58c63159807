"""CPU placement for the benchmark's control-plane processes (fake apiserver, extender, scheduler, node agent).

Every step of ``bench.py`` is a chain of dependent loopback round trips between those
processes, so its time is mostly wake-up latency: a process woken on an idle core pays
the core's C-state exit and a cold cache, and the scheduler may move it between runs.
Pinning each process to its own physical core keeps the chain on warm cores and makes
run-to-run spread small (``profiles/r02_bench_stability.md``).

The GPU boxes are slices of a shared host: other jobs keep some CPUs busy, and their
threads and the host's interrupts land on the low-numbered CPUs too (``scripts/experiments/cpu_probe.py``
measured CPUs 0-7 at 0-31 % busy and ~300 interrupts/s each, with other CPUs pinned at
100 %). A process pinned to such a CPU waits for the other job's time slice: one such
wait cost a timed wave 14 ms. ``spread`` therefore samples per-CPU load first and
places the processes on the idlest physical cores, filling the L3 domain with the
most idle cores first. All ranks of one ``torchrun`` job share one plan through a
locked file (:func:`shared_plan`).

Only CPUs in this process's affinity mask are used; SMT siblings are skipped while
physical cores remain, unless ``smt`` slots are asked for (a 2-wide slot = one core, both threads).
"""
from __future__ import annotations

import fcntl
import json
import logging
import os
import tempfile
import time

log = logging.getLogger("gsx.cpuset")
IDLE = 0.05  # a CPU busier than this (other jobs, interrupts) over the sample window is avoided


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


def _proc_stat() -> dict[int, tuple[int, int]]:
    """cpu -> (total jiffies, idle + iowait jiffies)."""
    out = {}
    try:
        with open("/proc/stat") as f:
            for ln in f:
                if ln.startswith("cpu") and ln[3:4].isdigit():
                    p = ln.split()
                    v = [int(x) for x in p[1:]]
                    out[int(p[0][3:])] = (sum(v), v[3] + (v[4] if len(v) > 4 else 0))
    except OSError:
        pass
    return out


def sample_load(window: float = 0.3) -> dict[int, float]:
    """Busy fraction of every CPU over ``window`` seconds ({} when /proc/stat is unreadable)."""
    s0 = _proc_stat()
    if not s0:
        return {}
    time.sleep(window)
    s1 = _proc_stat()
    out = {}
    for c, (t1, i1) in s1.items():
        t0, i0 = s0.get(c, (t1, i1))
        dt = t1 - t0
        out[c] = 0.0 if dt <= 0 else max(0.0, min(1.0, 1.0 - (i1 - i0) / dt))
    return out


def _cores(allowed: list[int]) -> list[tuple[int, ...]]:
    """Physical cores among ``allowed``: each as its allowed SMT threads, lowest CPU first."""
    allowed_set = set(allowed)
    seen, cores = set(), []
    for c in sorted(allowed):
        sib = tuple(_read_list(f"/sys/devices/system/cpu/cpu{c}/topology/thread_siblings_list") or [c])
        if sib in seen:
            continue
        seen.add(sib)
        cores.append(tuple([c] + [s for s in sib if s != c and s in allowed_set]))
    return cores


def _order_cores(cores: list[tuple[int, ...]], load: dict[int, float] | None, need: int = 0) -> list[tuple[int, ...]]:
    """Best placement first.

    Without ``load``: cores of the largest L3 domain first, in CPU order. With ``load``: the ``need`` least
    busy cores of the L3 domain whose ``need`` least busy cores are the least busy in total (domains with
    fewer than ``need`` cores only when none has enough); then every other core, idle ones (every thread
    < ``IDLE`` busy) before busy ones, least busy first. CPU 0's core goes last either way (the kernel's
    housekeeping and many interrupts run there).
    """
    def busy(core):
        return max(load.get(c, 0.0) for c in core) if load else 0.0

    groups: dict[tuple, list[tuple[int, ...]]] = {}
    for core in cores:
        groups.setdefault(_group_key(core[0]), []).append(core)
    if not load:
        ordered = [core for _, cs in sorted(groups.items(), key=lambda kv: -len(kv[1])) for core in cs]
    else:
        cand = {k: sorted((c for c in cs if 0 not in c), key=lambda c: (busy(c), c)) for k, cs in groups.items()}

        def score(k):
            cs = cand[k]
            if need and len(cs) >= need:
                return (0, sum(busy(c) for c in cs[:need]), k)
            return (1, -sum(1 for c in cs if busy(c) < IDLE), k)

        first = cand[min(groups, key=score)][:need] if need and groups else []
        taken = set(first)
        ordered = first + sorted((c for c in cores if c not in taken), key=lambda c: (busy(c) >= IDLE, busy(c), c))
    return [c for c in ordered if 0 not in c] + [c for c in ordered if 0 in c]


def physical_cpus(allowed: list[int] | None = None, load: dict[int, float] | None = None) -> list[int]:
    """Allowed CPUs, best placement first (:func:`_order_cores`): one per physical core, then the SMT siblings."""
    allowed = sorted(allowed if allowed is not None else os.sched_getaffinity(0))
    ordered = _order_cores(_cores(allowed), load)
    return [core[0] for core in ordered] + [c for core in ordered for c in core[1:]]


def plan(names: list[str], widths: dict[str, int] | None = None, mode: str = "spread",
         load: dict[int, float] | None = None, smt: bool = False, local: int | None = None) -> dict[str, list[int]]:
    """CPU list per process name.

    ``spread``: each process gets ``widths[name]`` (default 1) CPUs of its own, idlest physical cores first
    (``load`` sampled here unless given); ``static``: the same without the load sample (topology order);
    ``compact``: all processes share the first ``max(widths)`` cores; ``none``: {} (no pinning).
    ``smt``: a slot of width w takes ceil(w / 2) physical cores with their SMT siblings, so one process's
    threads share a core's caches (width 1 leaves the sibling unused); otherwise every CPU of a slot is a
    physical core of its own.  ``local``: the first ``local`` names (default all) should share one L3 domain
    (the chain of round trips); the rest go to the idlest cores anywhere.  Falls back to {} when there are not
    enough CPUs.
    """
    if mode == "none":
        return {}
    widths = widths or {}
    if mode == "spread" and load is None:
        load = sample_load()
    cores = _cores(sorted(os.sched_getaffinity(0)))
    if mode == "compact":
        cpus = physical_cpus(load=None)
        w = max((widths.get(n, 1) for n in names), default=1)
        return {n: cpus[:w] for n in names}
    per = {n: max(0, widths.get(n, 1)) for n in names}  # width 0: that process is not pinned
    near = names[:local] if local is not None else names
    if smt and all(len(c) >= 2 for c in cores):
        need = sum((w + 1) // 2 for w in per.values())
        ordered = _order_cores(cores, load if mode == "spread" else None, sum((per[n] + 1) // 2 for n in near))
        if len(ordered) < need:
            log.warning("CPU plan: %d physical cores asked for (%d processes), %d allowed: not pinning", need,
                        len(names), len(ordered))
            return {}
        out, i = {}, 0
        for n in names:
            k = (per[n] + 1) // 2
            out[n] = [c for core in ordered[i:i + k] for c in core[:2]][:per[n]]
            i += k
        return out
    need = sum(per.values())
    ordered = _order_cores(cores, load if mode == "spread" else None, sum(per[n] for n in near))
    cpus = [core[0] for core in ordered] + [c for core in ordered for c in core[1:]]
    if len(cpus) < need:
        log.warning("CPU plan: %d CPUs asked for (%d processes), %d allowed: not pinning", need, len(names),
                    len(cpus))
        return {}
    out, i = {}, 0
    for n in names:
        out[n] = cpus[i:i + per[n]]
        i += per[n]
    return out


def shared_plan(names: list[str], widths: dict[str, int] | None, mode: str, key: str,
                smt: bool = False, local: int | None = None) -> dict[str, list[int]]:
    """:func:`plan`, computed once per ``key`` and shared by every process that asks with that key.

    The ranks of one job sample the load at slightly different moments and could pick overlapping CPUs; the
    first rank to take the lock computes the plan, the others read it."""
    path = os.path.join(tempfile.gettempdir(), f"gsx-cpuplan-{key}.json")
    with open(path + ".lock", "a+") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        try:
            try:
                with open(path) as f:
                    got = json.load(f)
                if (got.get("names"), got.get("widths"), got.get("mode"), got.get("smt")) == (
                        names, widths or {}, mode, smt):
                    return {k: list(v) for k, v in got["plan"].items()}
            except (OSError, ValueError):
                pass
            out = plan(names, widths, mode, smt=smt, local=local)
            tmp = path + f".{os.getpid()}"
            with open(tmp, "w") as f:
                json.dump({"names": names, "widths": widths or {}, "mode": mode, "smt": smt, "plan": out}, f)
            os.replace(tmp, path)
            return out
        finally:
            fcntl.flock(lk, fcntl.LOCK_UN)


def forget_shared_plan(key: str) -> None:
    path = os.path.join(tempfile.gettempdir(), f"gsx-cpuplan-{key}.json")
    for p in (path, path + ".lock"):
        try:
            os.unlink(p)
        except OSError:
            pass


def pin_self(cpus: list[int] | None) -> None:
    """Pin the calling process (all threads created afterwards inherit it)."""
    if cpus:
        os.sched_setaffinity(0, set(cpus))
