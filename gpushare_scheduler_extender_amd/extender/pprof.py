"""``/debug/pprof/*`` covering the whole extender process: Python threads *and* the native ones.

The reference mounts Go's ``net/http/pprof`` on its API port (``pkg/routes/pprof.go:10-64``, paths with
trailing slashes); it sees every goroutine of the process that serves filter / bind.  Here filter and
bind run on C++ epoll loops and a bind pool, the informers on C++ reflector threads, so every endpoint
reports both sides (native side: ``native/engine/introspect.{h,cc}``):

* ``goroutine``    — every OS thread of the process: name (native threads are ``gsx-http-N``,
  ``gsx-bind-N``, ``gsx-refl-pods``, ...), state, CPU seconds, and its stack: Python frames for Python
  threads, a native backtrace (signal-sampled, symbolised) for the others; then the pending asyncio tasks;
* ``profile``      — statistical CPU profile of *all* threads for ``?seconds=N`` (default 5, max 60) at
  ``?hz=`` (default 100): collapsed stacks ``thread;frame;...;leaf count`` (flamegraph.pl / speedscope
  input), preceded by ``#`` lines with each thread's CPU seconds in the window, the native verb latency
  histograms (filter / bind / apiserver round trip) and the ledger mutex profile;
* ``trace``        — the same sampler at 1 kHz over ``?seconds`` (default 1);
* ``heap``         — ``tracemalloc`` top allocation sites (tracing starts on the first request;
  ``?start=0`` stops it) plus the process RSS;
* ``mutex``        — the ledger mutex (every filter / bind / informer update takes it): acquisitions,
  contended acquisitions, total / max wait and hold times;
* ``block``        — where binds waited: the native front end's bind-ordering waits and apiserver
  round-trip histogram;
* ``threadcreate`` — every OS thread with its name and CPU time; ``cmdline``, ``symbol``.
"""
from __future__ import annotations

import asyncio
import collections
import os
import sys
import threading
import time
import traceback
import tracemalloc

from aiohttp import web

PATHS = ["", "cmdline/", "profile/", "symbol/", "trace/", "heap/", "goroutine/", "block/", "threadcreate/", "mutex/"]
CLK_TCK = os.sysconf("SC_CLK_TCK")
_STATE = {"engine": None}


def _text(s: str) -> web.Response:
    return web.Response(text=s, content_type="text/plain")


def _engine_mod():
    try:
        from ..core.engine import native  # noqa: PLC0415

        return native()
    except Exception:  # noqa: BLE001 - no native engine: Python-only view
        return None


def os_threads() -> dict[int, dict]:
    """tid -> {comm, state, cpu_s} from /proc/self/task."""
    out = {}
    for t in os.listdir("/proc/self/task"):
        try:
            with open(f"/proc/self/task/{t}/stat") as f:
                raw = f.read()
            comm = raw[raw.index("(") + 1:raw.rindex(")")]
            rest = raw[raw.rindex(")") + 2:].split()
            out[int(t)] = {"comm": comm, "state": rest[0], "cpu_s": (int(rest[11]) + int(rest[12])) / CLK_TCK}
        except (OSError, ValueError, IndexError):
            continue
    return out


def _py_threads() -> dict[int, threading.Thread]:
    return {t.native_id: t for t in threading.enumerate() if t.native_id is not None}


def _py_stack(ident: int) -> list[str]:
    f = sys._current_frames().get(ident)  # noqa: SLF001
    stack = []
    while f is not None:
        stack.append(f"{f.f_code.co_name} ({f.f_code.co_filename.rsplit('/', 1)[-1]}:{f.f_lineno})")
        f = f.f_back
    return stack  # innermost first


def _native_stacks(tids: list[int] | None = None) -> dict[int, list[str]]:
    E = _engine_mod()
    if E is None or not hasattr(E, "native_stacks"):
        return {}
    return {tid: frames for tid, _comm, ok, frames in E.native_stacks(tids or [], 0.05) if ok}


async def index(request):
    lines = ["/debug/pprof/", ""]
    lines += [f"/debug/pprof/{p}" for p in PATHS if p]
    return _text("\n".join(lines) + "\n")


async def cmdline(request):
    return web.Response(body="\x00".join(sys.argv).encode(), content_type="text/plain")


async def symbol(request):
    """Go's pprof symbol protocol: GET -> ``num_symbols``; POST ``0xADDR+0xADDR...`` -> ``0xADDR name`` lines
    (native program counters of this process, symbolised from the loaded objects' symbol tables)."""
    E = _engine_mod()
    if request.method != "POST":
        return _text(f"num_symbols: {1 if E is not None else 0}\n")
    body = (await request.read()).decode(errors="replace")
    out = []
    for tok in body.replace("+", " ").split():
        try:
            pc = int(tok, 16)
        except ValueError:
            continue
        name = E.native_symbol(pc) if E is not None else ""
        if name:
            out.append(f"{tok} {name}")
    return _text("\n".join(out) + "\n")


async def goroutine(request):
    loop = asyncio.get_running_loop()
    threads = os_threads()
    py = _py_threads()
    native = await loop.run_in_executor(None, _native_stacks, [t for t in threads if t not in py])
    out = [f"threads: {len(threads)} ({len(py)} Python, {len(threads) - len(py)} native)", ""]
    for tid in sorted(threads):
        info = threads[tid]
        kind = "python" if tid in py else "native"
        out.append(f"thread {tid} [{info['comm']}] {kind} state={info['state']} cpu={info['cpu_s']:.3f}s")
        if tid in py:
            f = sys._current_frames().get(py[tid].ident)  # noqa: SLF001
            if f is not None:
                out.extend("  " + ln.rstrip() for ln in traceback.format_stack(f))
        else:
            out.extend(f"  {fr}" for fr in native.get(tid, ["<no sample>"]))
        out.append("")
    tasks = asyncio.all_tasks()
    out.append(f"asyncio tasks: {len(tasks)}")
    for task in tasks:
        out.append(f"task {task.get_name()} done={task.done()}")
        for fr in task.get_stack(limit=20):
            out.append(f"  {fr.f_code.co_filename}:{fr.f_lineno} {fr.f_code.co_name}")
        out.append("")
    return _text("\n".join(out) + "\n")


async def heap(request):
    rss = 0
    try:
        with open("/proc/self/status") as f:
            rss = next(int(ln.split()[1]) for ln in f if ln.startswith("VmRSS:"))
    except (OSError, StopIteration):
        pass
    if request.query.get("start") == "0":
        tracemalloc.stop()
        return _text("tracemalloc stopped\n")
    if not tracemalloc.is_tracing():
        tracemalloc.start(16)
        return _text(f"rss_kib={rss}\ntracemalloc started; request again for a snapshot\n")
    snap = tracemalloc.take_snapshot()
    stats = snap.statistics("lineno")[: int(request.query.get("top", "50"))]
    cur, peak = tracemalloc.get_traced_memory()
    lines = [f"heap profile: rss_kib={rss} python_current={cur} python_peak={peak}"]
    lines += [str(s) for s in stats]
    return _text("\n".join(lines) + "\n")


def sample_all(seconds: float, hz: float) -> tuple[collections.Counter, dict[int, dict], dict[int, dict]]:
    """Collapsed stacks of every thread of the process, sampled ``hz`` times per second (run off-loop)."""
    me = threading.get_native_id()
    counts: collections.Counter = collections.Counter()
    t0 = os_threads()
    end = time.monotonic() + seconds
    interval = 1.0 / hz
    while time.monotonic() < end:
        nxt = time.monotonic() + interval
        py = _py_threads()
        threads = os_threads()
        native = _native_stacks([t for t in threads if t not in py and t != me])
        frames_py = sys._current_frames()  # noqa: SLF001
        for tid, info in threads.items():
            if tid == me or info["state"] not in ("R", "D"):
                continue  # on-CPU profile: runnable / uninterruptible threads only
            if tid in py:
                f = frames_py.get(py[tid].ident)
                stack = []
                while f is not None:
                    stack.append(f"{f.f_code.co_name} ({f.f_code.co_filename.rsplit('/', 1)[-1]}:{f.f_lineno})")
                    f = f.f_back
            else:
                stack = native.get(tid)
                if not stack:
                    continue
            counts[";".join([info["comm"], *reversed(stack)])] += 1
        time.sleep(max(0.0, nxt - time.monotonic()))
    return counts, t0, os_threads()


def _header(t0: dict, t1: dict, seconds: float) -> list[str]:
    lines = [f"# window {seconds:.1f}s; per-thread CPU seconds (name tid cpu)"]
    for tid in sorted(t1):
        d = t1[tid]["cpu_s"] - t0.get(tid, {"cpu_s": 0.0})["cpu_s"]
        if d > 0:
            lines.append(f"#   {t1[tid]['comm']} {tid} {d:.3f}")
    eng = _STATE["engine"]
    if eng is not None:
        try:
            st = eng.server_stats()
        except Exception:  # noqa: BLE001 - not serving natively
            st = {}
        for name in ("filter_latency", "bind_latency", "api_latency"):
            h = st.get(name)
            if not h or not h["n"]:
                continue
            cells = " ".join(f"<={b * 1e3:g}ms:{c}" for b, c in zip(h["bounds"], h["counts"]) if c)
            tail = h["counts"][len(h["bounds"])]
            lines.append(f"# native {name}: n={h['n']} mean={1e3 * h['sum'] / h['n']:.3f}ms {cells}"
                         + (f" >{h['bounds'][-1] * 1e3:g}ms:{tail}" if tail else ""))
        m = eng.ledger_mutex()
        lines.append(f"# ledger mutex: acquisitions={m['acquisitions']} contended={m['contended']} "
                     f"wait={m['wait_s'] * 1e3:.3f}ms max_wait={m['max_wait_s'] * 1e6:.1f}us "
                     f"hold={m['hold_s'] * 1e3:.3f}ms max_hold={m['max_hold_s'] * 1e6:.1f}us")
    return lines


async def _profile(request, default_s: float, max_s: float, default_hz: float):
    seconds = min(max_s, float(request.query.get("seconds", str(default_s))))
    hz = min(1000.0, max(1.0, float(request.query.get("hz", str(default_hz)))))
    counts, t0, t1 = await asyncio.get_running_loop().run_in_executor(None, sample_all, seconds, hz)
    body = _header(t0, t1, seconds) + [f"{k} {v}" for k, v in counts.most_common()]
    return _text("\n".join(body) + "\n")


async def profile(request):
    return await _profile(request, 5.0, 60.0, 100.0)


async def trace(request):
    return await _profile(request, 1.0, 30.0, 1000.0)


async def threadcreate(request):
    ts = os_threads()
    py = _py_threads()
    lines = [f"threadcreate profile: total {len(ts)}"]
    lines += [f"{tid} {i['comm']} {'python' if tid in py else 'native'} cpu={i['cpu_s']:.3f}s"
              for tid, i in sorted(ts.items())]
    return _text("\n".join(lines) + "\n")


async def block(request):
    eng = _STATE["engine"]
    lines = ["block profile"]
    if eng is not None:
        try:
            st = eng.server_stats()
        except Exception:  # noqa: BLE001
            st = {}
        if st:
            lines.append(f"bind_order_waits={st.get('bind_order_waits', 0)} (equal-size binds for different GPUs "
                         f"of one node held back to keep ASSUME_TIME order)")
            h = st.get("api_latency") or {}
            if h.get("n"):
                lines.append(f"apiserver round trips: n={h['n']} total={h['sum']:.3f}s mean={1e3 * h['sum'] / h['n']:.3f}ms")
    return _text("\n".join(lines) + "\n")


async def mutex(request):
    eng = _STATE["engine"]
    if eng is None:
        return _text("mutex profile: no native engine\n")
    m = eng.ledger_mutex()
    return _text("mutex profile (ledger mutex: filter, bind reservations, informer updates)\n"
                 + "".join(f"{k}={v}\n" for k, v in m.items()))


def add_pprof(app: web.Application, engine=None):
    """pkg/routes/pprof.go:10-22 route table (trailing slashes kept; bare names also accepted)."""
    _STATE["engine"] = engine
    r = app.router
    r.add_get("/debug/pprof/", index)
    for name, h in (("cmdline", cmdline), ("profile", profile), ("symbol", symbol), ("trace", trace),
                    ("heap", heap), ("goroutine", goroutine), ("block", block), ("threadcreate", threadcreate),
                    ("mutex", mutex)):
        r.add_get(f"/debug/pprof/{name}/", h)
        r.add_get(f"/debug/pprof/{name}", h)
    r.add_post("/debug/pprof/symbol/", symbol)
    r.add_post("/debug/pprof/symbol", symbol)
