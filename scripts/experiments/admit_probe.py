"""Where a pod admission's time goes on the MI355X: fixed launch + sync cost, kernel time for the bench's
4 x 64 GiB slices at a 1 MiB stamp stride, the PodRuntime call without HTTP, and over HTTP."""
import json
import statistics
import time
import urllib.request

from gpushare_scheduler_extender_amd.core.engine import native
from gpushare_scheduler_extender_amd.ops import hip

GiB, MiB = 1 << 30, 1 << 20


def pct(xs, q):
    xs = sorted(xs)
    return xs[min(len(xs) - 1, int(q / 100 * len(xs)))]


def timeit(f, n=200):
    for _ in range(20):
        f()
    ts = []
    for _ in range(n):
        t = time.perf_counter()
        f()
        ts.append(time.perf_counter() - t)
    return {"p50_us": round(pct(ts, 50) * 1e6, 1), "p90_us": round(pct(ts, 90) * 1e6, 1),
            "mean_us": round(statistics.mean(ts) * 1e6, 1)}


out = {}
arena = 256 * GiB
buf = hip.DeviceBuffer(0, arena)
s = hip.Stream(0)
base = buf.addr(0)
small = [(base + i * 2 * MiB, 2 * MiB, 7 + i) for i in range(4)]
big = [(base + i * 64 * GiB, 64 * GiB, 7 + i) for i in range(4)]
out["tiny: stamp 1 + verify 4 (2 stamps each), 1 sync"] = timeit(lambda: hip.hbm_admit_n(s, small, 1, MiB))
out["tiny: stamp only (1 sync)"] = timeit(lambda: hip.hbm_admit_n(s, small[:1], 1, MiB, verify=False))
hip.hbm_admit_n(s, big, 4, MiB)
out["bench: stamp 1 x 64 GiB + verify 4 x 64 GiB @1 MiB"] = timeit(lambda: hip.hbm_admit_n(s, big, 1, MiB))
out["bench: stamp 1 x 64 GiB only @1 MiB"] = timeit(lambda: hip.hbm_admit_n(s, big[:1], 1, MiB, verify=False))
out["bench: verify 4 x 64 GiB only @1 MiB"] = timeit(lambda: hip.hbm_admit_n(s, big, 0, MiB))
out["bench @2 MiB stride: stamp 1 + verify 4"] = timeit(lambda: hip.hbm_admit_n(s, big, 1, 2 * MiB))
out["sync of an idle stream"] = timeit(lambda: s.sync())

rt = native().PodRuntime(0, arena, base, s.ptr, MiB, hip.lib()._name)
for i in range(3):
    rt.admit(f"r{i}", 64 * GiB, True)


def cycle():
    rt.admit("x", 64 * GiB, True)
    rt.release("x")


out["PodRuntime.admit + release, 3 resident (no HTTP)"] = timeit(cycle)
url = f"http://127.0.0.1:{rt.serve('127.0.0.1', 0)}"


def http_cycle():
    r = urllib.request.Request(url + "/v1/pods/y", data=json.dumps({"bytes": 64 * GiB}).encode(), method="POST")
    urllib.request.urlopen(r).read()
    rt.release("y")


out["HTTP POST /v1/pods (urllib, new connection each) + release"] = timeit(http_cycle, 100)
rt.stop()
s.sync()
s.destroy()
buf.free()
print(json.dumps(out, indent=1))
