"""Pod "container runtimes" for the node agent: where an admitted pod's gpu-mem physically lives.

kubelet + the container runtime start a pod's containers after the device
plugin's Allocate; here (no kubelet) the node agent does it through a
runtime:

* :class:`HbmArenaRuntime` — the MI355X path.  Each device holds one HBM
  arena sized to what the node advertises; an admitted pod gets a 2 MiB
  aligned slice — extents taken first-fit from the arena's holes, so a pod
  that fits the device's free bytes is admitted even when the arena is
  fragmented (the extender accounts a device as one number, like HBM behind
  the GPU's page tables) — the slice is stamped with the pod's tag by a HIP
  kernel and every resident pod's stamps are verified after each admission.
  A binpack decision that overcommits a device, or two pods sharing bytes,
  shows up as a failed admission or as bad stamps — on real HBM;
* :class:`LedgerRuntime` — the same slice accounting without a GPU
  (CPU tests, simulator).
"""
from __future__ import annotations

import hashlib
import threading

ALIGN = 2 << 20


class AdmissionError(Exception):
    pass


class _Slices:
    """Aligned slices of one arena, each a list of (offset, size) extents taken first-fit from the holes."""

    def __init__(self, capacity: int):
        self.capacity = capacity
        self.used: dict[str, list[tuple[int, int]]] = {}

    def alloc(self, uid: str, size: int) -> list[tuple[int, int]]:
        if uid in self.used:
            return self.used[uid]
        size = (size + ALIGN - 1) // ALIGN * ALIGN
        ext, pos, need = [], 0, size
        for off, sz in sorted(e for x in self.used.values() for e in x) + [(self.capacity, 0)]:
            if need and off > pos:
                n = min(need, off - pos)
                ext.append((pos, n))
                need -= n
            pos = max(pos, off + sz)
        if need:
            raise AdmissionError(f"arena exhausted: need {size} B, {size - need} free of {self.capacity}")
        self.used[uid] = ext
        return ext

    def free(self, uid: str) -> list[tuple[int, int]] | None:
        return self.used.pop(uid, None)

    def bytes_used(self) -> int:
        return sum(sz for x in self.used.values() for _, sz in x)


def pod_tag(uid: str) -> int:
    return int.from_bytes(hashlib.blake2b(uid.encode(), digest_size=8).digest(), "little") | 1


class LedgerRuntime:
    def __init__(self, capacities: dict[int, int]):
        self.slices = {d: _Slices(c) for d, c in capacities.items()}
        self.where: dict[str, int] = {}
        self.lock = threading.Lock()

    def start(self, uid: str, dev: int, nbytes: int, cus: list[int] | None = None) -> int:
        """Carve the pod's slice; returns the offset of its first extent."""
        with self.lock:
            if dev not in self.slices:
                raise AdmissionError(f"device {dev} not managed here")
            ext = self.slices[dev].alloc(uid, nbytes)
            self.where[uid] = dev
            return ext[0][0]

    def stop(self, uid: str) -> bool:
        with self.lock:
            dev = self.where.pop(uid, None)
            if dev is None:
                return False
            self.slices[dev].free(uid)
            return True

    def verify(self) -> int:
        return 0

    def resident_bytes(self, dev: int) -> int:
        return self.slices[dev].bytes_used()

    def close(self):
        pass


class HbmArenaRuntime(LedgerRuntime):
    def __init__(self, capacities: dict[int, int], stamp_stride: int = ALIGN, scrub_on_exit: bool = False):
        # default: one stamp per carve unit (every overlap of two slices covers at least one unit start)
        super().__init__(capacities)
        from ..ops import hip  # noqa: PLC0415

        self.hip = hip
        self.stride = stamp_stride
        self.scrub = scrub_on_exit
        self.arena = {d: hip.DeviceBuffer(d, c) for d, c in capacities.items()}
        self.stream = {d: hip.Stream(d) for d in capacities}
        self.stamps = 0
        self.verified = 0

    def start(self, uid: str, dev: int, nbytes: int, cus: list[int] | None = None) -> int:
        off = super().start(uid, dev, nbytes, cus)
        for o, size in self.slices[dev].used[uid]:
            self.hip.hbm_stamp(self.stream[dev], self.arena[dev].addr(o), size, self.stride, pod_tag(uid))
        self.stamps += 1
        return off

    def stop(self, uid: str) -> bool:
        with self.lock:
            dev = self.where.get(uid)
            ext = self.slices[dev].used.get(uid) if dev is not None else None
        if ext is not None and self.scrub:
            for o, size in ext:
                self.hip.hbm_fill(self.stream[dev], self.arena[dev].addr(o), size, 0)
        return super().stop(uid)

    def admit_sync(self, uid: str, dev: int, nbytes: int, cus=None, verify: bool = True) -> int:
        """Carve the slice, stamp it and verify every resident slice of the GPU: 2 launches, 1 sync."""
        LedgerRuntime.start(self, uid, dev, nbytes, cus)
        with self.lock:
            used = self.slices[dev].used
            mine = [(self.arena[dev].addr(o), sz, pod_tag(uid)) for o, sz in used[uid]]
            others = [(self.arena[dev].addr(o), sz, pod_tag(u)) for u, d in self.where.items() if d == dev and u != uid
                      for o, sz in used[u]] if verify else []
        bad = self.hip.hbm_admit_n(self.stream[dev], mine + others, len(mine), self.stride)
        self.stamps += 1
        self.verified += len(mine) + len(others)
        return bad if verify else 0

    def verify(self) -> int:
        """Verify every resident pod's stamps; returns the number of bad stamps."""
        bad = 0
        with self.lock:
            items = [(uid, dev, list(self.slices[dev].used[uid])) for uid, dev in self.where.items()]
        for uid, dev, ext in items:
            for off, size in ext:
                bad += self.hip.hbm_verify(self.stream[dev], self.arena[dev].addr(off), size, self.stride,
                                           pod_tag(uid))
            self.verified += 1
        return bad

    def sync(self):
        for s in self.stream.values():
            s.sync()

    def close(self):
        for s in self.stream.values():
            s.sync()
            s.destroy()
        for a in self.arena.values():
            a.free()


# ---------------------------------------------------------------- admission API used by the node agent

def admit_local(rt: LedgerRuntime, uid: str, dev: int, nbytes: int, cus=None, verify: bool = True) -> int:
    """Start a pod on a local runtime and (optionally) verify every resident slice; returns bad stamps."""
    fast = getattr(rt, "admit_sync", None)
    if fast is not None:
        return fast(uid, dev, nbytes, cus, verify)
    rt.start(uid, dev, nbytes, cus)
    return rt.verify() if verify else 0


class RuntimeShim:
    """Per-GPU runtime endpoint (the CRI-runtime role): the node agent starts / stops pods through it.

    ``POST /v1/pods/{uid}`` ``{"dev", "bytes", "cus", "verify"}`` -> ``{"bad"}`` (409 on admission failure),
    ``DELETE /v1/pods/{uid}``, ``GET /v1/stats``.  In ``bench.py`` every rank serves one for its GPU, so the
    HIP work for a pod runs in the process that owns that GPU.
    """

    def __init__(self, runtime: LedgerRuntime):
        from ..k8s.fasthttp import Server  # noqa: PLC0415

        self.runtime = runtime
        self.server = Server()
        self.server.route("POST", "/v1/pods/{uid}", self.h_start)
        self.server.route("DELETE", "/v1/pods/{uid}", self.h_stop)
        self.server.route("GET", "/v1/stats", self.h_stats)
        self.admitted = 0
        self.failed = 0
        self.bad = 0
        self.port = 0

    def h_start(self, request):
        from ..k8s.fasthttp import Response  # noqa: PLC0415

        b = request.json()
        uid = request.match_info["uid"]
        try:
            bad = admit_local(self.runtime, uid, int(b["dev"]), int(b["bytes"]), b.get("cus"),
                              bool(b.get("verify", True)))
        except AdmissionError as e:
            self.failed += 1
            return Response.json({"error": str(e)}, 409)
        self.admitted += 1
        self.bad += bad
        return Response.json({"bad": bad})

    def h_stop(self, request):
        from ..k8s.fasthttp import Response  # noqa: PLC0415

        ok = self.runtime.stop(request.match_info["uid"])
        return Response(b"", 200 if ok else 404)

    def h_stats(self, request):
        from ..k8s.fasthttp import Response  # noqa: PLC0415

        return Response.json({"admitted": self.admitted, "failed": self.failed, "bad": self.bad})

    async def start(self, host: str = "127.0.0.1", port: int = 0) -> str:
        self.port = await self.server.start(host, port)
        return f"http://{host}:{self.port}"

    async def stop(self):
        await self.server.stop()


class RemoteRuntime:
    """Node-agent side of :class:`RuntimeShim`: device index -> shim URL."""

    def __init__(self, endpoints: dict[int, str]):
        from ..k8s.fasthttp import Client  # noqa: PLC0415

        self.endpoints = dict(endpoints)
        self.clients = {d: Client(u, timeout=60.0) for d, u in self.endpoints.items()}
        self.where: dict[str, int] = {}

    async def admit(self, uid: str, dev: int, nbytes: int, cus=None, verify: bool = True) -> int:
        import json  # noqa: PLC0415

        c = self.clients.get(dev)
        if c is None:
            raise AdmissionError(f"no runtime endpoint for GPU {dev}")
        r = await c.request("POST", f"/v1/pods/{uid}", json.dumps({"dev": dev, "bytes": nbytes, "cus": cus,
                                                                    "verify": verify}).encode())
        body = r.json() or {}
        if r.status != 200:
            raise AdmissionError(body.get("error", f"runtime HTTP {r.status}"))
        self.where[uid] = dev
        return int(body.get("bad", 0))

    async def release(self, uid: str) -> bool:
        dev = self.where.pop(uid, None)
        if dev is None or dev not in self.clients:
            return False
        r = await self.clients[dev].request("DELETE", f"/v1/pods/{uid}")
        return r.status == 200

    async def close(self):
        for c in self.clients.values():
            await c.close()


class ProcessRuntime:
    """Container-runtime stand-in that runs each admitted pod's command as a child process.

    The child gets exactly the container environment the device plugin's
    Allocate returned (``HIP_VISIBLE_DEVICES``/``ROCR_VISIBLE_DEVICES``,
    ``SHARED_GPU_MEM_*``, ``HSA_CU_MASK``/``GSX_CU_MASK``) on top of this
    process's environment — the "Allocate output applied by a launcher" of
    SURVEY.md §7.3 slice B.  Children are started with fork+exec in the child
    (``asyncio.create_subprocess_exec``), never by replacing this process.
    """

    wants_envs = True
    mount_mode = "all"  # children run on the host and see every GPU: HIP_VISIBLE_DEVICES = host index

    def __init__(self, command: list[str], extra_env: dict | None = None, cwd: str | None = None):
        self.command = list(command)
        self.extra_env = dict(extra_env or {})
        self.cwd = cwd
        self.procs: dict = {}
        self.envs: dict[str, dict] = {}
        self.admitted = 0
        self.failed = 0
        self.bad = 0

    async def admit(self, uid: str, dev: int, nbytes: int, cus=None, verify: bool = True,
                    envs: dict | None = None) -> int:
        import asyncio  # noqa: PLC0415
        import os  # noqa: PLC0415

        env = dict(os.environ)
        env.update(self.extra_env)
        env.update(envs or {})
        try:
            proc = await asyncio.create_subprocess_exec(*self.command, env=env, cwd=self.cwd,
                                                        stdout=asyncio.subprocess.PIPE,
                                                        stderr=asyncio.subprocess.PIPE)
        except OSError as e:
            self.failed += 1
            raise AdmissionError(f"cannot start container: {e}") from e
        self.procs[uid] = proc
        self.envs[uid] = dict(envs or {})
        self.admitted += 1
        return 0

    async def wait(self, uid: str, timeout: float) -> tuple[int, str, str]:
        import asyncio  # noqa: PLC0415

        proc = self.procs[uid]
        so, se = await asyncio.wait_for(proc.communicate(), timeout)
        return proc.returncode, so.decode(errors="replace"), se.decode(errors="replace")

    async def release(self, uid: str) -> bool:
        proc = self.procs.pop(uid, None)
        if proc is None:
            return False
        if proc.returncode is None:
            proc.terminate()
            try:
                await proc.wait()
            except Exception:  # noqa: BLE001
                pass
        return True

    def verify(self) -> int:
        return 0

    def close(self):
        for p in self.procs.values():
            if p.returncode is None:
                p.kill()
