"""The sample pod workload: a PyTorch-ROCm / HIP GEMM loop that stays inside its GPU share.

Self-contained (the container image holds this file, ``run.sh`` and the ``libgsx_kernels.so`` its Dockerfile
builds; nothing else of this repository): counterpart of the reference's sample container
(``samples/docker/main.py``: TF1 with ``per_process_gpu_memory_fraction`` from ``SHARED_GPU_MEM_DEV`` /
``_CONTAINER``, a tiny matmul forever).  Here:

* the memory share becomes ``torch.cuda.set_per_process_memory_fraction`` (allocated / device total), so the
  caching allocator refuses to grow past the pod's gpu-mem;
* a CU partition handed out by the device plugin (``GSX_CU_MASK`` words) is applied by running the work on a
  ``hipExtStreamCreateWithCUMask`` stream; ``HSA_CU_MASK`` (set by the plugin too) restricts every queue of the
  process, including torch's own;
* the compute is the bf16 MFMA GEMM of ``libgsx_kernels.so`` (``--kernel gsx``, found next to this file, at
  ``$GSX_KERNELS_LIB``, or in the repository's build tree) or ``torch.matmul`` / hipBLASLt (``--kernel torch``);
  ``auto`` (default) takes the MFMA kernel when the library is there and says so when it falls back.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time
from pathlib import Path

HERE = Path(__file__).resolve().parent


def parse_mask(s: str) -> list[int]:
    return [int(x, 16) for x in s.split(",") if x]


def kernels_lib_path() -> Path | None:
    """libgsx_kernels.so: $GSX_KERNELS_LIB, next to this file (the image), or the repository's build tree."""
    cands = [os.environ.get("GSX_KERNELS_LIB", ""), str(HERE / "libgsx_kernels.so"),
             str(HERE.parents[1] / "gpushare_scheduler_extender_amd" / "_native" / "libgsx_kernels.so")
             if len(HERE.parents) > 1 else ""]
    for c in cands:
        if c and Path(c).is_file():
            return Path(c)
    return None


class Kernels:
    """The slice of libgsx_kernels.so (native/kernels/gsx_kernels.hip) the workload uses."""

    def __init__(self, path: Path):
        L = ctypes.CDLL(str(path))
        vp, u32p, i32 = ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint32), ctypes.c_int
        for name, args in {"gsx_stream_create": [i32, u32p, i32, ctypes.POINTER(vp)], "gsx_stream_destroy": [vp],
                           "gsx_stream_sync": [vp], "gsx_gemm_bf16_nt": [vp, vp, vp, vp, i32, i32, i32]}.items():
            f = getattr(L, name)
            f.argtypes, f.restype = args, i32
        L.gsx_last_error.argtypes, L.gsx_last_error.restype = [], ctypes.c_char_p
        self.L, self.path = L, path

    def _ck(self, rc: int, what: str):
        if rc != 0:
            raise RuntimeError(f"{what}: {(self.L.gsx_last_error() or b'').decode()}")

    def stream(self, dev: int, cu_mask: list[int] | None = None) -> ctypes.c_void_p:
        h = ctypes.c_void_p()
        arr = (ctypes.c_uint32 * len(cu_mask))(*cu_mask) if cu_mask else None
        self._ck(self.L.gsx_stream_create(dev, arr, len(cu_mask or []), ctypes.byref(h)), "stream_create")
        return h

    def gemm(self, s, a: int, b: int, c: int, m: int, n: int, k: int):
        self._ck(self.L.gsx_gemm_bf16_nt(s, ctypes.c_void_p(a), ctypes.c_void_p(b), ctypes.c_void_p(c), m, n, k),
                 "gemm_bf16_nt")

    def sync(self, s):
        self._ck(self.L.gsx_stream_sync(s), "stream_sync")

    def destroy(self, s):
        self.L.gsx_stream_destroy(s)


def run(total: float, allocated: float, *, kernel: str = "auto", size: int = 8192, seconds: float = 0.0,
        iters: int = 0, report_every: float = 5.0, touch: bool = False, quiet: bool = False,
        probe_limit: bool = False) -> dict:
    import torch

    lib_path = kernels_lib_path()
    if kernel == "auto":
        kernel = "gsx" if lib_path is not None else "torch"
        if lib_path is None and not quiet:
            print("[workload] libgsx_kernels.so not found: torch.matmul (hipBLASLt) instead", flush=True)
    kl = None
    if kernel == "gsx" or os.environ.get("GSX_CU_MASK"):
        if lib_path is None:
            if kernel == "gsx":
                raise SystemExit("--kernel gsx: libgsx_kernels.so not found (GSX_KERNELS_LIB, next to main.py)")
        else:
            kl = Kernels(lib_path)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    frac = 1.0 if not total else max(0.0, min(1.0, allocated / total))
    torch.cuda.set_per_process_memory_fraction(frac, dev)
    stream = None
    hip_stream = None
    if os.environ.get("GSX_CU_MASK") and kl is not None:
        hip_stream = kl.stream(0, parse_mask(os.environ["GSX_CU_MASK"]))
        stream = torch.cuda.ExternalStream(hip_stream.value, device=dev)
    hold = None
    if touch:
        # claim (most of) the share so co-resident pods really contend for HBM
        hold = torch.empty(int(allocated * (1 << 30) * 0.9) // 2, dtype=torch.bfloat16, device=dev)
        hold.fill_(1)
    m = n = k = size
    a = torch.randn(m, k, device=dev, dtype=torch.bfloat16)
    b = torch.randn(n, k, device=dev, dtype=torch.bfloat16)
    c = torch.empty(m, n, device=dev, dtype=torch.bfloat16)
    own = None
    if kernel == "gsx":
        gs = hip_stream if hip_stream is not None else kl.stream(0)
        own = None if hip_stream is not None else gs

        def step():
            kl.gemm(gs, a.data_ptr(), b.data_ptr(), c.data_ptr(), m, n, k)

        def sync():
            kl.sync(gs)
    else:
        def step():
            if stream is not None:
                with torch.cuda.stream(stream):
                    torch.matmul(a, b.t(), out=c)
            else:
                torch.matmul(a, b.t(), out=c)

        def sync():
            (stream or torch.cuda.current_stream()).synchronize()
    torch.cuda.synchronize()
    for _ in range(3):
        step()
    sync()
    start_at = float(os.environ.get("GSX_START_AT", "0") or 0)
    if start_at:  # co-resident pods start their timed loops together (isolation bench)
        time.sleep(max(0.0, start_at - time.time()))
    flops = 2.0 * m * n * k
    done = 0
    t0 = last = time.perf_counter()
    last_done = 0
    while True:
        for _ in range(10):
            step()
        done += 10
        sync()
        now = time.perf_counter()
        if now - last >= report_every:
            r = (done - last_done) * flops / (now - last) / 1e12
            if not quiet:
                print(f"[workload] {r:.1f} TFLOP/s  share={allocated}/{total} GiB frac={frac:.3f}", flush=True)
            last, last_done = now, done
        if (seconds and now - t0 >= seconds) or (iters and done >= iters):
            break
    el = time.perf_counter() - t0
    out = {"tflops": done * flops / el / 1e12, "iters": done, "seconds": el, "fraction": frac,
           "cu_mask": os.environ.get("GSX_CU_MASK", ""), "kernel": kernel, "size": size,
           "kernels_lib": str(kl.path) if kl is not None else "",
           "visible_devices": os.environ.get("HIP_VISIBLE_DEVICES", ""),
           "device_total_bytes": torch.cuda.get_device_properties(dev).total_memory}
    if probe_limit and allocated:
        # the share is a ceiling: one more share-sized tensor must be refused by the caching allocator
        try:
            extra = torch.empty(int(allocated * (1 << 30)) // 2, dtype=torch.bfloat16, device=dev)
            del extra
            out["limit_enforced"] = False
        except torch.cuda.OutOfMemoryError:
            out["limit_enforced"] = True
    del hold
    for s in (hip_stream, own):
        if s is not None:
            kl.destroy(s)
    return out


def main(argv=None) -> int:
    p = os.environ.get("GSX_ENV_PREFIX", "SHARED_GPU_MEM")
    ap = argparse.ArgumentParser(description="GEMM loop inside the pod's GPU share (the gpushare sample workload)")
    ap.add_argument("--total", type=float, default=float(os.environ.get(f"{p}_DEV", "0") or 0),
                    help="the GPU's gpu-mem (the device plugin's *_DEV env)")
    ap.add_argument("--allocated", type=float, default=float(os.environ.get(f"{p}_CONTAINER", "0") or 0),
                    help="this container's share (the device plugin's *_CONTAINER env)")
    ap.add_argument("--kernel", default="auto", choices=["auto", "gsx", "torch"])
    ap.add_argument("--size", type=int, default=8192)
    ap.add_argument("--seconds", type=float, default=0.0, help="0 = run forever (like the reference sample)")
    ap.add_argument("--iters", type=int, default=0)
    ap.add_argument("--touch", action="store_true")
    ap.add_argument("--json", action="store_true")
    ap.add_argument("--probe-limit", action="store_true", help="check that the memory share is enforced")
    a = ap.parse_args(argv)
    res = run(a.total, a.allocated, kernel=a.kernel, size=a.size, seconds=a.seconds, iters=a.iters, touch=a.touch,
              quiet=a.json, probe_limit=a.probe_limit)
    print(json.dumps(res) if a.json else res, flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
